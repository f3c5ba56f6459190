"""Config C4 for a kernel trace: the whole product, then one rank's eighth (rows [0, n/8)), each called
a few times after warm-up, with a host wall time per call; rocprofv3 separates the two by order."""
import sys
import time

sys.path.insert(0, 'sparse-linear-algebra-tests_amd')
import slat  # noqa: E402

ctx = slat.Context(0)
A = slat.torus_thinned_device(100, 3.0, slat.StdRng(), ctx)
P = A.matmul(A).matmul(A)
n = P.n
B = A.prepare() if len(sys.argv) < 2 or sys.argv[1] != "plain" else A  # (plain: B's image built per call)
for label, lo, hi in (("full", 0, n), ("eighth", 0, n // 8)):
    for _ in range(5):
        P.matmul_rowblock(lo, hi, B, 0)
    ctx.sync()
    ts = []
    for i in range(10):
        t0 = time.perf_counter()
        C = P.matmul_rowblock(lo, hi, B, 0)
        ts.append((time.perf_counter() - t0) * 1e3)
        del C
    ts.sort()
    print(f"C4 {label}: median {ts[5]:.4f} ms min {ts[0]:.4f} ms", flush=True)
