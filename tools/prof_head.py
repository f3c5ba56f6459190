"""The headline step (30^3 torus, C = A^6 * A, u32) for a kernel trace: 20 warm-up calls, then 40 timed
synchronous calls with the host wall time per call."""
import sys
import time

sys.path.insert(0, 'sparse-linear-algebra-tests_amd')
import slat  # noqa: E402

ctx = slat.Context(0)
A = slat.torus_thinned_device(30, 3.0, slat.StdRng(), ctx)
P = A
for _ in range(5):
    P = P.matmul(A)
for _ in range(20):
    P.matmul(A).nnz()
ctx.sync()
t0 = time.perf_counter()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
    C = P.matmul(A)
    C.nnz()
    del C
print(f"headline: {(time.perf_counter() - t0) / (int(sys.argv[1]) if len(sys.argv) > 1 else 40) * 1e3:.4f} ms per call", flush=True)
