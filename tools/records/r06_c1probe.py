import os, sys, time
sys.path.insert(0, "sparse-linear-algebra-tests_amd")
import slat
ctx = slat.Context(0)
A = slat.torus_thinned_device(30, 3.0, slat.StdRng(), ctx)
for _ in range(300):
    A.matmul(A).nnz()
ctx.sync()
t = time.perf_counter()
for _ in range(512):
    C = A.matmul(A); C.nnz(); del C
ctx.sync()
print(f"C1 {(time.perf_counter() - t) / 512 * 1e6:.1f} us per call (python)")
