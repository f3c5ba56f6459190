#!/usr/bin/env python3
"""Host-side cost of one SpGEMM call: a tiny product (fixed overhead: API + launches + sync) and the
phases of bench.py's step on its workload. Experiments only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
import numpy as np  # noqa: E402

import slat  # noqa: E402


def per_call(fn, reps=200):
    for _ in range(10):
        fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps * 1e6


ctx = slat.Context(0)
T = slat.CsrMatrix.from_host(slat.torus_thinned(4, 3.0, slat.StdRng()), ctx)
print(f"tiny 4^3 A*A: {per_call(lambda: T.matmul(T)):.1f} us/call, "
      f"with TIMING {per_call(lambda: T._spgemm(T, slat.FLAG_TIMING)):.1f} us/call")
A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()), ctx)
P = A
for _ in range(5):
    P = P.matmul(A)
n = A.n
ph = np.zeros(4)
for i in range(60):
    t0 = time.perf_counter()
    C = P.matmul_rowblock(0, n, A, slat.FLAG_TIMING)
    t1 = time.perf_counter()
    C.nnz()
    del C
    t2 = time.perf_counter()
    st = ctx.stats()
    t3 = time.perf_counter()
    if i >= 10:
        ph += [t1 - t0, t2 - t1, t3 - t2, t3 - t0]
ph = ph / 50 * 1e6
print(f"A^6*A step: call {ph[0]:.1f} us, nnz+free {ph[1]:.1f} us, stats {ph[2]:.1f} us, total {ph[3]:.1f} us; "
      f"device_total {st['total_ms'] * 1e3:.1f} us, numeric {st['numeric_ms'] * 1e3:.1f} us")
