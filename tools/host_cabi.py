#!/usr/bin/env python3
"""Per-call time of the headline step (30^3 A^6 * A) and of C1 (A * A) through the Python mirror
(CsrMatrix.matmul, then nnz and the release of C) against the same call made straight through the
C ABI with prebuilt views (slat_spgemm_csr_u32 + slat_csr_free, what a Rust binding pays). Experiments only."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
import slat  # noqa: E402
from slat import _lib as L  # noqa: E402


def per_call(fn, reps):
    for _ in range(50):
        fn()
    slat.default_context(0).sync()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        best = min(best, (time.perf_counter() - t) / reps * 1e6)
    return best


ctx = slat.default_context(0)
A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()), ctx)
P = A
for _ in range(5):
    P = P.matmul(A)
lib = L.lib()
for name, X in (("A^6*A", P), ("C1 A*A", A)):
    def mirror():
        c = X.matmul(A)
        c.nnz()
        del c
    xa, xb = X._cview(), A._cview()
    out = L.CsrOwned()

    def direct():
        st = lib.slat_spgemm_csr_u32(ctx.ptr, C.byref(xa), C.byref(xb), C.byref(out), 0)
        if st:
            raise RuntimeError(st)
        _ = out.nnz
        lib.slat_csr_free(ctx.ptr, C.byref(out))
    reps = 400 if name.startswith("C1") else 200
    print(f"{name}: python mirror {per_call(mirror, reps):.1f} us/call, C ABI {per_call(direct, reps):.1f} us/call",
          flush=True)
