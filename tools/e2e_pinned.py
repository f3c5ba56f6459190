#!/usr/bin/env python3
"""The drop-in's host-resident call with page-locked operands and a pooled page-locked output (bench.py's
e2e "pinned" leg) on the headline step (30^3 torus, C = A^6 * A, u32), split: H2D of A^6, the whole
call, D2H of C alone. One JSON line per library (SLAT_LIB_PATH)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
import numpy as np  # noqa: E402

import slat  # noqa: E402


def med(fn, n=15):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 3), round(ts[0], 3)


def main():
    ctx = slat.default_context(0)
    A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()), ctx)
    P = A
    for _ in range(5):
        P = P.matmul(A)

    def pin(x):
        y = slat.pinned_empty(len(x), x.dtype)
        y[:] = x
        return y
    hP0, hA0 = P.host(), A.host()
    pP = slat.HostCsr(hP0.n, pin(hP0.row_ptr), pin(hP0.col_idx), pin(hP0.values), hP0.dtype)
    pA = slat.HostCsr(hA0.n, pin(hA0.row_ptr), pin(hA0.col_idx), pin(hA0.values), hA0.dtype)
    pool, seq = {}, [0]

    def pooled(n, dt):  # one buffer per (position in the call: row_ptr, col, val; size), reused
        key = (seq[0] % 3, n, np.dtype(dt).str)
        seq[0] += 1
        if key not in pool:
            pool[key] = slat.pinned_empty(n, dt)
        return pool[key]
    out = {"lib": os.environ.get("SLAT_LIB_PATH", "libslat.so")}
    out["e2e_pinned_ms"] = med(lambda: slat.spgemm_host(pP, pA, ctx, alloc=pooled))
    out["h2d_P_pinned_ms"] = med(lambda: slat.CsrMatrix.from_host(pP, ctx))
    C = P.matmul(A)
    out["product_ms"] = med(lambda: P.matmul(A))
    import ctypes
    from slat import _lib as L
    seq[0] = 0
    rp, col, val = pooled(C.n + 1, np.uint64), pooled(max(C.nnz(), 1), np.uint32), pooled(max(C.nnz(), 1), np.uint32)

    def d2h():
        v = L.lib().slat_csr_view_of(ctypes.byref(C._m))
        L.check(L.lib().slat_csr_to_host(ctx.ptr, ctypes.byref(v), rp.ctypes.data, col.ctypes.data, val.ctypes.data),
                ctx.ptr)
    out["d2h_C_pinned_ms"] = med(d2h)
    d2h()
    h = C.host()
    out["same"] = bool(np.array_equal(rp, h.row_ptr) and np.array_equal(col[:C.nnz()], h.col_idx) and
                       np.array_equal(val[:C.nnz()], h.values))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
