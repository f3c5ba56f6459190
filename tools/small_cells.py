#!/usr/bin/env python3
"""Per-call wall time of small products (config C3's small cells: tori of side 5..15 at several e/n,
C = A^2, u32 and Sat64), the one-kernel small path against the regular pipeline (SLAT_FLAG_NO_TINY),
alternating; every result checked against the other path's. Two clocks: through the Python mirror
(_spgemm: views, result object, the previous result's free), and at the C ABI (slat_spgemm +
slat_csr_free on pre-built views: what a Rust caller of include/slat.h pays, plus ~1 us of ctypes)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sparse-linear-algebra-tests_amd"))
import slat  # noqa: E402


def per_call(fn, reps):
    for _ in range(20):
        fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps * 1e6


def abi_call(d, flags):
    from slat import _lib as L
    lib, cp = L.lib(), d._ctx.ptr
    a = d._cview()
    out = L.CsrOwned()
    ra, ro = C.byref(a), C.byref(out)

    def fn():
        st = lib.slat_spgemm(cp, ra, ra, ro, flags)
        lib.slat_csr_free(cp, ro)
        assert st == 0
    return fn


def main():
    ctx = slat.Context(0)
    print("side,epn,dtype,nnz_C,tiny_us,regular_us,tiny_mode,abi_tiny_us,abi_regular_us")
    for side in (5, 10, 15):
        for epn in (2.0, 3.0, 4.0, 8.0, 26.0):
            h = slat.torus_thinned(side, epn, slat.StdRng())
            for name, cls, dt in (("u32", slat.CsrMatrix, slat.U32), ("sat64", slat.MagnusMatrix, slat.SAT64)):
                d = cls.from_host(slat.HostCsr(h.n, h.row_ptr, h.col_idx, h.values.astype(np.uint64 if dt == slat.SAT64 else np.uint32), dt), ctx)
                a, b = d._spgemm(d), d._spgemm(d, slat.FLAG_NO_TINY)
                ha, hb = a.host(), b.host()
                assert all(np.array_equal(x, y) for x, y in ((ha.row_ptr, hb.row_ptr), (ha.col_idx, hb.col_idx), (ha.values, hb.values)))
                d._spgemm(d)
                mode = ctx.stats()["mode"]
                tt = [], [], [], []
                ft, fr = abi_call(d, 0), abi_call(d, slat.FLAG_NO_TINY)
                for _ in range(3):
                    tt[0].append(per_call(lambda: d._spgemm(d), 200))
                    tt[1].append(per_call(lambda: d._spgemm(d, slat.FLAG_NO_TINY), 200))
                    tt[2].append(per_call(ft, 200))
                    tt[3].append(per_call(fr, 200))
                print(f"{side},{epn},{name},{a.nnz()},{min(tt[0]):.1f},{min(tt[1]):.1f},{mode},{min(tt[2]):.1f},{min(tt[3]):.1f}",
                      flush=True)


if __name__ == "__main__":
    main()
