#!/usr/bin/env python3
"""The drop-in's host-resident call on the headline step (C = A^6 * A, 30^3 torus, u32): H2D of both
operands, the product, D2H of C into fresh pageable numpy arrays (np.empty per call, as a Rust Vec),
plus the two copies alone. One JSON line; run once per library (SLAT_LIB_PATH) / knob setting.
--mean K: the mean over K calls after one warm-up (bench.py's e2e timing) as e2e_mean_ms too."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
import numpy as np  # noqa: E402

import slat  # noqa: E402


def med(fn, n=10):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 3), round(ts[0], 3)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--mean", type=int, default=0)
    ap.add_argument("--quick", action="store_true", help="the end-to-end call only")
    args = ap.parse_args()
    ctx = slat.default_context(0)
    A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()), ctx)
    P = A
    for _ in range(5):
        P = P.matmul(A)
    hP0, hA0 = P.host(), A.host()
    hP = slat.HostCsr(hP0.n, hP0.row_ptr.copy(), hP0.col_idx.copy(), hP0.values.copy(), hP0.dtype)
    hA = slat.HostCsr(hA0.n, hA0.row_ptr.copy(), hA0.col_idx.copy(), hA0.values.copy(), hA0.dtype)
    C = P.matmul(A)
    out = {"lib": os.environ.get("SLAT_LIB_PATH", "libslat.so"), "mode": os.environ.get("SLAT_HOSTIO", "ring"),
           "threads": os.environ.get("SLAT_HOST_THREADS", "default")}
    nnz = [0]

    def e2e():
        nnz[0] = slat.spgemm_host(hP, hA, ctx).nnz

    out["e2e_ms"] = med(e2e)
    if args.mean:
        e2e()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(args.mean):
            e2e()
        ctx.sync()
        out["e2e_mean_ms"] = round((time.perf_counter() - t0) / args.mean * 1e3, 4)
    if args.quick:
        out["nnz"] = nnz[0]
        print(json.dumps(out), flush=True)
        return
    out["h2d_P_ms"] = med(lambda: slat.CsrMatrix.from_host(hP, ctx))

    def d2h():
        C._host = None
        C.host()
    out["d2h_C_ms"] = med(d2h)
    out["nnz"] = nnz[0]
    h = slat.spgemm_host(hP, hA, ctx)
    w = C.host()
    out["same"] = bool(np.array_equal(h.row_ptr, w.row_ptr) and np.array_equal(h.col_idx, w.col_idx) and
                       np.array_equal(h.values, w.values))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
