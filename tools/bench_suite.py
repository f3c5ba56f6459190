#!/usr/bin/env python3
"""Every BASELINE.json config on one MI355X, next to the oracle's matmul_par on the host cores.

  C1  30^3 torus (3 e/n, seed [42;32]) A^2, u32                    (configs[0])
  C2  30^3 torus A^2 ... A^7 repeated exponentiation, u32          (configs[1]; bench.py's headline is A^7)
  C3  the bench_matmul_magnus sweep: sides {5,10,20,30} x e/n {2,3,4,8,26}, one StdRng shared
      across the grid (src/graph_magnus.rs:792-929), A^2 per cell, u32   (configs[2])
  C4  100^3 torus A^3 * A on ONE GPU (the 8-GPU strong-scaling case's single-GPU point)  (configs[3])
  C5  f64 R-MAT power-law graph (a,b,c = .57,.19,.19), A * A, bit-exact vs the oracle   (configs[4])

GPU time per cell = mean wall time of synchronous device-resident calls (warm-up first), the same
region bench.py times; the numeric kernel's HIP-event time gives the roofline fraction
(SURVEY.md §8(d) algorithmic bytes / kernel time / 8 TB/s). CPU = oracle/oracle.c orc_matmul_par
(the restated CsrMatrix::matmul_par) on `--threads` host threads. Every GPU result is checked
against the CPU result of the same cell (bit-exact arrays). Writes JSON to --out and a markdown
table to stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402  (the CPU baseline and checker only)
import slat  # noqa: E402

HBM = 8000.0


def alg_bytes(za, zb, zc, n, vs):
    return (4 + vs) * (za + zb + zc) + 8 * 3 * (n + 1)


def gpu_time(fn, warm=3, iters=20, min_s=0.05):
    for _ in range(warm):
        fn()
    n, t0 = 0, time.perf_counter()
    while n < iters or time.perf_counter() - t0 < min_s:
        fn()
        n += 1
    return (time.perf_counter() - t0) / n


def cpu_time(fn, budget_s, max_iters=10):
    fn()  # warm-up (the reference: 1 warm-up + timed iterations)
    n, t0 = 0, time.perf_counter()
    while n < 1 or (n < max_iters and time.perf_counter() - t0 < budget_s):
        fn()
        n += 1
    return (time.perf_counter() - t0) / n


def to_dev(o: O.Csr, cls, ctx):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, cls.DTYPE), ctx)


def same(dev, orc, rtol=0.0) -> bool:
    h = dev.host()
    rp, col, val = orc.arrays()
    if rtol:
        return (np.array_equal(h.row_ptr, rp) and np.array_equal(h.col_idx, col)
                and np.allclose(h.values, val, rtol=rtol, atol=0))
    if val.dtype == np.float64:
        return (np.array_equal(h.row_ptr, rp) and np.array_equal(h.col_idx, col)
                and np.array_equal(h.values.view(np.uint64), val.view(np.uint64)))
    return np.array_equal(h.row_ptr, rp) and np.array_equal(h.col_idx, col) and np.array_equal(h.values, val)


def cell(name, dA, dB, oA, oB, args, vs=4, check=True, flags=0, rtol=0.0):
    """One product: GPU time, kernel times, CPU time, parity (bit-exact, or within rtol)."""
    ctx = dA._ctx
    C = dA._spgemm(dB, slat.FLAG_TIMING | flags)
    nnz = C.nnz()
    t_gpu = gpu_time(lambda: dA._spgemm(dB, flags).nnz())
    # kernel times: a few TIMING calls
    ks = []
    for _ in range(5):
        dA._spgemm(dB, slat.FLAG_TIMING | flags)
        ks.append(ctx.stats())
    num_ms = float(np.median([k["numeric_ms"] for k in ks]))
    dev_ms = float(np.median([k["total_ms"] for k in ks]))
    n = oA.n
    byt = alg_bytes(oA.nnz, oB.nnz, nnz, n, vs)
    rec = {"cell": name, "n": n, "nnz_a": oA.nnz, "nnz_b": oB.nnz, "nnz_c": nnz, "gpu_ms": t_gpu * 1e3,
           "gnnz_s": nnz / t_gpu / 1e9, "numeric_ms": num_ms, "device_ms": dev_ms,
           "numeric_hbm_frac": byt / (num_ms * 1e-3) / 1e9 / HBM if num_ms > 0 else None,
           "pipeline_hbm_frac": byt / (dev_ms * 1e-3) / 1e9 / HBM if dev_ms > 0 else None,
           "alg_bytes": byt}
    if args.cpu and oA.nnz * 1.0 < args.cpu_max_nnz:
        want = O.matmul_par(oA, oB, args.threads)
        t_cpu = cpu_time(lambda: O.matmul_par(oA, oB, args.threads), args.cpu_budget)
        rec.update({"cpu_ms": t_cpu * 1e3, "cpu_gnnz_s": nnz / t_cpu / 1e9, "speedup": t_cpu / t_gpu})
        if check:
            rec["bit_exact" if not rtol else f"within_rtol_{rtol:g}"] = bool(same(C, want, rtol))
    print(json.dumps(rec), file=sys.stderr, flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/suite.json")
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
    ap.add_argument("--cpu-budget", type=float, default=2.0, help="seconds of timed CPU calls per cell")
    ap.add_argument("--cpu-max-nnz", type=float, default=3e7, help="skip the CPU leg above this nnz(A)")
    ap.add_argument("--no-cpu", dest="cpu", action="store_false")
    ap.add_argument("--only", default="GEN,C1,C2,C3,C4,C5,RG,DN")
    ap.add_argument("--rmat-scale", type=int, default=16)
    ap.add_argument("--rmat-deg", type=int, default=16)
    args = ap.parse_args()
    only = set(args.only.split(","))
    ctx = slat.Context(0)
    out = {"threads": args.threads, "cells": []}
    M = slat.CsrMatrix

    if "GEN" in only:
        # the reference's input generators (lattice + thin, seed [42;32]): host library vs device
        for side in (30, 100):
            t0 = time.perf_counter()
            h = slat.torus_thinned(side, 3.0, slat.StdRng())
            th = time.perf_counter() - t0
            d = slat.torus_thinned_device(side, 3.0, slat.StdRng(), ctx)  # warm-up
            t0 = time.perf_counter()
            d = slat.torus_thinned_device(side, 3.0, slat.StdRng(), ctx)
            td = time.perf_counter() - t0
            same_arrays = bool(np.array_equal(d.host().col_idx, h.col_idx) and np.array_equal(d.host().row_ptr, h.row_ptr))
            rec = {"cell": f"GEN torus{side} thinned 3 e/n", "n": h.n, "nnz_c": h.nnz, "host_ms": th * 1e3,
                   "device_ms": td * 1e3, "identical": same_arrays}
            print(json.dumps(rec), file=sys.stderr, flush=True)
            out.setdefault("generators", []).append(rec)
    if only & {"C1", "C2"}:
        oA = O.torus_thinned(30, 3.0, O.Rng())
        dA = to_dev(oA, M, ctx)
        oP, dP = oA, dA
        for k in range(2, 8):
            if k > 2 and "C2" not in only:
                break
            out["cells"].append(cell(f"C{1 if k == 2 else 2} torus30 A^{k}", dP, dA, oP, oA, args))
            oP = O.matmul_seq(oP, oA)
            dP = dP.matmul(dA)
    if "C3" in only:
        rng = O.Rng()  # ONE rng shared across the grid (src/graph_magnus.rs:800)
        for s in [5, 10, 20, 30]:
            full = O.lattice([s, s, s], True)
            for epn in [2.0, 3.0, 4.0, 8.0, 26.0]:
                density = epn / (full.nnz / full.n)
                oA = O.thin(full, rng, density) if density < 1.0 else full
                dA = to_dev(oA, M, ctx)
                out["cells"].append(cell(f"C3 sweep side={s} e/n={epn:g}", dA, dA, oA, oA, args))
    if "C4" in only:
        oA = O.torus_thinned(100, 3.0, O.Rng())
        dA = to_dev(oA, M, ctx)
        dP = dA.matmul(dA).matmul(dA)
        h = dP.host()
        oP = O.from_arrays(h.row_ptr, h.col_idx, h.values, O.U32) if args.cpu else _shape(h)
        out["cells"].append(cell("C4 torus100 A^3*A (1 GPU)", dP, dA, oP, oA, args))
    if "C5" in only:
        scale, deg = args.rmat_scale, args.rmat_deg
        h = slat.host_rmat(scale, (1 << scale) * deg)
        oA = O.from_arrays(h.row_ptr, h.col_idx, h.values, O.F64)
        dA = slat.CsrF64.from_host(h, ctx)
        out["cells"].append(cell(f"C5 rmat scale={scale} deg={deg} f64 A*A, any order (rtol 1e-12)", dA, dA, oA, oA,
                                 args, vs=8, flags=slat.FLAG_F64_ANY_ORDER, rtol=1e-12))
        out["cells"].append(cell(f"C5 rmat scale={scale} deg={deg} f64 A*A, reference fold order", dA, dA, oA, oA,
                                 args, vs=8))
    if "RG" in only:
        # the real-graph path (bench_real_graphs / analyze_graph_structure, src/graph_csr.rs:1427-1549)
        # on synthetic stand-ins (the .edges files are absent): a power-law R-MAT graph made
        # undirected, and a randomly numbered 50^3 torus. Edges -> device CSR, RCM, A^2 before/after.
        g = np.random.default_rng(11)
        h = slat.host_rmat(16, (1 << 16) * 8)
        rows = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
        t = O.torus_thinned(50, 3.0, O.Rng())
        tp = g.permutation(t.n).astype(np.uint32)
        inv = np.empty_like(tp)
        inv[tp] = np.arange(t.n, dtype=np.uint32)
        trp, tcol, _ = t.arrays()
        trows = np.repeat(np.arange(t.n, dtype=np.uint32), np.diff(trp).astype(np.int64))
        for name, n, src, dst in [("rmat16 undirected", h.n, rows, h.col_idx),
                                  ("torus50 renumbered", t.n, inv[trows], inv[tcol])]:
            t0 = time.perf_counter()
            dA = M.from_edges_device(n, src, dst, True, ctx)
            t_build = time.perf_counter() - t0
            oA = O.from_edges_undirected(n, np.stack([src, dst], 1)) if args.cpu else None
            bw0 = dA.bandwidth_stats()
            t0 = time.perf_counter()
            p = dA.rcm_order()
            t_order = time.perf_counter() - t0
            dR = dA.clone()
            t0 = time.perf_counter()
            dR.permute(p)
            t_perm = time.perf_counter() - t0
            bw1 = dR.bandwidth_stats()
            rec = {"graph": name, "n": n, "nnz": dA.nnz(), "from_edges_ms": t_build * 1e3, "rcm_order_ms": t_order * 1e3,
                   "permute_ms": t_perm * 1e3, "bandwidth_before": bw0, "bandwidth_after": bw1}
            if oA is not None:
                rec["from_edges_exact"] = bool(same(dA, oA))
                rec["rcm_order_equal"] = bool(np.array_equal(p, O.rcm_order(oA)))
                oR = O.permute(oA, p)
            else:
                oR = _shape(dR.host())
                oA = _shape(dA.host())
            c0 = cell(f"RG {name} A^2", dA, dA, oA, oA, args)
            c1 = cell(f"RG {name} A^2 after RCM", dR, dR, oR, oR, args)
            rec.update({"a2_ms": c0["gpu_ms"], "a2_rcm_ms": c1["gpu_ms"]})
            out["cells"] += [c0, c1]
            print(json.dumps(rec), file=sys.stderr, flush=True)
            out.setdefault("real_graph", []).append(rec)
    if "DN" in only:
        # einsum_sparse_driven (einsum-dyn/src/sparse.rs:70-148): sparse x sparse into a dense
        # output resident on the device (a library buffer), checked against the oracle
        Cc = slat._lib.C
        oA = O.torus_thinned(30, 3.0, O.Rng())
        dA = to_dev(oA, M, ctx)
        oP = O.matmul_seq(O.matmul_seq(oA, oA), oA)
        dP = to_dev(oP, M, ctx)
        h = slat.host_rmat(14, (1 << 14) * 16)
        oR = O.from_arrays(h.row_ptr, h.col_idx, h.values, O.F64)
        dR = slat.CsrF64.from_host(h, ctx)
        for name, da, db, oa, ob, ndt in [("torus30 A*A u32", dA, dA, oA, oA, np.uint32),
                                          ("torus30 A^3*A u32", dP, dA, oP, oA, np.uint32),
                                          ("rmat14 A*A f64", dR, dR, oR, oR, np.float64)]:
            n = oa.n
            got = np.zeros((n, n), ndt)
            buf = Cc.c_void_p()
            slat.lib().slat_device_alloc(ctx.ptr, got.nbytes, Cc.byref(buf))
            slat.lib().slat_device_copy(ctx.ptr, buf, got.ctypes.data, got.nbytes, 0)

            def call():
                va, vb = da.view(), db.view()
                rc = slat.lib().slat_spgemm_dense(ctx.ptr, Cc.byref(va), Cc.byref(vb), buf, n, 0, slat.DEVICE)
                assert rc == 0
            call()
            t = gpu_time(call)
            slat.lib().slat_device_copy(ctx.ptr, got.ctypes.data, buf, got.nbytes, 1)
            slat.lib().slat_device_free(ctx.ptr, buf)
            want = O.einsum_sparse_driven(oa, ob, np.zeros((n, n), ndt))
            same_ = bool(np.array_equal(got.view(np.uint64) if ndt == np.float64 else got,
                                        want.view(np.uint64) if ndt == np.float64 else want))
            products = O.flops(oa, ob)
            rec = {"cell": f"DN {name}", "n": n, "gpu_ms": t * 1e3, "products": products,
                   "gprod_s": products / t / 1e9, "bit_exact": same_}
            if args.cpu:
                tc = cpu_time(lambda: O.einsum_sparse_driven(oa, ob, np.zeros((n, n), ndt)), args.cpu_budget, 3)
                rec.update({"cpu_1thr_ms": tc * 1e3, "speedup": tc / t})
            print(json.dumps(rec), file=sys.stderr, flush=True)
            out.setdefault("dense_out", []).append(rec)

    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"| cell | nnz(C) | GPU ms | GNNZ/s | numeric HBM frac | pipeline HBM frac | CPU ms ({args.threads} thr) "
          f"| CPU GNNZ/s | speedup | bit-exact |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in out["cells"]:
        f = lambda k, fmt: (fmt % r[k]) if r.get(k) is not None else "-"  # noqa: E731
        print(f"| {r['cell']} | {r['nnz_c']} | {r['gpu_ms']:.3f} | {r['gnnz_s']:.2f} | {f('numeric_hbm_frac', '%.3f')} "
              f"| {f('pipeline_hbm_frac', '%.3f')} | {f('cpu_ms', '%.2f')} | {f('cpu_gnnz_s', '%.3f')} "
              f"| {f('speedup', '%.0f')} | {r.get('bit_exact', r.get('within_rtol_1e-12', '-'))} |")
    for r in out.get("real_graph", []):
        print(f"\n{r['graph']}: n {r['n']}, nnz {r['nnz']}; from_edges {r['from_edges_ms']:.1f} ms, rcm order (host) "
              f"{r['rcm_order_ms']:.1f} ms, permute {r['permute_ms']:.1f} ms; bandwidth max/avg {r['bandwidth_before'][0]}/"
              f"{r['bandwidth_before'][1]:.0f} -> {r['bandwidth_after'][0]}/{r['bandwidth_after'][1]:.0f}; "
              f"A^2 {r['a2_ms']:.3f} -> {r['a2_rcm_ms']:.3f} ms; exact {r.get('from_edges_exact', '-')}, "
              f"same order {r.get('rcm_order_equal', '-')}")
    for r in out.get("dense_out", []):
        print(f"\n{r['cell']}: GPU {r['gpu_ms']:.3f} ms ({r['gprod_s']:.2f} G products/s), "
              f"oracle 1 thread {r.get('cpu_1thr_ms', float('nan')):.1f} ms, bit-exact {r['bit_exact']}")
    for g in out.get("generators", []):
        print(f"\n{g['cell']}: host library {g['host_ms']:.1f} ms, device {g['device_ms']:.1f} ms, identical {g['identical']}")


class _shape:
    """n / nnz of a host matrix (cells whose CPU leg is skipped)."""

    def __init__(self, h):
        self.n, self.nnz = h.n, h.nnz


if __name__ == "__main__":
    main()
