#!/usr/bin/env python3
"""The reference's real-graph drivers on the MI355X engine (src/graph_csr.rs:1228-1468).

  chain     bench_real_graphs (:1427-1468): A = CsrMatrix::from_edges (directed), A^k = A^(k-1) * A
            for k = 2..14 with 1 untimed call then ITERS = 1 timed call per step, stopping after the
            first output past MAX_NNZ = 4.4e9. CSV `graph,nodes,edges,step,nnz_out,csr_par_us` plus
            GNNZ/s. Outputs past 2^32 entries run the 64-bit-offset kernels. Every step is checked on
            sampled rows against an exact host restatement (saturating u32 sums of the row's products)
            and, at --check-full sizes, against the oracle's whole product.
  diameter  bench_diameter (:1228-1319): R0 = from_edges_undirected + I, repeated squaring until the
            pattern is stable, then linear refinement; the per-step log of the reference, then
            slat_diameter's answer (the same algorithm as one library call) beside it.

The reference's inputs (gen-graphs/{cora,nell,ogbn_arxiv}.edges) are not in the repository and no
network is available, so the default graphs are seeded synthetic stand-ins: directed R-MAT power-law
graphs (a,b,c = .57,.19,.19). `--edges FILE ...` runs real edge files through load_edges instead.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import slat  # noqa: E402

MAX_POWER = 14
MAX_NNZ = 4_400_000_000
U32MAX = np.uint64(0xFFFFFFFF)


def rmat(scale: int, deg: int, seed: int):
    h = slat.host_rmat(scale, (1 << scale) * deg, seed=bytes([seed] * 32))
    src = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
    return h.n, src, h.col_idx.copy()


def graphs(args):
    for f in args.edges:
        n, s, d = slat.load_edges(f)
        yield os.path.basename(f).split(".")[0], n, s, d
    if not args.edges:
        for spec in args.rmat:
            scale, deg = (int(x) for x in spec.split(":"))
            n, s, d = rmat(scale, deg, args.seed)
            yield f"rmat{scale}_d{deg}", n, s, d


def dev_rows(m, rows):
    """(cols, vals) of the given rows of a device matrix, copied row by row (no full D2H)."""
    L = slat.lib()
    ctx = m._ctx
    v = m.view()
    rp = np.empty(2, np.uint64)
    out = []
    for r in rows:
        L.slat_device_copy(ctx.ptr, rp.ctypes.data, C.c_void_p(v.row_ptr + 8 * int(r)), 16, 1)
        s, e = int(rp[0]), int(rp[1])
        col = np.empty(max(e - s, 1), np.uint32)
        val = np.empty(max(e - s, 1), np.uint32)
        if e > s:
            L.slat_device_copy(ctx.ptr, col.ctypes.data, C.c_void_p(v.col_idx + 4 * s), 4 * (e - s), 1)
            L.slat_device_copy(ctx.ptr, val.ctypes.data, C.c_void_p(v.values + 4 * s), 4 * (e - s), 1)
        out.append((col[:e - s], val[:e - s]))
    return out


def exact_rows(p_rows, a):
    """C[i,:] = sum_k P[i,k] * A[k,:] with CsrMatrix's saturating u32 semantics (src/graph_csr.rs:29-37):
    each product clamped to u32::MAX, the sum clamped (order-free: all values are non-negative)."""
    out = []
    for pc, pv in p_rows:
        if len(pc) == 0:
            out.append((np.zeros(0, np.uint32), np.zeros(0, np.uint32)))
            continue
        s = a.row_ptr[pc].astype(np.int64)
        e = a.row_ptr[pc.astype(np.int64) + 1].astype(np.int64)
        lens = e - s
        idx = np.repeat(s - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        cols = a.col_idx[idx]
        prod = np.minimum(np.repeat(pv.astype(np.uint64), lens) * a.values[idx].astype(np.uint64), U32MAX)
        uc, inv = np.unique(cols, return_inverse=True)
        acc = np.zeros(len(uc), np.uint64)
        np.add.at(acc, inv, prod)
        out.append((uc.astype(np.uint32), np.minimum(acc, U32MAX).astype(np.uint32)))
    return out


def chain(args, ctx):
    print("graph,nodes,edges,step,nnz_out,csr_par_us,gnnz_per_s,idx64,sampled_rows_exact", flush=True)
    rng = np.random.default_rng(5)
    for name, n, s, d in graphs(args):
        A = slat.CsrMatrix.from_edges_device(n, s, d, False, ctx)
        ah = A.host()
        full_ok = None
        if A.nnz() * 1.0 <= args.check_full:
            import oracle_py as O
            oA = O.from_edges(n, np.stack([s, d], 1))
            oP = oA
        prev = A
        for step in range(2, MAX_POWER + 1):
            result = prev.matmul_par(A)  # the reference's first (untimed) call
            nnz_out = result.nnz()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                r2 = prev.matmul_par(A)
                del r2
            t_us = int((time.perf_counter() - t0) * 1e6) // args.iters
            rows = rng.choice(n, size=min(args.sample, n), replace=False)
            got = dev_rows(result, rows)
            want = exact_rows(dev_rows(prev, rows), ah)
            ok = all(np.array_equal(g[0], w[0]) and np.array_equal(g[1], w[1]) for g, w in zip(got, want))
            if A.nnz() * 1.0 <= args.check_full and nnz_out * 1.0 <= args.check_full * 50:
                oP = O.matmul_seq(oP, oA)
                h = result.host()
                rp, col, val = oP.arrays()
                full_ok = bool(np.array_equal(h.row_ptr, rp) and np.array_equal(h.col_idx, col)
                               and np.array_equal(h.values, val))
                ok = ok and full_ok
            idx64 = prev.nnz() >= 0xFFFFFFFF or nnz_out >= 0xFFFFFFFF
            print(f"{name},{n},{len(s)},{step},{nnz_out},{t_us},{nnz_out / max(t_us, 1) / 1e3:.3f},{int(idx64)},"
                  f"{ok}" + ("" if full_ok is None else f" (whole product: {full_ok})"), flush=True)
            if not ok:
                raise AssertionError(f"{name} A^{step}: GPU result differs")
            prev = result
            del result
            if nnz_out > MAX_NNZ:
                break
        if args.past_cap and prev.nnz() >= 0xFFFFFFFF:
            # beyond the reference's protocol: one more product whose LEFT operand holds >= 2^32
            # entries, so the 64-bit-offset kernels run (no timed repeat: memory)
            t0 = time.perf_counter()
            result = prev.matmul_par(A)
            t_us = int((time.perf_counter() - t0) * 1e6)
            rows = rng.choice(n, size=min(args.sample, n), replace=False)
            got = dev_rows(result, rows)
            want = exact_rows(dev_rows(prev, rows), ah)
            ok = all(np.array_equal(g[0], w[0]) and np.array_equal(g[1], w[1]) for g, w in zip(got, want))
            print(f"{name},{n},{len(s)},{step + 1} (past the cap: nnz(A^{step}) = {prev.nnz()}),{result.nnz()},{t_us},"
                  f"{result.nnz() / max(t_us, 1) / 1e3:.3f},1,{ok}", flush=True)
            if not ok:
                raise AssertionError(f"{name} A^{step + 1}: GPU result differs")
            del result
        del prev


def same_pattern(x, y):
    return x.same_pattern(y)


def diameter(args, ctx):
    for name, n, s, d in graphs(args):
        a_sym = slat.CsrMatrix.from_edges_device(n, s, d, True, ctx)
        r0 = a_sym.add(slat.CsrMatrix.identity(n, ctx))
        print(f"\n[{name}] n={n}, edges={len(s)} (undirected nnz={a_sym.nnz()})", flush=True)
        current, reach, prev_saved, prev_reach, squarings = r0.clone(), 1, r0.clone(), 0, 0
        while True:
            t0 = time.perf_counter()
            nxt = current.matmul_par(current)
            t_ms = (time.perf_counter() - t0) * 1e3
            squarings += 1
            print(f"  squaring {squarings}: reach <={reach * 2}, nnz={nxt.nnz()}, {t_ms:.2f} ms", flush=True)
            if same_pattern(nxt, current):
                print(f"  stabilised: diameter in ({prev_reach}, {reach * 2}]")
                break
            prev_saved, prev_reach, current, reach = current, reach, nxt, reach * 2
        if prev_reach == 0:
            d_log = 1
            print("  diameter = 1 (or 0 if isolated nodes)")
        else:
            refine, dd = prev_saved, prev_reach
            while True:
                t0 = time.perf_counter()
                nxt = refine.matmul_par(r0)
                t_ms = (time.perf_counter() - t0) * 1e3
                dd += 1
                print(f"  refine d={dd}: nnz={nxt.nnz()}, {t_ms:.2f} ms", flush=True)
                if same_pattern(nxt, refine):
                    d_log = dd - 1
                    print(f"  diameter = {d_log}")
                    break
                refine = nxt
        t0 = time.perf_counter()
        dlib = a_sym.diameter()
        t_lib = (time.perf_counter() - t0) * 1e3
        print(f"  slat_diameter: {dlib} in {t_lib:.1f} ms; agrees with the log: {dlib[0] == d_log}", flush=True)
        if dlib[0] != d_log:
            raise AssertionError("slat_diameter differs from the logged driver")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["chain", "diameter"])
    ap.add_argument("--edges", nargs="*", default=[], help="edge files (load_edges format) instead of R-MAT")
    ap.add_argument("--rmat", nargs="*", default=["12:8", "17:8"], help="scale:degree of the synthetic graphs")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--past-cap", action="store_true", help="chain: one more step after the 4.4e9 cap (idx64 left operand)")
    ap.add_argument("--sample", type=int, default=64, help="rows checked against the exact restatement per step")
    ap.add_argument("--check-full", type=float, default=2e5,
                    help="also compare whole products with the oracle while nnz(A) is at most this")
    args = ap.parse_args()
    ctx = slat.default_context(0)
    chain(args, ctx) if args.mode == "chain" else diameter(args, ctx)


if __name__ == "__main__":
    main()
