#!/usr/bin/env python3
"""The reference's two benchmark harnesses, re-run with the MI355X engine in the reference's CSV format.

  sweep   bench_matmul_magnus (src/graph_magnus.rs:792-929): sides {5,10,20,30} x e/n {2,3,4,8,26},
          ONE StdRng([42;32]) shared across the grid in loop order (the BTreeMap-path `thin`, no
          draws at e/n 26), C = A^2 per cell; 1 warm-up call whose results are cross-checked (equal
          nnz everywhere, equal values on the first 10x10 block, :859-880), then 10 timed calls per
          implementation, mean in integer microseconds. Header = README.md:21, so the reference's
          plot_surface.py reads the output unchanged. Labelled extension cells follow in a second
          block (not in the reference grid): larger tori and CsrMatrix::random graphs, nnz(C) up to
          ~50M (BASELINE.json config 3's "random graph, nnz 10k-50M").
  repeat  bench_repeated_exponentiation (src/graph_magnus.rs:701-788): 30^3 torus thinned to 3 e/n,
          A^k = A^(k-1) * A for k = 2..7; 1 warm-up + 3 timed calls per implementation. Header =
          :734, plus the engine's columns (GNNZ/s and the numeric kernel's HBM roofline fraction).

Column mapping (the reference's implementations are Rust and cannot run here; each column names the
implementation that stands in for it):
  orig_btree_us  oracle/oracle.c CsrMatrix::matmul restatement, 1 thread (no BTreeMap port: the
                 slowest baseline this repo has; x_* columns divide it by each time)
  csr_us         GPU CsrMatrix::matmul      (slat_spgemm_csr_u32)
  csr_par_us     GPU CsrMatrix::matmul_par  (the same engine call: the reference's seq and par give
                 equal results)
  sprs_us        oracle CsrMatrix::matmul_par restatement on --threads host threads
  magnus_seq_us  GPU MagnusMatrix::matmul_seq (slat_spgemm_csr_sat64, Sat64 values)
  magnus_par_us  GPU MagnusMatrix::matmul     (the same Sat64 engine call)
In `repeat`, csr_us / csr_par_us are the oracle's seq / par restatements (the columns the README
table's CSR seq / CSR par figures come from) and magnus_seq_us / magnus_par_us the GPU Sat64 path;
gpu_u32_us is the GPU CsrMatrix path. Every GPU result is checked bit-exact against the oracle.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402  (the CPU baselines and the checker only)
import slat  # noqa: E402

HBM = 8000.0
SWEEP_HEADER = ("side,nodes,e_per_n,nnz,components,orig_btree_us,csr_us,csr_par_us,sprs_us,magnus_seq_us,"
                "magnus_par_us,x_csr,x_csr_par,x_sprs,x_magnus_seq,x_magnus_par")
EXTRA = "gnnz_per_s,hbm_gbps,roofline_frac,n_gpus"
REPEAT_HEADER = "step,nnz,csr_us,csr_par_us,magnus_seq_us,magnus_par_us,x_csr_par,x_magnus_seq,x_magnus_par"


def mean_us(fn, iters: int) -> int:
    """The reference's timing: Instant around `iters` calls, integer division (src/graph_magnus.rs:884-906)."""
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return int((time.perf_counter() - t0) * 1e6) // iters


def components(o: O.Csr) -> int:
    """CsrMatrix::num_components (src/graph_csr.rs:605-657): union-find over the entries as undirected edges."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components
    rp, col, val = o.arrays()
    m = csr_matrix((np.ones(len(col)), col.astype(np.int64), rp.astype(np.int64)), shape=(o.n, o.n))
    return int(connected_components(m, directed=False)[0])


def dev(o: O.Csr, cls, ctx):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, slat.U32).astype(cls.DTYPE), ctx)


def check(got, want: O.Csr, what: str):
    h = got.host()
    rp, col, val = want.arrays()
    ok = (np.array_equal(h.row_ptr, rp) and np.array_equal(h.col_idx, col)
          and np.array_equal(h.values.astype(np.uint64), val.astype(np.uint64)))
    if not ok:
        raise AssertionError(f"{what}: GPU result differs from the oracle")


def numeric_frac(P, B, nnz_c: int, vs: int) -> tuple[float, float]:
    """numeric kernel HIP-event time -> (achieved GB/s, fraction of 8 TB/s) on SURVEY §8(d) bytes."""
    ms = []
    for _ in range(5):
        P._spgemm(B, slat.FLAG_TIMING)
        ms.append(P._ctx.stats()["numeric_ms"])
    t = float(np.median(ms)) * 1e-3
    byt = (4 + vs) * (P.nnz() + B.nnz() + nnz_c) + 8 * 3 * (P.n + 1)
    gbs = byt / t / 1e9 if t > 0 else float("nan")
    return gbs, gbs / HBM


def sweep_cell(label, s, epn, oA, args, ctx):
    n = oA.n
    dA = dev(oA, slat.CsrMatrix, ctx)
    mA = dev(oA, slat.MagnusMatrix, ctx)
    # warm-up + verification (one call each)
    want = O.matmul_seq(oA, oA)
    c_csr, c_par = dA.matmul(dA), dA.matmul_par(dA)
    c_mseq, c_mpar = mA.matmul_seq(mA), mA.matmul(mA)
    want_par = O.matmul_par(oA, oA, args.threads)
    for c in (c_csr, c_par, c_mseq, c_mpar):
        assert c.nnz() == want.nnz == want_par.nnz, f"nnz mismatch (s={s}, epn={epn})"
    for c in (c_csr, c_par, c_mseq, c_mpar):
        check(c, want, f"s={s} e/n={epn}")
    nnz_c = want.nnz
    del c_csr, c_par, c_mseq, c_mpar
    it = args.iters
    t_bt = mean_us(lambda: O.matmul_seq(oA, oA), it)
    t_csr = mean_us(lambda: dA.matmul(dA).nnz(), it)
    t_par = mean_us(lambda: dA.matmul_par(dA).nnz(), it)
    t_sprs = mean_us(lambda: O.matmul_par(oA, oA, args.threads), it)
    t_mseq = mean_us(lambda: mA.matmul_seq(mA).nnz(), it)
    t_mpar = mean_us(lambda: mA.matmul(mA).nnz(), it)
    x = lambda t: f"{t_bt / t:.4f}" if t > 0 else "inf"  # noqa: E731
    gbs, frac = numeric_frac(dA, dA, nnz_c, 4)
    gnnz = nnz_c / max(t_par, 1) / 1e3
    return (f"{s},{n},{epn:.0f},{oA.nnz},{components(oA)},{t_bt},{t_csr},{t_par},{t_sprs},{t_mseq},{t_mpar},"
            f"{x(t_csr)},{x(t_par)},{x(t_sprs)},{x(t_mseq)},{x(t_mpar)},{gnnz:.4f},{gbs:.1f},{frac:.4f},1")


def sweep(args, ctx):
    print(f"# bench_matmul_magnus grid (src/graph_magnus.rs:792-929) on the MI355X engine; {args.threads} host threads;"
          f" 1 warm-up + {args.iters} timed calls; columns: see tools/bench_protocol.py")
    print(SWEEP_HEADER + "," + EXTRA, flush=True)
    rng = O.Rng()  # ONE rng across the grid (src/graph_magnus.rs:800)
    for s in [5, 10, 20, 30]:
        full = O.lattice([s, s, s], True)
        for epn in [2.0, 3.0, 4.0, 8.0, 26.0]:
            density = epn / (full.nnz / full.n)
            oA = O.thin(full, rng, density) if density < 1.0 else full
            print(sweep_cell("grid", s, epn, oA, args, ctx), flush=True)
    if args.extension:
        print("# extension cells (NOT in the reference grid): larger tori, fresh StdRng([42;32]) per side, and"
              " CsrMatrix::random(n, m) graphs (src/graph_csr.rs:163-174; side column = 0)")
        print(SWEEP_HEADER + "," + EXTRA, flush=True)
        for s in args.ext_sides:
            full = O.lattice([s, s, s], True)
            rng = O.Rng()
            for epn in [2.0, 3.0, 4.0, 8.0]:
                density = epn / (full.nnz / full.n)
                oA = O.thin(full, rng, density)
                print(sweep_cell("ext", s, epn, oA, args, ctx), flush=True)
        rng = O.Rng()
        for n, m in args.ext_random:
            oA = O.random(rng, n, m)
            print(sweep_cell("ext", 0, m / n, oA, args, ctx), flush=True)


def repeat(args, ctx):
    print(f"# bench_repeated_exponentiation (src/graph_magnus.rs:701-788) on the MI355X engine: 30^3 torus, 3 e/n,"
          f" seed [42;32]; 1 warm-up + {args.repeat_iters} timed calls; csr_us / csr_par_us = oracle seq / par on"
          f" {args.threads} host threads, magnus_* = GPU Sat64 (MagnusMatrix), gpu_u32_us = GPU CsrMatrix")
    print(REPEAT_HEADER + ",gpu_u32_us,x_gpu_u32,sat64_gnnz_per_s,sat64_roofline_frac,u32_gnnz_per_s,u32_roofline_frac",
          flush=True)
    oA = O.torus_thinned(30, 3.0, O.Rng())
    dA, mA = dev(oA, slat.CsrMatrix, ctx), dev(oA, slat.MagnusMatrix, ctx)
    oP, dP, mP = oA, dA, mA
    for step in range(2, 8):
        want = O.matmul_seq(oP, oA)
        r_par = O.matmul_par(oP, oA, args.threads)
        r_u32, r_mseq, r_mpar = dP.matmul(dA), mP.matmul_seq(mA), mP.matmul(mA)
        for c in (r_u32, r_mseq, r_mpar):
            assert c.nnz() == want.nnz == r_par.nnz, f"step {step}: nnz mismatch"
            check(c, want, f"A^{step}")
        it = args.repeat_iters
        t_csr = mean_us(lambda: O.matmul_seq(oP, oA), it)
        t_par = mean_us(lambda: O.matmul_par(oP, oA, args.threads), it)
        t_mseq = mean_us(lambda: mP.matmul_seq(mA).nnz(), it)
        t_mpar = mean_us(lambda: mP.matmul(mA).nnz(), it)
        t_u32 = mean_us(lambda: dP.matmul(dA).nnz(), it)
        x = lambda t: f"{t_csr / t:.4f}" if t > 0 else "inf"  # noqa: E731
        _, f64frac = numeric_frac(mP, mA, want.nnz, 8)
        _, u32frac = numeric_frac(dP, dA, want.nnz, 4)
        # GNNZ/s from longer runs than the 3-call protocol (the GPU clocks up under load)
        tg_m = mean_us(lambda: mP.matmul(mA).nnz(), 50)
        tg_u = mean_us(lambda: dP.matmul(dA).nnz(), 50)
        print(f"{step},{want.nnz},{t_csr},{t_par},{t_mseq},{t_mpar},{x(t_par)},{x(t_mseq)},{x(t_mpar)},{t_u32},"
              f"{x(t_u32)},{want.nnz / max(tg_m, 1) / 1e3:.3f},{f64frac:.4f},{want.nnz / max(tg_u, 1) / 1e3:.3f},"
              f"{u32frac:.4f}", flush=True)
        oP, dP, mP = want, r_u32, r_mseq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["sweep", "repeat"])
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
    ap.add_argument("--iters", type=int, default=10, help="timed calls per implementation (sweep: 10)")
    ap.add_argument("--repeat-iters", type=int, default=3, help="timed calls per step (repeat: 3)")
    ap.add_argument("--extension", action="store_true", help="sweep: add the labelled extension cells")
    ap.add_argument("--ext-sides", type=int, nargs="*", default=[46, 64, 100])
    ap.add_argument("--ext-random", type=lambda v: tuple(int(x) for x in v.split(":")), nargs="*",
                    default=[(10000, 50000), (100000, 500000), (1000000, 4000000), (2000000, 10000000)],
                    help="n:m pairs for CsrMatrix::random")
    args = ap.parse_args()
    ctx = slat.default_context(0)
    sweep(args, ctx) if args.mode == "sweep" else repeat(args, ctx)


if __name__ == "__main__":
    main()
