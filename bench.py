#!/usr/bin/env python3
"""bench.py — GNNZ/s of the MI355X SpGEMM on the reference's headline workload.

Workload (BASELINE.json configs[1], the one the metric is quoted on): the 30^3 Moore torus
thinned to 3 edges/node with StdRng seed [42;32] (src/graph_magnus.rs:707-719), one step =
C = A^6 · A (the A^7 step of bench_repeated_exponentiation, src/graph_magnus.rs:740-772), u32
saturating values, nnz(C) = 11,736,555. Inputs are device-resident before the timed region; each
step is one complete synchronous SpGEMM call (symbolic, scan, C allocation, numeric, nnz read-back)
and its output is released inside the step.

N > 1 (torchrun, one rank per GPU): `--scaling strong` (default) — config C4, the 100^3 torus,
C = A^3·A, whose rows are split across the ranks into flops-balanced blocks cut on the device
(north_star: >= 6x strong scaling at 8 GPUs). Rank 0 builds A and A^3 and broadcasts them over
RCCL (libslat's slat_bcast_csr, outside the timed region); each rank then times its row block with
no data-path collective (C stays row-distributed, the next power's left operand). Rank 0 also times
the whole product alone on its GPU afterwards and reports the speedup. `--gather` adds the
allgatherv of C's row blocks over RCCL (slat_allgather_rows), timed separately as gather_ms.
`--scaling weak` is the labelled extra: one 30^3 torus per rank (the block-diagonal matrix).
value = output nnz of all ranks / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))

import numpy as np  # noqa: E402

import slat  # noqa: E402
from slat import dist as slat_dist  # noqa: E402

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
README_CSR_PAR_A7_GNNZ = 11736555 / 40.5e-3 / 1e9   # README.md:46, unstated hardware: 0.290 GNNZ/s


def algorithmic_bytes(nnz_a: int, nnz_b: int, nnz_c: int, n: int, vsize: int) -> int:
    """compulsory traffic, each array touched once."""
    return (4 + vsize) * (nnz_a + nnz_b + nnz_c) + 8 * 3 * (n + 1)


def build_inputs(side: int, power: int, ctx):
    A = slat.CsrMatrix.from_host(slat.torus_thinned(side, 3.0, slat.StdRng()), ctx)
    P = A
    for _ in range(2, power):
        P = P.matmul(A)
    return A, P


def cpu_baseline(side: int, power: int, seconds: float = 12.0):
    """Oracle restatement of CsrMatrix::matmul_par (oracle/, kind 'port') on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    A = O.torus_thinned(side, 3.0, O.Rng())
    P = A
    for _ in range(2, power):
        P = O.matmul_seq(P, A)
    C = O.matmul_par(P, A, threads)  # warm-up (reference: 1 warm-up + timed iterations)
    nnz = C.nnz
    del C
    iters, t0 = 0, time.perf_counter()
    while True:
        O.matmul_par(P, A, threads)
        iters += 1
        el = time.perf_counter() - t0
        if (el >= seconds and iters >= 3) or iters >= 200:
            break
    per = el / iters
    return {"value": nnz / per / 1e9, "unit": "GNNZ/s", "cores": threads, "kind": "port",
            "sample": f"A^{power - 1}*A on {side}^3 torus (nnz(C)={nnz}), {iters} timed calls after 1 warm-up, "
                      f"{per * 1e3:.2f} ms/call, oracle/oracle.c orc_matmul_par with {threads} threads"}


def load_pmc(workload: str):
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50, help="untimed steps; the GPU needs ~10 ms of load to clock up")
    ap.add_argument("--side", type=int, default=30)
    ap.add_argument("--power", type=int, default=7, help="C = A^(power-1) * A")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="N > 1 default: strong (config C4 split over the ranks); weak = one torus per rank")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--timing-every", type=int, default=4,
                    help="record the per-kernel HIP events (roofline) on every k-th timed step; the event "
                         "records cost host time, so the other steps run without them")
    ap.add_argument("--gather", action="store_true",
                    help="N > 1: after the timed region, assemble C's row blocks on every rank (allgatherv over "
                         "RCCL) and report its time as config.gather_ms")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one rank per GPU; SLAT_DIST_BACKEND=gloo rehearses the multi-rank flow with ranks sharing the
    # visible GPU(s) (the metric's runs use RCCL, "nccl")
    backend = os.environ.get("SLAT_DIST_BACKEND", "nccl")
    dev_index = local
    # SLAT_FORCE_DIST=1: the multi-rank code path even at world size 1 (one-GPU rehearsal)
    if world > 1 or os.environ.get("SLAT_FORCE_DIST"):
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dev_index = local % max(1, torch.cuda.device_count())
            dist.init_process_group(backend)
    coll_dev = f"cuda:{local}" if backend == "nccl" else "cpu"

    ctx = slat.Context(dev_index)
    scaling = args.scaling or ("strong" if dist is not None else "weak")
    side, power = args.side, args.power
    if scaling == "strong" and dist is not None and side == 30 and power == 7:
        side, power = 100, 4  # config C4: 100^3 torus, C = A^3 * A split over the ranks
    comm = None
    if dist is not None and scaling == "strong" and backend == "nccl":
        # rank 0 builds the operands; B (= A) and the left operand reach the others over RCCL
        # (one broadcast per array, outside the timed region)
        comm = slat_dist.Comm(ctx)
        A, P = build_inputs(side, power, ctx) if rank == 0 else (None, None)
        A = comm.bcast(A, slat.CsrMatrix)
        P = comm.bcast(P, slat.CsrMatrix)
    else:
        A, P = build_inputs(side, power, ctx)
    n = A.n
    row_lo, row_hi = 0, n
    if scaling == "strong" and dist is not None:
        # flops-balanced 1-D row blocks of the left operand, cut on the device
        cuts = slat_dist.device_cuts(P, A, world)
        row_lo, row_hi = cuts[rank], cuts[rank + 1]

    def step(flags=0):
        C = P.matmul_rowblock(row_lo, row_hi, A, flags)
        nz = C.nnz()
        del C
        return nz

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()
        ctx.sync()

    barrier()
    sym, scan, num, tot, abl = [], [], [], [], []
    t0 = time.perf_counter()
    nnz_c = 0
    every = max(1, args.timing_every)
    for i in range(args.steps):
        if i % every == 0:  # HIP events around each kernel of this step, on the library's stream
            nnz_c = step(slat.FLAG_TIMING)
            st = ctx.stats()
            sym.append(st["symbolic_ms"]), scan.append(st["scan_ms"]), num.append(st["numeric_ms"])
            tot.append(st["total_ms"])
            abl.append(st["compact_ms"])
        else:
            nnz_c = step()
    barrier()
    elapsed = time.perf_counter() - t0
    stats = ctx.stats()

    units = nnz_c * args.steps
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        u = torch.tensor([units], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        units = int(u.item())

    value = units / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3

    single_ms = None
    if dist is not None and scaling == "strong":
        # the same product on one GPU (rank 0 alone), for the strong-scaling speedup
        dist.barrier()
        if rank == 0:
            k = max(5, min(args.steps, 20))
            for _ in range(3):
                P.matmul_rowblock(0, n, A, 0)
            ctx.sync()
            ts = time.perf_counter()
            for _ in range(k):
                C1 = P.matmul_rowblock(0, n, A, 0)
                del C1
            ctx.sync()
            single_ms = (time.perf_counter() - ts) / k * 1e3
        dist.barrier()

    gather_ms, gather_nnz = None, None
    if dist is not None and args.gather:
        # not part of the SpGEMM metric: C row blocks stay distributed for the next step (§8(e))
        import torch
        C = P.matmul_rowblock(row_lo, row_hi, A, 0)
        if comm is not None:
            # device-resident allgatherv over RCCL (libslat): u32 columns, native-width values
            comm.allgather_rows(C)  # warm-up (RCCL connection setup)
            dist.barrier()
            tg = time.perf_counter()
            full = comm.allgather_rows(C)
            dist.barrier()
            gather_ms = (time.perf_counter() - tg) * 1e3
            gather_nnz = full.nnz()
            del full
        else:  # CPU rehearsal (gloo): the host restatement of the assembly
            hc = C.host()
            dist.barrier()
            tg = time.perf_counter()
            slat_dist.gather_blocks(hc.row_ptr, hc.col_idx, hc.values, device=torch.device(coll_dev))
            dist.barrier()
            gather_ms = (time.perf_counter() - tg) * 1e3
            gather_nnz = None
        del C

    if rank == 0:
        nnz_a = P.nnz() if row_hi - row_lo == n else int(P.row_ptr[row_hi] - P.row_ptr[row_lo])
        alg = algorithmic_bytes(nnz_a, A.nnz(), nnz_c, row_hi - row_lo, 4)
        num_ms = float(np.mean(num))
        achieved = alg / (max(num_ms, 1e-6) * 1e-3) / 1e9
        pmc = load_pmc(f"torus{side}_a{power}")
        traffic = pmc.get("numeric_bytes_per_launch") if pmc else None
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                    "kernel": "k_numeric", "algorithmic_bytes": alg, "timed_steps": len(num),
                    "kernel_ms": {"symbolic": round(float(np.mean(sym)), 4), "scan": round(float(np.mean(scan)), 4),
                                  "numeric": round(num_ms, 4), "device_total": round(float(np.mean(tot)), 4)},
                    "pipeline_frac": round(alg / (max(float(np.mean(tot)), 1e-6) * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
        cpu = None
        if not args.no_cpu and world == 1:
            cpu = cpu_baseline(side, power, args.cpu_seconds)
        workload = f"{side}^3 Moore torus thinned to 3 e/n (seed [42;32]), C = A^{power - 1} * A, u32 saturating"
        out = {
            "metric": "GNNZ/s (output nnz/s) for A×A on 30³ Moore torus, 1/2/4/8 GPUs",
            "value": round(value, 4), "unit": "GNNZ/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": round(value / README_CSR_PAR_A7_GNNZ, 2) if (side, power) == (30, 7) else None,
            "dtype": "u32", "data": "synthetic (reference generator: ChaCha12 StdRng seed [42;32])",
            "config": {"workload": workload, "nnz_c": nnz_c, "n": n, "rows": [row_lo, row_hi],
                       "partition": "block-diagonal, one torus per rank" if scaling == "weak" else "flops-balanced row blocks",
                       "capacity": stats["capacity"], "mode": stats["mode"], "window_words": stats["window_words"],
                       **({"ablated_ms": round(float(np.mean(abl)), 4)} if os.environ.get("SLAT_ABLATE") else {}),
                       **({"gather_ms": round(gather_ms, 3)} if gather_ms is not None else {}),
                       **({"gather_nnz": gather_nnz} if gather_nnz is not None else {}),
                       **({"single_gpu_ms": round(single_ms, 4), "strong_speedup": round(single_ms / ms_per_step, 3)}
                          if single_ms is not None else {})},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
