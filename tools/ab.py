#!/usr/bin/env python3
"""A/B of library builds on the headline (30^3 A^6*A, u32) and C4 (100^3 A^3*A) workloads.

usage: python tools/ab.py [--reps R] [--c4] VARIANT...   (VARIANT = "tree" for the in-tree
libslat.so, NAME for tools/var/libslat_NAME.so, or NAME:ENV=VAL,ENV=VAL for an env knob)

Each (rep, variant) runs in a child process (SLAT_LIB_PATH selects the build), in alternating order,
so clock drift and box-to-box spread fall on every variant alike. A child prints one JSON line:
ms per call over the timed calls and the mean per-kernel HIP-event times of every 4th call.
Every child checks its last output's nnz against the golden count.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(c4: bool, steps: int, only_c4: bool = False, sat64: bool = False, chain: bool = False):
    sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
    import numpy as np

    import slat
    ctx = slat.Context(0)
    out = {}
    legs = ([] if only_c4 else [("a7", 30, 7, steps)]) + ([("c4", 100, 4, max(10, steps // 10))] if c4 or only_c4 else [])
    legs += [("s7", 30, 7, steps)] if sat64 else []
    # the 30^3 chain's other steps A^(k-1) * A (C1 = a2): the fixed cost per call and per row
    legs += [(f"a{k}", 30, k, steps) for k in range(2, 7)] if chain else []
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    for name, side, power, k in legs:
        A = slat.torus_thinned_device(side, 3.0, slat.StdRng(), ctx)
        if name == "s7":  # MagnusMatrix (Sat64) on the same torus
            A = slat.MagnusMatrix.from_host(A.host().astype(slat.SAT64), ctx)
        P = A
        for _ in range(2, power):
            P = P.matmul(A)
        for _ in range(max(5, k // 4)):
            P.matmul(A)
        ctx.sync()
        sym, num, tot = [], [], []
        t0 = time.perf_counter()
        nz = 0
        for i in range(k):
            if i % 4 == 0:
                C = P._spgemm(A, slat.FLAG_TIMING)
                st = ctx.stats()
                sym.append(st["symbolic_ms"]), num.append(st["numeric_ms"]), tot.append(st["total_ms"])
            else:
                C = P._spgemm(A)
            nz = C.nnz()
            del C
        ctx.sync()
        el = (time.perf_counter() - t0) / k * 1e3
        gold = [e for e in want[f"torus{side}_powers"] if e["k"] == power][0]["nnz"]
        out[name] = {"ms": round(el, 4), "sym": round(float(np.mean(sym)), 4), "num": round(float(np.mean(num)), 4),
                     "dev": round(float(np.mean(tot)), 4), "ok": nz == gold}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--only-c4", action="store_true", help="child: the C4 leg alone")
    ap.add_argument("--sat64", action="store_true", help="add the Sat64 (MagnusMatrix) A^6*A leg")
    ap.add_argument("--chain", action="store_true", help="add the 30^3 chain's A^2 ... A^6 legs")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a.c4, a.steps, a.only_c4, a.sat64, a.chain)
        return
    res = {}
    for r in range(a.reps):
        order = a.variants if r % 2 == 0 else a.variants[::-1]
        for v in order:
            name, _, knobs = v.partition(":")
            env = dict(os.environ)
            env.pop("SLAT_LIB_PATH", None)
            if name != "tree":
                env["SLAT_LIB_PATH"] = os.path.join(ROOT, "tools", "var", f"libslat_{name}.so")
            for kv in filter(None, knobs.split(",")):
                k, _, val = kv.partition("=")
                env[k] = val
            cmd = ([sys.executable, os.path.abspath(__file__), "--child", "--steps", str(a.steps)] + (["--c4"] if a.c4 else [])
                   + (["--sat64"] if a.sat64 else []) + (["--chain"] if a.chain else []))
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(f"{v}: FAILED rc={p.returncode}\n{p.stderr[-3000:]}", flush=True)
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            print(v, json.dumps(d), flush=True)
    print("summary (mean over reps):")
    for v, ds in res.items():
        line = [v]
        for leg in ds[0]:
            for f in ("ms", "sym", "num"):
                line.append(f"{leg}.{f}={sum(d[leg][f] for d in ds) / len(ds):.4f}")
            line.append(f"{leg}.ok={all(d[leg]['ok'] for d in ds)}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
