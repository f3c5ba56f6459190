#!/usr/bin/env python3
"""A/B of library builds / env knobs on the power-law and long-row products (the fat-row and
window categories): RG = R-MAT 2^16 undirected u32 A^2, C5 = R-MAT 2^16 (and --big: 2^18) degree 16
f64 A*A in any order and in the reference's fold order, chain = directed R-MAT 2^14 A^4 * A.

usage: python tools/ab_heavy.py [--reps R] [--big] [--legs rg,c5any,...] VARIANT...  (VARIANT as in
tools/ab.py: "tree", NAME for tools/var/libslat_NAME.so, NAME:ENV=VAL,... for env knobs);
python tools/ab_heavy.py --child [--big] [--legs ...] runs the legs once in this process (profiling)

Children alternate in order; each prints the best-of-2 ms per leg (after one warm-up call), its
symbolic / numeric event split, and the output nnz against the known count.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NNZ = {"rg": 164123598, "c5any": 163990080, "c5ord": 163990080, "chain": 84295215,
       "c5big_any": 1277823132, "c5big_ord": 1277823132}


def child(big: bool, legs=None):
    sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
    import numpy as np

    import slat
    ctx = slat.Context(0)
    out = {}

    def run(name, a, b, flags=0, reps=2):
        if legs and name not in legs:
            return
        best, st, nz = 1e30, None, 0
        c = a._spgemm(b, flags)
        del c
        for _ in range(reps):
            ctx.sync()
            t0 = time.perf_counter()
            c = a._spgemm(b, slat.FLAG_TIMING | flags)
            t = (time.perf_counter() - t0) * 1e3
            nz = c.nnz()
            del c
            if t < best:
                best, st = t, ctx.stats()
        out[name] = {"ms": round(best, 3), "sym": round(st["symbolic_ms"], 3), "num": round(st["numeric_ms"], 3),
                     "ok": nz == NNZ[name]}

    want = lambda *ns: not legs or any(n in legs for n in ns)  # noqa: E731
    if want("rg"):
        h = slat.host_rmat(16, (1 << 16) * 8)
        rows = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
        a = slat.CsrMatrix.from_edges_device(h.n, rows, h.col_idx, True, ctx)
        run("rg", a, a)
        del a
    if want("c5any", "c5ord"):
        f = slat.CsrF64.from_host(slat.host_rmat(16, (1 << 16) * 16), ctx)
        run("c5any", f, f, slat.FLAG_F64_ANY_ORDER)
        run("c5ord", f, f, 0, 1)
        del f
    if want("chain"):
        h = slat.host_rmat(14, (1 << 14) * 8)
        rows = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
        d = slat.CsrMatrix.from_edges_device(h.n, rows, h.col_idx, False, ctx)
        p = d.matmul(d).matmul(d).matmul(d)
        run("chain", p, d)
        del p, d
    if big and want("c5big_any", "c5big_ord"):
        f = slat.CsrF64.from_host(slat.host_rmat(18, (1 << 18) * 16), ctx)
        run("c5big_any", f, f, slat.FLAG_F64_ANY_ORDER, 1)
        run("c5big_ord", f, f, 0, 1)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--legs", default="", help="comma-separated subset of the legs")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    legs = [x for x in a.legs.split(",") if x]
    if a.child:
        child(a.big, legs)
        return
    res = {}
    for r in range(a.reps):
        for v in (a.variants if r % 2 == 0 else a.variants[::-1]):
            name, _, knobs = v.partition(":")
            env = dict(os.environ)
            env.pop("SLAT_LIB_PATH", None)
            if name != "tree":
                env["SLAT_LIB_PATH"] = os.path.join(ROOT, "tools", "var", f"libslat_{name}.so")
            for kv in filter(None, knobs.split(",")):
                k, _, val = kv.partition("=")
                env[k] = val
            cmd = ([sys.executable, os.path.abspath(__file__), "--child"] + (["--big"] if a.big else [])
                   + (["--legs", a.legs] if legs else []))
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(f"{v}: FAILED rc={p.returncode}\n{p.stderr[-3000:]}", flush=True)
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            print(v, json.dumps(d), flush=True)
    print("summary (best over reps, ms):")
    for v, ds in res.items():
        print("  ".join([v] + [f"{leg}={min(d[leg]['ms'] for d in ds):.3f}(num {min(d[leg]['num'] for d in ds):.3f})"
                               f"{'' if all(d[leg]['ok'] for d in ds) else '!BAD'}" for leg in ds[0]]), flush=True)


if __name__ == "__main__":
    main()
