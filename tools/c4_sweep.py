#!/usr/bin/env python3
"""C4 whole against one eighth (tools/c4_eighth.py) under env-knob settings of a variant library, each
setting in its own process, alternated over --reps rounds. usage: c4_sweep.py --lib L [--reps R] SETTING..."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("settings", nargs="+")
a = ap.parse_args()
for rep in range(a.reps):
    for st in a.settings:
        env = dict(os.environ, SLAT_LIB_PATH=os.path.join(ROOT, a.lib))
        if st != "-":
            for kv in st.split(","):
                k, v = kv.split("=")
                env[k] = v
        r = subprocess.run([sys.executable, "tools/c4_eighth.py"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-2000:], flush=True)
            sys.exit(r.returncode)
        print(json.dumps({"rep": rep, "setting": st, "out": json.loads(r.stdout.strip().splitlines()[-1])}), flush=True)
