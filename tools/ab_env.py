#!/usr/bin/env python3
"""A/B of one variant library's A/B knobs (environment values) on config C4 (whole and one rank's
eighth, tools/c4_eighth.py) and the R-MAT 2^16 leg (tools/ab_heavy.py --child --legs rg): each setting
in its own process, settings alternated over --reps rounds. Prints one JSON line per run.
usage: python tools/ab_env.py --lib tools/var/libslat_X.so [--reps R] KNOB=V[,KNOB=V] ... ('-' = none)"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
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
            for cmd in (["tools/c4_eighth.py"], ["tools/ab_heavy.py", "--child", "--legs", "rg"]):
                r = subprocess.run([sys.executable] + cmd, cwd=ROOT, env=env, capture_output=True, text=True,
                                   timeout=240)
                if r.returncode != 0:
                    print(r.stdout[-2000:], r.stderr[-2000:], flush=True)
                    sys.exit(r.returncode)
                line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
                print(json.dumps({"rep": rep, "setting": st, "leg": cmd[0], "out": json.loads(line)}), flush=True)


if __name__ == "__main__":
    main()
