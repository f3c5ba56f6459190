#!/usr/bin/env python3
"""Counters of the last K dispatches of kernels matching a substring (e.g. an ablated launch and the
real one of the same step). usage: pmc_dispatches.py 'glob' substring K"""
import csv
import glob
import sys
from collections import defaultdict

rows = defaultdict(dict)
for p in glob.glob(sys.argv[1], recursive=True):
    for r in csv.DictReader(open(p)):
        if sys.argv[2] in r["Kernel_Name"]:
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for d in sorted(rows)[-int(sys.argv[3]):]:
    print(d, {k: int(v) for k, v in sorted(rows[d].items())})
