"""The bench_suite GEN leg verbatim (sides 30 then 100 on one context), repeated."""
import sys
import numpy as np
sys.path.insert(0, 'sparse-linear-algebra-tests_amd'); sys.path.insert(0, 'tools')
import slat  # noqa: E402
from check_generators_util import diff  # noqa: E402

for rep in range(3):
    ctx = slat.Context(0)
    for side in (30, 100):
        h = slat.torus_thinned(side, 3.0, slat.StdRng())
        d = slat.torus_thinned_device(side, 3.0, slat.StdRng(), ctx)
        diff(f"rep {rep} side {side} warm-up", d, h)
        d = slat.torus_thinned_device(side, 3.0, slat.StdRng(), ctx)
        diff(f"rep {rep} side {side} timed", d, h)
    del d, ctx
