#!/usr/bin/env python3
"""Phase split of the numeric kernels on the 30^3 chain's first steps (A*A, A^2*A), for a
-DSLAT_PHASES=1 variant build (SLAT_LIB_PATH): the library prints one `phases(...)` line per call on
stderr (cycles per batch / row, summed over waves). usage: python tools/phases_chain.py [calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
import slat  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = slat.Context(0)
    A = slat.torus_thinned_device(30, 3.0, slat.StdRng(), ctx)
    P = A
    for k in (2, 3):
        for i in range(calls):
            ctx.sync()
            t0 = time.perf_counter()
            C = P._spgemm(A, slat.FLAG_TIMING)
            st = ctx.stats()
            print(f"a{k} call {i}: {1e3 * (time.perf_counter() - t0):.1f} us nnz {C.nnz()} "
                  f"sym {1e3 * st['symbolic_ms']:.1f} num {1e3 * st['numeric_ms']:.1f}", file=sys.stderr, flush=True)
        P = P.matmul(A)


if __name__ == "__main__":
    main()
