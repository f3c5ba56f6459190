#!/usr/bin/env python3
"""Phase split of k_numeric on the headline step (30^3 torus, C = A^6 * A) for a -DSLAT_PHASES=1
variant build (SLAT_LIB_PATH): the library prints one `phases(...)` line per call on stderr (cycles
per row, summed over waves, then divided by the rows). usage: python tools/phases_a7.py [calls]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-linear-algebra-tests_amd"))
import slat  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ctx = slat.Context(0)
    A = slat.torus_thinned_device(30, 3.0, slat.StdRng(), ctx)
    P = A
    for _ in range(5):
        P = P.matmul(A)
    for i in range(calls):
        C = P._spgemm(A, slat.FLAG_TIMING)
        st = ctx.stats()
        print(f"a7 call {i}: nnz {C.nnz()} sym {1e3 * st['symbolic_ms']:.1f} num {1e3 * st['numeric_ms']:.1f} us",
              file=sys.stderr, flush=True)
        del C


if __name__ == "__main__":
    main()
