import sys, numpy as np
sys.path.insert(0,'sparse-linear-algebra-tests_amd'); sys.path.insert(0,'oracle')
import slat, oracle_py as O
ctx = slat.default_context(0)
for side in (48, 50, 64, 100):
    L = slat.CsrMatrix.lattice([side]*3, True, ctx)
    o = O.lattice([side]*3, True); rp, col, val = o.arrays(); h = L.host()
    print(side, side**3*27, L.nnz(), o.nnz, np.array_equal(h.row_ptr, rp), np.array_equal(h.col_idx, col), np.array_equal(h.values, val), flush=True)
