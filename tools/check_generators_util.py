import numpy as np


def diff(what, d, h):
    g = d.host()
    same_rp = np.array_equal(g.row_ptr, h.row_ptr)
    same_col = g.col_idx.shape == h.col_idx.shape and np.array_equal(g.col_idx, h.col_idx)
    same_val = g.values.shape == h.values.shape and np.array_equal(g.values, h.values)
    msg = f"{what}: nnz {d.nnz()} vs {h.nnz} rp {same_rp} col {same_col} val {same_val}"
    if not same_rp:
        r = int(np.argmax(g.row_ptr != h.row_ptr))
        msg += f" first rp diff at row {r}: {g.row_ptr[r]} vs {h.row_ptr[r]}"
    elif not same_col:
        k = int(np.argmax(g.col_idx != h.col_idx))
        r = int(np.searchsorted(h.row_ptr, k, side='right') - 1)
        msg += f" first col diff at {k} (row {r}): {g.col_idx[k]} vs {h.col_idx[k]};"
        msg += f" row dev {g.col_idx[h.row_ptr[r]:h.row_ptr[r+1]]} host {h.col_idx[h.row_ptr[r]:h.row_ptr[r+1]]}"
        msg += f" ndiff {int((g.col_idx != h.col_idx).sum())}"
    print(msg, flush=True)
    return same_rp and same_col and same_val
