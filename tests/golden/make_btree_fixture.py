"""Copies the reference's own B-tree layout output into a fixture: btree_overhead.csv (the printout of
src/dense_btree.rs:418-426 `print_overhead_csv`: n, internal_len, total_len of
DenseBTree::from_sorted(0..n) for n = 1..10000) as tests/golden/btree_overhead.npz. Run in the
container that holds /root/reference; the fixture is data (inputs and outputs), not source."""
import os
import sys

import numpy as np

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/btree_overhead.csv"
rows = np.loadtxt(src, delimiter=",", skiprows=1, dtype=np.int64)
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "btree_overhead.npz")
np.savez_compressed(out, n=rows[:, 0], internal_len=rows[:, 1], total_len=rows[:, 2])
print(out, rows.shape)
