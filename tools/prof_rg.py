"""rmat16 undirected A^2 (the RG cell) a few times, for a rocprofv3 kernel trace; u32 and f64 any-order."""
import sys

import numpy as np

sys.path.insert(0, 'sparse-linear-algebra-tests_amd')
import slat  # noqa: E402

ctx = slat.Context(0)
h = slat.host_rmat(16, (1 << 16) * 8)
rows = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
a = slat.CsrMatrix.from_edges_device(h.n, rows, h.col_idx, True, ctx)
for _ in range(3):
    c = a._spgemm(a, slat.FLAG_TIMING)
    print("u32", c.nnz(), ctx.stats(), flush=True)
af = slat.CsrF64.from_host(a.host().astype(slat.F64), ctx)
for _ in range(3):
    c = af._spgemm(af, slat.FLAG_TIMING | slat.FLAG_F64_ANY_ORDER)
    print("f64any", c.nnz(), ctx.stats(), flush=True)
