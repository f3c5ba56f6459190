"""Power-law / dense-row products for a rocprofv3 kernel trace: the RG cell (R-MAT 2^16 undirected,
A^2), config C5 (R-MAT 2^16 f64, reference order and any order) and a dense-output chain step
(directed R-MAT 2^14, A^5 = A^4 * A)."""
import sys
import time

import numpy as np

sys.path.insert(0, 'sparse-linear-algebra-tests_amd')
import slat  # noqa: E402

ctx = slat.Context(0)


def run(name, a, b, flags=0, reps=2):
    for _ in range(reps):
        t0 = time.perf_counter()
        c = a._spgemm(b, slat.FLAG_TIMING | flags)
        t = (time.perf_counter() - t0) * 1e3
        s = ctx.stats()
        print(f"{name}: {t:.2f} ms nnz {c.nnz()} sym {s['symbolic_ms']:.2f} scan {s['scan_ms']:.2f} "
              f"num {s['numeric_ms']:.2f} mode {s['mode']} ww {s['window_words']}", flush=True)


h = slat.host_rmat(16, (1 << 16) * 8)
rows = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
a = slat.CsrMatrix.from_edges_device(h.n, rows, h.col_idx, True, ctx)
run("RG rmat16 undirected u32 A^2", a, a)
f = slat.CsrF64.from_host(slat.host_rmat(16, (1 << 16) * 16), ctx)
run("C5 rmat16 deg16 f64 any", f, f, slat.FLAG_F64_ANY_ORDER)
run("C5 rmat16 deg16 f64 ordered", f, f, 0, 1)
h = slat.host_rmat(14, (1 << 14) * 8)
rows = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
d = slat.CsrMatrix.from_edges_device(h.n, rows, h.col_idx, False, ctx)
p = d.matmul(d).matmul(d).matmul(d)
run("chain rmat14 A^4*A", p, d)
