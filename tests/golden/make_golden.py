#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (runs in the dev container only).

This is an INDEPENDENT restatement (numpy + scipy.sparse) of the reference's input generators and
SpGEMM, used to pin both the C oracle and the HIP path:

* ChaCha12 StdRng (rand 0.9.2 / rand_chacha 0.9.0, reference Cargo.lock:851-895), vectorised over
  blocks; f64 draws = (next_u64 >> 12) * 2^-52 (rand's UniformFloat::sample_single over 0.0..1.0).
* CsrMatrix::lattice (src/graph_csr.rs:177-222) and CsrMatrix::thin (src/graph_csr.rs:225-247),
  whose draw pattern equals SparseCountMatrix::thin (src/graph.rs:143-154).
* A^k = A^(k-1) * A via scipy int64 matmul (exact: no value at these sizes reaches 2^32), as in
  bench_repeated_exponentiation (src/graph_magnus.rs:701-788), and the sweep grid of
  bench_matmul_magnus (src/graph_magnus.rs:792-929) with ONE rng shared across the grid.

External pin: the A..A^7 nnz sequence below rounds to every nnz figure printed in the reference's
README.md:41-46 (252k, 655k, 1.57M, 3.38M, 6.59M, 11.7M) — checked in tests/test_golden.py.

Outputs (small): golden.json (nnz sequences, flops, SHA-256 of canonical arrays) and
small_cells.npz (full arrays for the small sweep cells and the hand-computed unit cases).
Canonical bytes: row_ptr as little-endian u64, col as u32, values as u32 (u32 semantics).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = bytes([42] * 32)
MASK = np.uint64(0xFFFFFFFF)


def _rotl(x, n):
    return ((x << np.uint32(n)) | (x >> np.uint32(32 - n))).astype(np.uint32)


def chacha12_blocks(key_words: np.ndarray, first: int, count: int) -> np.ndarray:
    """`count` ChaCha12 blocks with 64-bit counters first..first+count-1, stream 0 -> (count,16) u32."""
    s = np.zeros((count, 16), dtype=np.uint32)
    s[:, 0:4] = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)
    s[:, 4:12] = key_words
    ctr = np.arange(first, first + count, dtype=np.uint64)
    s[:, 12] = (ctr & MASK).astype(np.uint32)
    s[:, 13] = (ctr >> np.uint64(32)).astype(np.uint32)
    x = [s[:, i].copy() for i in range(16)]

    def qr(a, b, c, d):
        with np.errstate(over="ignore"):
            x[a] = x[a] + x[b]; x[d] = _rotl(x[d] ^ x[a], 16)
            x[c] = x[c] + x[d]; x[b] = _rotl(x[b] ^ x[c], 12)
            x[a] = x[a] + x[b]; x[d] = _rotl(x[d] ^ x[a], 8)
            x[c] = x[c] + x[d]; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(6):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    with np.errstate(over="ignore"):
        out = np.stack(x, axis=1) + s
    return out.astype(np.uint32)


class StdRng:
    """Stream of f64 draws; only u64-aligned reads happen on the reference path."""

    def __init__(self, seed: bytes = SEED):
        self.key = np.frombuffer(seed, dtype="<u4").astype(np.uint32)
        self.word = 0  # words consumed

    def f64(self, count: int) -> np.ndarray:
        w0 = self.word
        w1 = w0 + 2 * count
        b0, b1 = w0 // 16, (w1 + 15) // 16
        words = chacha12_blocks(self.key, b0, max(b1 - b0, 0)).reshape(-1)[w0 - 16 * b0: w1 - 16 * b0]
        self.word = w1
        lo = words[0::2].astype(np.uint64)
        hi = words[1::2].astype(np.uint64)
        u = lo | (hi << np.uint64(32))
        return (u >> np.uint64(12)).astype(np.float64) * (1.0 / 4503599627370496.0)


def lattice(dims, torus=True) -> sp.csr_matrix:
    dims = list(dims)
    nd = len(dims)
    total = int(np.prod(dims))
    strides = [1] * nd
    for i in range(nd - 2, -1, -1):
        strides[i] = strides[i + 1] * dims[i + 1]
    node = np.arange(total, dtype=np.int64)
    coord = [(node // strides[d]) % dims[d] for d in range(nd)]
    rows, cols = [], []
    for off in range(3 ** nd):
        tmp, deltas = off, []
        for d in range(nd):
            deltas.append(tmp % 3 - 1)
            tmp //= 3
        if all(dl == 0 for dl in deltas):
            continue
        nb = np.zeros(total, dtype=np.int64)
        ok = np.ones(total, dtype=bool)
        for d in range(nd):
            c = coord[d] + deltas[d]
            if torus:
                c = np.mod(c, dims[d])
            else:
                ok &= (c >= 0) & (c < dims[d])
            nb += c * strides[d]
        rows.append(node[ok]); cols.append(nb[ok])
    r = np.concatenate(rows); c = np.concatenate(cols)
    m = sp.coo_matrix((np.ones(len(r), dtype=np.int64), (r, c)), shape=(total, total)).tocsr()
    m.sum_duplicates(); m.sort_indices()
    return m


def thin(m: sp.csr_matrix, rng: StdRng, density: float) -> sp.csr_matrix:
    m = m.tocsr(); m.sort_indices()
    n = m.shape[0]
    rows = np.repeat(np.arange(n), np.diff(m.indptr))
    cols = m.indices.astype(np.int64)
    vals = m.data
    upper = rows <= cols                 # a draw happens only for r <= c (row-major order)
    draws = rng.f64(int(upper.sum()))
    keep = np.zeros(len(rows), dtype=bool)
    keep[np.flatnonzero(upper)] = draws < density
    kr, kc, kv = rows[keep], cols[keep], vals[keep]
    off = kr != kc
    mt = m.T.tocsr()                     # value of (c, r) = m[c, r]
    rev = np.asarray(m[kc[off], kr[off]]).reshape(-1)
    pos = rev > 0
    R = np.concatenate([kr, kc[off][pos]]); Cc = np.concatenate([kc, kr[off][pos]])
    V = np.concatenate([kv, rev[pos]])
    del mt
    out = sp.coo_matrix((V.astype(np.int64), (R, Cc)), shape=m.shape).tocsr()
    out.sum_duplicates(); out.eliminate_zeros(); out.sort_indices()
    return out


def matmul(a: sp.csr_matrix, b: sp.csr_matrix) -> sp.csr_matrix:
    c = (a @ b).tocsr()
    c.sum_duplicates(); c.eliminate_zeros(); c.sort_indices()
    return c


def flops(a: sp.csr_matrix, b: sp.csr_matrix) -> int:
    blen = np.diff(b.indptr)
    return int(blen[a.indices].sum())


def digest(m: sp.csr_matrix, vdtype="<u4") -> dict:
    rp = np.asarray(m.indptr, dtype="<u8").tobytes()
    col = np.asarray(m.indices, dtype="<u4").tobytes()
    assert m.data.max(initial=0) < 2 ** 32
    val = np.asarray(m.data, dtype=vdtype).tobytes()
    return {"n": int(m.shape[0]), "nnz": int(m.nnz),
            "row_ptr": hashlib.sha256(rp).hexdigest(), "col": hashlib.sha256(col).hexdigest(),
            "val": hashlib.sha256(val).hexdigest(), "max": int(m.data.max(initial=0)),
            "max_row": int(np.diff(m.indptr).max(initial=0))}


def main(with_100: bool = False):
    g = {"seed": list(SEED), "note": "see make_golden.py docstring"}
    small = {}

    # C1/C2: 30^3 torus thinned to 3 e/n, A^k = A^(k-1) * A (src/graph_magnus.rs:707-787)
    rng = StdRng()
    full = lattice([30, 30, 30])
    A = thin(full, rng, 3.0 / (full.nnz / full.shape[0]))
    powers = [A]
    rep = [{"k": 1, **digest(A)}]
    for k in range(2, 8):
        P = matmul(powers[-1], A)
        rep.append({"k": k, "flops": flops(powers[-1], A), **digest(P)})
        powers.append(P)
        print("30^3 A^%d nnz=%d" % (k, P.nnz), file=sys.stderr)
    g["torus30_powers"] = rep
    small["torus30_A_row_ptr"] = A.indptr.astype(np.uint64)
    small["torus30_A_col"] = A.indices.astype(np.uint32)
    del powers

    # C3: sweep grid, ONE rng across the grid, epn 26 = full lattice, no draws
    rng = StdRng()
    sweep = []
    for s in [5, 10, 20, 30]:
        full = lattice([s, s, s])
        full_epn = full.nnz / full.shape[0]
        for epn in [2.0, 3.0, 4.0, 8.0, 26.0]:
            density = epn / full_epn
            Acell = full if density >= 1.0 else thin(full, rng, density)
            C2 = matmul(Acell, Acell)
            sweep.append({"side": s, "e_per_n": epn, "A": digest(Acell), "A2": digest(C2),
                          "flops": flops(Acell, Acell)})
            if s == 5 or (s == 10 and epn <= 3.0):
                tag = "sweep_s%d_e%d" % (s, int(epn))
                small[tag + "_row_ptr"] = Acell.indptr.astype(np.uint64)
                small[tag + "_col"] = Acell.indices.astype(np.uint32)
                small[tag + "_A2_row_ptr"] = C2.indptr.astype(np.uint64)
                small[tag + "_A2_col"] = C2.indices.astype(np.uint32)
                small[tag + "_A2_val"] = C2.data.astype(np.uint32)
    g["sweep"] = sweep

    if with_100:  # C4: 100^3 torus, fresh seed, A^4 = A^3 * A
        rng = StdRng()
        full = lattice([100, 100, 100])
        A = thin(full, rng, 3.0 / (full.nnz / full.shape[0]))
        del full
        rep = [{"k": 1, **digest(A)}]
        P = A
        for k in range(2, 5):
            f = flops(P, A)
            P = matmul(P, A)
            rep.append({"k": k, "flops": f, **digest(P)})
            print("100^3 A^%d nnz=%d" % (k, P.nnz), file=sys.stderr)
        g["torus100_powers"] = rep
    else:
        old = os.path.join(HERE, "golden.json")
        if os.path.exists(old):
            prev = json.load(open(old))
            if "torus100_powers" in prev:
                g["torus100_powers"] = prev["torus100_powers"]

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "small_cells.npz"), **small)


if __name__ == "__main__":
    main(with_100="--with-100" in sys.argv)
