"""The product's host constructors (libslat.so: ChaCha12 StdRng, lattice, thin, from_coo) against the
golden digests and the oracle. CPU only."""
import numpy as np

import oracle_py as O
import slat
from helpers import assert_digest, digest


def test_rng_matches_oracle():
    a, b = slat.StdRng(), O.Rng()
    assert [a.next_u64() for _ in range(300)] == [b.next_u64() for _ in range(300)]
    a, b = slat.StdRng(bytes(range(32))), O.Rng(bytes(range(32)))
    assert [a.random_f64() for _ in range(100)] == [b.next_f64() for _ in range(100)]


def test_torus30_input(golden):
    A = slat.torus_thinned(30, 3.0, slat.StdRng())
    assert_digest(digest(A.row_ptr, A.col_idx, A.values), golden["torus30_powers"][0], "A")


def test_sweep_inputs(golden):
    rng = slat.StdRng()
    cells = iter(golden["sweep"])
    for s in [5, 10, 20, 30]:
        full = slat.host_lattice([s, s, s], True)
        for epn in [2.0, 3.0, 4.0, 8.0, 26.0]:
            cell = next(cells)
            density = epn / (full.nnz / full.n)
            A = slat.host_thin(full, rng, density) if density < 1.0 else full
            assert_digest(digest(A.row_ptr, A.col_idx, A.values), cell["A"], f"s={s} epn={epn}")


def test_from_coo_dedup_and_zero_drop():
    h = slat.host_from_coo(4, [0, 0, 1, 1, 3], [2, 2, 0, 1, 3], [1, 2, 5, 0, 7])
    assert h.row_ptr.tolist() == [0, 1, 2, 2, 3]
    assert h.col_idx.tolist() == [2, 0, 3]
    assert h.values.tolist() == [3, 5, 7]


def test_lattice_against_oracle():
    for dims, torus in [([5], False), ([5], True), ([3, 3], True), ([4, 3], False), ([2, 2, 2], False), ([2, 3, 2], True)]:
        h = slat.host_lattice(dims, torus)
        o = O.lattice(dims, torus)
        rp, col, val = o.arrays()
        np.testing.assert_array_equal(h.row_ptr, rp)
        np.testing.assert_array_equal(h.col_idx, col)
        np.testing.assert_array_equal(h.values, val)


def test_rmat_is_seeded_and_positive():
    a = slat.host_rmat(10, 8000)
    b = slat.host_rmat(10, 8000)
    np.testing.assert_array_equal(a.col_idx, b.col_idx)
    assert a.values.min() >= 0.5 and a.n == 1024
