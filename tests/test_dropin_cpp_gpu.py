"""The C++ drop-in (include/slat.hpp): a C++ program written against the reference's names
(CsrMatrix::matmul / matmul_par / add / power_until_stable / reachability_sum /
connected_components, MagnusMatrix::matmul / matmul_seq, linalg Csr<f64>::matmul_par) with host
vectors in and out, run as its own process (tests/cpp/dropin, built by __graft_entry__.build()).
Every product it writes is checked here against the oracle: bit-exact for u32 / Sat64 and the f64
left fold."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "dropin")


def load(d, name, col_dt, val_dt):
    rp = np.fromfile(os.path.join(d, name + ".rp"), np.uint64)
    col = np.fromfile(os.path.join(d, name + ".col"), col_dt)
    val = np.fromfile(os.path.join(d, name + ".val"), val_dt)
    return rp, col, val


def same(got, want: O.Csr, what):
    rp, col, val = want.arrays()
    np.testing.assert_array_equal(got[0], rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(got[1].astype(np.uint64), col.astype(np.uint64), err_msg=f"{what} col_idx")
    if val.dtype == np.float64:
        np.testing.assert_array_equal(got[2].view(np.uint64), val.view(np.uint64), err_msg=f"{what} f64 bits")
    else:
        np.testing.assert_array_equal(got[2], val, err_msg=f"{what} values")


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built (make -C tests/cpp, or __graft_entry__.build())")
    d = str(tmp_path_factory.mktemp("dropin"))
    r = subprocess.run([BIN, d, "3"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stderr[-3000:]
    summary = {}
    with open(os.path.join(d, "summary.txt")) as f:
        for line in f:
            k, *v = line.split()
            summary[k] = v
    return d, summary


@pytest.mark.gpu
def test_cpp_csr_matmul_c1_and_a3(run):
    d, s = run
    a = O.torus_thinned(30, 3.0, O.Rng())
    same(load(d, "torus30_a1", np.uint32, np.uint32), a, "C++ thin(lattice) input")
    a2 = O.matmul_seq(a, a)
    assert int(s["a2_nnz"][0]) == a2.nnz == 251590  # README.md:41
    same(load(d, "torus30_a2", np.uint32, np.uint32), a2, "C++ CsrMatrix::matmul A^2 (C1)")
    assert s["a2_par_equal"] == ["1"]  # matmul_par gives the same arrays
    same(load(d, "torus30_a3", np.uint32, np.uint32), O.matmul_seq(a2, a), "C++ A^3")
    assert s["threads_equal"] == ["1"]  # one context per host thread


@pytest.mark.gpu
def test_cpp_saturating_chains(run):
    d, s = run
    n = 64
    base = O.add(O.from_edges(n, [(i, i + 1) for i in range(n - 1)]), O.identity(n))
    want, iters = O.power_until_stable(base)
    assert int(s["chain_u32_iters"][0]) == iters == 7  # test_power_until_stable_chain
    same(load(d, "chain_u32_stable", np.uint32, np.uint32), want, "C++ power_until_stable (u32 saturating)")
    m = O.convert(base, O.SAT64)
    for _ in range(7):
        m = O.matmul_seq(m, m)
    got = load(d, "chain_sat64_sq7", np.uint64, np.uint64)
    same(got, m, "C++ MagnusMatrix matmul / matmul_seq chain (Sat64)")
    assert int((got[2] == np.iinfo(np.uint64).max).sum()) == 1176  # SURVEY §8(c) golden 2
    a = O.convert(O.torus_thinned(30, 3.0, O.Rng()), O.SAT64)
    same(load(d, "torus30_sat64_a2", np.uint64, np.uint64), O.matmul_seq(a, a), "C++ MagnusMatrix A^2")


@pytest.mark.gpu
def test_cpp_drivers_f64_and_errors(run):
    d, s = run
    tri = O.from_edges(6, [(0, 1), (1, 2), (2, 0), (3, 4)])
    want, k = O.reachability_sum(tri)
    assert int(s["tri_reach_k"][0]) == k
    same(load(d, "tri_reach", np.uint32, np.uint32), want, "C++ reachability_sum")
    comp = O.connected_components(O.from_edges_undirected(6, [(0, 1), (1, 2), (3, 4)]))
    assert [int(x) for x in s["components"]] == [int(x) for x in comp]
    f = O.from_arrays(np.array([0, 2, 3, 5], np.uint64), np.array([0, 2, 1, 0, 1], np.uint32),
                      np.array([0.1, 0.7, 1.3, -2.5, 0.3]), O.F64)
    same(load(d, "f64_sq", np.uint32, np.float64), O.matmul_seq(f, f), "C++ Csr<f64>::matmul_par")
    assert s["mismatch_status"] == ["2"]  # SLAT_EDIM where the reference panics


@pytest.mark.gpu
def test_cpp_e2e_headline_step(run):
    """The drop-in's host-vector cost of the headline step A^6 * A (PCIe both ways included)."""
    _, s = run
    assert int(s["e2e_a7_nnz"][0]) == 11736555
    assert float(s["e2e_a7_ms"][0]) > 0
