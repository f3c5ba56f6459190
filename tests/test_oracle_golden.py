"""The oracle (C restatement, oracle/) pinned against the golden vectors and the reference's own
known-answer tests. CPU only."""
import numpy as np
import pytest

import oracle_py as O
from helpers import assert_digest, digest

# README.md:41-46 prints nnz(C) rounded: 252k, 655k, 1.57M, 3.38M, 6.59M, 11.7M.
README_NNZ = {2: (252e3, 1e3), 3: (655e3, 1e3), 4: (1.57e6, 1e4), 5: (3.38e6, 1e4), 6: (6.59e6, 1e4),
              7: (11.7e6, 1e5)}


# RFC 8439 appendix A.1, test vectors #1 and #2: ChaCha20 keystream for the all-zero key and nonce,
# block counters 0 and 1 (the SURVEY.md section 8(c) probe's "ade0b876..., block 1 bee7079f")
RFC8439_ZERO_KEY = {
    0: "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
       "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586",
    1: "9f07e7be5551387a98ba977c732d080dcb0f29a048e3656912c6533e32ee7aed"
       "29b721769ce64e43d57133b074d839d531ed1f28510afb45ace10a1f4b794d6f",
}


def test_chacha12_zero_key_vector():
    """The oracle's ChaCha core (the one StdRng's ChaCha12 runs with 6 double rounds) run with 10
    double rounds reproduces the RFC 8439 ChaCha20 zero-key keystream, so the quarter round, the
    state layout (constants, key words, 64-bit counter in words 12-13, zero stream) and the final
    addition are right; the 12-round StdRng then only differs in the round count."""
    import struct
    for ctr, hexs in RFC8439_ZERO_KEY.items():
        words = O.chacha_block([0] * 8, ctr, 10)
        assert struct.pack("<16I", *words).hex() == hexs, f"block {ctr}"
    assert O.chacha_block([0] * 8, 0, 10)[0] == 0xADE0B876
    assert O.chacha_block([0] * 8, 1, 10)[0] == 0xBEE7079F
    # the 12-round core is a different function of the same state, and StdRng's first draws come
    # from its block 0 words 0-1 (seed [42;32])
    k42 = [0x2A2A2A2A] * 8
    b12 = O.chacha_block(k42, 0, 6)
    assert b12 != O.chacha_block(k42, 0, 10)
    r = O.Rng()
    assert r.next_u64() == b12[0] | (b12[1] << 32)
    assert r.next_u64() == b12[2] | (b12[3] << 32)


def test_readme_nnz_sequence_pins_oracle(golden):
    rng = O.Rng()
    A = O.torus_thinned(30, 3.0, rng)
    assert A.nnz == 81434
    P = A
    for k in range(2, 8):
        P = O.matmul_seq(P, A)
        want, tol = README_NNZ[k]
        assert abs(P.nnz - want) <= tol / 2 + 1, (k, P.nnz)
        assert P.nnz == golden["torus30_powers"][k - 1]["nnz"]


def test_oracle_matches_scipy_digests(golden):
    rng = O.Rng()
    A = O.torus_thinned(30, 3.0, rng)
    assert_digest(digest(*A.arrays()), golden["torus30_powers"][0], "A")
    P = A
    for k in range(2, 6):
        P = O.matmul_seq(P, A)
        assert_digest(digest(*P.arrays()), golden["torus30_powers"][k - 1], f"A^{k}")


def test_oracle_sweep_grid(golden):
    rng = O.Rng()  # ONE rng shared across the grid (src/graph_magnus.rs:800)
    cells = iter(golden["sweep"])
    for s in [5, 10, 20]:
        full = O.lattice([s, s, s], True)
        for epn in [2.0, 3.0, 4.0, 8.0, 26.0]:
            cell = next(cells)
            density = epn / (full.nnz / full.n)
            A = O.thin(full, rng, density) if density < 1.0 else full
            assert_digest(digest(*A.arrays()), cell["A"], f"s={s} epn={epn} A")
            C = O.matmul_seq(A, A)
            assert_digest(digest(*C.arrays()), cell["A2"], f"s={s} epn={epn} A2")


def test_par_equals_seq_u32():
    rng = O.Rng()
    A = O.torus_thinned(20, 4.0, rng)
    A3 = O.matmul_seq(O.matmul_seq(A, A), A)
    for a, b in [(A, A), (A3, A)]:
        s = O.matmul_seq(a, b).arrays()
        p = O.matmul_par(a, b, 4).arrays()
        for x, y in zip(s, p):
            np.testing.assert_array_equal(x, y)


# --- hand-computed known answers from the reference's unit tests (src/graph_csr.rs:878-1145) ---
@pytest.mark.parametrize("dtype", [O.U32, O.SAT64, O.F64])
def test_reference_unit_cases(dtype):
    m = O.from_edges(3, [(0, 1), (1, 2)], dtype)
    r = O.matmul_seq(m, O.identity(3, dtype))
    assert r.get(0, 1) == 1 and r.get(1, 2) == 1 and r.get(0, 2) == 0 and r.nnz == 2
    t = O.from_edges(3, [(0, 1), (1, 2), (2, 0)], dtype)
    t2 = O.matmul_seq(t, t)
    assert t2.get(0, 2) == 1 and t2.get(1, 0) == 1 and t2.get(2, 1) == 1
    t3 = O.matmul_seq(t2, t)
    assert t3.get(0, 0) == 1 and t3.get(1, 1) == 1 and t3.get(2, 2) == 1
    assert O.from_edges(2, [(0, 1), (0, 1)], dtype).get(0, 1) == 2
    d = O.from_edges(4, [(0, 1), (0, 2), (1, 3), (2, 3)], dtype)
    assert O.matmul_seq(d, d).get(0, 3) == 2


def test_lattice_counts():
    assert O.lattice([5], False).nnz == 8
    assert O.lattice([5], True).nnz == 10
    assert O.lattice([3, 3], True).nnz == 72
    assert O.lattice([2, 2, 2], False).nnz == 56


def test_saturation_chain():
    """test_power_until_stable_chain (src/graph_csr.rs:931-939): (I+N)^(2^k) on a 64-chain saturates
    u32 at iterations 6/7 and Sat64 at 7 (counts from SURVEY §8(c) golden 2)."""
    n = 64
    for dtype, want in [(O.U32, {6: 1568, 7: 1711}), (O.SAT64, {7: 1176})]:
        m = O.from_edges(n, [(i, i + 1) for i in range(n - 1)], dtype)
        cur = O.add(m, O.identity(n, dtype))
        it = 0
        while True:
            nxt = O.matmul_seq(cur, cur)
            it += 1
            rp0, c0, _ = cur.arrays()
            rp1, c1, v1 = nxt.arrays()
            mx = 0xFFFFFFFF if dtype == O.U32 else 0xFFFFFFFFFFFFFFFF
            if it in want:
                assert int((v1 == mx).sum()) == want[it], (dtype, it)
            if nxt.nnz == cur.nnz and np.array_equal(rp0, rp1) and np.array_equal(c0, c1):
                break
            cur = nxt
        assert it == 7
