"""The oracle's restatements of the SpGEMM consumers (oracle.c: orc_reachability_sum,
orc_power_until_stable, orc_connected_components; src/graph_csr.rs:545-603) pinned by the
reference's own unit-test answers (src/graph_csr.rs:918-965, 1096-1106). CPU only."""
import oracle_py as O


def undirected(n, edges):
    e = [(a, b) for a, b in edges] + [(b, a) for a, b in edges if a != b]
    return O.from_edges(n, e)


def test_reachability_chain():
    s, k = O.reachability_sum(O.from_edges(4, [(0, 1), (1, 2), (2, 3)]))
    for a, b in [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]:
        assert s.get(a, b) > 0
    assert s.get(3, 0) == 0 and s.get(2, 0) == 0
    assert k == 4


def test_power_until_stable_chain():
    n = 64
    m = O.from_edges(n, [(i, i + 1) for i in range(n - 1)])
    _, iters = O.power_until_stable(O.add(m, O.identity(n)))
    assert iters <= 8


def test_connected_components():
    c = O.connected_components(undirected(6, [(0, 1), (1, 2), (2, 0), (3, 4), (4, 5), (5, 3)]))
    assert c[0] == c[1] == c[2] and c[3] == c[4] == c[5] and c[0] != c[3]
    assert len(set(O.connected_components(O.from_edges(5, [])).tolist())) == 5
    c = O.connected_components(undirected(4, [(0, 1), (1, 2), (2, 3)]))
    assert c[0] == c[1] == c[2] == c[3]


def test_identity():
    i = O.identity(4, O.SAT64)
    assert i.nnz == 4 and all(i.get(k, k) == 1 for k in range(4))
