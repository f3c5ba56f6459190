"""The reference's constructors on the device: CsrMatrix::from_coo,
lattice and thin (src/graph_csr.rs:83-129, 177-247) through slat_csr_from_coo / slat_csr_lattice /
slat_csr_thin, against the oracle's restatements and the golden digests. Bar: bit-exact arrays
(f64 duplicate sums use values whose sums are exact in any order), the same RNG stream position
afterwards as the host StdRng."""
import numpy as np
import pytest

import oracle_py as O
import slat
from helpers import assert_digest, digest

pytestmark = pytest.mark.gpu

CLS = {O.U32: slat.CsrMatrix, O.SAT64: slat.MagnusMatrix, O.F64: slat.CsrF64}


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def assert_same(dev, orc: O.Csr, what=""):
    h = dev.host()
    rp, col, val = orc.arrays()
    assert dev.nnz() == orc.nnz, f"{what}: nnz {dev.nnz()} != {orc.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(h.col_idx, col, err_msg=f"{what} col_idx")
    if val.dtype == np.float64:
        np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=f"{what} f64 bits")
    else:
        np.testing.assert_array_equal(h.values, val, err_msg=f"{what} values")


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64, O.F64])
@pytest.mark.parametrize("n,nt", [(1, 1), (7, 40), (1000, 5000), (50_000, 400_000)])
def test_from_coo_matches_oracle(ctx, dtype, n, nt):
    g = np.random.default_rng(n + nt)
    r = g.integers(0, n, nt)
    c = g.integers(0, n, nt)
    if dtype == O.F64:
        v = g.integers(-4, 5, nt).astype(np.float64) * 0.5  # duplicate sums exact in any order; zeros drop
    else:
        v = g.integers(0, 6, nt)  # zeros and duplicates
    want = O.from_coo(n, r, c, v, dtype)
    got = CLS[dtype].from_coo_device(n, r, c, v, ctx)
    assert_same(got, want, f"from_coo n={n} nt={nt}")


def test_from_coo_u32_wrapping_sum_and_errors(ctx):
    # 0xFFFFFFFF + 1 wraps to 0 (`+=` in a release build) and the entry is dropped
    r, c = [0, 0, 1, 1], [1, 1, 0, 0]
    v = [0xFFFFFFFF, 1, 3, 4]
    assert_same(slat.CsrMatrix.from_coo_device(2, r, c, v, ctx), O.from_coo(2, r, c, v, O.U32), "wrap")
    with pytest.raises(slat.SlatError):
        slat.CsrMatrix.from_coo_device(2, [0, 2], [0, 0], [1, 1], ctx)
    e = slat.CsrMatrix.from_coo_device(5, [], [], [], ctx)
    assert e.nnz() == 0 and e.n == 5


@pytest.mark.parametrize("dims,torus", [([5], False), ([5], True), ([2, 2], True), ([3, 3], True),
                                        ([2, 2, 2], False), ([4, 5, 6], True), ([3, 4, 2, 3], False)])
def test_lattice_matches_oracle(ctx, dims, torus):
    assert_same(slat.CsrMatrix.lattice(dims, torus, ctx), O.lattice(dims, torus), f"lattice {dims} {torus}")


def test_thin_matches_oracle_and_stream(ctx):
    # one generator shared by consecutive thins (the sweep's pattern, src/graph_magnus.rs:800)
    rng_d, rng_o = slat.StdRng(), O.Rng()
    for s, epn in [(5, 2.0), (5, 4.0), (10, 3.0), (12, 8.0)]:
        full_d = slat.CsrMatrix.lattice([s, s, s], True, ctx)
        full_o = O.lattice([s, s, s], True)
        dens = epn / (full_o.nnz / full_o.n)
        assert_same(full_d.thin(rng_d, dens), O.thin(full_o, rng_o, dens), f"thin {s} {epn}")
    assert rng_d.next_u64() == rng_o.next_u64()  # both generators at the same stream position


def test_torus30_device_generator_golden(ctx, golden):
    a = slat.torus_thinned_device(30, 3.0, slat.StdRng(), ctx)
    h = a.host()
    assert_digest(digest(h.row_ptr, h.col_idx, h.values), golden["torus30_powers"][0], "30^3 A (device)")


def test_torus100_device_generator_golden(ctx, golden):
    a = slat.torus_thinned_device(100, 3.0, slat.StdRng(), ctx)
    h = a.host()
    assert_digest(digest(h.row_ptr, h.col_idx, h.values), golden["torus100_powers"][0], "100^3 A (device)")


def test_generators_small_then_large_same_context(golden):
    # the sequence that exposed lost writes in the stream-ordered pool (DESIGN.md "Device memory"):
    # a 30^3 generation frees scratch, then the 100^3 lattice grows past it, on one fresh context
    c = slat.Context(0)
    for rep in range(2):
        a = slat.torus_thinned_device(30, 3.0, slat.StdRng(), c)
        h = a.host()
        assert_digest(digest(h.row_ptr, h.col_idx, h.values), golden["torus30_powers"][0], f"30^3 A rep {rep}")
        del a
        b = slat.torus_thinned_device(100, 3.0, slat.StdRng(), c)
        h = b.host()
        assert_digest(digest(h.row_ptr, h.col_idx, h.values), golden["torus100_powers"][0], f"100^3 A rep {rep}")
        del b


def test_from_coo_rejects_2_31_triplets():
    """The device sort counts items in an int: 2^31 triplets or more -> SLAT_ENOTSUP before any device
    work (a wrapped negative count would sort nothing)."""
    import ctypes as C
    ctx = slat.default_context(0)
    buf = C.c_void_p()
    slat.lib().slat_device_alloc(ctx.ptr, 4096, C.byref(buf))
    out = slat._lib.CsrOwned()
    for nt in (1 << 31, (1 << 32) - 1, 1 << 32):
        rc = slat.lib().slat_csr_from_coo(ctx.ptr, 1000, nt, buf, buf, buf, slat.U32, slat.DEVICE, C.byref(out))
        assert rc == 5, (nt, rc)  # SLAT_ENOTSUP
    slat.lib().slat_device_free(ctx.ptr, buf)
