/*
 * slat.hpp — header-only C++ drop-in over the C ABI (slat.h) with the reference's types, method
 * names, argument meaning and failure behaviour:
 *
 *   reference (Rust)                                        here
 *   graph_csr::CsrMatrix        src/graph_csr.rs:39-53      slat::CsrMatrix  (n u32, row_ptr usize,
 *                                                            col_idx u32, values u32 saturating)
 *     ::matmul                  src/graph_csr.rs:306-346      CsrMatrix::matmul      -> slat_spgemm_csr_u32
 *     ::matmul_par              src/graph_csr.rs:350-484      CsrMatrix::matmul_par  -> slat_spgemm_csr_u32
 *     ::add / identity / from_coo / from_edges / lattice / thin / get / nnz
 *     ::reachability_sum / power_until_stable / connected_components (:545-603), written exactly as the
 *       reference writes them: loops over matmul / add on host values (their call sites are unchanged)
 *   graph_magnus::MagnusMatrix  src/graph_magnus.rs:11-14    slat::MagnusMatrix (n usize, mat: row_ptr,
 *                                                            col_idx usize, values Sat64 = u64)
 *     ::matmul (parallel)       src/graph_magnus.rs:224-232   MagnusMatrix::matmul     -> slat_magnus_matmul
 *     ::matmul_seq              src/graph_magnus.rs:234-242   MagnusMatrix::matmul_seq -> slat_magnus_matmul
 *   linalg::csr::Csr<u32, V>    linalg/src/csr.rs:93-98      slat::Csr<V>, V = uint32_t | uint64_t | double
 *     ::matmul / matmul_par     linalg/src/csr.rs:308-466     Csr<V>::matmul / matmul_par -> slat_spgemm_csr_*
 *
 * Ownership and threading follow the reference: inputs are borrowed (`const&`), the result is a new
 * owned value in host vectors, nothing is cached across calls. Each host thread gets its own device
 * context on first use (a thread_local slat_ctx on device slat::thread_device(), default 0): calls
 * from several threads never share a stream. Where the reference panics (`assert_eq!(self.n,
 * other.n)`, src/graph_csr.rs:307,351) a slat::Error is thrown; its status() is the C ABI's code
 * (SLAT_EDIM for a shape mismatch).
 *
 * Host-resident operands cross PCIe on every call (H2D of both operands, D2H of the result), as the
 * reference's Vec in / Vec out signature implies; chains that can stay on the device should use the C
 * ABI's device views instead (slat_csr_view_of of the previous product).
 */
#ifndef SLAT_HPP
#define SLAT_HPP

#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "slat.h"

namespace slat {

static_assert(sizeof(size_t) == 8, "usize row pointers are 64-bit (the reference's targets)");

using NodeId = uint32_t;  // src/graph_csr.rs:14
using Val = uint32_t;     // src/graph_csr.rs:17

class Error : public std::runtime_error {
  public:
    Error(slat_status s, const std::string &what) : std::runtime_error(what), status_(s) {}
    slat_status status() const { return status_; }

  private:
    slat_status status_;
};

namespace detail {

inline int &device_slot() {
    thread_local int dev = 0;
    return dev;
}

struct ThreadCtx {
    slat_ctx *p = nullptr;
    ~ThreadCtx() {
        if (p) slat_ctx_destroy(p);
    }
};

inline ThreadCtx &thread_ctx_holder() {
    thread_local ThreadCtx h;
    return h;
}

inline void check(slat_status s, slat_ctx *ctx) {
    if (s == SLAT_OK) return;
    std::string msg = std::string("slat: ") + slat_status_string(s);
    if (ctx) {
        const char *d = slat_last_error(ctx);
        if (d && *d) msg += std::string(" (") + d + ")";
    }
    throw Error(s, msg);
}

}  // namespace detail

// The device this thread's context opens (before its first call; later changes are ignored).
inline void set_thread_device(int device) { detail::device_slot() = device; }
inline int thread_device() { return detail::device_slot(); }

// This thread's context, created on first use.
inline slat_ctx *thread_ctx() {
    detail::ThreadCtx &h = detail::thread_ctx_holder();
    if (!h.p) detail::check(slat_ctx_create(detail::device_slot(), &h.p), nullptr);
    return h.p;
}

// MATMUL_PROGRESS.store(on) (src/graph_csr.rs:11): the library's pass summary lines per product.
inline void set_matmul_progress(bool on) { (void)slat_set_matmul_progress(on ? 1 : 0); }

// rand 0.9 StdRng (ChaCha12) as the reference seeds it: StdRng::from_seed([42; 32]) by default.
class StdRng {
  public:
    explicit StdRng(const uint8_t seed[32]) { slat_rng_seed(&s_, seed); }
    static StdRng from_seed(uint8_t byte = 42) {
        uint8_t seed[32];
        std::memset(seed, byte, sizeof seed);
        return StdRng(seed);
    }
    uint64_t next_u64() { return slat_rng_next_u64(&s_); }
    double random_f64() { return slat_rng_next_f64(&s_); }
    slat_rng *raw() { return &s_; }

  private:
    slat_rng s_;
};

namespace detail {

template <typename V>
constexpr int32_t dtype_of() {
    static_assert(std::is_same<V, uint32_t>::value || std::is_same<V, uint64_t>::value || std::is_same<V, double>::value,
                  "values are u32, Sat64 (u64) or f64");
    return std::is_same<V, uint32_t>::value ? SLAT_U32 : std::is_same<V, uint64_t>::value ? SLAT_SAT64 : SLAT_F64;
}

template <typename V>
slat_csr_view host_view(uint64_t n_rows, uint64_t n_cols, const std::vector<size_t> &row_ptr,
                        const std::vector<uint32_t> &col_idx, const std::vector<V> &values) {
    slat_csr_view v;
    std::memset(&v, 0, sizeof v);
    v.n_rows = n_rows;
    v.n_cols = n_cols;
    v.nnz = col_idx.size();
    v.row_ptr = reinterpret_cast<const uint64_t *>(row_ptr.data());
    v.col_idx = col_idx.data();
    v.values = values.data();
    v.dtype = dtype_of<V>();
    v.residency = SLAT_HOST;
    v.max_row_nnz = 0;
    return v;
}

// C = A * B for host-resident CSR operands into fresh host vectors; the device result is freed
template <typename V>
void spgemm_host(const slat_csr_view &a, const slat_csr_view &b, std::vector<size_t> &row_ptr,
                 std::vector<uint32_t> &col_idx, std::vector<V> &values) {
    slat_ctx *ctx = thread_ctx();
    slat_csr c;
    std::memset(&c, 0, sizeof c);
    slat_status s = dtype_of<V>() == SLAT_U32     ? slat_spgemm_csr_u32(ctx, &a, &b, &c, 0)
                    : dtype_of<V>() == SLAT_SAT64 ? slat_spgemm_csr_sat64(ctx, &a, &b, &c, 0)
                                                  : slat_spgemm_csr_f64(ctx, &a, &b, &c, 0);
    check(s, ctx);
    try {
        row_ptr.resize(c.n_rows + 1);
        col_idx.resize(c.nnz);
        values.resize(c.nnz);
        const slat_csr_view cv = slat_csr_view_of(&c);
        check(slat_csr_to_host(ctx, &cv, reinterpret_cast<uint64_t *>(row_ptr.data()), col_idx.data(), values.data()),
              ctx);
    } catch (...) {
        slat_csr_free(ctx, &c);
        throw;
    }
    slat_csr_free(ctx, &c);
}

struct HostCsrOwner {
    slat_host_csr h;
    HostCsrOwner() { std::memset(&h, 0, sizeof h); }
    ~HostCsrOwner() { slat_host_csr_free(&h); }
    HostCsrOwner(const HostCsrOwner &) = delete;
    HostCsrOwner &operator=(const HostCsrOwner &) = delete;
};

template <typename V>
void take_host(const slat_host_csr &h, std::vector<size_t> &row_ptr, std::vector<uint32_t> &col_idx, std::vector<V> &values) {
    row_ptr.assign(reinterpret_cast<const size_t *>(h.row_ptr), reinterpret_cast<const size_t *>(h.row_ptr) + h.n + 1);
    col_idx.assign(h.col_idx, h.col_idx + h.nnz);
    values.assign(static_cast<const V *>(h.values), static_cast<const V *>(h.values) + h.nnz);
}

}  // namespace detail

// ---------------------------------------------------------------------------------------------
// graph_csr::CsrMatrix (src/graph_csr.rs:39-53)
// ---------------------------------------------------------------------------------------------
struct CsrMatrix {
    NodeId n = 0;
    std::vector<size_t> row_ptr{0};
    std::vector<NodeId> col_idx;
    std::vector<Val> values;
    std::optional<std::vector<NodeId>> perm;  // not propagated by matmul (src/graph_csr.rs:345,483)

    // CsrMatrix::new (src/graph_csr.rs:56-65): the empty n x n matrix
    static CsrMatrix empty(NodeId n) {
        CsrMatrix m;
        m.n = n;
        m.row_ptr.assign((size_t)n + 1, 0);
        return m;
    }
    // CsrMatrix::identity (src/graph_csr.rs:68-80)
    static CsrMatrix identity(NodeId n) {
        CsrMatrix m;
        m.n = n;
        m.row_ptr.resize((size_t)n + 1);
        m.col_idx.resize(n);
        m.values.assign(n, 1u);
        for (NodeId i = 0; i <= n; ++i) m.row_ptr[i] = i;
        for (NodeId i = 0; i < n; ++i) m.col_idx[i] = i;
        return m;
    }
    // CsrMatrix::from_coo (src/graph_csr.rs:83-129): sort by (row, col), sum duplicates, drop zeros
    static CsrMatrix from_coo(NodeId n, const std::vector<std::tuple<NodeId, NodeId, Val>> &triplets) {
        std::vector<uint32_t> r(triplets.size()), c(triplets.size()), v(triplets.size());
        for (size_t i = 0; i < triplets.size(); ++i) std::tie(r[i], c[i], v[i]) = triplets[i];
        detail::HostCsrOwner o;
        detail::check(slat_host_from_coo(n, triplets.size(), r.data(), c.data(), v.data(), SLAT_U32, &o.h), nullptr);
        CsrMatrix m;
        m.n = n;
        detail::take_host(o.h, m.row_ptr, m.col_idx, m.values);
        return m;
    }
    // CsrMatrix::from_edges (src/graph_csr.rs:131-135): value 1 per edge, duplicates summed
    static CsrMatrix from_edges(NodeId n, const std::vector<std::pair<NodeId, NodeId>> &edges) {
        std::vector<std::tuple<NodeId, NodeId, Val>> t;
        t.reserve(edges.size());
        for (const auto &e : edges) t.emplace_back(e.first, e.second, 1u);
        return from_coo(n, t);
    }
    // CsrMatrix::from_edges_undirected (src/graph_csr.rs:138-147): each edge and its mirror (r != c)
    static CsrMatrix from_edges_undirected(NodeId n, const std::vector<std::pair<NodeId, NodeId>> &edges) {
        std::vector<std::tuple<NodeId, NodeId, Val>> t;
        t.reserve(edges.size() * 2);
        for (const auto &e : edges) {
            t.emplace_back(e.first, e.second, 1u);
            if (e.first != e.second) t.emplace_back(e.second, e.first, 1u);
        }
        return from_coo(n, t);
    }
    // CsrMatrix::lattice (src/graph_csr.rs:177-222)
    static CsrMatrix lattice(const std::vector<size_t> &dims, bool torus) {
        std::vector<uint64_t> d(dims.begin(), dims.end());
        detail::HostCsrOwner o;
        detail::check(slat_host_lattice(d.data(), (int)d.size(), torus ? 1 : 0, &o.h), nullptr);
        CsrMatrix m;
        m.n = (NodeId)o.h.n;
        detail::take_host(o.h, m.row_ptr, m.col_idx, m.values);
        return m;
    }
    // CsrMatrix::thin (src/graph_csr.rs:225-247): the same draws from the same StdRng stream
    CsrMatrix thin(StdRng &rng, double density) const {
        slat_host_csr in;
        std::memset(&in, 0, sizeof in);
        in.n = n;
        in.nnz = col_idx.size();
        in.row_ptr = const_cast<uint64_t *>(reinterpret_cast<const uint64_t *>(row_ptr.data()));
        in.col_idx = const_cast<uint32_t *>(col_idx.data());
        in.values = const_cast<uint32_t *>(values.data());
        in.dtype = SLAT_U32;
        detail::HostCsrOwner o;
        detail::check(slat_host_thin(&in, rng.raw(), density, &o.h), nullptr);
        CsrMatrix m;
        m.n = n;
        detail::take_host(o.h, m.row_ptr, m.col_idx, m.values);
        return m;
    }

    size_t nnz() const { return col_idx.size(); }
    // CsrMatrix::get (src/graph_csr.rs:250-258): binary search in the sorted row
    Val get(NodeId r, NodeId c) const {
        const auto b = col_idx.begin() + (std::ptrdiff_t)row_ptr[r], e = col_idx.begin() + (std::ptrdiff_t)row_ptr[r + 1];
        const auto it = std::lower_bound(b, e, c);
        return it != e && *it == c ? values[(size_t)(it - col_idx.begin())] : 0u;
    }

    // CsrMatrix::matmul (src/graph_csr.rs:306-346) on the GPU: the same result bit for bit
    CsrMatrix matmul(const CsrMatrix &other) const { return product(other); }
    // CsrMatrix::matmul_par (src/graph_csr.rs:350-484): the same call (identical results)
    CsrMatrix matmul_par(const CsrMatrix &other) const { return product(other); }

    // CsrMatrix::add (src/graph_csr.rs:487-542) on the GPU (saturating union of sorted rows)
    CsrMatrix add(const CsrMatrix &other) const {
        slat_ctx *ctx = thread_ctx();
        const slat_csr_view a = detail::host_view(n, n, row_ptr, col_idx, values);
        const slat_csr_view b = detail::host_view(other.n, other.n, other.row_ptr, other.col_idx, other.values);
        slat_csr c;
        std::memset(&c, 0, sizeof c);
        detail::check(slat_csr_add(ctx, &a, &b, &c), ctx);
        CsrMatrix out;
        out.n = n;
        try {
            out.row_ptr.resize((size_t)n + 1);
            out.col_idx.resize(c.nnz);
            out.values.resize(c.nnz);
            const slat_csr_view cv = slat_csr_view_of(&c);
            detail::check(slat_csr_to_host(ctx, &cv, reinterpret_cast<uint64_t *>(out.row_ptr.data()), out.col_idx.data(),
                                           out.values.data()),
                          ctx);
        } catch (...) {
            slat_csr_free(ctx, &c);
            throw;
        }
        slat_csr_free(ctx, &c);
        return out;
    }

    // The reference's SpGEMM consumers (src/graph_csr.rs:545-603), written as the reference writes
    // them: their matmul / add call sites are the ones above, unchanged.
    std::pair<CsrMatrix, size_t> reachability_sum() const {
        CsrMatrix sum = *this, power = *this;
        size_t k = 1;
        for (;;) {
            power = power.matmul(*this);
            k += 1;
            CsrMatrix new_sum = sum.add(power);
            if (new_sum.nnz() == sum.nnz()) return {new_sum, k};
            sum = std::move(new_sum);
        }
    }
    std::pair<CsrMatrix, size_t> power_until_stable() const {
        CsrMatrix current = *this;
        size_t k = 0;
        for (;;) {
            CsrMatrix next = current.matmul(current);
            k += 1;
            if (next.nnz() == current.nnz() && next.col_idx == current.col_idx && next.row_ptr == current.row_ptr)
                return {next, k};
            current = std::move(next);
        }
    }
    std::vector<size_t> connected_components() const {
        const CsrMatrix with_id = add(identity(n));
        const CsrMatrix closure = with_id.power_until_stable().first;
        std::vector<size_t> component((size_t)n, SIZE_MAX);
        size_t next_id = 0;
        for (NodeId i = 0; i < n; ++i) {
            if (component[i] != SIZE_MAX) continue;
            component[i] = next_id;
            for (NodeId j = i + 1; j < n; ++j)
                if (closure.get(i, j) > 0 && closure.get(j, i) > 0) component[j] = next_id;
            next_id += 1;
        }
        return component;
    }

  private:
    CsrMatrix product(const CsrMatrix &other) const {
        if (n != other.n)  // assert_eq!(self.n, other.n) (src/graph_csr.rs:307,351)
            throw Error(SLAT_EDIM, "slat: dimension mismatch (self.n != other.n)");
        const slat_csr_view a = detail::host_view(n, n, row_ptr, col_idx, values);
        const slat_csr_view b = detail::host_view(other.n, other.n, other.row_ptr, other.col_idx, other.values);
        CsrMatrix c;
        c.n = n;
        detail::spgemm_host<Val>(a, b, c.row_ptr, c.col_idx, c.values);
        return c;  // perm: None (src/graph_csr.rs:345)
    }
};

// ---------------------------------------------------------------------------------------------
// graph_magnus::MagnusMatrix (src/graph_magnus.rs:11-14): magnus::SparseMatrixCSR<Sat64>
// ---------------------------------------------------------------------------------------------
struct SparseMatrixCSR {  // the magnus crate's layout (row_ptr, col_idx usize; values Sat64)
    size_t n_rows = 0, n_cols = 0;
    std::vector<size_t> row_ptr{0};
    std::vector<size_t> col_idx;
    std::vector<uint64_t> values;
    size_t nnz() const { return col_idx.size(); }
};

struct MagnusMatrix {
    size_t n = 0;
    SparseMatrixCSR mat;

    static MagnusMatrix empty(size_t n) {  // MagnusMatrix::new (src/graph_magnus.rs:17-22)
        MagnusMatrix m;
        m.n = n;
        m.mat.n_rows = m.mat.n_cols = n;
        m.mat.row_ptr.assign(n + 1, 0);
        return m;
    }
    // MagnusMatrix::from_edges (src/graph_magnus.rs:78-82): value 1 per edge, duplicates summed
    static MagnusMatrix from_edges(size_t n, const std::vector<std::pair<size_t, size_t>> &edges) {
        std::vector<uint32_t> r(edges.size()), c(edges.size());
        std::vector<uint64_t> v(edges.size(), 1);
        for (size_t i = 0; i < edges.size(); ++i) {
            r[i] = (uint32_t)edges[i].first;
            c[i] = (uint32_t)edges[i].second;
        }
        detail::HostCsrOwner o;
        detail::check(slat_host_from_coo(n, edges.size(), r.data(), c.data(), v.data(), SLAT_SAT64, &o.h), nullptr);
        MagnusMatrix m;
        m.n = n;
        m.mat.n_rows = m.mat.n_cols = n;
        m.mat.row_ptr.assign(reinterpret_cast<const size_t *>(o.h.row_ptr), reinterpret_cast<const size_t *>(o.h.row_ptr) + n + 1);
        m.mat.col_idx.assign(o.h.col_idx, o.h.col_idx + o.h.nnz);  // widened to usize
        m.mat.values.assign((const uint64_t *)o.h.values, (const uint64_t *)o.h.values + o.h.nnz);
        return m;
    }
    // the MagnusMatrix of a CsrMatrix's entries (the benches build both from one generator's
    // triplets, src/graph_magnus.rs:720-729)
    static MagnusMatrix from_csr(const CsrMatrix &a) {
        MagnusMatrix m;
        m.n = a.n;
        m.mat.n_rows = m.mat.n_cols = a.n;
        m.mat.row_ptr = a.row_ptr;
        m.mat.col_idx.assign(a.col_idx.begin(), a.col_idx.end());
        m.mat.values.assign(a.values.begin(), a.values.end());
        return m;
    }

    size_t nnz() const { return mat.nnz(); }
    uint64_t get(size_t r, size_t c) const {
        const auto b = mat.col_idx.begin() + (std::ptrdiff_t)mat.row_ptr[r], e = mat.col_idx.begin() + (std::ptrdiff_t)mat.row_ptr[r + 1];
        const auto it = std::lower_bound(b, e, c);
        return it != e && *it == c ? mat.values[(size_t)(it - mat.col_idx.begin())] : 0u;
    }

    // MagnusMatrix::matmul (magnus_spgemm_parallel, src/graph_magnus.rs:224-232) on the GPU
    MagnusMatrix matmul(const MagnusMatrix &other) const { return product(other); }
    // MagnusMatrix::matmul_seq (magnus_spgemm, src/graph_magnus.rs:234-242): the same result
    MagnusMatrix matmul_seq(const MagnusMatrix &other) const { return product(other); }

  private:
    static slat_magnus_view view(const MagnusMatrix &m) {
        slat_magnus_view v;
        std::memset(&v, 0, sizeof v);
        v.n_rows = m.mat.n_rows;
        v.n_cols = m.mat.n_cols;
        v.nnz = m.mat.col_idx.size();
        v.row_ptr = reinterpret_cast<const uint64_t *>(m.mat.row_ptr.data());
        v.col_idx = reinterpret_cast<const uint64_t *>(m.mat.col_idx.data());
        v.values = m.mat.values.data();
        v.residency = SLAT_HOST;
        return v;
    }
    MagnusMatrix product(const MagnusMatrix &other) const {
        if (n != other.n) throw Error(SLAT_EDIM, "slat: dimension mismatch (self.n != other.n)");
        slat_ctx *ctx = thread_ctx();
        const slat_magnus_view a = view(*this), b = view(other);
        slat_magnus c;
        std::memset(&c, 0, sizeof c);
        detail::check(slat_magnus_matmul(ctx, &a, &b, &c, 0), ctx);
        MagnusMatrix out;
        out.n = n;
        out.mat.n_rows = c.n_rows;
        out.mat.n_cols = c.n_cols;
        try {
            out.mat.row_ptr.resize(c.n_rows + 1);
            out.mat.col_idx.resize(c.nnz);
            out.mat.values.resize(c.nnz);
            detail::check(slat_magnus_to_host(ctx, &c, reinterpret_cast<uint64_t *>(out.mat.row_ptr.data()),
                                              reinterpret_cast<uint64_t *>(out.mat.col_idx.data()), out.mat.values.data()),
                          ctx);
        } catch (...) {
            slat_magnus_free(ctx, &c);
            throw;
        }
        slat_magnus_free(ctx, &c);
        return out;
    }
};

// ---------------------------------------------------------------------------------------------
// linalg::csr::Csr<u32, V> (linalg/src/csr.rs:93-98), square matrices; V = u32 / u64 (saturating)
// or f64 (the reference's left fold in A-row order, bit for bit)
// ---------------------------------------------------------------------------------------------
template <typename V>
struct Csr {
    std::vector<size_t> shape{0, 0};
    std::vector<size_t> row_ptr{0};
    std::vector<uint32_t> col_idx;
    std::vector<V> values;

    size_t nnz() const { return col_idx.size(); }
    // Csr::matmul (linalg/src/csr.rs:308-356); the square check of :309-311 throws SLAT_EDIM
    Csr matmul(const Csr &other) const { return product(other); }
    // Csr::matmul_par (linalg/src/csr.rs:361-466): the same result
    Csr matmul_par(const Csr &other) const { return product(other); }

  private:
    Csr product(const Csr &other) const {
        if (shape.size() != 2 || other.shape.size() != 2 || shape[0] != shape[1] || other.shape[0] != other.shape[1] ||
            shape[1] != other.shape[0])
            throw Error(SLAT_EDIM, "slat: matmul needs square matrices of one size");
        const slat_csr_view a = detail::host_view(shape[0], shape[1], row_ptr, col_idx, values);
        const slat_csr_view b = detail::host_view(other.shape[0], other.shape[1], other.row_ptr, other.col_idx, other.values);
        Csr c;
        c.shape = {shape[0], other.shape[1]};
        detail::spgemm_host<V>(a, b, c.row_ptr, c.col_idx, c.values);
        return c;
    }
};

}  // namespace slat

#endif  // SLAT_HPP
