// dropin.cpp — the C++ drop-in (include/slat.hpp) driven the way the reference's own code drives
// CsrMatrix / MagnusMatrix / Csr: host values in, host values out, the reference's method names.
// tests/test_dropin_cpp_gpu.py runs it and checks every written product against the oracle.
//
// usage: dropin OUT_DIR [e2e_iters]
//   writes OUT_DIR/<name>.{rp,col,val} (raw little-endian arrays) and OUT_DIR/summary.txt
#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <thread>

#include "slat.hpp"

static std::string g_dir;

template <typename T>
static void dump(const std::string &name, const std::vector<T> &v) {
    std::ofstream f(g_dir + "/" + name, std::ios::binary);
    f.write(reinterpret_cast<const char *>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
}
static void dump_csr(const std::string &name, const slat::CsrMatrix &m) {
    dump(name + ".rp", m.row_ptr), dump(name + ".col", m.col_idx), dump(name + ".val", m.values);
}
static void dump_magnus(const std::string &name, const slat::MagnusMatrix &m) {
    dump(name + ".rp", m.mat.row_ptr), dump(name + ".col", m.mat.col_idx), dump(name + ".val", m.mat.values);
}

// bench_repeated_exponentiation's input (src/graph_magnus.rs:707-719): the 30^3 Moore torus thinned
// to 3 edges per node with StdRng::from_seed([42; 32])
static slat::CsrMatrix torus30() {
    slat::StdRng rng = slat::StdRng::from_seed(42);
    const slat::CsrMatrix full = slat::CsrMatrix::lattice({30, 30, 30}, true);
    return full.thin(rng, 3.0 / ((double)full.nnz() / full.n));
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s OUT_DIR [e2e_iters]\n", argv[0]);
        return 2;
    }
    g_dir = argv[1];
    const int e2e_iters = argc > 2 ? std::atoi(argv[2]) : 0;
    std::FILE *sum = std::fopen((g_dir + "/summary.txt").c_str(), "w");
    try {
        // C1: A^2 on the 30^3 torus through matmul and matmul_par (src/graph_csr.rs:306,350)
        const slat::CsrMatrix a = torus30();
        dump_csr("torus30_a1", a);
        const slat::CsrMatrix a2 = a.matmul(a);
        const slat::CsrMatrix a2p = a.matmul_par(a);
        dump_csr("torus30_a2", a2);
        std::fprintf(sum, "a_nnz %zu\na2_nnz %zu\na2_par_equal %d\n", a.nnz(), a2.nnz(),
                     (int)(a2.row_ptr == a2p.row_ptr && a2.col_idx == a2p.col_idx && a2.values == a2p.values));
        const slat::CsrMatrix a3 = a2.matmul(a);
        dump_csr("torus30_a3", a3);

        // the saturating 64-chain (test_power_until_stable_chain, src/graph_csr.rs:931-939): (I + N)
        // squared until the pattern is stable, u32 through the reference's own power_until_stable
        std::vector<std::pair<slat::NodeId, slat::NodeId>> chain;
        for (slat::NodeId i = 0; i + 1 < 64; ++i) chain.emplace_back(i, i + 1);
        const slat::CsrMatrix in = slat::CsrMatrix::from_edges(64, chain).add(slat::CsrMatrix::identity(64));
        const auto stable = in.power_until_stable();
        dump_csr("chain_u32_stable", stable.first);
        std::fprintf(sum, "chain_u32_iters %zu\n", stable.second);

        // the same chain as MagnusMatrix (Sat64 values, usize columns): 7 squarings via matmul (the
        // parallel MAGNUS call) alternating with matmul_seq, as the reference's benches call both
        std::vector<std::pair<size_t, size_t>> chain64;
        for (size_t i = 0; i + 1 < 64; ++i) chain64.emplace_back(i, i + 1);
        for (size_t i = 0; i < 64; ++i) chain64.emplace_back(i, i);
        slat::MagnusMatrix m = slat::MagnusMatrix::from_edges(64, chain64);
        for (int k = 0; k < 7; ++k) m = (k % 2) ? m.matmul_seq(m) : m.matmul(m);
        dump_magnus("chain_sat64_sq7", m);
        const slat::MagnusMatrix mt = slat::MagnusMatrix::from_csr(a);
        dump_magnus("torus30_sat64_a2", mt.matmul(mt));

        // reachability_sum and connected_components, the reference's bodies over matmul / add
        const slat::CsrMatrix tri = slat::CsrMatrix::from_edges(6, {{0, 1}, {1, 2}, {2, 0}, {3, 4}});
        const auto reach = tri.reachability_sum();
        dump_csr("tri_reach", reach.first);
        std::fprintf(sum, "tri_reach_k %zu\n", reach.second);
        const std::vector<size_t> comp = slat::CsrMatrix::from_edges_undirected(6, {{0, 1}, {1, 2}, {3, 4}}).connected_components();
        std::fprintf(sum, "components");
        for (size_t c : comp) std::fprintf(sum, " %zu", c);
        std::fprintf(sum, "\n");

        // linalg Csr<u32, f64>: the left fold in A-row order
        slat::Csr<double> f;
        f.shape = {3, 3};
        f.row_ptr = {0, 2, 3, 5};
        f.col_idx = {0, 2, 1, 0, 1};
        f.values = {0.1, 0.7, 1.3, -2.5, 0.3};
        const slat::Csr<double> f2 = f.matmul_par(f);
        dump("f64_sq.rp", f2.row_ptr), dump("f64_sq.col", f2.col_idx), dump("f64_sq.val", f2.values);

        // assert_eq!(self.n, other.n) panics in the reference: here slat::Error with SLAT_EDIM
        int status = -1;
        try {
            (void)slat::CsrMatrix::empty(3).matmul(slat::CsrMatrix::empty(4));
        } catch (const slat::Error &e) {
            status = (int)e.status();
        }
        std::fprintf(sum, "mismatch_status %d\n", status);

        // two host threads, each with its own context (thread_local), the same product
        slat::CsrMatrix t1, t2;
        std::thread th1([&] { t1 = a2.matmul(a); }), th2([&] { t2 = a.matmul(a2); });
        th1.join(), th2.join();
        std::fprintf(sum, "threads_equal %d\n", (int)(t1.col_idx == a3.col_idx && t1.values == a3.values &&
                                                       t2.row_ptr == a3.row_ptr && t2.nnz() == a3.nnz()));

        // the drop-in's end-to-end cost on the headline step (A^6 * A with host vectors in and out:
        // H2D of both operands, the product, D2H of C into fresh vectors)
        if (e2e_iters > 0) {
            slat::CsrMatrix p = a;
            for (int k = 2; k < 7; ++k) p = p.matmul(a);
            slat::CsrMatrix c = p.matmul(a);  // warm-up
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < e2e_iters; ++i) c = p.matmul(a);
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / e2e_iters;
            std::fprintf(sum, "e2e_a7_nnz %zu\ne2e_a7_ms %.4f\n", c.nnz(), ms);
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "dropin: %s\n", e.what());
        std::fclose(sum);
        return 1;
    }
    std::fclose(sum);
    std::puts("dropin ok");
    return 0;
}
