/*
 * oracle.h — CPU restatement of the reference SpGEMM path. TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker and the `cpu_baseline` leg of bench.py. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline may load it. The product path
 * (libslat.so) never links or calls it.
 *
 * What it restates (reference = imlvts/sparse-linear-algebra-tests, read-only at /root/reference):
 *   orc_rng_*        rand 0.9.2 StdRng = rand_chacha 0.9.0 ChaCha12Rng (Cargo.lock:851-895),
 *                    f64 draws as rand's UniformFloat::sample_single: (next_u64 >> 12) * 2^-52.
 *   orc_lattice      CsrMatrix::lattice          src/graph_csr.rs:177-222
 *   orc_thin         CsrMatrix::thin             src/graph_csr.rs:225-247 (same draw pattern as
 *                    SparseCountMatrix::thin, src/graph.rs:143-154)
 *   orc_random       CsrMatrix::random           src/graph_csr.rs:163-174; integer draws as rand 0.9's
 *                    `random_range(0..n)` for usize: UniformUsize -> UniformInt<u32> (n <= u32::MAX),
 *                    Canon's method on next_u32 words (rand_core BlockRng word order). Pinned by the
 *                    nnz the reference's einsum study prints for random(1000, 5000) / (2000, 10000)
 *                    after three 4/26 thins from seed [42;32] (SPARSE_EINSUM_APPROACHES.md:127-132,
 *                    configs src/graph_csr.rs:1652-1669).
 *   orc_from_coo     CsrMatrix::from_coo         src/graph_csr.rs:83-129
 *   orc_matmul_seq   CsrMatrix::matmul           src/graph_csr.rs:306-346   (u32 saturating)
 *                    same algorithm on Sat64     src/graph_sprs.rs:15-86    (u64 saturating)
 *                    linalg Csr<u32,f64>::matmul linalg/src/csr.rs:308-356  (f64, left fold)
 *   orc_matmul_par   CsrMatrix::matmul_par       src/graph_csr.rs:350-484   (two-pass, threads)
 *   orc_add          CsrMatrix::add              src/graph_csr.rs:487-542
 *   orc_identity     CsrMatrix::identity         src/graph_csr.rs:68-80
 *   orc_reachability_sum      CsrMatrix::reachability_sum      src/graph_csr.rs:545-559
 *   orc_power_until_stable    CsrMatrix::power_until_stable    src/graph_csr.rs:562-577
 *   orc_connected_components  CsrMatrix::connected_components  src/graph_csr.rs:580-603
 *   orc_rcm_order    CsrMatrix::rcm              src/graph_csr.rs:663-722 (the order it permutes by;
 *                    ties of the degree sort in column order: the reference's sort_unstable leaves
 *                    them unspecified, so tie order is unpinned)
 *   orc_permute      CsrMatrix::permute          src/graph_csr.rs:726-783 (perm[new] = old)
 *   orc_bandwidth_stats CsrMatrix::bandwidth_stats src/graph_csr.rs:802-818
 *   orc_load_edges   load_edges                  src/graph_csr.rs:1209-1224
 *   orc_einsum_sparse_driven einsum_sparse_driven einsum-dyn/src/sparse.rs:70-148 (dense output)
 *
 * Parity pin: see tests/golden/ (nnz sequence that rounds to README.md:41-46, SHA-256 of the
 * arrays computed independently by tests/golden/make_golden.py with numpy+scipy).
 */
#ifndef SLAT_ORACLE_H
#define SLAT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_U32 = 0, ORC_SAT64 = 1, ORC_F64 = 2 };

typedef struct {
    uint64_t n;        /* square n x n */
    uint64_t nnz;
    int32_t dtype;     /* ORC_U32 / ORC_SAT64 / ORC_F64 */
    int32_t _pad;
    uint64_t *row_ptr; /* n+1 */
    uint32_t *col;     /* nnz */
    void *val;         /* nnz x (4 | 8 | 8) bytes */
} orc_csr;

typedef struct {
    uint32_t key[8];
    uint64_t counter;  /* next block counter */
    uint32_t buf[64];  /* 4 blocks, like rand_chacha's 4-block refill */
    uint32_t idx;      /* next word in buf; 64 = empty */
} orc_rng;

void orc_rng_seed(orc_rng *r, const uint8_t seed[32]);
uint64_t orc_rng_next_u64(orc_rng *r);
uint32_t orc_rng_next_u32(orc_rng *r);
uint32_t orc_rng_range_u32(orc_rng *r, uint32_t lo, uint32_t hi);
double orc_rng_next_f64(orc_rng *r);
int orc_random(orc_rng *rng, uint32_t n, uint64_t m, orc_csr *out);
void orc_chacha12_block(const uint32_t key[8], uint64_t counter, uint32_t out[16]);
void orc_chacha_block(const uint32_t key[8], uint64_t counter, int double_rounds, uint32_t out[16]);

void orc_csr_free(orc_csr *m);
int orc_from_coo(uint64_t n, uint64_t ntrip, const uint32_t *rows, const uint32_t *cols,
                 const void *vals, int dtype, orc_csr *out);
int orc_lattice(const uint64_t *dims, int ndim, int torus, orc_csr *out);
int orc_thin(const orc_csr *m, orc_rng *rng, double density, orc_csr *out);
int orc_convert(const orc_csr *m, int dtype, orc_csr *out);
int orc_matmul_seq(const orc_csr *a, const orc_csr *b, orc_csr *out);
int orc_matmul_par(const orc_csr *a, const orc_csr *b, int nthreads, orc_csr *out);
int orc_add(const orc_csr *a, const orc_csr *b, orc_csr *out);
uint64_t orc_flops(const orc_csr *a, const orc_csr *b);
int orc_identity(uint64_t n, int dtype, orc_csr *out);
int orc_power_until_stable(const orc_csr *a, uint64_t *k, orc_csr *out);
int orc_reachability_sum(const orc_csr *a, uint64_t *k, orc_csr *out);
int orc_connected_components(const orc_csr *a, uint64_t *component);
/* perm (n entries, malloc'd) = the order rcm() permutes by; -1 if that order is not a permutation
 * (a directed graph whose peripheral BFS re-enters a finished component: the reference panics) */
int orc_rcm_order(const orc_csr *a, uint32_t *perm);
int orc_permute(const orc_csr *a, const uint32_t *perm, orc_csr *out);
void orc_bandwidth_stats(const orc_csr *a, uint64_t *max_bw, double *avg_bw);
/* "<a> <b>" per non-empty line; n = max id + 1; src and dst arrays malloc-ed. -1 on a malformed line. */
int orc_einsum_sparse_driven(const orc_csr *a, const orc_csr *b, void *out, uint64_t ld, int trans);
int orc_load_edges(const char *path, uint64_t *n, uint64_t *n_edges, uint32_t **src, uint32_t **dst);

#ifdef __cplusplus
}
#endif
#endif
