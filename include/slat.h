/*
 * slat.h — C ABI of the MI355X-native SpGEMM engine (libslat.so, gfx950).
 *
 * Drop-in boundary for the reference's SpGEMM path (imlvts/sparse-linear-algebra-tests):
 *
 *   reference (Rust)                                          replaced by
 *   CsrMatrix::matmul       src/graph_csr.rs:306-346         slat_spgemm_csr_u32 (flags 0)
 *   CsrMatrix::matmul_par   src/graph_csr.rs:350-484         slat_spgemm_csr_u32 (same result)
 *   MagnusMatrix::matmul    src/graph_magnus.rs:224-232      slat_spgemm_csr_sat64
 *   MagnusMatrix::matmul_seq src/graph_magnus.rs:234-242     slat_spgemm_csr_sat64
 *   MagnusMatrix (usize cols) src/graph_magnus.rs:11-14,224-242  slat_magnus_matmul
 *   linalg Csr<u32,f64>::matmul{,_par} linalg/src/csr.rs:308-466  slat_spgemm_csr_f64
 *   CsrMatrix::from_coo     src/graph_csr.rs:83-129          slat_csr_from_coo (device) / slat_host_from_coo
 *   CsrMatrix::lattice      src/graph_csr.rs:177-222         slat_csr_lattice (device) / slat_host_lattice
 *   CsrMatrix::thin         src/graph_csr.rs:225-247         slat_csr_thin (device) / slat_host_thin
 *   CsrMatrix::random       src/graph_csr.rs:163-174         slat_host_random
 *   CsrMatrix::add          src/graph_csr.rs:487-542         slat_csr_add
 *   CsrMatrix::identity     src/graph_csr.rs:68-80           slat_csr_identity
 *   CsrMatrix::reachability_sum    src/graph_csr.rs:545-559  slat_reachability_sum
 *   CsrMatrix::power_until_stable  src/graph_csr.rs:562-577  slat_power_until_stable
 *   CsrMatrix::connected_components src/graph_csr.rs:580-603 slat_connected_components
 *   bench_diameter (driver) src/graph_csr.rs:1228-1319       slat_diameter
 *   CsrMatrix::from_edges{,_undirected} src/graph_csr.rs:132-147 slat_csr_from_edges
 *   CsrMatrix::rcm          src/graph_csr.rs:663-722         slat_rcm_order + slat_csr_permute
 *   CsrMatrix::permute / unpermute src/graph_csr.rs:726-799  slat_csr_permute
 *   CsrMatrix::bandwidth_stats src/graph_csr.rs:802-818      slat_bandwidth_stats
 *   load_edges (tests)      src/graph_csr.rs:1209-1224       slat_load_edges
 *   einsum_sparse_driven    einsum-dyn/src/sparse.rs:70-148  slat_spgemm_dense
 *   assert_eq!(self.n, other.n) panics (graph_csr.rs:307,351)  -> SLAT_EDIM
 *
 * Conventions:
 *   * Inputs are borrowed read-only views (`&self`, `&Self`); device- or host-resident.
 *   * The output is a freshly allocated, library-owned device matrix; release it with
 *     slat_csr_free. Nothing is cached across calls except scratch in the context.
 *   * Layout = the reference's: row_ptr u64 (usize) [n_rows+1], col_idx u32 (NodeId) sorted and
 *     unique within a row, values u32 (saturating) | u64 (Sat64, saturating) | f64; no explicit
 *     zeros in outputs. slat_spgemm_csr_sat64 takes MagnusMatrix with u32 column ids;
 *     slat_magnus_matmul takes its usize (u64) column ids as they are.
 *   * Results equal CsrMatrix::matmul bit for bit (u32 / Sat64; order-independent because values
 *     are non-negative) and the linalg f64 left fold in A-row order bit for bit (f64).
 *   * One slat_ctx per host thread / stream. Calls are synchronous on the context's stream.
 */
#ifndef SLAT_H
#define SLAT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SLAT_OK = 0,
    SLAT_EINVAL = 1,   /* bad argument / malformed CSR / dtype mismatch */
    SLAT_EDIM = 2,     /* shape mismatch (the reference panics: assert_eq!(self.n, other.n)) */
    SLAT_EOOM = 3,     /* device or host allocation failed */
    SLAT_EHIP = 4,     /* HIP runtime error */
    SLAT_ENOTSUP = 5,  /* unsupported combination */
    SLAT_ENODEV = 6    /* no usable gfx950 device */
} slat_status;

typedef enum { SLAT_U32 = 0, SLAT_SAT64 = 1, SLAT_F64 = 2 } slat_dtype;

typedef enum { SLAT_DEVICE = 0, SLAT_HOST = 1 } slat_residency;

/* spgemm flags */
#define SLAT_FLAG_TIMING      0x1u  /* record per-kernel HIP events; read with slat_get_stats */
#define SLAT_FLAG_EXACT_ALLOC 0x2u  /* size C exactly (extra mid-call sync) instead of by bound */
#define SLAT_FLAG_STATS       0x4u  /* also count scalar products (flops) for slat_get_stats */
/* f64 only: sum each output's products in any order (LDS / global atomics) instead of the
 * reference's left fold in A-row order; results then agree with the reference within the stated
 * tolerance (relative 1e-12 for same-sign values), not bit for bit (config C5). */
#define SLAT_FLAG_F64_ANY_ORDER 0x8u
/* the 64-bit-offset kernel instances even when every offset fits 32 bits (they run by themselves
 * once nnz(A) or nnz(B) reaches 2^32; the flag lets small inputs test them) */
#define SLAT_FLAG_IDX64 0x10u
/* the regular multi-kernel pipeline even for a small product (which otherwise runs as one kernel,
 * slat_tiny.hip); results are identical either way (tests run both) */
#define SLAT_FLAG_NO_TINY 0x20u
/* fat rows (MAGNUS's coarse category, >= 8192 products) accumulate from their products bucketed by
 * accumulator chunk in HBM (MAGNUS's fine-level reordering) instead of per-chunk walks over B split by
 * chunk, the default, which measured faster; results are identical */
#define SLAT_FLAG_FAT_BUCKETS 0x40u

typedef struct slat_ctx slat_ctx;

/* Borrowed CSR view. row_ptr holds absolute offsets into col_idx/values (a row block of a larger
 * matrix is a view with row_ptr advanced, n_rows reduced). max_row_nnz = 0 means unknown. */
typedef struct {
    uint64_t n_rows, n_cols, nnz;
    const uint64_t *row_ptr;
    const uint32_t *col_idx;
    const void *values;
    int32_t dtype;      /* slat_dtype */
    int32_t residency;  /* slat_residency */
    uint64_t max_row_nnz;
} slat_csr_view;

/* Library-owned device CSR. capacity >= nnz entries are allocated for col_idx/values. `alloc` is
 * private to the library (how the arrays were allocated: one block or several); treat the whole
 * struct as read-only and release it with slat_csr_free. */
typedef struct {
    uint64_t n_rows, n_cols, nnz, capacity, max_row_nnz;
    uint64_t *row_ptr;
    uint32_t *col_idx;
    void *values;
    int32_t dtype;
    int32_t device;
    int32_t alloc;
    int32_t _pad;
} slat_csr;

typedef struct {
    uint64_t nnz;          /* nnz(C) of the last call */
    uint64_t flops;        /* scalar products (only with SLAT_FLAG_STATS) */
    uint64_t capacity;     /* entries allocated for C */
    double symbolic_ms;    /* kernel durations (only with SLAT_FLAG_TIMING) */
    double scan_ms;
    double numeric_ms;
    double compact_ms;
    double total_ms;       /* first event to last event on the stream */
    uint32_t mode;         /* bits: 1 = 32-bit offsets, 2 = B's ELL image, 4 = the one-kernel small path,
                              8 = the lane kernel, 16 = the stored-bitmap numeric pass (MODE 4),
                              32 = a speculative wide launch (no listed-row launches) that held,
                              64 = a speculative wide launch that listed a row and was rerun */
    uint32_t window_words; /* LDS bitmap words per window */
    uint32_t exact_alloc;  /* 1 if the mid-call-sync path was taken */
    uint32_t dropped_rows; /* rows that lost explicit zeros in the numeric pass */
} slat_stats;

/* --- context ------------------------------------------------------------------------------ */
slat_status slat_ctx_create(int device, slat_ctx **out);
slat_status slat_ctx_destroy(slat_ctx *ctx);
slat_status slat_ctx_set_stream(slat_ctx *ctx, void *hip_stream); /* NULL = the ctx's own stream */
void *slat_ctx_stream(slat_ctx *ctx);
const char *slat_status_string(slat_status s);
const char *slat_last_error(slat_ctx *ctx);
slat_status slat_get_stats(slat_ctx *ctx, slat_stats *out);
slat_status slat_sync(slat_ctx *ctx);
/* MATMUL_PROGRESS (src/graph_csr.rs:10-11, 355-358, 392-408, 465-481): a process-wide switch; while
 * on, every SpGEMM call prints the reference's pass summary lines to stderr,
 * "  symbolic: done in <s>s (<rows/s> rows/s)" and "  numeric:  done in ...", from HIP events
 * around the passes (a device call has no per-row progress to report). Also on when the environment
 * variable SLAT_MATMUL_PROGRESS is set at first use. Returns the previous setting. */
int slat_set_matmul_progress(int on);

/* --- matrices ----------------------------------------------------------------------------- */
slat_status slat_csr_create(slat_ctx *ctx, const slat_csr_view *src, slat_csr *out); /* copy H2D/D2D */
slat_status slat_csr_to_host(slat_ctx *ctx, const slat_csr_view *src, uint64_t *row_ptr,
                             uint32_t *col_idx, void *values);
slat_status slat_csr_free(slat_ctx *ctx, slat_csr *m);
slat_csr_view slat_csr_view_of(const slat_csr *m);
slat_status slat_csr_max_row_nnz(slat_ctx *ctx, const slat_csr_view *m, uint64_t *out);

/* --- SpGEMM: C = A * B ---------------------------------------------------------------------- */
slat_status slat_spgemm(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C,
                        uint32_t flags);
slat_status slat_spgemm_csr_u32(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B,
                                slat_csr *C, uint32_t flags);
slat_status slat_spgemm_csr_sat64(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B,
                                  slat_csr *C, uint32_t flags);
slat_status slat_spgemm_csr_f64(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B,
                                slat_csr *C, uint32_t flags);
/* Rows [row_begin, row_end) of A times B -> C with (row_end - row_begin) local rows: the 1-D
 * row-block partition used across GPUs. */
slat_status slat_spgemm_rowblock(slat_ctx *ctx, const slat_csr_view *A, uint64_t row_begin,
                                 uint64_t row_end, const slat_csr_view *B, slat_csr *C, uint32_t flags);

/* A prepared right operand: B's padded ELL image and value summary, which every call otherwise
 * builds from B (a few microseconds at 27 000 rows, ~28 us at 10^6), built once for many products
 * with the same B: the replicated B of the multi-GPU row blocks, an A^k chain's A.
 * The handle borrows B's device arrays: they must stay alive and unchanged while it is used. Results
 * are identical to slat_spgemm_rowblock with the plain view. */
typedef struct slat_bprep slat_bprep;
slat_status slat_bprep_create(slat_ctx *ctx, const slat_csr_view *B, slat_bprep **out);
slat_status slat_bprep_free(slat_ctx *ctx, slat_bprep *p);
slat_status slat_spgemm_rowblock_prepared(slat_ctx *ctx, const slat_csr_view *A, uint64_t row_begin,
                                          uint64_t row_end, const slat_bprep *B, slat_csr *C, uint32_t flags);

/* --- MagnusMatrix in its own layout (src/graph_magnus.rs:11-14) --------------------------------
 * magnus::SparseMatrixCSR<Sat64>: row_ptr usize, col_idx usize (8-byte ids), values Sat64 (u64).
 * slat_magnus_matmul replaces MagnusMatrix::matmul / matmul_seq (src/graph_magnus.rs:224-242)
 * without narrowing or widening the Rust Vecs on the host: the columns are narrowed to u32 on the
 * device (a column id >= n_cols -> SLAT_EINVAL; n_cols >= 2^32 -> SLAT_ENOTSUP), the Sat64 SpGEMM
 * runs, and C's columns come back as u64. Release the result with slat_magnus_free. */
typedef struct {
    uint64_t n_rows, n_cols, nnz;
    const uint64_t *row_ptr;
    const uint64_t *col_idx;
    const uint64_t *values;
    int32_t residency; /* slat_residency */
    int32_t _pad;
    uint64_t max_row_nnz; /* 0 = unknown */
} slat_magnus_view;

typedef struct {
    uint64_t n_rows, n_cols, nnz, capacity, max_row_nnz;
    uint64_t *row_ptr;
    uint64_t *col_idx;
    uint64_t *values;
    int32_t device;
    int32_t _pad;
    uint8_t _owner[96]; /* private: the blocks that hold the arrays */
} slat_magnus;

slat_status slat_magnus_matmul(slat_ctx *ctx, const slat_magnus_view *A, const slat_magnus_view *B,
                               slat_magnus *C, uint32_t flags);
slat_status slat_magnus_free(slat_ctx *ctx, slat_magnus *m);
/* MagnusMatrix's SpGEMM consumers in the same layout (src/graph_magnus.rs:245-359): add (per-row
 * sorted union, Sat64 sums, exact zeros dropped), reachability_sum (A + A^2 + ... until nnz repeats;
 * *k = last power), power_until_stable (repeated squaring until the pattern is stable; *k =
 * squarings) and connected_components (closure of A + I; `component` = host array of n_rows u64).
 * The same device kernels as the u32-column entry points, with the columns narrowed / widened. */
slat_status slat_magnus_add(slat_ctx *ctx, const slat_magnus_view *A, const slat_magnus_view *B, slat_magnus *C);
slat_status slat_magnus_reachability_sum(slat_ctx *ctx, const slat_magnus_view *A, slat_magnus *sum, uint64_t *k);
slat_status slat_magnus_power_until_stable(slat_ctx *ctx, const slat_magnus_view *A, slat_magnus *out, uint64_t *k);
slat_status slat_magnus_connected_components(slat_ctx *ctx, const slat_magnus_view *A, uint64_t *component);
slat_status slat_magnus_to_host(slat_ctx *ctx, const slat_magnus *m, uint64_t *row_ptr, uint64_t *col_idx,
                                uint64_t *values);
slat_magnus_view slat_magnus_view_of(const slat_magnus *m);

/* --- CsrBTreeMatrix in its own layout (src/graph_csr_btree.rs:44-52) -----------------------------
 * DenseBTreeList (src/dense_btree.rs:269-330) packs each row as [internal separator nodes | sorted
 * data] into one flat `nodes` Vec<NodeId>. Row r's columns are nodes[data_off[r] ..
 * data_off[r] + (data_start[r+1] - data_start[r])), with data_off[r] = its NodeEntry's offset +
 * internal_len, and its values are values[data_start[r] ..] (data_start[r] = NodeEntry::data_start,
 * data_start[n_rows] = total_data_len() = nnz). slat_spgemm_btree replaces CsrBTreeMatrix::matmul_par
 * (src/graph_csr_btree.rs:350-479): the columns are gathered into CSR order on the device, the u32
 * SpGEMM runs, and C is returned as CSR, the arrays matmul_par passes to from_flat (:99). A slice
 * outside nodes / nnz or a column >= n_cols -> SLAT_EINVAL. */
typedef struct {
    uint64_t n_rows, n_cols, nnz, n_nodes;
    const uint64_t *data_start; /* n_rows + 1 */
    const uint64_t *data_off;   /* n_rows */
    const uint32_t *nodes;      /* n_nodes: separators and data of every row */
    const uint32_t *values;     /* nnz (Val = u32) */
    int32_t residency;          /* slat_residency, for all four arrays */
    int32_t _pad;
    uint64_t max_row_nnz; /* 0 = unknown */
} slat_btree_view;

slat_status slat_spgemm_btree(slat_ctx *ctx, const slat_btree_view *A, const slat_btree_view *B, slat_csr *C,
                              uint32_t flags);

/* --- multi-GPU row blocks over RCCL -------------------------------------------
 * One process per GPU. The reference splits matmul_par's output rows over rayon threads
 * (src/graph_csr.rs:350-484); here rank r computes C rows [cuts[r], cuts[r+1]) with
 * slat_spgemm_rowblock, B replicated. All calls are collective over the communicator (every rank
 * calls them, in the same order) and run on the context's stream. */
typedef struct slat_comm slat_comm;
/* ncclGetUniqueId into id[128], on one rank; share it with the others out of band. */
slat_status slat_comm_id(uint8_t id[128]);
slat_status slat_comm_create(slat_ctx *ctx, int nranks, int rank, const uint8_t id[128], slat_comm **out);
slat_status slat_comm_destroy(slat_comm *comm);
/* Flops-balanced 1-D row cuts of A*B on the device (not collective): cuts[0..parts] (host array),
 * cuts[r] = the first row whose running product count reaches r/parts of the total. */
slat_status slat_rowblock_cuts(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, uint32_t parts,
                               uint64_t *cuts);
/* The root's matrix on every rank (non-roots: *m is overwritten with a new library-owned matrix). */
slat_status slat_bcast_csr(slat_ctx *ctx, slat_comm *comm, slat_csr *m, int root);
/* Allgatherv of the ranks' C row blocks, in rank order, into a new library-owned matrix `full` on every
 * rank: row_ptr rebased on the device; payload nnz * (4 + value bytes) + rows * 8. */
slat_status slat_allgather_rows(slat_ctx *ctx, slat_comm *comm, const slat_csr_view *block, slat_csr *full);
/* The same assembly of row blocks that all live on this context's device (not collective): blocks
 * [0, nblocks) stacked in order into a new library-owned matrix, each block's row_ptr taken relative
 * to its first entry (views into a larger matrix allowed), row_ptr rebased on the device. */
slat_status slat_concat_rows(slat_ctx *ctx, const slat_csr_view *blocks, uint32_t nblocks, slat_csr *full);

/* --- the reference's SpGEMM consumers, device-resident --------------
 * Square matrices (n_rows == n_cols) for the iterated drivers; host views are staged to the device.
 * Loop decisions (nnz, pattern equality) are the only host round trips. */
/* CsrMatrix::add (src/graph_csr.rs:487-542), MagnusMatrix::add (src/graph_magnus.rs:245-300):
 * per-row sorted union; equal columns combine with the saturating add (u32 / Sat64) or f64 `+`,
 * a sum of exactly zero is dropped, unmatched entries are copied. Shape mismatch -> SLAT_EDIM. */
slat_status slat_csr_add(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C);
/* CsrMatrix::identity (src/graph_csr.rs:68-80): n x n, values 1. */
slat_status slat_csr_identity(slat_ctx *ctx, uint64_t n, int32_t dtype, slat_csr *out);
/* *equal = 1 iff nnz, row_ptr and col_idx agree (the stability test of power_until_stable,
 * src/graph_csr.rs:567-569). Device-resident views only. */
slat_status slat_csr_pattern_equal(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B,
                                   int32_t *equal);
/* CsrMatrix::reachability_sum (src/graph_csr.rs:545-559): sum = A + A^2 + ... until nnz(sum)
 * repeats; *k = the last power added. */
slat_status slat_reachability_sum(slat_ctx *ctx, const slat_csr_view *A, slat_csr *sum, uint64_t *k);
/* CsrMatrix::power_until_stable (src/graph_csr.rs:562-577): repeated squaring until the pattern
 * is stable; *k = squarings. */
slat_status slat_power_until_stable(slat_ctx *ctx, const slat_csr_view *A, slat_csr *out, uint64_t *k);
/* CsrMatrix::connected_components (src/graph_csr.rs:580-603): closure of A + I, then component ids
 * numbered by smallest member; `component` = host array of n_rows u64 (usize). */
slat_status slat_connected_components(slat_ctx *ctx, const slat_csr_view *A, uint64_t *component);

/* bench_diameter's algorithm (src/graph_csr.rs:1228-1319) on the device: A = the undirected graph
 * (from_edges_undirected); R0 = A + I squared until its pattern is stable, then the last power
 * before stabilisation times R0 until stable. *diameter = the largest finite distance (1 when R0 is
 * already its own closure); *squarings / *refinements = the products of each phase (may be NULL). */
slat_status slat_diameter(slat_ctx *ctx, const slat_csr_view *A, uint64_t *diameter, uint64_t *squarings,
                          uint64_t *refinements);

/* --- host-side input generators (the reference's constructors) ------------------------------ */
/* Host CSR owned by the library (malloc); free with slat_host_csr_free. */
typedef struct {
    uint64_t n, nnz;
    uint64_t *row_ptr;
    uint32_t *col_idx;
    void *values;
    int32_t dtype;
    int32_t _pad;
} slat_host_csr;

typedef struct { uint8_t opaque[512]; } slat_rng; /* rand 0.9 StdRng (ChaCha12) state */

void slat_rng_seed(slat_rng *rng, const uint8_t seed[32]);
uint64_t slat_rng_next_u64(slat_rng *rng);
uint32_t slat_rng_next_u32(slat_rng *rng);
/* rand 0.9 `rng.random_range(lo..hi)` for usize / u32 bounds below 2^32 (lo < hi). */
uint32_t slat_rng_range_u32(slat_rng *rng, uint32_t lo, uint32_t hi);
double slat_rng_next_f64(slat_rng *rng);
/* CsrMatrix::from_coo (src/graph_csr.rs:83-129): sort, merge duplicates by summing, drop zeros. */
slat_status slat_host_from_coo(uint64_t n, uint64_t ntrip, const uint32_t *rows, const uint32_t *cols,
                               const void *vals, int32_t dtype, slat_host_csr *out);
/* CsrMatrix::lattice (src/graph_csr.rs:177-222). */
slat_status slat_host_lattice(const uint64_t *dims, int ndim, int torus, slat_host_csr *out);
/* CsrMatrix::thin (src/graph_csr.rs:225-247). */
slat_status slat_host_thin(const slat_host_csr *m, slat_rng *rng, double density, slat_host_csr *out);
/* CsrMatrix::random (src/graph_csr.rs:163-174): random directed graph, n >= 2 nodes, m edge draws
 * without self-loops, duplicates summed (u32 values). */
slat_status slat_host_random(slat_rng *rng, uint32_t n, uint64_t m, slat_host_csr *out);
/* Seeded R-MAT power-law graph with f64 values uniform in [0.5, 1.5) (config C5; not in the
 * reference, which has no power-law generator). */
slat_status slat_host_rmat(uint32_t scale, uint64_t n_edges, double a, double b, double c,
                           const uint8_t seed[32], slat_host_csr *out);
void slat_host_csr_free(slat_host_csr *m);

/* --- the reference's constructors on the device ------------------------ */
/* CsrMatrix::from_coo (src/graph_csr.rs:83-129): sort by (row, col), sum duplicates (u32 / u64
 * wrapping like the reference's release build; f64 in input order), drop zeros. Triplet arrays
 * rows, cols u32 and vals (u32 | u64 | f64 per dtype) are device or host memory per `residency`.
 * A row or column id >= n -> SLAT_EINVAL (the reference panics on the index). */
slat_status slat_csr_from_coo(slat_ctx *ctx, uint64_t n, uint64_t ntrip, const uint32_t *rows,
                              const uint32_t *cols, const void *vals, int32_t dtype, int32_t residency,
                              slat_csr *out);
/* CsrMatrix::lattice (src/graph_csr.rs:177-222), built on the device (u32 values 1). */
slat_status slat_csr_lattice(slat_ctx *ctx, const uint64_t *dims, int ndim, int torus, slat_csr *out);
/* CsrMatrix::thin (src/graph_csr.rs:225-247) of a device matrix: the same draws as the host StdRng
 * (one f64 per entry with row <= col, row-major order), each computed from its stream position;
 * *rng ends where the reference's generator would. */
slat_status slat_csr_thin(slat_ctx *ctx, const slat_csr_view *m, slat_rng *rng, double density,
                          slat_csr *out);

/* --- the real-graph path -------------------------------------------- */
/* load_edges (src/graph_csr.rs:1209-1224): "<a> <b>" per non-empty line (further tokens ignored);
 * n = max id + 1; *src, *dst are malloc'd host arrays of *n_edges ids (free: slat_edges_free).
 * Unreadable file or malformed line -> SLAT_EINVAL (the reference panics). */
slat_status slat_load_edges(const char *path, uint64_t *n, uint64_t *n_edges, uint32_t **src, uint32_t **dst);
void slat_edges_free(uint32_t *src, uint32_t *dst);
/* CsrMatrix::from_edges (undirected = 0) / from_edges_undirected (= 1), src/graph_csr.rs:132-147:
 * u32 value 1 per edge (and per mirrored edge r != c), then from_coo (duplicates summed). */
slat_status slat_csr_from_edges(slat_ctx *ctx, uint64_t n, uint64_t n_edges, const uint32_t *src,
                                const uint32_t *dst, int32_t undirected, int32_t residency, slat_csr *out);
/* The order CsrMatrix::rcm (src/graph_csr.rs:663-722) permutes by, perm[new] = old, into the host
 * array perm[n]. Degree ties keep column order (the reference's unstable sort leaves them open).
 * An order that is not a permutation (possible on directed graphs) -> SLAT_EINVAL. */
slat_status slat_rcm_order(slat_ctx *ctx, const slat_csr_view *m, uint32_t *perm);
/* CsrMatrix::permute (src/graph_csr.rs:726-783), perm[new] = old (device or host per
 * perm_residency); out = rows and columns renumbered, columns sorted, explicit zeros kept.
 * unpermute is permute by the inverse. perm not a permutation of 0..n -> SLAT_EINVAL. */
slat_status slat_csr_permute(slat_ctx *ctx, const slat_csr_view *m, const uint32_t *perm, int32_t perm_residency,
                             slat_csr *out);
/* CsrMatrix::bandwidth_stats (src/graph_csr.rs:802-818): max |r-c| and mean |r-c| over entries. */
slat_status slat_bandwidth_stats(slat_ctx *ctx, const slat_csr_view *m, uint64_t *max_bw, double *avg_bw);

/* --- sparse x sparse with a dense output ---------------------------- */
/* einsum_sparse_driven (einsum-dyn/src/sparse.rs:70-148), "ab,bc->ac" (transpose = 0) or
 * "ab,bc->ca" (1): every output entry that some product touches is overwritten with its sum,
 * untouched entries keep their content. `out` is row-major with leading dimension ld, device or
 * host memory per out_residency. Values: SLAT_U32 as plain u32 (wrapping `+=` and `*`, the einsum
 * tests' T) or SLAT_F64 (the reference's left fold, bit-exact); SLAT_SAT64 -> SLAT_ENOTSUP. */
slat_status slat_spgemm_dense(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, void *out, uint64_t ld,
                              int32_t transpose, int32_t out_residency);
/* Device buffers for dense operands (the context's block cache) and host <-> device copies
 * (to_host = 1: device src -> host dst; 0: host src -> device dst), synchronous. */
slat_status slat_device_alloc(slat_ctx *ctx, uint64_t bytes, void **p);
slat_status slat_device_free(slat_ctx *ctx, void *p);
slat_status slat_device_copy(slat_ctx *ctx, void *dst, const void *src, uint64_t bytes, int32_t to_host);
/* Page-locked host memory (hipHostMalloc): host views and slat_csr_to_host destinations in such
 * buffers move over PCIe by DMA at full rate; pageable buffers are staged by the runtime. */
slat_status slat_host_alloc(uint64_t bytes, void **p);
slat_status slat_host_free(void *p);


#ifdef __cplusplus
}
#endif
#endif /* SLAT_H */
