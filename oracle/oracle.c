/*
 * oracle.c — CPU restatement of the reference SpGEMM path. TEST INFRASTRUCTURE ONLY
 * (parity checker + bench.py cpu_baseline). See oracle.h for the file:line map.
 * Plain C11 + pthreads; built by oracle/Makefile into oracle/liboracle.so.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* ChaCha12 StdRng (rand 0.9.2 / rand_chacha 0.9.0 / rand_core 0.9.5, Cargo.lock:851-895).    */
/* Key = seed as 8 LE words; words 12-13 = 64-bit block counter from 0; words 14-15 = stream 0. */
/* rand_chacha refills 4 blocks (64 words) at a time; next_u64 = lo | hi << 32 of consecutive  */
/* words. Only u64 draws are made on the reference's path, so the read index stays even.      */
/* ------------------------------------------------------------------------------------------ */
#define ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
#define QR(a, b, c, d)                                                                             \
    a += b; d ^= a; d = ROTL(d, 16);                                                              \
    c += d; b ^= c; b = ROTL(b, 12);                                                              \
    a += b; d ^= a; d = ROTL(d, 8);                                                               \
    c += d; b ^= c; b = ROTL(b, 7);

/* the ChaCha block function with `double_rounds` double rounds (ChaCha12: 6; ChaCha20: 10, which the
 * tests use to check the core against the RFC 8439 zero-key keystream) */
void orc_chacha_block(const uint32_t key[8], uint64_t counter, int double_rounds, uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 8; ++i) s[4 + i] = key[i];
    s[12] = (uint32_t)counter;
    s[13] = (uint32_t)(counter >> 32);
    s[14] = 0;
    s[15] = 0;
    uint32_t x[16];
    memcpy(x, s, sizeof x);
    for (int r = 0; r < double_rounds; ++r) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

void orc_chacha12_block(const uint32_t key[8], uint64_t counter, uint32_t out[16]) {
    orc_chacha_block(key, counter, 6, out); /* 12 rounds = 6 double rounds */
}

void orc_rng_seed(orc_rng *r, const uint8_t seed[32]) {
    for (int i = 0; i < 8; ++i)
        r->key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) |
                    ((uint32_t)seed[4 * i + 2] << 16) | ((uint32_t)seed[4 * i + 3] << 24);
    r->counter = 0;
    r->idx = 64;
}

static void orc_rng_refill(orc_rng *r) {
    for (int b = 0; b < 4; ++b) orc_chacha12_block(r->key, r->counter + (uint64_t)b, r->buf + 16 * b);
    r->counter += 4;
    r->idx = 0;
}

/* rand_core 0.9 BlockRng::next_u64: two consecutive words; at the last word of the buffer the
 * low half is that word and the high half the first word of the next refill. */
uint64_t orc_rng_next_u64(orc_rng *r) {
    if (r->idx >= 64) orc_rng_refill(r);
    if (r->idx == 63) {
        const uint64_t lo = r->buf[63];
        orc_rng_refill(r);
        r->idx = 1;
        return lo | ((uint64_t)r->buf[0] << 32);
    }
    uint64_t lo = r->buf[r->idx], hi = r->buf[r->idx + 1];
    r->idx += 2;
    return lo | (hi << 32);
}

/* rand_core 0.9 BlockRng::next_u32: one word. */
uint32_t orc_rng_next_u32(orc_rng *r) {
    if (r->idx >= 64) orc_rng_refill(r);
    return r->buf[r->idx++];
}

/* rand 0.9 `random_range(lo..hi)` for usize / u32 with hi <= u32::MAX: UniformUsize samples as
 * u32 (portable across pointer widths), UniformInt<u32>::sample_single_inclusive(lo, hi - 1) by
 * Canon's method — one u32 draw widened-multiplied by the range; only when the low half exceeds
 * 2^32 - range a second draw's high half is added to it, and its carry bumps the result. */
uint32_t orc_rng_range_u32(orc_rng *r, uint32_t lo, uint32_t hi) {
    const uint32_t range = hi - lo; /* (hi - 1) - lo + 1; 0 = the full u32 range */
    if (range == 0) return orc_rng_next_u32(r);
    const uint64_t m = (uint64_t)orc_rng_next_u32(r) * range;
    uint32_t result = (uint32_t)(m >> 32);
    const uint32_t lo_order = (uint32_t)m;
    if (lo_order > (uint32_t)(0u - range)) {
        const uint32_t new_hi = (uint32_t)(((uint64_t)orc_rng_next_u32(r) * range) >> 32);
        if ((uint32_t)(lo_order + new_hi) < lo_order) result += 1;
    }
    return lo + result;
}

/* rand 0.9 `random_range(0.0..1.0)` for f64: value1_2 - 1.0 with 52 random mantissa bits. */
double orc_rng_next_f64(orc_rng *r) {
    return (double)(orc_rng_next_u64(r) >> 12) * (1.0 / 4503599627370496.0);
}

/* ------------------------------------------------------------------------------------------ */
/* CSR helpers                                                                                */
/* ------------------------------------------------------------------------------------------ */
static size_t vsize(int dtype) { return dtype == ORC_U32 ? 4 : 8; }

void orc_csr_free(orc_csr *m) {
    if (!m) return;
    free(m->row_ptr);
    free(m->col);
    free(m->val);
    m->row_ptr = NULL;
    m->col = NULL;
    m->val = NULL;
    m->nnz = 0;
}

typedef struct {
    uint64_t key; /* row << 32 | col */
    uint64_t v;   /* value bits (u32 / u64 / f64) */
} trip;

static int trip_cmp(const void *a, const void *b) {
    uint64_t x = ((const trip *)a)->key, y = ((const trip *)b)->key;
    return (x > y) - (x < y);
}

/* CsrMatrix::from_coo (src/graph_csr.rs:83-129): sort by (r,c), merge duplicates by summing
 * (plain `+=`, wrapping in a release build), drop zero values. */
static int from_trips(uint64_t n, trip *t, uint64_t nt, int dtype, orc_csr *out) {
    qsort(t, nt, sizeof(trip), trip_cmp);
    uint64_t nd = 0;
    for (uint64_t i = 0; i < nt; ++i) {
        if (nd > 0 && t[nd - 1].key == t[i].key) {
            if (dtype == ORC_F64) {
                double a, b;
                memcpy(&a, &t[nd - 1].v, 8);
                memcpy(&b, &t[i].v, 8);
                a += b;
                memcpy(&t[nd - 1].v, &a, 8);
            } else if (dtype == ORC_U32) {
                t[nd - 1].v = (uint32_t)(t[nd - 1].v + t[i].v);
            } else {
                t[nd - 1].v += t[i].v;
            }
        } else {
            t[nd++] = t[i];
        }
    }
    out->n = n;
    out->dtype = dtype;
    out->row_ptr = (uint64_t *)calloc(n + 1, 8);
    out->col = (uint32_t *)malloc((nd ? nd : 1) * 4);
    out->val = malloc((nd ? nd : 1) * vsize(dtype));
    if (!out->row_ptr || !out->col || !out->val) return -1;
    uint64_t k = 0, cur = 0;
    for (uint64_t i = 0; i < nd; ++i) {
        int zero;
        if (dtype == ORC_F64) {
            double a;
            memcpy(&a, &t[i].v, 8);
            zero = (a == 0.0);
        } else {
            zero = (t[i].v == 0);
        }
        if (zero) continue;
        uint64_t r = t[i].key >> 32;
        while (cur <= r) out->row_ptr[cur++] = k;
        out->col[k] = (uint32_t)t[i].key;
        if (dtype == ORC_U32)
            ((uint32_t *)out->val)[k] = (uint32_t)t[i].v;
        else
            ((uint64_t *)out->val)[k] = t[i].v;
        ++k;
    }
    while (cur <= n) out->row_ptr[cur++] = k;
    out->nnz = k;
    return 0;
}

int orc_from_coo(uint64_t n, uint64_t ntrip, const uint32_t *rows, const uint32_t *cols,
                 const void *vals, int dtype, orc_csr *out) {
    trip *t = (trip *)malloc((ntrip ? ntrip : 1) * sizeof(trip));
    if (!t) return -1;
    for (uint64_t i = 0; i < ntrip; ++i) {
        t[i].key = ((uint64_t)rows[i] << 32) | cols[i];
        if (dtype == ORC_U32)
            t[i].v = ((const uint32_t *)vals)[i];
        else
            memcpy(&t[i].v, (const uint8_t *)vals + 8 * i, 8);
    }
    int rc = from_trips(n, t, ntrip, dtype, out);
    free(t);
    return rc;
}

/* CsrMatrix::lattice (src/graph_csr.rs:177-222): row-major strides, 3^d offsets decoded base-3
 * with dimension 0 as the least-significant digit, self excluded, torus wraps with rem_euclid. */
int orc_lattice(const uint64_t *dims, int ndim, int torus, orc_csr *out) {
    uint64_t total = 1;
    for (int d = 0; d < ndim; ++d) total *= dims[d];
    uint64_t strides[16];
    if (ndim > 16) return -1;
    for (int d = 0; d < ndim; ++d) strides[d] = 1;
    for (int d = ndim - 2; d >= 0; --d) strides[d] = strides[d + 1] * dims[d + 1];
    uint64_t nnb = 1;
    for (int d = 0; d < ndim; ++d) nnb *= 3;
    trip *t = (trip *)malloc((total * nnb > 0 ? total * nnb : 1) * sizeof(trip));
    if (!t) return -1;
    uint64_t nt = 0;
    uint64_t coord[16] = {0};
    for (uint64_t node = 0; node < total; ++node) {
        for (uint64_t off = 0; off < nnb; ++off) {
            uint64_t tmp = off, neighbor = 0;
            int all_zero = 1, valid = 1;
            for (int d = 0; d < ndim; ++d) {
                int64_t delta = (int64_t)(tmp % 3) - 1;
                tmp /= 3;
                if (delta != 0) all_zero = 0;
                int64_t c = (int64_t)coord[d] + delta;
                if (torus) {
                    int64_t m = (int64_t)dims[d];
                    c = ((c % m) + m) % m;
                } else if (c < 0 || c >= (int64_t)dims[d]) {
                    valid = 0;
                    break;
                }
                neighbor += (uint64_t)c * strides[d];
            }
            if (all_zero || !valid) continue;
            t[nt].key = (node << 32) | neighbor;
            t[nt].v = 1;
            ++nt;
        }
        for (int d = ndim - 1; d >= 0; --d) {
            coord[d] += 1;
            if (coord[d] < dims[d]) break;
            coord[d] = 0;
        }
    }
    int rc = from_trips(total, t, nt, ORC_U32, out);
    free(t);
    return rc;
}

static uint64_t get_bits(const orc_csr *m, uint64_t r, uint32_t c) {
    uint64_t lo = m->row_ptr[r], hi = m->row_ptr[r + 1];
    while (lo < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if (m->col[mid] < c)
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo < m->row_ptr[r + 1] && m->col[lo] == c) {
        if (m->dtype == ORC_U32) return ((uint32_t *)m->val)[lo];
        return ((uint64_t *)m->val)[lo];
    }
    return 0;
}

/* CsrMatrix::thin (src/graph_csr.rs:225-247): row-major scan; one f64 draw only when r <= c
 * (the `&&` short-circuits), keep (r,c) and mirror (c,r) if present. */
int orc_thin(const orc_csr *m, orc_rng *rng, double density, orc_csr *out) {
    trip *t = (trip *)malloc((m->nnz ? m->nnz : 1) * sizeof(trip));
    if (!t) return -1;
    uint64_t nt = 0;
    for (uint64_t r = 0; r < m->n; ++r) {
        for (uint64_t idx = m->row_ptr[r]; idx < m->row_ptr[r + 1]; ++idx) {
            uint32_t c = m->col[idx];
            uint64_t v = m->dtype == ORC_U32 ? ((uint32_t *)m->val)[idx] : ((uint64_t *)m->val)[idx];
            if (r <= c && orc_rng_next_f64(rng) < density) {
                t[nt].key = (r << 32) | c;
                t[nt].v = v;
                ++nt;
                if (r != c) {
                    uint64_t rev = get_bits(m, c, (uint32_t)r);
                    if (rev > 0) {
                        t[nt].key = ((uint64_t)c << 32) | r;
                        t[nt].v = rev;
                        ++nt;
                    }
                }
            }
        }
    }
    int rc = from_trips(m->n, t, nt, m->dtype, out);
    free(t);
    return rc;
}

/* CsrMatrix::random (src/graph_csr.rs:163-174): m draws of r in 0..n, c in 0..n-1 bumped past r
 * (no self-loops), value 1, then from_coo (duplicates summed). u32 values. */
int orc_random(orc_rng *rng, uint32_t n, uint64_t m, orc_csr *out) {
    if (n < 2) return -1; /* assert!(nu >= 2) */
    trip *t = (trip *)malloc((m ? m : 1) * sizeof(trip));
    if (!t) return -1;
    for (uint64_t i = 0; i < m; ++i) {
        const uint32_t r = orc_rng_range_u32(rng, 0, n);
        uint32_t c = orc_rng_range_u32(rng, 0, n - 1);
        if (c >= r) c += 1;
        t[i].key = ((uint64_t)r << 32) | c;
        t[i].v = 1;
    }
    int rc = from_trips(n, t, m, ORC_U32, out);
    free(t);
    return rc;
}

/* Value-type conversion (u32 -> Sat64 / f64), used to feed the same structure to every path. */
int orc_convert(const orc_csr *m, int dtype, orc_csr *out) {
    out->n = m->n;
    out->nnz = m->nnz;
    out->dtype = dtype;
    out->row_ptr = (uint64_t *)malloc((m->n + 1) * 8);
    out->col = (uint32_t *)malloc((m->nnz ? m->nnz : 1) * 4);
    out->val = malloc((m->nnz ? m->nnz : 1) * vsize(dtype));
    if (!out->row_ptr || !out->col || !out->val) return -1;
    memcpy(out->row_ptr, m->row_ptr, (m->n + 1) * 8);
    memcpy(out->col, m->col, m->nnz * 4);
    for (uint64_t i = 0; i < m->nnz; ++i) {
        uint64_t u;
        double f;
        if (m->dtype == ORC_U32) {
            u = ((uint32_t *)m->val)[i];
            f = (double)u;
        } else if (m->dtype == ORC_SAT64) {
            u = ((uint64_t *)m->val)[i];
            f = (double)u;
        } else {
            f = ((double *)m->val)[i];
            u = (uint64_t)f;
        }
        if (dtype == ORC_U32)
            ((uint32_t *)out->val)[i] = (uint32_t)u;
        else if (dtype == ORC_SAT64)
            ((uint64_t *)out->val)[i] = u;
        else
            ((double *)out->val)[i] = f;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Semiring scalars: sadd/smul (src/graph_csr.rs:29-37), Sat64 (src/graph_sprs.rs:29-51),     */
/* f64 plain +,* (linalg/src/csr.rs:81-85).                                                    */
/* ------------------------------------------------------------------------------------------ */
static inline uint32_t sadd32(uint32_t a, uint32_t b) {
    uint32_t s = a + b;
    return s < a ? 0xFFFFFFFFu : s;
}
static inline uint32_t smul32(uint32_t a, uint32_t b) {
    uint64_t p = (uint64_t)a * b;
    return p > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)p;
}
static inline uint64_t sadd64(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    return s < a ? ~0ull : s;
}
static inline uint64_t smul64(uint64_t a, uint64_t b) {
    unsigned __int128 p = (unsigned __int128)a * b;
    return (p >> 64) ? ~0ull : (uint64_t)p;
}

/* Small in-place unstable sort of u32 (stand-in for Rust's sort_unstable on nz_cols). */
static void sort_u32(uint32_t *a, int64_t n) {
    while (n > 24) {
        uint32_t x = a[0], y = a[n / 2], z = a[n - 1];
        uint32_t p = x < y ? (y < z ? y : (x < z ? z : x)) : (x < z ? x : (y < z ? z : y));
        int64_t i = 0, j = n - 1;
        for (;;) {
            while (a[i] < p) ++i;
            while (a[j] > p) --j;
            if (i >= j) break;
            uint32_t t = a[i];
            a[i] = a[j];
            a[j] = t;
            ++i;
            --j;
        }
        /* recurse on the smaller half, loop on the larger */
        if (j + 1 < n - (j + 1)) {
            sort_u32(a, j + 1);
            a += j + 1;
            n -= j + 1;
        } else {
            sort_u32(a + j + 1, n - (j + 1));
            n = j + 1;
        }
    }
    for (int64_t i = 1; i < n; ++i) {
        uint32_t v = a[i];
        int64_t j = i - 1;
        while (j >= 0 && a[j] > v) {
            a[j + 1] = a[j];
            --j;
        }
        a[j + 1] = v;
    }
}

/* Append a column to nz_cols, growing it (explicit zero values can re-push a column). */
#define NZ_PUSH(j)                                                                                 \
    do {                                                                                           \
        if (nz_len == nz_cap) {                                                                    \
            nz_cap *= 2;                                                                           \
            uint32_t *nz2_ = (uint32_t *)realloc(nz, nz_cap * 4);                                  \
            if (!nz2_) abort();                                                                    \
            nz = nz2_;                                                                             \
        }                                                                                          \
        nz[nz_len++] = (j);                                                                        \
    } while (0)

/* Growable output buffers for the sequential matmul. */
typedef struct {
    uint32_t *col;
    uint8_t *val;
    uint64_t len, cap;
} obuf;

static int obuf_push(obuf *o, uint32_t c, const void *v, size_t vs) {
    if (o->len == o->cap) {
        uint64_t nc = o->cap ? o->cap * 2 : 1024;
        uint32_t *nc_ = (uint32_t *)realloc(o->col, nc * 4);
        uint8_t *nv = (uint8_t *)realloc(o->val, nc * vs);
        if (!nc_ || !nv) return -1;
        o->col = nc_;
        o->val = nv;
        o->cap = nc;
    }
    o->col[o->len] = c;
    memcpy(o->val + o->len * vs, v, vs);
    o->len++;
    return 0;
}

/* CsrMatrix::matmul (src/graph_csr.rs:306-346) — dense accumulator, nz_cols pushed when the
 * accumulator is zero, sort_unstable, emit non-zero values, clear. Same loop for Sat64 and for
 * linalg Csr<u32,f64>::matmul (linalg/src/csr.rs:308-356). */
int orc_matmul_seq(const orc_csr *a, const orc_csr *b, orc_csr *out) {
    if (a->n != b->n || a->dtype != b->dtype) return -2;
    const uint64_t n = a->n;
    const int dt = a->dtype;
    const size_t vs = vsize(dt);
    out->n = n;
    out->dtype = dt;
    out->row_ptr = (uint64_t *)malloc((n + 1) * 8);
    uint8_t *acc = (uint8_t *)calloc(n ? n : 1, vs);
    uint32_t *nz = (uint32_t *)malloc((n ? n : 1) * 4 * 2 + 64);
    if (!out->row_ptr || !acc || !nz) return -1;
    uint64_t nz_cap = (n ? n : 1) * 2 + 16, nz_len = 0; /* f64 may re-push a column */
    obuf o = {0};
    out->row_ptr[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        for (uint64_t idx = a->row_ptr[i]; idx < a->row_ptr[i + 1]; ++idx) {
            uint32_t k = a->col[idx];
            for (uint64_t jdx = b->row_ptr[k]; jdx < b->row_ptr[k + 1]; ++jdx) {
                uint32_t j = b->col[jdx];
                if (dt == ORC_U32) {
                    uint32_t *ac = (uint32_t *)acc;
                    if (ac[j] == 0) NZ_PUSH(j);
                    ac[j] = sadd32(ac[j], smul32(((uint32_t *)a->val)[idx], ((uint32_t *)b->val)[jdx]));
                } else if (dt == ORC_SAT64) {
                    uint64_t *ac = (uint64_t *)acc;
                    if (ac[j] == 0) NZ_PUSH(j);
                    ac[j] = sadd64(ac[j], smul64(((uint64_t *)a->val)[idx], ((uint64_t *)b->val)[jdx]));
                } else {
                    double *ac = (double *)acc;
                    if (ac[j] == 0.0) NZ_PUSH(j);
                    double prod = ((double *)a->val)[idx] * ((double *)b->val)[jdx];
                    ac[j] = ac[j] + prod;
                }
            }
        }
        sort_u32(nz, (int64_t)nz_len);
        for (uint64_t q = 0; q < nz_len; ++q) {
            uint32_t j = nz[q];
            if (dt == ORC_U32) {
                uint32_t v = ((uint32_t *)acc)[j];
                if (v != 0 && obuf_push(&o, j, &v, 4)) return -1;
                ((uint32_t *)acc)[j] = 0;
            } else if (dt == ORC_SAT64) {
                uint64_t v = ((uint64_t *)acc)[j];
                if (v != 0 && obuf_push(&o, j, &v, 8)) return -1;
                ((uint64_t *)acc)[j] = 0;
            } else {
                double v = ((double *)acc)[j];
                if (v != 0.0 && obuf_push(&o, j, &v, 8)) return -1;
                ((double *)acc)[j] = 0.0;
            }
        }
        nz_len = 0;
        out->row_ptr[i + 1] = o.len;
    }
    free(acc);
    free(nz);
    out->nnz = o.len;
    out->col = o.col ? o.col : (uint32_t *)malloc(4);
    out->val = o.val ? (void *)o.val : malloc(8);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* CsrMatrix::matmul_par (src/graph_csr.rs:350-484): pass 1 symbolic (bool mask), serial       */
/* prefix sum, zeroed exact-size outputs, pass 2 numeric into disjoint row slices. rayon's      */
/* work-stealing `par_iter` is replaced by a dynamic row-chunk scheduler over pthreads.         */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const orc_csr *a, *b;
    uint64_t *nnz_row;
    uint64_t *row_ptr;
    uint32_t *ocol;
    uint8_t *oval;
    atomic_uint_fast64_t next;
    int pass;
} par_job;

#define PAR_CHUNK 64

static void *par_worker(void *arg) {
    par_job *J = (par_job *)arg;
    const orc_csr *a = J->a, *b = J->b;
    const uint64_t n = a->n;
    const int dt = a->dtype;
    const size_t vs = vsize(dt);
    if (J->pass == 1) {
        uint8_t *mask = (uint8_t *)calloc(n ? n : 1, 1);
        for (;;) {
            uint64_t r0 = atomic_fetch_add(&J->next, PAR_CHUNK);
            if (r0 >= n) break;
            uint64_t r1 = r0 + PAR_CHUNK < n ? r0 + PAR_CHUNK : n;
            for (uint64_t i = r0; i < r1; ++i) {
                uint64_t count = 0;
                for (uint64_t idx = a->row_ptr[i]; idx < a->row_ptr[i + 1]; ++idx) {
                    uint32_t k = a->col[idx];
                    for (uint64_t jdx = b->row_ptr[k]; jdx < b->row_ptr[k + 1]; ++jdx) {
                        uint32_t j = b->col[jdx];
                        if (!mask[j]) {
                            mask[j] = 1;
                            ++count;
                        }
                    }
                }
                J->nnz_row[i] = count;
                for (uint64_t idx = a->row_ptr[i]; idx < a->row_ptr[i + 1]; ++idx) {
                    uint32_t k = a->col[idx];
                    for (uint64_t jdx = b->row_ptr[k]; jdx < b->row_ptr[k + 1]; ++jdx) mask[b->col[jdx]] = 0;
                }
            }
        }
        free(mask);
    } else {
        uint8_t *acc = (uint8_t *)calloc(n ? n : 1, vs);
        uint64_t nz_cap = (n ? n : 1) * 2 + 16;
        uint32_t *nz = (uint32_t *)malloc(nz_cap * 4);
        for (;;) {
            uint64_t r0 = atomic_fetch_add(&J->next, PAR_CHUNK);
            if (r0 >= n) break;
            uint64_t r1 = r0 + PAR_CHUNK < n ? r0 + PAR_CHUNK : n;
            for (uint64_t i = r0; i < r1; ++i) {
                uint64_t nz_len = 0;
                for (uint64_t idx = a->row_ptr[i]; idx < a->row_ptr[i + 1]; ++idx) {
                    uint32_t k = a->col[idx];
                    for (uint64_t jdx = b->row_ptr[k]; jdx < b->row_ptr[k + 1]; ++jdx) {
                        uint32_t j = b->col[jdx];
                        if (dt == ORC_U32) {
                            uint32_t *ac = (uint32_t *)acc;
                            if (ac[j] == 0) NZ_PUSH(j);
                            ac[j] = sadd32(ac[j], smul32(((uint32_t *)a->val)[idx], ((uint32_t *)b->val)[jdx]));
                        } else if (dt == ORC_SAT64) {
                            uint64_t *ac = (uint64_t *)acc;
                            if (ac[j] == 0) NZ_PUSH(j);
                            ac[j] = sadd64(ac[j], smul64(((uint64_t *)a->val)[idx], ((uint64_t *)b->val)[jdx]));
                        } else {
                            double *ac = (double *)acc;
                            if (ac[j] == 0.0) NZ_PUSH(j);
                            ac[j] = ac[j] + ((double *)a->val)[idx] * ((double *)b->val)[jdx];
                        }
                    }
                }
                sort_u32(nz, (int64_t)nz_len);
                uint64_t pos = J->row_ptr[i];
                for (uint64_t q = 0; q < nz_len; ++q) {
                    uint32_t j = nz[q];
                    int nonzero;
                    if (dt == ORC_F64)
                        nonzero = ((double *)acc)[j] != 0.0;
                    else if (dt == ORC_U32)
                        nonzero = ((uint32_t *)acc)[j] != 0;
                    else
                        nonzero = ((uint64_t *)acc)[j] != 0;
                    if (nonzero) {
                        J->ocol[pos] = j;
                        memcpy(J->oval + pos * vs, acc + (uint64_t)j * vs, vs);
                        ++pos;
                    }
                    memset(acc + (uint64_t)j * vs, 0, vs);
                }
            }
        }
        free(acc);
        free(nz);
    }
    return NULL;
}

int orc_matmul_par(const orc_csr *a, const orc_csr *b, int nthreads, orc_csr *out) {
    if (a->n != b->n || a->dtype != b->dtype) return -2;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    const uint64_t n = a->n;
    par_job J;
    J.a = a;
    J.b = b;
    J.nnz_row = (uint64_t *)calloc(n ? n : 1, 8);
    J.pass = 1;
    atomic_init(&J.next, 0);
    pthread_t th[1024];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, par_worker, &J);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    uint64_t *row_ptr = (uint64_t *)malloc((n + 1) * 8);
    row_ptr[0] = 0;
    for (uint64_t i = 0; i < n; ++i) row_ptr[i + 1] = row_ptr[i] + J.nnz_row[i];
    const uint64_t total = row_ptr[n];
    const size_t vs = vsize(a->dtype);
    J.row_ptr = row_ptr;
    J.ocol = (uint32_t *)calloc(total ? total : 1, 4);
    J.oval = (uint8_t *)calloc(total ? total : 1, vs);
    J.pass = 2;
    atomic_store(&J.next, 0);
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, par_worker, &J);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(J.nnz_row);
    out->n = n;
    out->nnz = total;
    out->dtype = a->dtype;
    out->row_ptr = row_ptr;
    out->col = J.ocol;
    out->val = J.oval;
    return 0;
}

/* CsrMatrix::add (src/graph_csr.rs:487-542): per-row sorted merge; equal columns combine with
 * sadd and are dropped if the sum is zero. */
int orc_add(const orc_csr *a, const orc_csr *b, orc_csr *out) {
    if (a->n != b->n || a->dtype != b->dtype) return -2;
    const uint64_t n = a->n;
    const int dt = a->dtype;
    const size_t vs = vsize(dt);
    out->n = n;
    out->dtype = dt;
    out->row_ptr = (uint64_t *)malloc((n + 1) * 8);
    obuf o = {0};
    out->row_ptr[0] = 0;
    const uint8_t *av = (const uint8_t *)a->val, *bv = (const uint8_t *)b->val;
    for (uint64_t r = 0; r < n; ++r) {
        uint64_t ai = a->row_ptr[r], ae = a->row_ptr[r + 1], bi = b->row_ptr[r], be = b->row_ptr[r + 1];
        while (ai < ae && bi < be) {
            uint32_t ac = a->col[ai], bc = b->col[bi];
            if (ac < bc) {
                obuf_push(&o, ac, av + ai * vs, vs);
                ++ai;
            } else if (ac > bc) {
                obuf_push(&o, bc, bv + bi * vs, vs);
                ++bi;
            } else {
                uint8_t tmp[8];
                int nz;
                if (dt == ORC_U32) {
                    uint32_t v = sadd32(((const uint32_t *)av)[ai], ((const uint32_t *)bv)[bi]);
                    memcpy(tmp, &v, 4);
                    nz = v != 0;
                } else if (dt == ORC_SAT64) {
                    uint64_t v = sadd64(((const uint64_t *)av)[ai], ((const uint64_t *)bv)[bi]);
                    memcpy(tmp, &v, 8);
                    nz = v != 0;
                } else {
                    double v = ((const double *)av)[ai] + ((const double *)bv)[bi];
                    memcpy(tmp, &v, 8);
                    nz = v != 0.0;
                }
                if (nz) obuf_push(&o, ac, tmp, vs);
                ++ai;
                ++bi;
            }
        }
        for (; ai < ae; ++ai) obuf_push(&o, a->col[ai], av + ai * vs, vs);
        for (; bi < be; ++bi) obuf_push(&o, b->col[bi], bv + bi * vs, vs);
        out->row_ptr[r + 1] = o.len;
    }
    out->nnz = o.len;
    out->col = o.col ? o.col : (uint32_t *)malloc(4);
    out->val = o.val ? (void *)o.val : malloc(8);
    return 0;
}

/* Number of scalar products of a*b (Σ_i Σ_{k∈A_i} nnz(B_k)). */
uint64_t orc_flops(const orc_csr *a, const orc_csr *b) {
    uint64_t f = 0;
    for (uint64_t idx = 0; idx < a->nnz; ++idx) {
        uint32_t k = a->col[idx];
        f += b->row_ptr[k + 1] - b->row_ptr[k];
    }
    return f;
}

/* ---------------------------------------------------------------------------------------------
 * The reference's SpGEMM consumers, restated over orc_matmul_seq / orc_add.
 * ------------------------------------------------------------------------------------------- */
static int orc_clone(const orc_csr *m, orc_csr *out) { return orc_convert(m, m->dtype, out); }

/* CsrMatrix::identity (src/graph_csr.rs:68-80): values 1. */
int orc_identity(uint64_t n, int dtype, orc_csr *out) {
    const size_t vs = vsize(dtype);
    out->n = n;
    out->nnz = n;
    out->dtype = dtype;
    out->row_ptr = (uint64_t *)malloc((n + 1) * 8);
    out->col = (uint32_t *)malloc(n ? n * 4 : 4);
    out->val = malloc(n ? n * vs : 8);
    for (uint64_t i = 0; i <= n; ++i) out->row_ptr[i] = i;
    for (uint64_t i = 0; i < n; ++i) {
        out->col[i] = (uint32_t)i;
        if (dtype == ORC_U32) ((uint32_t *)out->val)[i] = 1;
        else if (dtype == ORC_SAT64) ((uint64_t *)out->val)[i] = 1;
        else ((double *)out->val)[i] = 1.0;
    }
    return 0;
}

/* next.nnz() == cur.nnz() && row_ptr == && col_idx == (src/graph_csr.rs:567-569) */
static int same_pattern(const orc_csr *a, const orc_csr *b) {
    return a->nnz == b->nnz && a->n == b->n && memcmp(a->row_ptr, b->row_ptr, (a->n + 1) * 8) == 0 &&
           (a->nnz == 0 || memcmp(a->col, b->col, a->nnz * 4) == 0);
}

/* CsrMatrix::power_until_stable (src/graph_csr.rs:562-577): repeated squaring until the pattern
 * of the square equals the pattern of the matrix; *k = squarings done. */
int orc_power_until_stable(const orc_csr *a, uint64_t *k, orc_csr *out) {
    orc_csr cur;
    int rc = orc_clone(a, &cur);
    if (rc) return rc;
    *k = 0;
    for (;;) {
        orc_csr next;
        if ((rc = orc_matmul_seq(&cur, &cur, &next))) {
            orc_csr_free(&cur);
            return rc;
        }
        *k += 1;
        const int stable = same_pattern(&next, &cur);
        orc_csr_free(&cur);
        cur = next;
        if (stable) break;
    }
    *out = cur;
    return 0;
}

/* CsrMatrix::reachability_sum (src/graph_csr.rs:545-559): A + A^2 + ... until nnz(sum) repeats;
 * *k = the last power added. */
int orc_reachability_sum(const orc_csr *a, uint64_t *k, orc_csr *out) {
    orc_csr power, sum;
    int rc;
    if ((rc = orc_clone(a, &power))) return rc;
    if ((rc = orc_clone(a, &sum))) {
        orc_csr_free(&power);
        return rc;
    }
    *k = 1;
    for (;;) {
        orc_csr np, ns;
        if ((rc = orc_matmul_seq(&power, a, &np))) break;
        orc_csr_free(&power);
        power = np;
        *k += 1;
        if ((rc = orc_add(&sum, &power, &ns))) break;
        const int done = ns.nnz == sum.nnz;
        orc_csr_free(&sum);
        sum = ns;
        if (done) break;
    }
    orc_csr_free(&power);
    if (rc) {
        orc_csr_free(&sum);
        return rc;
    }
    *out = sum;
    return 0;
}

static int has_entry(const orc_csr *m, uint64_t r, uint32_t c) {
    uint64_t lo = m->row_ptr[r], hi = m->row_ptr[r + 1];
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (m->col[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    return lo < m->row_ptr[r + 1] && m->col[lo] == c;  /* stored entries are non-zero */
}

/* CsrMatrix::connected_components (src/graph_csr.rs:580-603): closure of A + I by
 * power_until_stable, then ids in order of each component's smallest node. */
int orc_connected_components(const orc_csr *a, uint64_t *component) {
    orc_csr id, with_id, closure;
    uint64_t k;
    int rc;
    if ((rc = orc_identity(a->n, a->dtype, &id))) return rc;
    rc = orc_add(a, &id, &with_id);
    orc_csr_free(&id);
    if (rc) return rc;
    rc = orc_power_until_stable(&with_id, &k, &closure);
    orc_csr_free(&with_id);
    if (rc) return rc;
    const uint64_t n = a->n;
    for (uint64_t i = 0; i < n; ++i) component[i] = UINT64_MAX;
    uint64_t next_id = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (component[i] != UINT64_MAX) continue;
        const uint64_t cid = next_id++;
        component[i] = cid;
        for (uint64_t j = i + 1; j < n; ++j)
            if (has_entry(&closure, i, (uint32_t)j) && has_entry(&closure, j, (uint32_t)i)) component[j] = cid;
    }
    orc_csr_free(&closure);
    return 0;
}

/* ---- CsrMatrix::rcm order (src/graph_csr.rs:663-722) ------------------------------------------
 * For every unvisited seed in id order: a plain BFS (neighbours in column order) whose last popped
 * node is the start; then a BFS from the start that visits each node's unvisited neighbours by
 * ascending degree (ties in column order); the concatenated visit order, reversed. */
static uint64_t deg_of(const orc_csr *a, uint64_t v) { return a->row_ptr[v + 1] - a->row_ptr[v]; }

int orc_rcm_order(const orc_csr *a, uint32_t *perm) {
    const uint64_t n = a->n;
    uint8_t *visited = calloc(n ? n : 1, 1);
    uint64_t *stamp = calloc(n ? n : 1, 8); /* vis2 of seed s: stamp == s + 1 */
    uint64_t *queue = malloc((n + 2) * 8);
    uint64_t *order = malloc((2 * n + 1) * 8);
    uint64_t *nbrs = malloc((n ? n : 1) * 8);
    uint64_t olen = 0;
    int rc = 0;
    for (uint64_t seed = 0; seed < n; ++seed) {
        if (visited[seed]) continue;
        uint64_t qh = 0, qt = 0, last = seed;
        stamp[seed] = seed + 1;
        queue[qt++] = seed;
        while (qh < qt) {
            const uint64_t u = queue[qh++];
            last = u;
            for (uint64_t i = a->row_ptr[u]; i < a->row_ptr[u + 1]; ++i) {
                const uint64_t v = a->col[i];
                if (stamp[v] != seed + 1) {
                    stamp[v] = seed + 1;
                    queue[qt++] = v;
                }
            }
        }
        const uint64_t start = last;
        qh = qt = 0;
        queue[qt++] = start;
        visited[start] = 1;
        while (qh < qt) {
            const uint64_t u = queue[qh++];
            if (olen >= 2 * n) { rc = -1; goto done; }
            order[olen++] = u;
            uint64_t k = 0;
            for (uint64_t i = a->row_ptr[u]; i < a->row_ptr[u + 1]; ++i)
                if (!visited[a->col[i]]) nbrs[k++] = a->col[i];
            /* stable insertion sort by degree (k is a row length) */
            for (uint64_t x = 1; x < k; ++x) {
                const uint64_t v = nbrs[x], dv = deg_of(a, v);
                uint64_t y = x;
                while (y > 0 && deg_of(a, nbrs[y - 1]) > dv) { nbrs[y] = nbrs[y - 1]; --y; }
                nbrs[y] = v;
            }
            for (uint64_t x = 0; x < k; ++x)
                if (!visited[nbrs[x]]) {
                    visited[nbrs[x]] = 1;
                    if (qt > n) { rc = -1; goto done; }
                    queue[qt++] = nbrs[x];
                }
        }
    }
    if (olen != n) { rc = -1; goto done; }
    for (uint64_t i = 0; i < n; ++i) perm[i] = (uint32_t)order[n - 1 - i];
done:
    free(visited); free(stamp); free(queue); free(order); free(nbrs);
    return rc;
}

/* CsrMatrix::permute (src/graph_csr.rs:726-783): new row inv[r] holds row r's entries with
 * columns inv[c], sorted by column (a permutation has no duplicate columns, so order is unique) */
int orc_permute(const orc_csr *a, const uint32_t *perm, orc_csr *out) {
    const uint64_t n = a->n, nnz = a->nnz;
    const size_t vs = a->dtype == ORC_U32 ? 4 : 8;
    uint32_t *inv = malloc((n ? n : 1) * 4);
    for (uint64_t i = 0; i < n; ++i) inv[perm[i]] = (uint32_t)i;
    out->n = n;
    out->nnz = nnz;
    out->dtype = a->dtype;
    out->row_ptr = calloc(n + 1, 8);
    out->col = malloc((nnz ? nnz : 1) * 4);
    out->val = malloc((nnz ? nnz : 1) * vs);
    for (uint64_t r = 0; r < n; ++r) out->row_ptr[inv[r] + 1] = a->row_ptr[r + 1] - a->row_ptr[r];
    for (uint64_t i = 1; i <= n; ++i) out->row_ptr[i] += out->row_ptr[i - 1];
    for (uint64_t r = 0; r < n; ++r) {
        const uint64_t nr = inv[r], s = a->row_ptr[r], e = a->row_ptr[r + 1];
        uint64_t pos = out->row_ptr[nr];
        for (uint64_t i = s; i < e; ++i, ++pos) {
            /* insertion into the sorted prefix of the new row */
            const uint32_t c = inv[a->col[i]];
            uint64_t y = pos;
            while (y > out->row_ptr[nr] && out->col[y - 1] > c) {
                out->col[y] = out->col[y - 1];
                memcpy((char *)out->val + y * vs, (char *)out->val + (y - 1) * vs, vs);
                --y;
            }
            out->col[y] = c;
            memcpy((char *)out->val + y * vs, (const char *)a->val + i * vs, vs);
        }
    }
    free(inv);
    return 0;
}

void orc_bandwidth_stats(const orc_csr *a, uint64_t *max_bw, double *avg_bw) {
    uint64_t mx = 0, sum = 0;
    for (uint64_t r = 0; r < a->n; ++r)
        for (uint64_t i = a->row_ptr[r]; i < a->row_ptr[r + 1]; ++i) {
            const uint64_t c = a->col[i], d = r > c ? r - c : c - r;
            if (d > mx) mx = d;
            sum += d;
        }
    *max_bw = mx;
    *avg_bw = (double)sum / (double)(a->nnz ? a->nnz : 1);
}

/* load_edges (src/graph_csr.rs:1209-1224): lines trimmed, empty ones skipped, the first two
 * whitespace-separated tokens parsed as u32 (further tokens ignored) */
int orc_load_edges(const char *path, uint64_t *n, uint64_t *n_edges, uint32_t **src, uint32_t **dst) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    uint64_t cap = 1024, m = 0;
    uint32_t *s = malloc(cap * 4), *d = malloc(cap * 4), max_id = 0;
    char line[4096];
    int rc = 0;
    while (fgets(line, sizeof line, f)) {
        char *p = line;
        uint64_t v[2];
        int got = 0;
        while (got < 2) {
            while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n' || *p == '\f' || *p == '\v') ++p;
            if (!*p) break;
            if (*p == '+') ++p; /* str::parse::<u32> takes a leading '+' */
            if (*p < '0' || *p > '9') { rc = -1; goto done; }
            uint64_t x = 0;
            while (*p >= '0' && *p <= '9') {
                x = x * 10 + (uint64_t)(*p++ - '0');
                if (x > 0xFFFFFFFFull) { rc = -1; goto done; }
            }
            if (*p && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n' && *p != '\f' && *p != '\v') { rc = -1; goto done; }
            v[got++] = x;
        }
        if (got == 0) continue;
        if (got == 1) { rc = -1; goto done; }
        if (m == cap) { cap *= 2; s = realloc(s, cap * 4); d = realloc(d, cap * 4); }
        s[m] = (uint32_t)v[0];
        d[m] = (uint32_t)v[1];
        if (s[m] > max_id) max_id = s[m];
        if (d[m] > max_id) max_id = d[m];
        ++m;
    }
    if (max_id == 0xFFFFFFFFu) rc = -1;
done:
    fclose(f);
    if (rc) { free(s); free(d); return rc; }
    *n = (uint64_t)max_id + 1;
    *n_edges = m;
    *src = s;
    *dst = d;
    return 0;
}

/* einsum_sparse_driven (einsum-dyn/src/sparse.rs:70-148), "ab,bc->ac" (trans 0) or "->ca" (1):
 * a dense accumulator per A row, touched columns listed when their accumulator reads 0, written
 * out and cleared. u32 = plain wrapping u32 (the einsum tests' T); f64 = the same left fold. */
int orc_einsum_sparse_driven(const orc_csr *a, const orc_csr *b, void *out, uint64_t ld, int trans) {
    if (a->dtype != b->dtype || a->dtype == ORC_SAT64) return -1;
    const uint64_t m = b->n;
    const int f = a->dtype == ORC_F64;
    double *accd = calloc(m ? m : 1, 8);
    uint32_t *accu = calloc(m ? m : 1, 4);
    uint64_t *nz = malloc((m ? m : 1) * 8 * 4 + 64), nzcap = (m ? m : 1) * 4, nn = 0;
    for (uint64_t i = 0; i < a->n; ++i) {
        nn = 0;
        for (uint64_t e = a->row_ptr[i]; e < a->row_ptr[i + 1]; ++e) {
            const uint64_t k = a->col[e];
            for (uint64_t t = b->row_ptr[k]; t < b->row_ptr[k + 1]; ++t) {
                const uint64_t j = b->col[t];
                const int zero = f ? accd[j] == 0.0 : accu[j] == 0;
                if (zero) {
                    if (nn == nzcap) { nzcap *= 2; nz = realloc(nz, nzcap * 8); }
                    nz[nn++] = j;
                }
                if (f) {
                    volatile double p = ((const double *)a->val)[e] * ((const double *)b->val)[t];
                    accd[j] = accd[j] + p;
                } else {
                    accu[j] += ((const uint32_t *)a->val)[e] * ((const uint32_t *)b->val)[t];
                }
            }
        }
        for (uint64_t q = 0; q < nn; ++q) {
            const uint64_t j = nz[q], at = trans ? j * ld + i : i * ld + j;
            if (f) { ((double *)out)[at] = accd[j]; accd[j] = 0.0; }
            else { ((uint32_t *)out)[at] = accu[j]; accu[j] = 0; }
        }
    }
    free(accd); free(accu); free(nz);
    return 0;
}
