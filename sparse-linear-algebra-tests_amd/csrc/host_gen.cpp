// host_gen.cpp — host-side constructors of the reference API (product code, not the oracle).
//
//   slat_rng_*          rand 0.9.2 StdRng = ChaCha12Rng (rand_chacha 0.9.0, Cargo.lock:851-895):
//                       key = seed words (LE), 64-bit block counter in words 12-13, stream 0,
//                       4-block refills; f64 draw = (next_u64 >> 12) * 2^-52 (UniformFloat).
//   slat_host_from_coo  CsrMatrix::from_coo   src/graph_csr.rs:83-129 (row counting sort + per-row
//                       column sort, duplicates summed, zeros dropped)
//   slat_host_lattice   CsrMatrix::lattice    src/graph_csr.rs:177-222
//   slat_host_thin      CsrMatrix::thin       src/graph_csr.rs:225-247
//   slat_host_random    CsrMatrix::random     src/graph_csr.rs:163-174 (rand 0.9 integer
//                       random_range: UniformUsize -> u32 Canon's method, BlockRng word order)
//   slat_host_rmat      seeded R-MAT for the f64 power-law config (not in the reference)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "slat.h"

namespace {

struct Rng {
    uint32_t key[8];
    uint64_t counter;
    uint32_t buf[64];
    uint32_t idx;
};
static_assert(sizeof(Rng) <= sizeof(slat_rng), "slat_rng too small");

inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

void chacha12(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    uint32_t x[16];
    std::memcpy(x, s, sizeof x);
    auto qr = [&](int a, int b, int c, int d) {
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 6; ++r) {
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

Rng *R(slat_rng *r) { return reinterpret_cast<Rng *>(r); }

size_t vsz(int32_t dt) { return dt == SLAT_U32 ? 4 : 8; }

struct Trip {
    uint32_t r, c;
    uint64_t v;  // value bits
};

bool is_zero(uint64_t bits, int32_t dt) {
    if (dt == SLAT_F64) {
        double d;
        std::memcpy(&d, &bits, 8);
        return d == 0.0;
    }
    return bits == 0;
}

uint64_t add_bits(uint64_t x, uint64_t y, int32_t dt) {
    if (dt == SLAT_F64) {
        double a, b;
        std::memcpy(&a, &x, 8);
        std::memcpy(&b, &y, 8);
        a += b;
        uint64_t o;
        std::memcpy(&o, &a, 8);
        return o;
    }
    if (dt == SLAT_U32) return (uint32_t)(x + y);  // plain `+=` (wraps in release)
    return x + y;
}

slat_status build(uint64_t n, std::vector<Trip> &t, int32_t dt, slat_host_csr *out) {
    std::memset(out, 0, sizeof *out);
    // counting sort by row, then sort columns inside each row
    std::vector<uint64_t> cnt(n + 1, 0);
    for (const Trip &x : t) {
        if (x.r >= n || x.c >= n) return SLAT_EINVAL;
        cnt[x.r + 1]++;
    }
    for (uint64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    std::vector<Trip> s(t.size());
    {
        std::vector<uint64_t> pos(cnt.begin(), cnt.end() - 1);
        for (const Trip &x : t) s[pos[x.r]++] = x;
    }
    out->n = n;
    out->dtype = dt;
    out->row_ptr = (uint64_t *)std::malloc((n + 1) * 8);
    out->col_idx = (uint32_t *)std::malloc(std::max<size_t>(t.size(), 1) * 4);
    out->values = std::malloc(std::max<size_t>(t.size(), 1) * vsz(dt));
    if (!out->row_ptr || !out->col_idx || !out->values) return SLAT_EOOM;
    uint64_t k = 0;
    out->row_ptr[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        Trip *b = s.data() + cnt[r], *e = s.data() + cnt[r + 1];
        std::sort(b, e, [](const Trip &x, const Trip &y) { return x.c < y.c; });  // ties: duplicates
        for (Trip *p = b; p < e;) {
            uint64_t v = p->v;
            const uint32_t c = p->c;
            // merge duplicates in input order (stable semantics irrelevant: addition of one type)
            for (++p; p < e && p->c == c; ++p) v = add_bits(v, p->v, dt);
            if (is_zero(v, dt)) continue;
            out->col_idx[k] = c;
            if (dt == SLAT_U32)
                ((uint32_t *)out->values)[k] = (uint32_t)v;
            else
                std::memcpy((uint8_t *)out->values + 8 * k, &v, 8);
            ++k;
        }
        out->row_ptr[r + 1] = k;
    }
    out->nnz = k;
    return SLAT_OK;
}

uint64_t get_bits(const slat_host_csr *m, uint64_t r, uint32_t c) {
    const uint32_t *b = m->col_idx + m->row_ptr[r], *e = m->col_idx + m->row_ptr[r + 1];
    const uint32_t *p = std::lower_bound(b, e, c);
    if (p == e || *p != c) return 0;
    const uint64_t i = (uint64_t)(p - m->col_idx);
    if (m->dtype == SLAT_U32) return ((const uint32_t *)m->values)[i];
    uint64_t v;
    std::memcpy(&v, (const uint8_t *)m->values + 8 * i, 8);
    return v;
}

}  // namespace

extern "C" {

void slat_rng_seed(slat_rng *rng, const uint8_t seed[32]) {
    Rng *r = R(rng);
    for (int i = 0; i < 8; ++i)
        r->key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
                    ((uint32_t)seed[4 * i + 3] << 24);
    r->counter = 0;
    r->idx = 64;
}

static void refill(Rng *r) {
    for (int b = 0; b < 4; ++b) chacha12(r->key, r->counter + (uint64_t)b, r->buf + 16 * b);
    r->counter += 4;
    r->idx = 0;
}

// rand_core 0.9 BlockRng::next_u64: two consecutive words; from the buffer's last word, the low
// half is that word and the high half the first word of the next refill
uint64_t slat_rng_next_u64(slat_rng *rng) {
    Rng *r = R(rng);
    if (r->idx >= 64) refill(r);
    if (r->idx == 63) {
        const uint64_t lo = r->buf[63];
        refill(r);
        r->idx = 1;
        return lo | ((uint64_t)r->buf[0] << 32);
    }
    const uint64_t lo = r->buf[r->idx], hi = r->buf[r->idx + 1];
    r->idx += 2;
    return lo | (hi << 32);
}

// rand_core 0.9 BlockRng::next_u32: one word
uint32_t slat_rng_next_u32(slat_rng *rng) {
    Rng *r = R(rng);
    if (r->idx >= 64) refill(r);
    return r->buf[r->idx++];
}

// rand 0.9 `random_range(lo..hi)` for usize / u32 with hi <= u32::MAX: UniformUsize samples as u32,
// UniformInt<u32>::sample_single_inclusive(lo, hi - 1) by Canon's method (a second draw only when
// the low half of the first product exceeds 2^32 - range; its carry bumps the result)
uint32_t slat_rng_range_u32(slat_rng *rng, uint32_t lo, uint32_t hi) {
    const uint32_t range = hi - lo;  // 0 = the whole u32 range
    if (range == 0) return slat_rng_next_u32(rng);
    const uint64_t m = (uint64_t)slat_rng_next_u32(rng) * range;
    uint32_t result = (uint32_t)(m >> 32);
    const uint32_t lo_order = (uint32_t)m;
    if (lo_order > 0u - range) {
        const uint32_t new_hi = (uint32_t)(((uint64_t)slat_rng_next_u32(rng) * range) >> 32);
        if ((uint32_t)(lo_order + new_hi) < lo_order) result += 1;
    }
    return lo + result;
}

double slat_rng_next_f64(slat_rng *rng) {
    return (double)(slat_rng_next_u64(rng) >> 12) * (1.0 / 4503599627370496.0);
}

// Stream position of a StdRng (slat_internal.hpp): the key and the index of the next keystream word,
// so a device generator can draw the same values; advance = `draws` u64 draws later, in the state the
// host generator would be in after making them itself.
void slat_rng_position(const slat_rng *rng, uint32_t key[8], uint64_t *word) {
    const Rng *r = reinterpret_cast<const Rng *>(rng);
    std::memcpy(key, r->key, 32);
    *word = r->idx >= 64 ? r->counter * 16 : (r->counter - 4) * 16 + r->idx;
}

void slat_rng_advance(slat_rng *rng, uint64_t draws) {
    Rng *r = R(rng);
    uint32_t key[8];
    uint64_t w;
    slat_rng_position(rng, key, &w);
    w += 2 * draws;  // f64 draws: two words each
    r->counter = (w / 64) * 4;
    r->idx = 64;
    if (w % 64) {  // mid-refill: the 4 blocks holding word w, read position inside them
        for (int b = 0; b < 4; ++b) chacha12(r->key, r->counter + (uint64_t)b, r->buf + 16 * b);
        r->counter += 4;
        r->idx = (uint32_t)(w % 64);
    }
}

void slat_host_csr_free(slat_host_csr *m) {
    if (!m) return;
    std::free(m->row_ptr);
    std::free(m->col_idx);
    std::free(m->values);
    std::memset(m, 0, sizeof *m);
}

slat_status slat_host_from_coo(uint64_t n, uint64_t ntrip, const uint32_t *rows, const uint32_t *cols,
                               const void *vals, int32_t dtype, slat_host_csr *out) {
    if (!out || (ntrip && (!rows || !cols || !vals)) || dtype < SLAT_U32 || dtype > SLAT_F64) return SLAT_EINVAL;
    std::vector<Trip> t(ntrip);
    for (uint64_t i = 0; i < ntrip; ++i) {
        t[i].r = rows[i];
        t[i].c = cols[i];
        if (dtype == SLAT_U32)
            t[i].v = ((const uint32_t *)vals)[i];
        else
            std::memcpy(&t[i].v, (const uint8_t *)vals + 8 * i, 8);
    }
    return build(n, t, dtype, out);
}

slat_status slat_host_lattice(const uint64_t *dims, int ndim, int torus, slat_host_csr *out) {
    if (!dims || ndim < 1 || ndim > 16 || !out) return SLAT_EINVAL;
    uint64_t total = 1, nnb = 1;
    for (int d = 0; d < ndim; ++d) {
        total *= dims[d];
        nnb *= 3;
    }
    if (total > 0xFFFFFFFFull) return SLAT_EINVAL;
    std::vector<uint64_t> strides(ndim, 1);
    for (int d = ndim - 2; d >= 0; --d) strides[d] = strides[d + 1] * dims[d + 1];
    std::vector<Trip> t;
    t.reserve(total * (nnb - 1));
    std::vector<uint64_t> coord(ndim, 0);
    for (uint64_t node = 0; node < total; ++node) {
        for (uint64_t off = 0; off < nnb; ++off) {
            uint64_t tmp = off, nb = 0;
            bool all_zero = true, valid = true;
            for (int d = 0; d < ndim; ++d) {
                const int64_t delta = (int64_t)(tmp % 3) - 1;  // dimension 0 = least significant digit
                tmp /= 3;
                if (delta) all_zero = false;
                int64_t c = (int64_t)coord[d] + delta;
                const int64_t m = (int64_t)dims[d];
                if (torus) {
                    c = ((c % m) + m) % m;
                } else if (c < 0 || c >= m) {
                    valid = false;
                    break;
                }
                nb += (uint64_t)c * strides[d];
            }
            if (all_zero || !valid) continue;
            t.push_back({(uint32_t)node, (uint32_t)nb, 1});
        }
        for (int d = ndim - 1; d >= 0; --d) {
            if (++coord[d] < dims[d]) break;
            coord[d] = 0;
        }
    }
    return build(total, t, SLAT_U32, out);
}

slat_status slat_host_thin(const slat_host_csr *m, slat_rng *rng, double density, slat_host_csr *out) {
    if (!m || !rng || !out) return SLAT_EINVAL;
    std::vector<Trip> t;
    t.reserve(m->nnz);
    for (uint64_t r = 0; r < m->n; ++r) {
        for (uint64_t idx = m->row_ptr[r]; idx < m->row_ptr[r + 1]; ++idx) {
            const uint32_t c = m->col_idx[idx];
            uint64_t v;
            if (m->dtype == SLAT_U32)
                v = ((const uint32_t *)m->values)[idx];
            else
                std::memcpy(&v, (const uint8_t *)m->values + 8 * idx, 8);
            // `r <= c && rng.random_range(0.0..1.0) < density`: one draw only when r <= c
            if (r <= c && slat_rng_next_f64(rng) < density) {
                t.push_back({(uint32_t)r, c, v});
                if (r != c) {
                    const uint64_t rev = get_bits(m, c, (uint32_t)r);
                    if (!is_zero(rev, m->dtype)) t.push_back({c, (uint32_t)r, rev});
                }
            }
        }
    }
    return build(m->n, t, m->dtype, out);
}

// CsrMatrix::random (src/graph_csr.rs:163-174): m edges r in 0..n, c in 0..n-1 bumped past r (no
// self-loops), value 1, duplicates summed by from_coo
slat_status slat_host_random(slat_rng *rng, uint32_t n, uint64_t m, slat_host_csr *out) {
    if (!rng || !out || n < 2) return SLAT_EINVAL;  // assert!(nu >= 2)
    std::vector<Trip> t(m);
    for (uint64_t i = 0; i < m; ++i) {
        const uint32_t r = slat_rng_range_u32(rng, 0, n);
        uint32_t c = slat_rng_range_u32(rng, 0, n - 1);
        if (c >= r) c += 1;
        t[i] = {r, c, 1};
    }
    return build(n, t, SLAT_U32, out);
}

slat_status slat_host_rmat(uint32_t scale, uint64_t n_edges, double a, double b, double c, const uint8_t seed[32],
                           slat_host_csr *out) {
    if (!out || scale == 0 || scale > 31 || a < 0 || b < 0 || c < 0 || a + b + c > 1.0) return SLAT_EINVAL;
    slat_rng rng;
    slat_rng_seed(&rng, seed);
    const uint64_t n = 1ull << scale;
    std::vector<Trip> t(n_edges);
    for (uint64_t e = 0; e < n_edges; ++e) {
        uint32_t r = 0, col = 0;
        for (uint32_t lvl = 0; lvl < scale; ++lvl) {
            const double u = slat_rng_next_f64(&rng);
            const uint32_t bit = 1u << (scale - 1 - lvl);
            if (u < a) {
            } else if (u < a + b) {
                col |= bit;
            } else if (u < a + b + c) {
                r |= bit;
            } else {
                r |= bit;
                col |= bit;
            }
        }
        const double v = 0.5 + slat_rng_next_f64(&rng);  // strictly positive: no cancellation
        t[e].r = r;
        t[e].c = col;
        std::memcpy(&t[e].v, &v, 8);
    }
    return build(n, t, SLAT_F64, out);
}

}  // extern "C"

// load_edges (src/graph_csr.rs:1209-1224): the file read whole, lines trimmed, empty lines skipped,
// the first two whitespace-separated tokens parsed as u32 (an optional '+', like str::parse);
// n = max id + 1. A missing or malformed token -> SLAT_EINVAL (the reference panics).
extern "C" slat_status slat_load_edges(const char *path, uint64_t *n, uint64_t *n_edges, uint32_t **src,
                                       uint32_t **dst) {
    if (!path || !n || !n_edges || !src || !dst) return SLAT_EINVAL;
    FILE *f = std::fopen(path, "rb");
    if (!f) return SLAT_EINVAL;
    std::vector<char> buf;
    char chunk[1 << 16];
    size_t got;
    while ((got = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + got);
    std::fclose(f);
    buf.push_back('\n');
    auto space = [](char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v'; };
    std::vector<uint32_t> s, d;
    uint32_t max_id = 0;
    size_t i = 0;
    const size_t end = buf.size();
    while (i < end) {
        uint64_t v[2];
        int tokens = 0;
        while (true) {
            while (i < end && space(buf[i])) ++i;
            if (i >= end || buf[i] == '\n' || tokens == 2) break;
            if (buf[i] == '+') ++i;
            if (i >= end || buf[i] < '0' || buf[i] > '9') return SLAT_EINVAL;
            uint64_t x = 0;
            while (i < end && buf[i] >= '0' && buf[i] <= '9') {
                x = x * 10 + (uint64_t)(buf[i++] - '0');
                if (x > 0xFFFFFFFFull) return SLAT_EINVAL;
            }
            if (i < end && buf[i] != '\n' && !space(buf[i])) return SLAT_EINVAL;
            v[tokens++] = x;
        }
        while (i < end && buf[i] != '\n') ++i;  // further tokens are not read
        ++i;
        if (tokens == 0) continue;
        if (tokens == 1) return SLAT_EINVAL;
        s.push_back((uint32_t)v[0]);
        d.push_back((uint32_t)v[1]);
        max_id = std::max(max_id, std::max((uint32_t)v[0], (uint32_t)v[1]));
    }
    if (max_id == 0xFFFFFFFFu) return SLAT_EINVAL;  // max_id + 1 overflows NodeId
    *src = (uint32_t *)std::malloc(std::max<size_t>(s.size(), 1) * 4);
    *dst = (uint32_t *)std::malloc(std::max<size_t>(d.size(), 1) * 4);
    if (!*src || !*dst) {
        std::free(*src);
        std::free(*dst);
        return SLAT_EOOM;
    }
    if (!s.empty()) {
        std::memcpy(*src, s.data(), s.size() * 4);
        std::memcpy(*dst, d.data(), d.size() * 4);
    }
    *n = (uint64_t)max_id + 1;
    *n_edges = s.size();
    return SLAT_OK;
}

extern "C" void slat_edges_free(uint32_t *src, uint32_t *dst) {
    std::free(src);
    std::free(dst);
}
