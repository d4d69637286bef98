/*
 * oracle.c -- plain-C restatement of wasabipesto/nice's CPU field processing.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Never linked into nice_amd/.
 *
 * Arithmetic is exact for every n < 2^128 and base 2..128: n^2 and n^3 are
 * held in up to 6 u64 limbs.  (The reference's u128 / U256 fast paths wrap
 * for n far outside a base's valid range -- client_process.rs:84-85 for b40
 * above ~6.98e12, fixed_width.rs:88-125 above 2^85 -- release builds do not
 * check overflow, Cargo.toml [profile.release].  Inside every valid range all
 * arms agree with this exact version, and with the reference's GPU path.)
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint32_t u32;

#define MAXL 8 /* u64 limbs: n < 2^128 => n^3 < 2^384 (6 limbs) */

typedef struct {
    u64 l[MAXL];
    int top; /* index of the highest non-zero limb, -1 for zero */
} big;

static inline u128 mk(u64 lo, u64 hi) { return ((u128)hi << 64) | lo; }

static inline void big_set(big *b, u128 v) {
    memset(b, 0, sizeof(*b));
    b->l[0] = (u64)v;
    b->l[1] = (u64)(v >> 64);
    b->top = b->l[1] ? 1 : (b->l[0] ? 0 : -1);
}

/* r = a * m (schoolbook, u64 limbs). */
static inline void big_mul_u128(const big *a, u128 m, big *r) {
    u64 ml[2] = {(u64)m, (u64)(m >> 64)};
    memset(r, 0, sizeof(*r));
    r->top = -1;
    if (a->top < 0 || m == 0) return;
    for (int j = 0; j < 2; j++) {
        if (!ml[j]) continue;
        u64 carry = 0;
        for (int i = 0; i <= a->top; i++) {
            u128 cur = (u128)a->l[i] * ml[j] + r->l[i + j] + carry;
            r->l[i + j] = (u64)cur;
            carry = (u64)(cur >> 64);
        }
        int k = a->top + 1 + j;
        while (carry && k < MAXL) {
            u128 cur = (u128)r->l[k] + carry;
            r->l[k] = (u64)cur;
            carry = (u64)(cur >> 64);
            k++;
        }
    }
    for (int i = MAXL - 1; i >= 0; i--)
        if (r->l[i]) { r->top = i; break; }
}

/* In-place v /= d, returns v % d (d < 2^32).  Each u64 limb is divided in two
 * 32-bit halves so every quotient fits a u64 (same idea as fixed_width.rs:151-181). */
static inline __attribute__((always_inline)) u32 big_divrem(big *v, u64 d) {
    u64 rem = 0;
    for (int i = v->top; i >= 0; i--) {
        u64 limb = v->l[i];
        u64 hi = (rem << 32) | (limb >> 32);
        u64 qh = hi / d;
        u64 rh = hi - qh * d;
        u64 lo = (rh << 32) | (limb & 0xffffffffu);
        u64 ql = lo / d;
        rem = lo - ql * d;
        v->l[i] = (qh << 32) | ql;
    }
    while (v->top >= 0 && v->l[v->top] == 0) v->top--;
    return (u32)rem;
}

/* Digits of v, least significant first, until v reaches zero (malachite
 * to_digits_asc / the `while n != 0` loops).  Returns the count. */
static int big_digits_asc(big v, u32 base, u32 *out) {
    int n = 0;
    while (v.top >= 0) out[n++] = big_divrem(&v, base);
    return n;
}

/* ------------------------------------------------------------------------ */
/* base_range.rs:14-54                                                      */
/* ------------------------------------------------------------------------ */

/* Arbitrary-size natural as u32 limbs for b^e with e up to ~3*25+2. */
#define NATL 80
typedef struct { u32 l[NATL]; int n; } nat;

static void nat_pow(u32 b, u32 e, nat *r) {
    memset(r, 0, sizeof(*r));
    r->l[0] = 1; r->n = 1;
    for (u32 i = 0; i < e; i++) {
        u64 carry = 0;
        for (int j = 0; j < r->n; j++) {
            u64 cur = (u64)r->l[j] * b + carry;
            r->l[j] = (u32)cur; carry = cur >> 32;
        }
        if (carry) r->l[r->n++] = (u32)carry;
    }
}
/* r = x^p for x < 2^128 (p = 2 or 3), as nat. */
static void nat_from_pow(u128 x, int p, nat *r) {
    big t, s, c;
    big_set(&t, x);
    big_mul_u128(&t, x, &s);
    const big *src = &s;
    if (p == 3) { big_mul_u128(&s, x, &c); src = &c; }
    if (p == 1) src = &t;
    memset(r, 0, sizeof(*r));
    for (int i = 0; i < MAXL; i++) { r->l[2 * i] = (u32)src->l[i]; r->l[2 * i + 1] = (u32)(src->l[i] >> 32); }
    r->n = 2 * MAXL;
    while (r->n > 0 && r->l[r->n - 1] == 0) r->n--;
}
static int nat_cmp(const nat *a, const nat *b) {
    if (a->n != b->n) return a->n < b->n ? -1 : 1;
    for (int i = a->n - 1; i >= 0; i--)
        if (a->l[i] != b->l[i]) return a->l[i] < b->l[i] ? -1 : 1;
    return 0;
}
/* ceiling p-th root of v, or -1 status if it does not fit u128. */
static int nat_ceil_root(const nat *v, int p, u128 *out) {
    /* smallest x with x^p >= v; binary search over u128 */
    int bits = 0;
    for (int i = v->n - 1; i >= 0; i--)
        if (v->l[i]) { bits = 32 * i + (32 - __builtin_clz(v->l[i])); break; }
    int rb = (bits + p - 1) / p + 1;
    u128 lo = 0, hi = (rb >= 128) ? ~(u128)0 : ((u128)1 << rb);
    while (lo < hi) {
        u128 mid = lo + (hi - lo) / 2;
        nat m;
        nat_from_pow(mid, p, &m);
        if (nat_cmp(&m, v) >= 0) hi = mid; else lo = mid + 1;
    }
    nat chk;
    nat_from_pow(lo, p, &chk);
    if (nat_cmp(&chk, v) < 0) return -1; /* root >= 2^128 */
    *out = lo;
    return 0;
}
static int nat_to_u128(const nat *v, u128 *out) {
    if (v->n > 4) return -1;
    u128 r = 0;
    for (int i = v->n - 1; i >= 0; i--) r = (r << 32) | v->l[i];
    *out = r;
    return 0;
}

int oracle_base_range(u32 base, u64 *slo, u64 *shi, u64 *elo, u64 *ehi) {
    u32 k = base / 5;
    nat a, b;
    u128 s, e;
    int st = 0;
    switch (base % 5) {
    case 0:
        if (k == 0) return 0;
        nat_pow(base, 3 * k - 1, &a); st |= nat_ceil_root(&a, 3, &s);
        nat_pow(base, k, &b); st |= nat_to_u128(&b, &e);
        break;
    case 1:
        return 0;
    case 2:
        nat_pow(base, k, &a); st |= nat_to_u128(&a, &s);
        nat_pow(base, 3 * k + 1, &b); st |= nat_ceil_root(&b, 3, &e);
        break;
    case 3:
        nat_pow(base, 3 * k + 1, &a); st |= nat_ceil_root(&a, 3, &s);
        nat_pow(base, 2 * k + 1, &b); st |= nat_ceil_root(&b, 2, &e);
        break;
    default:
        nat_pow(base, 2 * k + 1, &a); st |= nat_ceil_root(&a, 2, &s);
        nat_pow(base, 3 * k + 2, &b); st |= nat_ceil_root(&b, 3, &e);
        break;
    }
    if (st) return -1;
    if (s >= e) return 0; /* FieldSize::new would reject it */
    *slo = (u64)s; *shi = (u64)(s >> 64);
    *elo = (u64)e; *ehi = (u64)(e >> 64);
    return 1;
}

/* number_stats.rs:15-17 */
u32 oracle_near_miss_cutoff(u32 base) {
    volatile float f = (float)base * 0.9f;
    return (u32)floorf(f);
}

/* ------------------------------------------------------------------------ */
/* client_process.rs:47-143: unique digits of n^2 and n^3                   */
/* ------------------------------------------------------------------------ */

static inline __attribute__((always_inline)) u32 nud_impl(u128 n, u32 base) {
    big t, sq, cu;
    big_set(&t, n);
    big_mul_u128(&t, n, &sq);
    big_mul_u128(&sq, n, &cu);
    u64 m0 = 0, m1 = 0;
    while (sq.top >= 0) {
        u32 d = big_divrem(&sq, base);
        if (d < 64) m0 |= 1ull << d; else m1 |= 1ull << (d - 64);
    }
    while (cu.top >= 0) {
        u32 d = big_divrem(&cu, base);
        if (d < 64) m0 |= 1ull << d; else m1 |= 1ull << (d - 64);
    }
    return (u32)(__builtin_popcountll(m0) + __builtin_popcountll(m1));
}
/* Constant-base instances so gcc strength-reduces the divisions, as the
 * reference's const-generic arms do (client_process.rs:48-67). */
static u32 nud_10(u128 n) { return nud_impl(n, 10); }
static u32 nud_40(u128 n) { return nud_impl(n, 40); }
static u32 nud_50(u128 n) { return nud_impl(n, 50); }
static u32 nud_80(u128 n) { return nud_impl(n, 80); }
static u32 nud_any(u128 n, u32 base) { return nud_impl(n, base); }

static inline u32 nud(u128 n, u32 base) {
    switch (base) {
    case 10: return nud_10(n);
    case 40: return nud_40(n);
    case 50: return nud_50(n);
    case 80: return nud_80(n);
    default: return nud_any(n, base);
    }
}

u32 oracle_num_unique_digits(u64 lo, u64 hi, u32 base) { return nud(mk(lo, hi), base); }

/* client_process.rs:222-413.  sq_ok (test statistic, may be NULL): set to 1
 * when n^2 alone has no repeated digit, i.e. the scan reached the cube. */
static inline __attribute__((always_inline)) int is_nice_impl2(u128 n, u32 base, int *sq_ok) {
    big t, sq, cu;
    big_set(&t, n);
    big_mul_u128(&t, n, &sq);
    u64 m0 = 0, m1 = 0;
    big s2 = sq;
    while (s2.top >= 0) {
        u32 d = big_divrem(&s2, base);
        u64 *w = d < 64 ? &m0 : &m1;
        u64 bit = 1ull << (d & 63);
        if (*w & bit) return 0;
        *w |= bit;
    }
    if (sq_ok) *sq_ok = 1;
    big_mul_u128(&sq, n, &cu);
    while (cu.top >= 0) {
        u32 d = big_divrem(&cu, base);
        u64 *w = d < 64 ? &m0 : &m1;
        u64 bit = 1ull << (d & 63);
        if (*w & bit) return 0;
        *w |= bit;
    }
    return 1;
}
static inline __attribute__((always_inline)) int is_nice_impl(u128 n, u32 base) {
    return is_nice_impl2(n, base, NULL);
}
static int isn_10(u128 n) { return is_nice_impl(n, 10); }
static int isn_40(u128 n) { return is_nice_impl(n, 40); }
static int isn_50(u128 n) { return is_nice_impl(n, 50); }
static int isn_80(u128 n) { return is_nice_impl(n, 80); }
static int isn_any(u128 n, u32 base) { return is_nice_impl(n, base); }
static inline int is_nice(u128 n, u32 base) {
    switch (base) {
    case 10: return isn_10(n);
    case 40: return isn_40(n);
    case 50: return isn_50(n);
    case 80: return isn_80(n);
    default: return isn_any(n, base);
    }
}
int oracle_is_nice(u64 lo, u64 hi, u32 base) { return is_nice(mk(lo, hi), base); }

u32 oracle_scan_depth(u64 lo, u64 hi, u32 base) {
    u128 n = mk(lo, hi);
    big t, sq, cu;
    big_set(&t, n);
    big_mul_u128(&t, n, &sq);
    big_mul_u128(&sq, n, &cu);
    u64 m[2] = {0, 0};
    u32 depth = 0;
    big *v[2] = {&sq, &cu};
    for (int p = 0; p < 2; p++) {
        while (v[p]->top >= 0) {
            u32 d = big_divrem(v[p], base);
            depth++;
            u64 bit = 1ull << (d & 63);
            if (m[d >> 6] & bit) return depth;
            m[d >> 6] |= bit;
        }
    }
    return depth;
}

/* ------------------------------------------------------------------------ */
/* client_process.rs:150-191: detailed                                      */
/* ------------------------------------------------------------------------ */

typedef struct {
    u64 *n;   /* pairs */
    u32 *u;
    size_t len, cap;
} misslist;

static void ml_push(misslist *m, u128 n, u32 u) {
    if (m->len == m->cap) {
        m->cap = m->cap ? 2 * m->cap : 64;
        m->n = realloc(m->n, 2 * m->cap * sizeof(u64));
        m->u = realloc(m->u, m->cap * sizeof(u32));
    }
    m->n[2 * m->len] = (u64)n;
    m->n[2 * m->len + 1] = (u64)(n >> 64);
    m->u[m->len] = u;
    m->len++;
}

#define DETAILED_LOOP(CALL)                                   \
    for (u128 n = s; n < e; n++) {                            \
        u32 u = CALL;                                         \
        hist[u]++;                                            \
        if (u > cutoff) ml_push(ml, n, u);                    \
    }

static void detailed_range(u128 s, u128 e, u32 base, u64 *hist, misslist *ml) {
    u32 cutoff = oracle_near_miss_cutoff(base);
    switch (base) {
    case 10: DETAILED_LOOP(nud_10(n)); break;
    case 40: DETAILED_LOOP(nud_40(n)); break;
    case 50: DETAILED_LOOP(nud_50(n)); break;
    case 80: DETAILED_LOOP(nud_80(n)); break;
    default: DETAILED_LOOP(nud_any(n, base)); break;
    }
}

static int emit_misses(const misslist *ml, u64 *miss_n, u32 *miss_u, size_t cap,
                       size_t *n_miss) {
    size_t c = ml->len < cap ? ml->len : cap;
    if (c) {
        memcpy(miss_n, ml->n, 2 * c * sizeof(u64));
        memcpy(miss_u, ml->u, c * sizeof(u32));
    }
    *n_miss = ml->len;
    return ml->len > cap ? 1 : 0;
}

int oracle_process_range_detailed(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base,
                                  u64 *hist, u64 *miss_n, u32 *miss_u, size_t cap,
                                  size_t *n_miss) {
    memset(hist, 0, (base + 1) * sizeof(u64));
    misslist ml = {0};
    detailed_range(mk(slo, shi), mk(elo, ehi), base, hist, &ml);
    int rc = emit_misses(&ml, miss_n, miss_u, cap, n_miss);
    free(ml.n); free(ml.u);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* client/src/main.rs:158-206: reference client chunking + rayon fan-out    */
/* ------------------------------------------------------------------------ */

static u128 client_chunk_size(u128 size) {
    const u128 def = 1000000, target = 100000;
    u128 mult = (size + def * target - 1) / (def * target);
    if (mult < 1) mult = 1;
    if (mult > 1000) mult = 1000;
    return def * mult;
}

typedef struct {
    u128 start, end, chunk;
    u64 nchunks;
    u32 base;
    int mode; /* 0 detailed, 1 niceonly */
    uint64_t floor_size;
    atomic_ullong next;
    /* per-chunk outputs */
    u64 **hists;
    misslist *lists;
    /* niceonly */
    u64 *stride_res; u64 stride_count; u64 stride_mod;
    u64 *cand_counts;
    u64 *range_counts;
    u64 *sq_counts; /* test statistic: candidates whose square has no repeat (or NULL) */
} job;

static uint64_t niceonly_range_impl(u128 s, u128 e, u32 base, const u64 *res, u64 R,
                                    u64 M, u64 floor_size, misslist *out, u64 *n_ranges,
                                    u64 *n_sq);

static void *worker(void *arg) {
    job *j = (job *)arg;
    for (;;) {
        u64 i = atomic_fetch_add(&j->next, 1);
        if (i >= j->nchunks) break;
        u128 s = j->start + (u128)i * j->chunk;
        u128 e = s + j->chunk < j->end ? s + j->chunk : j->end;
        if (j->mode == 0) {
            detailed_range(s, e, j->base, j->hists[i], &j->lists[i]);
        } else {
            j->cand_counts[i] = niceonly_range_impl(s, e, j->base, j->stride_res,
                                                    j->stride_count, j->stride_mod,
                                                    j->floor_size, &j->lists[i],
                                                    &j->range_counts[i],
                                                    j->sq_counts ? &j->sq_counts[i] : NULL);
        }
    }
    return NULL;
}

static void run_job(job *j, int threads) {
    if (threads < 1) threads = 1;
    pthread_t th[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, j);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

int oracle_process_field_detailed_mt(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base,
                                     int threads, u64 *hist, u64 *miss_n, u32 *miss_u,
                                     size_t cap, size_t *n_miss) {
    job j;
    memset(&j, 0, sizeof(j));
    j.start = mk(slo, shi); j.end = mk(elo, ehi); j.base = base; j.mode = 0;
    j.chunk = client_chunk_size(j.end - j.start);
    j.nchunks = (u64)((j.end - j.start + j.chunk - 1) / j.chunk);
    atomic_init(&j.next, 0);
    j.hists = calloc(j.nchunks, sizeof(u64 *));
    j.lists = calloc(j.nchunks, sizeof(misslist));
    for (u64 i = 0; i < j.nchunks; i++) j.hists[i] = calloc(base + 1, sizeof(u64));
    run_job(&j, threads);
    /* compile_results (main.rs:212-254): sum histograms; concat lists in chunk order */
    memset(hist, 0, (base + 1) * sizeof(u64));
    misslist all = {0};
    for (u64 i = 0; i < j.nchunks; i++) {
        for (u32 b = 0; b <= base; b++) hist[b] += j.hists[i][b];
        for (size_t q = 0; q < j.lists[i].len; q++)
            ml_push(&all, mk(j.lists[i].n[2 * q], j.lists[i].n[2 * q + 1]), j.lists[i].u[q]);
        free(j.hists[i]); free(j.lists[i].n); free(j.lists[i].u);
    }
    free(j.hists); free(j.lists);
    int rc = emit_misses(&all, miss_n, miss_u, cap, n_miss);
    free(all.n); free(all.u);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* residue_filter.rs:6-11, lsd_filter.rs:132-224, stride_filter.rs:40-155   */
/* ------------------------------------------------------------------------ */

u32 oracle_residue_filter(u32 base, u32 *out) {
    u32 m = base - 1;
    u32 target = base * (base - 1) / 2 % m;
    u32 c = 0;
    for (u32 r = 0; r < m; r++)
        if ((r * r + r * r * r) % m == target) out[c++] = r;
    return c;
}

/* lsd_filter.rs:132-148: digits of value, at most num_digits, stopping once
 * the remainder is zero.  Returns a bitmask (two words). */
static void extract_digit_set(u128 v, u32 base, u32 k, u64 m[2]) {
    m[0] = m[1] = 0;
    for (u32 i = 0; i < k; i++) {
        u32 d = (u32)(v % base);
        m[d >> 6] |= 1ull << (d & 63);
        v /= base;
        if (v == 0) break;
    }
}

int64_t oracle_lsd_bitmap(u32 base, u32 k, uint8_t *bitmap) {
    u64 mod = 1;
    for (u32 i = 0; i < k; i++) {
        mod *= base;
        if (mod > 0xffffffffull) return -1;
    }
    int64_t valid = 0;
    for (u64 s = 0; s < mod; s++) {
        u128 sq = ((u128)s * s) % mod;
        u128 cb = ((u128)s * s * s) % mod;
        u64 a[2], b[2];
        extract_digit_set(sq, base, k, a);
        extract_digit_set(cb, base, k, b);
        int ok = ((a[0] & b[0]) | (a[1] & b[1])) == 0;
        bitmap[s] = (uint8_t)ok;
        valid += ok;
    }
    return valid;
}

u64 oracle_stride_residues(u32 base, u32 k, u64 *modulus, u64 *residues, u64 cap) {
    u64 bk = 1;
    for (u32 i = 0; i < k; i++) bk *= base;
    u64 bm1 = base - 1;
    u64 M = bm1 * bk;
    *modulus = M;
    uint8_t *res_ok = calloc(bm1, 1);
    u32 rs[256];
    u32 nr = oracle_residue_filter(base, rs);
    for (u32 i = 0; i < nr; i++) res_ok[rs[i]] = 1;
    uint8_t *lsd = malloc(bk);
    oracle_lsd_bitmap(base, k, lsd);
    u64 c = 0;
    for (u64 r = 0; r < M; r++) {
        if (res_ok[r % bm1] && lsd[r % bk]) {
            if (c < cap) residues[c] = r;
            c++;
        }
    }
    free(res_ok);
    free(lsd);
    return c;
}

/* stride_filter.rs:99-124 */
static u128 first_valid_at_or_after(const u64 *res, u64 R, u64 M, u128 start, u64 *idx) {
    u64 r = (u64)(start % M);
    u64 lo = 0, hi = R; /* lower_bound */
    while (lo < hi) {
        u64 mid = (lo + hi) / 2;
        if (res[mid] < r) lo = mid + 1; else hi = mid;
    }
    u64 i = lo < R ? lo : 0;
    u64 tr = res[i];
    *idx = i;
    if (tr >= r) return start + (tr - r);
    return start + (M - r + tr);
}

/* ------------------------------------------------------------------------ */
/* msd_prefix_filter.rs:382-674                                             */
/* ------------------------------------------------------------------------ */

static int dup_digits(const u32 *d, int n) {
    u64 seen[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        u64 bit = 1ull << (d[i] & 63);
        if (seen[d[i] >> 6] & bit) return 1;
        seen[d[i] >> 6] |= bit;
    }
    return 0;
}
static int overlap_digits(const u32 *a, int na, const u32 *b, int nb) {
    u64 seen[4] = {0, 0, 0, 0};
    for (int i = 0; i < na; i++) seen[a[i] >> 6] |= 1ull << (a[i] & 63);
    for (int i = 0; i < nb; i++)
        if (seen[b[i] >> 6] & (1ull << (b[i] & 63))) return 1;
    return 0;
}
/* Common most-significant prefix length of two LSD-first digit arrays. */
static int common_msd_len(const u32 *a, int na, const u32 *b, int nb) {
    int m = na < nb ? na : nb, c = 0;
    for (int i = 0; i < m; i++) {
        if (a[na - 1 - i] == b[nb - 1 - i]) c++; else break;
    }
    return c;
}

#define MSD_LSD_K 2 /* MSD_LSD_OVERLAP_K_VALUE, msd_prefix_filter.rs:287 */

/* Study switch, not part of the restatement (scripts/filter_c_share.py):
 * 0 turns Filter C off.  Filter C judges a range by FIRST's two LSDs when
 * first / b^2 == last / b^2 -- a condition on the high digits, under which
 * n mod b^2 still varies across the range -- so it is sound only for ranges
 * of one number (which return before it); "off" is the sound filter. */
static int g_filter_c = 1;
void oracle_set_filter_c(int on) { g_filter_c = on; }

static int has_dup_msd_prefix(u128 s, u128 e, u32 base) {
    u128 first = s, last = e - 1;
    if (e - s == 1) return 0;
    big t, s_sq, e_sq, s_cu, e_cu;
    u32 dss[400], des[400], dsc[400], dec[400];
    big_set(&t, first); big_mul_u128(&t, first, &s_sq); big_mul_u128(&s_sq, first, &s_cu);
    big_set(&t, last); big_mul_u128(&t, last, &e_sq); big_mul_u128(&e_sq, last, &e_cu);
    int nss = big_digits_asc(s_sq, base, dss);
    int nes = big_digits_asc(e_sq, base, des);
    if (nss != nes) return 0;
    int cps = common_msd_len(dss, nss, des, nes);
    const u32 *sq_p = dss + (nss - cps);
    if (dup_digits(sq_p, cps)) return 1;
    int nsc = big_digits_asc(s_cu, base, dsc);
    int nec = big_digits_asc(e_cu, base, dec);
    if (nsc != nec) return 0;
    int cpc = common_msd_len(dsc, nsc, dec, nec);
    const u32 *cu_p = dsc + (nsc - cpc);
    if (dup_digits(cu_p, cpc)) return 1;
    if (overlap_digits(sq_p, cps, cu_p, cpc)) return 1;
    /* Filter C, msd_prefix_filter.rs:461-559 */
    u128 bk = 1;
    for (int i = 0; i < MSD_LSD_K; i++) bk *= base; /* saturating_pow cannot saturate here */
    if (g_filter_c && first / bk == last / bk) {
        int nls = nss < MSD_LSD_K ? nss : MSD_LSD_K;
        int nlc = nsc < MSD_LSD_K ? nsc : MSD_LSD_K;
        const u32 *lsd_sq = dss, *lsd_cu = dsc;
        if (overlap_digits(sq_p, cps, lsd_sq, nls) || overlap_digits(cu_p, cpc, lsd_cu, nlc) ||
            overlap_digits(sq_p, cps, lsd_cu, nlc) || overlap_digits(cu_p, cpc, lsd_sq, nls) ||
            dup_digits(lsd_sq, nls) || dup_digits(lsd_cu, nlc) ||
            overlap_digits(lsd_sq, nls, lsd_cu, nlc))
            return 1;
    }
    return 0;
}

int oracle_has_duplicate_msd_prefix(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base) {
    return has_dup_msd_prefix(mk(slo, shi), mk(elo, ehi), base);
}

typedef struct {
    u128 *s, *e;
    u64 len, cap;
} rangelist;

static void rl_push(rangelist *r, u128 s, u128 e) {
    if (r->len == r->cap) {
        r->cap = r->cap ? 2 * r->cap : 64;
        r->s = realloc(r->s, r->cap * sizeof(u128));
        r->e = realloc(r->e, r->cap * sizeof(u128));
    }
    r->s[r->len] = s; r->e[r->len] = e; r->len++;
}

/* msd_prefix_filter.rs:583-658 */
static void valid_ranges_rec(u128 s, u128 e, u32 base, u32 depth, u32 max_depth,
                             u128 min_size, u32 factor, rangelist *out) {
    if (depth >= max_depth) { rl_push(out, s, e); return; }
    if (e - s <= min_size) { rl_push(out, s, e); return; }
    if (has_dup_msd_prefix(s, e, base)) return;
    if (e - s < min_size * factor) { rl_push(out, s, e); return; }
    u128 cs = (e - s) / factor;
    for (u32 i = 0; i < factor; i++) {
        u128 ss = s + (u128)i * cs;
        u128 se = (i == factor - 1) ? e : ss + cs;
        if (ss < se) valid_ranges_rec(ss, se, base, depth + 1, max_depth, min_size, factor, out);
    }
}

u64 oracle_valid_ranges(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base, u64 floor_size,
                        u64 *out, u64 cap) {
    rangelist rl = {0};
    valid_ranges_rec(mk(slo, shi), mk(elo, ehi), base, 0, 22, floor_size, 2, &rl);
    for (u64 i = 0; i < rl.len && i < cap; i++) {
        out[4 * i] = (u64)rl.s[i]; out[4 * i + 1] = (u64)(rl.s[i] >> 64);
        out[4 * i + 2] = (u64)rl.e[i]; out[4 * i + 3] = (u64)(rl.e[i] >> 64);
    }
    u64 n = rl.len;
    free(rl.s); free(rl.e);
    return n;
}

/* client_process.rs:439-465 + stride_filter.rs:139-155 */
static uint64_t niceonly_range_impl(u128 s, u128 e, u32 base, const u64 *res, u64 R,
                                    u64 M, u64 floor_size, misslist *out, u64 *n_ranges,
                                    u64 *n_sq) {
    if (n_ranges) *n_ranges = 0;
    if (n_sq) *n_sq = 0;
    if (R == 0) return 0;
    rangelist rl = {0};
    valid_ranges_rec(s, e, base, 0, 22, floor_size, 2, &rl);
    if (n_ranges) *n_ranges = rl.len;
    uint64_t cands = 0;
    for (u64 q = 0; q < rl.len; q++) {
        u64 idx;
        u128 n = first_valid_at_or_after(res, R, M, rl.s[q], &idx);
        while (n < rl.e[q]) {
            cands++;
            int nice;
            if (n_sq) {
                int sq_ok = 0;
                nice = is_nice_impl2(n, base, &sq_ok);
                *n_sq += (u64)sq_ok;
            } else {
                nice = is_nice(n, base);
            }
            if (nice) ml_push(out, n, base);
            n += (idx + 1 < R) ? res[idx + 1] - res[idx] : M - res[idx] + res[0];
            idx = (idx + 1) % R;
        }
    }
    free(rl.s); free(rl.e);
    return cands;
}

static u64 *stride_table_alloc(u32 base, u32 k, u64 *R, u64 *M) {
    u64 n = oracle_stride_residues(base, k, M, NULL, 0);
    u64 *res = malloc((n ? n : 1) * sizeof(u64));
    oracle_stride_residues(base, k, M, res, n);
    *R = n;
    return res;
}

static u64 emit_nice(const misslist *ml, u64 *out, u64 cap) {
    for (u64 i = 0; i < ml->len && i < cap; i++) {
        out[2 * i] = ml->n[2 * i];
        out[2 * i + 1] = ml->n[2 * i + 1];
    }
    return ml->len;
}

u64 oracle_process_range_niceonly(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base, u32 k,
                                  u64 floor_size, u64 *out, u64 cap, u64 *n_candidates) {
    u64 R, M;
    u64 *res = stride_table_alloc(base, k, &R, &M);
    misslist ml = {0};
    u64 c = niceonly_range_impl(mk(slo, shi), mk(elo, ehi), base, res, R, M, floor_size, &ml,
                                NULL, NULL);
    if (n_candidates) *n_candidates = c;
    u64 n = emit_nice(&ml, out, cap);
    free(ml.n); free(ml.u); free(res);
    return n;
}

/* client/src/main.rs:120-254 (niceonly) with an explicit MSD chunk size
 * (0 -> the client rule) and floor (0 -> 250): a window of a larger field is
 * processed on that field's chunk grid when it starts on a grid point.
 * *n_ranges receives the number of MSD-surviving ranges (get_valid_ranges
 * output length summed over chunks, msd_prefix_filter.rs:665-674). */
u64 oracle_process_field_niceonly_sq(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base,
                                     int threads, u64 chunk, u64 floor_size, u64 *out,
                                     u64 cap, u64 *n_candidates, u64 *n_ranges, u64 *n_sq);

u64 oracle_process_field_niceonly_ex(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base,
                                     int threads, u64 chunk, u64 floor_size, u64 *out,
                                     u64 cap, u64 *n_candidates, u64 *n_ranges) {
    return oracle_process_field_niceonly_sq(slo, shi, elo, ehi, base, threads, chunk, floor_size,
                                            out, cap, n_candidates, n_ranges, NULL);
}

/* _ex plus the test statistic *n_sq: stride candidates whose square alone has
 * no repeated digit (get_is_nice reached the cube scan).  The GPU's in-range
 * test counts the same set (its square-survivor queue), which pins the
 * candidate enumeration and the digit test even where no number is nice. */
u64 oracle_process_field_niceonly_sq(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base,
                                     int threads, u64 chunk, u64 floor_size, u64 *out,
                                     u64 cap, u64 *n_candidates, u64 *n_ranges, u64 *n_sq) {
    job j;
    memset(&j, 0, sizeof(j));
    j.start = mk(slo, shi); j.end = mk(elo, ehi); j.base = base; j.mode = 1;
    j.floor_size = floor_size ? floor_size : 250; /* MSD_RECURSIVE_MIN_RANGE_SIZE, msd_prefix_filter.rs:282 */
    j.chunk = chunk ? (u128)chunk : client_chunk_size(j.end - j.start);
    j.nchunks = (u64)((j.end - j.start + j.chunk - 1) / j.chunk);
    atomic_init(&j.next, 0);
    j.stride_res = stride_table_alloc(base, 2, &j.stride_count, &j.stride_mod);
    j.lists = calloc(j.nchunks, sizeof(misslist));
    j.cand_counts = calloc(j.nchunks, sizeof(u64));
    j.range_counts = calloc(j.nchunks, sizeof(u64));
    j.sq_counts = n_sq ? calloc(j.nchunks, sizeof(u64)) : NULL;
    run_job(&j, threads);
    misslist all = {0};
    u64 cands = 0, ranges = 0, sqs = 0;
    for (u64 i = 0; i < j.nchunks; i++) {
        for (size_t q = 0; q < j.lists[i].len; q++)
            ml_push(&all, mk(j.lists[i].n[2 * q], j.lists[i].n[2 * q + 1]), base);
        cands += j.cand_counts[i];
        ranges += j.range_counts[i];
        if (j.sq_counts) sqs += j.sq_counts[i];
        free(j.lists[i].n); free(j.lists[i].u);
    }
    if (n_candidates) *n_candidates = cands;
    if (n_ranges) *n_ranges = ranges;
    if (n_sq) *n_sq = sqs;
    u64 n = emit_nice(&all, out, cap);
    free(all.n); free(all.u); free(j.lists); free(j.cand_counts); free(j.range_counts);
    free(j.sq_counts);
    free(j.stride_res);
    return n;
}

u64 oracle_process_field_niceonly_mt(u64 slo, u64 shi, u64 elo, u64 ehi, u32 base,
                                     int threads, u64 *out, u64 cap, u64 *n_candidates) {
    return oracle_process_field_niceonly_ex(slo, shi, elo, ehi, base, threads, 0, 0, out, cap,
                                            n_candidates, NULL);
}
