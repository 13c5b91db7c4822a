/*
 * oracle/fec_oracle.c -- TEST INFRASTRUCTURE ONLY.  See fec_oracle.h.
 *
 * Clean-room restatement of p-quic/pquic plugins/fec scheme arithmetic, written from
 * the reference's behaviour (file:line cited per function), not copied from it.
 */
#define _GNU_SOURCE
#include "fec_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------------------------
 * GF(2^8) with reduction polynomial x^8+x^4+x^3+x^2+1 (0x11D).
 * gf256/swif_symbol.c:16-29: shift-and-add multiply; the carry out of bit 7 is
 * folded back with ^0x1d.  generated_table_code.c:4-10 fills the full 256x256 table
 * from that formula; :12-14 assigns a literal inverse table with inv[0] = 0.  Here
 * the inverse is derived from the product table (pinned against the reference's
 * literal table by tests/golden/gf256_tables.json).
 * ---------------------------------------------------------------------------------- */
static uint8_t g_mul[256][256];
static uint8_t g_inv[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static uint8_t gf_mul_formula(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        b >>= 1;
        uint8_t carry = a & 0x80;
        a = (uint8_t)(a << 1);
        if (carry) a ^= 0x1d;
    }
    return p;
}

static void gf_init(void) {
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++) g_mul[a][b] = gf_mul_formula((uint8_t)a, (uint8_t)b);
    g_inv[0] = 0;
    for (int a = 1; a < 256; a++)
        for (int b = 1; b < 256; b++)
            if (g_mul[a][b] == 1) { g_inv[a] = (uint8_t)b; break; }
}

static inline void gf_ready(void) { pthread_once(&g_once, gf_init); }

void oracle_gf_tables(uint8_t *mul, uint8_t *inv) {
    gf_ready();
    if (mul) memcpy(mul, g_mul, sizeof g_mul);
    if (inv) memcpy(inv, g_inv, sizeof g_inv);
}

uint8_t oracle_gf_mul(uint8_t a, uint8_t b) { gf_ready(); return g_mul[a][b]; }

/* symbol_add_scaled / symbol_sub_scaled (swif_symbol.c:39-47, swif_symbol.h:40):
 * dst[i] ^= coef * src[i] for i < n. */
static inline void sym_add_scaled(uint8_t *dst, uint8_t coef, const uint8_t *src, size_t n) {
    const uint8_t *row = g_mul[coef];
    for (size_t i = 0; i < n; i++) dst[i] ^= row[src[i]];
}

/* symbol_mul (swif_symbol.c:63-69) */
static inline void sym_mul(uint8_t *dst, uint8_t coef, size_t n) {
    const uint8_t *row = g_mul[coef];
    for (size_t i = 0; i < n; i++) dst[i] = row[dst[i]];
}

/* symbol_is_zero (swif_symbol.c:49-59) */
static inline int sym_is_zero(const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) if (p[i]) return 0;
    return 1;
}

/* ------------------------------------------------------------------------------------
 * TinyMT32, the 127-bit generator vendored at prng/tinymt32.c.  Parameters are the
 * ones both RLC pluglets set before init: mat1 0x8f7011ee, mat2 0xfc78ff1f,
 * tmat 0x3793fdff (rlc_fec_scheme_generate_gf256.c:27-29, rlc_fec_scheme_gf256.c:146-148).
 * ---------------------------------------------------------------------------------- */
#define TMT_MAT1 0x8f7011eeu
#define TMT_MAT2 0xfc78ff1fu
#define TMT_TMAT 0x3793fdffu

typedef struct { uint32_t s0, s1, s2, s3; } tmt_t;

/* tinymt32_next_state (tinymt32.c:60-76): SH0 = 1, SH1 = 10, MASK = 0x7fffffff */
static inline void tmt_next(tmt_t *t) {
    uint32_t y = t->s3;
    uint32_t x = (t->s0 & 0x7fffffffu) ^ t->s1 ^ t->s2;
    x ^= x << 1;
    y ^= (y >> 1) ^ x;
    t->s0 = t->s1;
    t->s1 = t->s2;
    t->s2 = x ^ (y << 10);
    t->s3 = y;
    uint32_t m = (uint32_t)(-(int32_t)(y & 1u));
    t->s1 ^= m & TMT_MAT1;
    t->s2 ^= m & TMT_MAT2;
}

/* tinymt32_temper (tinymt32.c:84-97), additive form (LINEARITY_CHECK unset) */
static inline uint32_t tmt_temper(const tmt_t *t) {
    uint32_t t1 = t->s0 + (t->s2 >> 8);
    uint32_t t0 = t->s3 ^ t1;
    t0 ^= (uint32_t)(-(int32_t)(t1 & 1u)) & TMT_TMAT;
    return t0;
}

/* tinymt32_init (tinymt32.c:301-315): 7 mixing rounds, period certification,
 * 8 state advances. */
static inline void tmt_init(tmt_t *t, uint32_t seed) {
    uint32_t st[4] = {seed, TMT_MAT1, TMT_MAT2, TMT_TMAT};
    for (uint32_t i = 1; i < 8; i++) {
        uint32_t p = st[(i - 1) & 3];
        st[i & 3] ^= i + 1812433253u * (p ^ (p >> 30));
    }
    if ((st[0] & 0x7fffffffu) == 0 && st[1] == 0 && st[2] == 0 && st[3] == 0) {
        st[0] = 'T'; st[1] = 'I'; st[2] = 'N'; st[3] = 'Y';
    }
    t->s0 = st[0]; t->s1 = st[1]; t->s2 = st[2]; t->s3 = st[3];
    for (int i = 0; i < 8; i++) tmt_next(t);
}

uint32_t oracle_tinymt32_first(uint32_t seed) {
    tmt_t t; tmt_init(&t, seed); tmt_next(&t); return tmt_temper(&t);
}

void oracle_tinymt32_stream(uint32_t seed, int n, uint32_t *out) {
    tmt_t t; tmt_init(&t, seed);
    for (int i = 0; i < n; i++) { tmt_next(&t); out[i] = tmt_temper(&t); }
}

/* get_coefs (rlc_fec_scheme_generate_gf256.c:9-17 == rlc_fec_scheme_gf256.c:117-125):
 * low byte of each draw, 0 replaced by 1. */
void oracle_rlc_coefs(uint32_t seed, int n, uint8_t *coefs) {
    tmt_t t; tmt_init(&t, seed);
    for (int i = 0; i < n; i++) {
        tmt_next(&t);
        uint8_t c = (uint8_t)tmt_temper(&t);
        coefs[i] = c ? c : 1;
    }
}

/* Seed = repair_fpid.source_fpid.raw: packed {u8 symbol_number; u24 fec_block_number}
 * little-endian (fec.h:44-50,63-75; rlc_fec_scheme_generate_gf256.c:308-312). */
uint32_t oracle_rlc_seed(uint32_t fbn, uint32_t repair_index) {
    return ((fbn & 0xffffffu) << 8) | (repair_index & 0xffu);
}

/* ------------------------------------------------------------------------------------
 * RLC encode, fec_generate_repair_symbols (rlc_fec_scheme_generate_gf256.c:24-77).
 * Precondition r > 0 && k >= 1 (current == total is implied by src[] non-NULL) else 1.
 * Sources are zero-padded to max_length = max(data_length) (:41-45, :51-55); each
 * repair has data_length max_length and data sum_j coef_i[j] * S_j.
 * ---------------------------------------------------------------------------------- */
int oracle_rlc_encode_block(uint32_t fbn, int k, int r, const uint8_t *const *src,
                            const uint16_t *src_len, uint8_t *const *rep, uint16_t *rep_len) {
    gf_ready();
    if (r == 0 || k < 1) return 1;
    for (int j = 0; j < k; j++) if (!src[j]) return 1;
    uint16_t max_len = 0;
    for (int j = 0; j < k; j++) if (src_len[j] > max_len) max_len = src_len[j];
    uint8_t coefs[256];
    for (int i = 0; i < r; i++) {
        oracle_rlc_coefs(oracle_rlc_seed(fbn, (uint32_t)i), k, coefs);
        memset(rep[i], 0, max_len);
        for (int j = 0; j < k; j++) sym_add_scaled(rep[i], coefs[j], src[j], src_len[j]);
        rep_len[i] = max_len;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------
 * XOR encode (xor_fec_scheme_generate.c:41-78): needs r == 1, k >= 1; the repair is
 * the XOR of the zero-extended sources, length max(data_length).
 * ---------------------------------------------------------------------------------- */
int oracle_xor_encode_block(int k, int r, const uint8_t *const *src, const uint16_t *src_len,
                            uint8_t *rep, uint16_t *rep_len) {
    if (r != 1 || k < 1) return 1;
    for (int j = 0; j < k; j++) if (!src[j]) return 1;
    uint16_t max_len = 0;
    for (int j = 0; j < k; j++) if (src_len[j] > max_len) max_len = src_len[j];
    memset(rep, 0, max_len);
    for (int j = 0; j < k; j++)
        for (uint16_t t = 0; t < src_len[j]; t++) rep[t] ^= src[j][t];
    *rep_len = max_len;
    return 0;
}

/* ------------------------------------------------------------------------------------
 * XOR recover (xor_fec_scheme.c:41-74).  Proceeds only when total_repair_symbols == 1
 * and current_ss + current_rs == total_ss (:45-49, else returns 1).  The missing index
 * is the LAST NULL source (:54-58); its data starts as the repair (length = repair
 * length) and is XORed with every present source over min(lengths) (:12-33, :65-70).
 * A proceeding call with the repair absent would dereference NULL: REF_UB.
 * ---------------------------------------------------------------------------------- */
int oracle_xor_decode_block(int k, int r, const uint8_t *const *src, const uint16_t *src_len,
                            const uint8_t *const *rep, const uint16_t *rep_len,
                            uint8_t *out, uint16_t *out_len, int *recovered_index) {
    *recovered_index = -1;
    int cur_ss = 0, cur_rs = 0;
    for (int j = 0; j < k; j++) cur_ss += src[j] != NULL;
    for (int i = 0; i < r; i++) cur_rs += rep[i] != NULL;
    if (r != 1 || cur_ss + cur_rs != k) return ORACLE_DEC_NOTHING;
    if (!rep[0]) return ORACLE_DEC_REF_UB;
    int missing = 0;
    for (int j = 0; j < k; j++) if (!src[j]) missing = j;
    uint16_t len = rep_len[0];
    memcpy(out, rep[0], len);
    for (int j = 0; j < k; j++) {
        if (!src[j]) continue;
        uint16_t n = src_len[j] < len ? src_len[j] : len;
        for (uint16_t t = 0; t < n; t++) out[t] ^= src[j][t];
    }
    *out_len = len;
    *recovered_index = missing;
    return ORACLE_DEC_RECOVERED;
}

/* ------------------------------------------------------------------------------------
 * RLC recover, fec_recover (rlc_fec_scheme_gf256.c:134-251) with gaussElimination
 * (:51-115), sort_system (:28-40) and cmp_eq (:20-25).
 * ---------------------------------------------------------------------------------- */
#define MAXK 256

int oracle_rlc_decode_block(uint32_t fbn, int k, int r, const uint8_t *const *src,
                            const uint16_t *src_len, const uint8_t *const *rep,
                            const uint16_t *rep_len, const uint32_t *rep_seed,
                            uint8_t *const *out, uint16_t *out_len, uint8_t *recovered) {
    gf_ready();
    for (int j = 0; j < k; j++) recovered[j] = 0;
    int cur_ss = 0, cur_rs = 0;
    for (int j = 0; j < k; j++) cur_ss += src[j] != NULL;
    for (int i = 0; i < r; i++) cur_rs += rep[i] != NULL;
    /* :140-144 */
    if (r == 0 || cur_ss == k || cur_ss + cur_rs < k) return ORACLE_DEC_NOTHING;

    int n_unk = k - cur_ss;
    int n_eq = n_unk < cur_rs ? n_unk : cur_rs;              /* :151-152 */
    int first = 0;
    while (!rep[first]) first++;                               /* :174-184 */
    size_t L = rep_len[first];                                 /* :186 */

    uint8_t *x = calloc((size_t)n_unk, L ? L : 1);             /* unknowns, zeroed :188-191 */
    uint8_t *ct = calloc((size_t)n_eq, L ? L : 1);             /* constant terms */
    uint8_t A[MAXK][MAXK];
    int ctrow[MAXK], arow[MAXK];                               /* row permutation (swap) */
    uint8_t undet[MAXK];
    memset(undet, 0, sizeof undet);
    int ret = ORACLE_DEC_RECOVERED;

    /* build the system, :194-212: first n_eq present repairs in index order */
    uint8_t coefs[MAXK];
    int e = 0;
    for (int i = 0; i < r && e < n_eq; i++) {
        if (!rep[i]) continue;
        /* bytes past max_length land in the allocator slot's slack and are never read
         * again (memory.c:181-191 hands out 2100-B slots): truncation semantics */
        memcpy(ct + (size_t)e * L, rep[i], rep_len[i] < L ? rep_len[i] : L);
        uint32_t seed = rep_seed ? rep_seed[i] : oracle_rlc_seed(fbn, (uint32_t)i);
        oracle_rlc_coefs(seed, k, coefs);
        int u = 0;
        for (int j = 0; j < k; j++) {
            if (src[j]) {
                sym_add_scaled(ct + (size_t)e * L, coefs[j], src[j], src_len[j] < L ? src_len[j] : L);
            } else if (u < n_unk) {
                A[e][u++] = coefs[j];
            }
        }
        e++;
    }
    for (int i = 0; i < n_eq; i++) { arow[i] = i; ctrow[i] = i; }

    /* sort_system :28-40 -- selection sort, row i takes the (first) row with the
     * largest value in column i among rows i..n_eq-1. Rows are swapped by pointer. */
#define AR(i) A[arow[i]]
    for (int i = 0; i < n_eq; i++) {
        int mx = i;
        for (int j = i + 1; j < n_eq; j++)
            if (AR(mx)[i] < AR(j)[i]) mx = j;
        int t = arow[i]; arow[i] = arow[mx]; arow[mx] = t;
        t = ctrow[i]; ctrow[i] = ctrow[mx]; ctrow[mx] = t;
    }
#define CT(i) (ct + (size_t)ctrow[i] * L)
    /* forward elimination, no re-pivoting :54-70 (inv[0] == 0 makes term 0) */
    for (int i = 0; i < n_eq - 1; i++) {
        for (int kk = i + 1; kk < n_eq; kk++) {
            uint8_t term = g_mul[AR(kk)[i]][g_inv[AR(i)[i]]];
            for (int j = 0; j < n_unk; j++) AR(kk)[j] ^= g_mul[term][AR(i)[j]];
            sym_add_scaled(CT(kk), term, CT(i), L);
        }
    }
    /* back substitution :71-114 */
    int cand = n_unk - 1;
    for (int i = n_eq - 1; i >= 0; i--) {
        while (cand >= 0 && AR(i)[cand] == 0) undet[cand--] = 1;
        if (cand < 0) { ret = ORACLE_DEC_REF_UB; goto done; }   /* my_memcpy(x[-1], ...) */
        uint8_t *xc = x + (size_t)cand * L;
        memcpy(xc, CT(i), L);
        for (int j = 0; j < cand; j++)
            if (AR(i)[j] != 0) { undet[cand] = 1; break; }
        for (int j = cand + 1; j < n_unk; j++) {
            if (AR(i)[j] != 0) {
                if (undet[j]) undet[cand] = 1;
                else { sym_add_scaled(xc, AR(i)[j], x + (size_t)j * L, L); AR(i)[j] = 0; }
            }
        }
        if (sym_is_zero(xc, L) || AR(i)[cand] == 0) {
            undet[cand] = 1;
        } else if (!undet[cand]) {
            uint8_t iv = g_inv[AR(i)[cand]];
            sym_mul(xc, iv, L);
            AR(i)[cand] = g_mul[AR(i)[cand]][iv];
        }
        cand--;
    }
    if (cand >= 0) memset(undet, 1, (size_t)cand + 1);

    /* insert recovered symbols :218-236 */
    {
        int u = 0;
        for (int j = 0; j < k; j++) {
            if (src[j]) continue;
            const uint8_t *xu = x + (size_t)u * L;
            if (!undet[u] && !sym_is_zero(xu, L)) {
                memcpy(out[j], xu, L);
                out_len[j] = (uint16_t)L;
                recovered[j] = 1;
            }
            u++;
        }
    }
#undef AR
#undef CT
done:
    free(x);
    free(ct);
    if (ret == ORACLE_DEC_REF_UB) for (int j = 0; j < k; j++) recovered[j] = 0;
    return ret;
}

/* ------------------------------------------------------------------------------------
 * Batched drivers over the fixed layout; pthreads over disjoint block ranges.
 * ---------------------------------------------------------------------------------- */
int oracle_cpu_count(void) {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) return CPU_COUNT(&set);
    long n = sysconf(_SC_NPROCESSORS_ONLN);
    return n > 0 ? (int)n : 1;
}

typedef struct {
    int op;
    uint8_t *src; const uint8_t *csrc; uint8_t *rep; const uint8_t *crep;
    uint64_t b0, b1;
    int k, r, L;
    uint32_t fbn_base;
    const uint64_t *sp, *rp;
    uint8_t *status; uint64_t *recovered;
} job_t;

static void run_range(job_t *jb) {
    const uint8_t *sp[MAXK]; uint16_t sl[MAXK];
    const uint8_t *rpp[MAXK]; uint16_t rl[MAXK];
    uint8_t *outp[MAXK]; uint16_t ol[MAXK]; uint8_t recd[MAXK];
    uint8_t *rep_out[MAXK];
    size_t L = (size_t)jb->L;
    for (uint64_t b = jb->b0; b < jb->b1; b++) {
        uint32_t fbn = (uint32_t)((jb->fbn_base + b) & 0xffffffu);
        const uint8_t *sb = (jb->op == 0 || jb->op == 2) ? jb->csrc + b * jb->k * L : jb->src + b * jb->k * L;
        for (int j = 0; j < jb->k; j++) { sp[j] = sb + j * L; sl[j] = (uint16_t)L; }
        if (jb->op == 0) {               /* rlc encode */
            for (int i = 0; i < jb->r; i++) rep_out[i] = jb->rep + (b * jb->r + i) * L;
            oracle_rlc_encode_block(fbn, jb->k, jb->r, sp, sl, rep_out, rl);
        } else if (jb->op == 2) {        /* xor encode */
            oracle_xor_encode_block(jb->k, 1, sp, sl, jb->rep + b * L, rl);
        } else {                         /* decode */
            for (int j = 0; j < jb->k; j++) {
                if (!((jb->sp[b * 2 + (j >> 6)] >> (j & 63)) & 1)) sp[j] = NULL;
                outp[j] = jb->src + (b * jb->k + j) * L;
            }
            for (int i = 0; i < jb->r; i++) {
                rpp[i] = ((jb->rp[b * 2 + (i >> 6)] >> (i & 63)) & 1) ? jb->crep + (b * jb->r + i) * L : NULL;
                rl[i] = (uint16_t)L;
            }
            uint64_t m[2] = {0, 0};
            int st;
            if (jb->op == 1) {
                st = oracle_rlc_decode_block(fbn, jb->k, jb->r, sp, sl, rpp, rl, NULL, outp, ol, recd);
                for (int j = 0; j < jb->k; j++) if (recd[j]) m[j >> 6] |= 1ull << (j & 63);
            } else {
                int idx;
                uint8_t tmp[65536];
                st = oracle_xor_decode_block(jb->k, jb->r, sp, sl, rpp, rl, tmp, ol, &idx);
                if (st == ORACLE_DEC_RECOVERED) {
                    memcpy(jb->src + (b * jb->k + idx) * L, tmp, L);
                    m[idx >> 6] |= 1ull << (idx & 63);
                }
            }
            jb->status[b] = (uint8_t)st;
            jb->recovered[b * 2] = m[0];
            jb->recovered[b * 2 + 1] = m[1];
        }
    }
}

static void *thread_main(void *p) { run_range((job_t *)p); return NULL; }

static int run_batch(job_t proto, uint64_t nblocks, int nthreads) {
    gf_ready();
    if (proto.k < 1 || proto.k > 255 || proto.r < 0 || proto.r > 255 || proto.L < 0 || proto.L > 65535) return -1;
    if (nthreads <= 0) nthreads = oracle_cpu_count();
    if ((uint64_t)nthreads > nblocks) nthreads = nblocks ? (int)nblocks : 1;
    pthread_t th[512];
    job_t jobs[512];
    if (nthreads > 512) nthreads = 512;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].b0 = nblocks * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].b1 = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, thread_main, &jobs[t]);
    run_range(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    return nthreads;
}

int oracle_rlc_encode_batch(const uint8_t *src, uint8_t *rep, uint64_t nblocks, int k, int r,
                            int L, uint32_t fbn_base, int nthreads) {
    job_t j = {0};
    j.op = 0; j.csrc = src; j.rep = rep; j.k = k; j.r = r; j.L = L; j.fbn_base = fbn_base;
    return run_batch(j, nblocks, nthreads);
}

int oracle_rlc_decode_batch(uint8_t *src, const uint8_t *rep, uint64_t nblocks, int k, int r,
                            int L, uint32_t fbn_base, const uint64_t *src_present,
                            const uint64_t *rep_present, uint8_t *status, uint64_t *recovered,
                            int nthreads) {
    job_t j = {0};
    j.op = 1; j.src = src; j.crep = rep; j.k = k; j.r = r; j.L = L; j.fbn_base = fbn_base;
    j.sp = src_present; j.rp = rep_present; j.status = status; j.recovered = recovered;
    return run_batch(j, nblocks, nthreads);
}

int oracle_xor_encode_batch(const uint8_t *src, uint8_t *rep, uint64_t nblocks, int k, int L,
                            int nthreads) {
    job_t j = {0};
    j.op = 2; j.csrc = src; j.rep = rep; j.k = k; j.r = 1; j.L = L;
    return run_batch(j, nblocks, nthreads);
}

int oracle_xor_decode_batch(uint8_t *src, const uint8_t *rep, uint64_t nblocks, int k, int L,
                            const uint64_t *src_present, const uint64_t *rep_present,
                            uint8_t *status, uint64_t *recovered, int nthreads) {
    job_t j = {0};
    j.op = 3; j.src = src; j.crep = rep; j.k = k; j.r = 1; j.L = L;
    j.sp = src_present; j.rp = rep_present; j.status = status; j.recovered = recovered;
    return run_batch(j, nblocks, nthreads);
}

/* ------------------------------------------------------------------------------------
 * Synthetic payload: counter-based SplitMix64, little-endian words.
 * ---------------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

void oracle_synth_fill(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t offset) {
    for (uint64_t i = 0; i < nbytes; i++) {
        uint64_t o = offset + i;
        uint64_t w = mix64(seed + ((o >> 3) + 1) * 0x9e3779b97f4a7c15ull);
        dst[i] = (uint8_t)(w >> (8 * (o & 7)));
    }
}
