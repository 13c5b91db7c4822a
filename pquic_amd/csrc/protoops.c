/*
 * pquic_amd/csrc/protoops.c -- PQUIC protocol operations for the FEC scheme hooks
 * (include/pquic_fec_protoops.h), host side in C like the reference pluglets.
 *
 * Each operation reads the fec_block_t the framework passes in, stages its symbols into a
 * zero-padded fixed-size row layout, runs the device engine through the host-resident
 * entry points of include/fecgpu.h (one block per call, synchronous like the reference),
 * and writes results back into the block with the caller's allocator.  The arithmetic
 * itself never runs on the CPU: if no gfx950 device is usable the operation fails with an
 * error code instead of computing.
 */
#include "pquic_fec_protoops.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "fecgpu.h"

_Static_assert(sizeof(pquic_source_fpid_t) == 4, "source_fpid_t is 4 bytes (fec.h:44-50)");
_Static_assert(sizeof(pquic_repair_fpid_t) == 8, "repair_fpid_t is 8 bytes (fec.h:63-75)");
_Static_assert(sizeof(pquic_source_symbol_t) == 16, "source_symbol_t layout (fec.h:104-114)");
_Static_assert(sizeof(pquic_repair_symbol_t) == 24, "repair_symbol_t layout (fec.h:91-102)");
_Static_assert(sizeof(pquic_fec_block_t) == 1608, "fec_block_t layout (fec.h:121-130)");

#define RLC_MAGIC 0x524c4347u /* "RLCG" */

struct pquic_fec_scheme {
    uint32_t magic;
    uint32_t device;
};

static pquic_fec_host_api_t g_api;
static int g_bound;
static int g_device;
static fecgpu_host_ctx_t *g_ctx;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pquic_fec_protoop_stats_t g_stats;

/* per-call staging (host), grown on demand */
static uint8_t *g_src, *g_rep;
static size_t g_src_cap, g_rep_cap;

int pquic_fec_bind_host(const pquic_fec_host_api_t *api, int device) {
    pthread_mutex_lock(&g_mu);
    if (api) {
        g_api = *api;
        g_bound = api->get_cnx && api->set_cnx && api->my_malloc && api->my_free;
    } else {
        g_bound = 0;
    }
    if (g_ctx && g_device != device) {
        fecgpu_host_ctx_destroy(g_ctx);
        g_ctx = NULL;
    }
    g_device = device;
    pthread_mutex_unlock(&g_mu);
    return g_bound ? 0 : -1;
}

void pquic_fec_protoop_stats(pquic_fec_protoop_stats_t *out) { *out = g_stats; }

int pquic_fec_layout(uint64_t out[8]) {
    out[0] = sizeof(pquic_fec_block_t);
    out[1] = sizeof(pquic_source_symbol_t);
    out[2] = sizeof(pquic_repair_symbol_t);
    out[3] = offsetof(pquic_fec_block_t, source_symbols);
    out[4] = offsetof(pquic_fec_block_t, repair_symbols);
    out[5] = offsetof(pquic_source_symbol_t, data);
    out[6] = offsetof(pquic_repair_symbol_t, data);
    out[7] = sizeof(pquic_repair_fpid_t);
    return 8;
}

static fecgpu_host_ctx_t *ctx(void) {
    if (!g_ctx) g_ctx = fecgpu_host_ctx_create(g_device, 1, 1u << 20);
    return g_ctx;
}

static int stage(size_t src_bytes, size_t rep_bytes) {
    if (src_bytes > g_src_cap) {
        uint8_t *p = realloc(g_src, src_bytes);
        if (!p) return -1;
        g_src = p;
        g_src_cap = src_bytes;
    }
    if (rep_bytes > g_rep_cap) {
        uint8_t *p = realloc(g_rep, rep_bytes);
        if (!p) return -1;
        g_rep = p;
        g_rep_cap = rep_bytes;
    }
    return 0;
}

static uint32_t pad4(uint32_t x) { return (x + 3u) & ~3u; }

/* malloc_repair_symbol (plugins/fec/fec.h:231-244): zeroed struct, fpid, zeroed data */
static pquic_repair_symbol_t *new_repair(picoquic_cnx_t *cnx, uint64_t fpid_raw, uint16_t len) {
    pquic_repair_symbol_t *s = g_api.my_malloc(cnx, sizeof *s);
    uint8_t *d = g_api.my_malloc(cnx, len);
    if (!s || !d) {
        if (s) g_api.my_free(cnx, s);
        if (d) g_api.my_free(cnx, d);
        return NULL;
    }
    memset(s, 0, sizeof *s);
    s->fpid.raw = fpid_raw;
    s->data = d;
    s->data_length = len;
    return s;
}

/* malloc_source_symbol (plugins/fec/fec.h:201-213) */
static pquic_source_symbol_t *new_source(picoquic_cnx_t *cnx, uint32_t fpid_raw, uint16_t len) {
    pquic_source_symbol_t *s = g_api.my_malloc(cnx, sizeof *s);
    uint8_t *d = g_api.my_malloc(cnx, len);
    if (!s || !d) {
        if (s) g_api.my_free(cnx, s);
        if (d) g_api.my_free(cnx, d);
        return NULL;
    }
    memset(s, 0, sizeof *s);
    s->fpid.raw = fpid_raw;
    s->data = d;
    s->data_length = len;
    return s;
}

/* ------------------------------------------------------------------ create_fec_schemes */

/* create_rlc_fec_scheme_gf256.c:46-59: outputs [0] receiver scheme, [1] sender scheme
 * (the same object); returns 0 or PICOQUIC_ERROR_MEMORY.  The 64 KiB multiplication and
 * inverse tables of the reference are not needed: the device derives products from
 * GF(2^8) bit planes. */
protoop_arg_t pquic_fec_rlc_create_fec_schemes(picoquic_cnx_t *cnx) {
    if (!g_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_scheme_t *fs = g_api.my_malloc(cnx, sizeof *fs);
    if (!fs) return PQUIC_ERROR_MEMORY;
    fs->magic = RLC_MAGIC;
    fs->device = (uint32_t)g_device;
    g_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 0, (protoop_arg_t)(uintptr_t)fs);
    g_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 1, (protoop_arg_t)(uintptr_t)fs);
    return 0;
}

/* create_xor_fec_scheme.c:4-9: both outputs NULL */
protoop_arg_t pquic_fec_xor_create_fec_schemes(picoquic_cnx_t *cnx) {
    if (!g_bound) return PQUIC_FEC_ERR_UNBOUND;
    g_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 0, 0);
    g_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 1, 0);
    return 0;
}

/* ------------------------------------------------------------------ generate */

static protoop_arg_t generate(picoquic_cnx_t *cnx, int xor_scheme) {
    if (!g_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_block_t *fb = (pquic_fec_block_t *)(uintptr_t)g_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 0);
    const int k = fb->total_source_symbols, r = fb->total_repair_symbols;
    /* rlc_fec_scheme_generate_gf256.c:34-39 / xor_fec_scheme_generate.c:45-50 */
    if ((xor_scheme ? r != 1 : r == 0) || k < 1 || fb->current_source_symbols != fb->total_source_symbols)
        return 1;
    uint16_t maxl = 0;
    for (int j = 0; j < k; j++)
        if (fb->source_symbols[j] && fb->source_symbols[j]->data_length > maxl) maxl = fb->source_symbols[j]->data_length;
    const uint32_t fbn = fb->fec_block_number & 0xffffffu;
    pthread_mutex_lock(&g_mu);
    g_stats.generate_calls++;
    const uint32_t L = pad4(maxl ? maxl : 1);
    int rc = stage((size_t)k * L, (size_t)r * L);
    fecgpu_host_ctx_t *c = rc ? NULL : ctx();
    if (c) {
        for (int j = 0; j < k; j++) {  /* zero-padded to max_length (:41-55) */
            uint8_t *row = g_src + (size_t)j * L;
            const pquic_source_symbol_t *ss = fb->source_symbols[j];
            uint16_t n = ss ? ss->data_length : 0;
            if (n) memcpy(row, ss->data, n);
            memset(row + n, 0, L - n);
        }
        rc = xor_scheme ? fecgpu_xor_encode_host(c, g_src, g_rep, 1, (uint32_t)k, L)
                        : fecgpu_rlc_encode_host(c, g_src, g_rep, 1, (uint32_t)k, (uint32_t)r, L, fbn, NULL);
    } else {
        rc = -1;
    }
    if (rc) {
        g_stats.errors++;
        pthread_mutex_unlock(&g_mu);
        return PQUIC_FEC_ERR_UNBOUND;
    }
    protoop_arg_t ret = 0;
    for (int i = 0; i < r; i++) {
        /* repair fpid: raw 0, fec_block_number, symbol_number = i, fec_scheme_specific 0
         * (rlc_fec_scheme_generate_gf256.c:57-61; xor_fec_scheme_generate.c:71-75) */
        pquic_repair_symbol_t *rs = new_repair(cnx, ((uint64_t)fbn << 8) | (uint64_t)(i & 0xff), maxl);
        if (!rs) { ret = PQUIC_ERROR_MEMORY; break; }
        memcpy(rs->data, g_rep + (size_t)i * L, maxl);
        fb->repair_symbols[i] = rs;
    }
    pthread_mutex_unlock(&g_mu);
    return ret;
}

protoop_arg_t pquic_fec_rlc_generate_repair_symbols(picoquic_cnx_t *cnx) { return generate(cnx, 0); }
protoop_arg_t pquic_fec_xor_generate_repair_symbols(picoquic_cnx_t *cnx) { return generate(cnx, 1); }

/* ------------------------------------------------------------------ recover */

/* rlc_fec_scheme_gf256.c:134-251 */
protoop_arg_t pquic_fec_rlc_recover(picoquic_cnx_t *cnx) {
    if (!g_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_block_t *fb = (pquic_fec_block_t *)(uintptr_t)g_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 0);
    const int k = fb->total_source_symbols, r = fb->total_repair_symbols;
    if (r == 0 || fb->current_source_symbols == fb->total_source_symbols ||
        fb->current_source_symbols + fb->current_repair_symbols < fb->total_source_symbols)
        return 0;  /* :140-144 */
    int first = -1;
    for (int i = 0; i < r; i++)
        if (fb->repair_symbols[i]) { first = i; break; }
    if (first < 0) return 0;
    const uint16_t maxl = fb->repair_symbols[first]->data_length;  /* :186 */
    const uint32_t fbn = fb->fec_block_number & 0xffffffu;
    pthread_mutex_lock(&g_mu);
    g_stats.recover_calls++;
    const uint32_t L = pad4(maxl ? maxl : 1);
    uint64_t sp[2] = {0, 0}, rp[2] = {0, 0}, rec[2] = {0, 0};
    uint8_t st = FECGPU_BLOCK_NOTHING;
    int rc = stage((size_t)k * L, (size_t)r * L);
    fecgpu_host_ctx_t *c = rc ? NULL : ctx();
    if (c) {
        for (int j = 0; j < k; j++) {
            uint8_t *row = g_src + (size_t)j * L;
            const pquic_source_symbol_t *ss = fb->source_symbols[j];
            uint16_t n = 0;
            if (ss) {  /* bytes past max_length are never read back (:205): truncate */
                n = ss->data_length < maxl ? ss->data_length : maxl;
                memcpy(row, ss->data, n);
                sp[j >> 6] |= 1ull << (j & 63);
            }
            memset(row + n, 0, L - n);
        }
        for (int i = 0; i < r; i++) {
            uint8_t *row = g_rep + (size_t)i * L;
            const pquic_repair_symbol_t *rs = fb->repair_symbols[i];
            uint16_t n = 0;
            if (rs) {
                /* the seed is the repair's own FPID (:200); the engine derives it from the
                 * block number and the slot, which the block framework keeps equal
                 * (block_framework_receiver.h:29-56, fec.h:292-299) */
                if (rs->fpid.f.source_fpid.raw != (((fbn << 8) | (uint32_t)(i & 0xff)))) { rc = -2; break; }
                n = rs->data_length < maxl ? rs->data_length : maxl;
                memcpy(row, rs->data, n);
                rp[i >> 6] |= 1ull << (i & 63);
            }
            memset(row + n, 0, L - n);
        }
        if (!rc)
            rc = fecgpu_rlc_decode_host(c, g_src, g_rep, 1, (uint32_t)k, (uint32_t)r, L, fbn, NULL, sp, rp, &st, rec);
    } else {
        rc = -1;
    }
    if (rc) {
        g_stats.errors++;
        pthread_mutex_unlock(&g_mu);
        return PQUIC_FEC_ERR_UNBOUND;
    }
    if (st == FECGPU_BLOCK_REF_UB) g_stats.ref_ub_blocks++;
    protoop_arg_t ret = 0;
    for (int j = 0; j < k && st == FECGPU_BLOCK_RECOVERED; j++) {  /* :218-236 */
        if (!((rec[j >> 6] >> (j & 63)) & 1)) continue;
        pquic_source_symbol_t *ss = new_source(cnx, (fbn << 8) + (uint8_t)j, maxl);
        if (!ss) continue;  /* the reference skips an unallocatable symbol (:222-226) */
        memcpy(ss->data, g_src + (size_t)j * L, maxl);
        fb->source_symbols[j] = ss;
        fb->current_source_symbols++;
        g_stats.recovered_symbols++;
    }
    pthread_mutex_unlock(&g_mu);
    return ret;
}

/* xor_fec_scheme.c:41-74 */
protoop_arg_t pquic_fec_xor_recover(picoquic_cnx_t *cnx) {
    if (!g_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_block_t *fb = (pquic_fec_block_t *)(uintptr_t)g_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 0);
    const int k = fb->total_source_symbols;
    if (fb->total_repair_symbols != 1 ||
        fb->current_source_symbols + fb->current_repair_symbols != fb->total_source_symbols)
        return 1;  /* :45-49 */
    const pquic_repair_symbol_t *rs = fb->repair_symbols[0];
    if (!rs) return 1;  /* the reference dereferences NULL here (:50-51) */
    const uint16_t maxl = rs->data_length;
    pthread_mutex_lock(&g_mu);
    g_stats.recover_calls++;
    const uint32_t L = pad4(maxl ? maxl : 1);
    uint64_t sp[2] = {0, 0}, rp[2] = {1, 0}, rec[2] = {0, 0};
    uint8_t st = FECGPU_BLOCK_NOTHING;
    int rc = stage((size_t)k * L, L);
    fecgpu_host_ctx_t *c = rc ? NULL : ctx();
    if (c) {
        for (int j = 0; j < k; j++) {
            uint8_t *row = g_src + (size_t)j * L;
            const pquic_source_symbol_t *ss = fb->source_symbols[j];
            uint16_t n = 0;
            if (ss) {
                n = ss->data_length < maxl ? ss->data_length : maxl;
                memcpy(row, ss->data, n);
                sp[j >> 6] |= 1ull << (j & 63);
            }
            memset(row + n, 0, L - n);
        }
        memcpy(g_rep, rs->data, maxl);
        memset(g_rep + maxl, 0, L - maxl);
        rc = fecgpu_xor_decode_host(c, g_src, g_rep, 1, (uint32_t)k, L, sp, rp, &st, rec);
    } else {
        rc = -1;
    }
    if (rc) {
        g_stats.errors++;
        pthread_mutex_unlock(&g_mu);
        return PQUIC_FEC_ERR_UNBOUND;
    }
    protoop_arg_t ret = 1;
    for (int j = 0; j < k && st == FECGPU_BLOCK_RECOVERED; j++) {
        if (!((rec[j >> 6] >> (j & 63)) & 1)) continue;
        pquic_source_symbol_t *ss = new_source(cnx, (fb->fec_block_number << 8) | (uint32_t)j, maxl);
        if (!ss) { ret = PQUIC_ERROR_MEMORY; break; }
        memcpy(ss->data, g_src + (size_t)j * L, maxl);
        fb->source_symbols[j] = ss;  /* current_source_symbols is NOT incremented (:72) */
        g_stats.recovered_symbols++;
        ret = 0;
    }
    pthread_mutex_unlock(&g_mu);
    return ret;
}
