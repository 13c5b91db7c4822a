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
#include "pquic_fec_frames.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "fec_core.h"
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

pquic_fec_host_api_t g_fec_api;
int g_fec_bound;
pquic_fec_protoop_stats_t g_fec_stats;
static int g_device;
static fecgpu_host_ctx_t *g_ctx;
/* the resident single-block service (fecgpu_block_svc_*): one block per call without a kernel launch;
 * calls it refuses (block too large for it, knob off) take the host path */
static fecgpu_block_svc_t *g_svc;
static int g_svc_failed;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

/* Per-call staging, page-locked (fecgpu_host_alloc) and grown on demand: the engine's host path
 * then runs zero-copy -- the kernels read the staged rows and write repairs / recovered rows and
 * the small per-block arrays (seeds, masks, status) in place over PCIe -- so a one-block call is
 * launches plus one synchronisation, with no copy stages. */
static uint8_t *g_src, *g_rep;
static size_t g_src_cap, g_rep_cap;
typedef struct {
    uint32_t seeds[PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK];
    uint64_t sp[2], rp[2], rec[2];
    uint8_t st;
} aux_t;
static aux_t *g_aux;

int pquic_fec_bind_host(const pquic_fec_host_api_t *api, int device) {
    pthread_mutex_lock(&g_mu);
    if (api) {
        g_fec_api = *api;
        g_fec_bound = api->get_cnx && api->set_cnx && api->my_malloc && api->my_free;
    } else {
        g_fec_bound = 0;
    }
    if (g_ctx && g_device != device) {
        fecgpu_host_ctx_destroy(g_ctx);
        g_ctx = NULL;
    }
    if (g_svc && g_device != device) {
        fecgpu_block_svc_destroy(g_svc);
        g_svc = NULL;
    }
    g_svc_failed = 0;
    g_device = device;
    pthread_mutex_unlock(&g_mu);
    return g_fec_bound ? 0 : -1;
}

void pquic_fec_protoop_stats(pquic_fec_protoop_stats_t *out) {
    out->generate_calls = __atomic_load_n(&g_fec_stats.generate_calls, __ATOMIC_RELAXED);
    out->recover_calls = __atomic_load_n(&g_fec_stats.recover_calls, __ATOMIC_RELAXED);
    out->recovered_symbols = __atomic_load_n(&g_fec_stats.recovered_symbols, __ATOMIC_RELAXED);
    out->ref_ub_blocks = __atomic_load_n(&g_fec_stats.ref_ub_blocks, __ATOMIC_RELAXED);
    out->errors = __atomic_load_n(&g_fec_stats.errors, __ATOMIC_RELAXED);
    pthread_mutex_lock(&g_mu);
    out->svc_deadline_misses = g_svc ? fecgpu_block_svc_deadline_misses(g_svc) : 0;
    pthread_mutex_unlock(&g_mu);
}

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

/* the worker ends within a poll of the quit flag; at exit it must not outlive the process's HIP state */
static void svc_atexit(void) {
    pthread_mutex_lock(&g_mu);
    fecgpu_block_svc_destroy(g_svc);
    g_svc = NULL;
    pthread_mutex_unlock(&g_mu);
}

static fecgpu_block_svc_t *svc(void) {
    static int at_exit;
    if (!g_svc && !g_svc_failed && !(g_svc = fecgpu_block_svc_create(g_device))) g_svc_failed = 1;
    if (g_svc && !at_exit) at_exit = !atexit(svc_atexit);
    return g_svc;
}

static int grow_pinned(uint8_t **p, size_t *cap, size_t need) {
    if (need <= *cap) return 0;
    size_t n = *cap ? *cap : 64 * 1024;
    while (n < need) n *= 2;
    uint8_t *q = fecgpu_host_alloc(n);
    if (!q) return -1;
    fecgpu_host_free(*p);
    *p = q;
    *cap = n;
    return 0;
}

static int stage(size_t src_bytes, size_t rep_bytes) {
    if (!g_aux && !(g_aux = fecgpu_host_alloc(sizeof *g_aux))) return -1;
    if (grow_pinned(&g_src, &g_src_cap, src_bytes) || grow_pinned(&g_rep, &g_rep_cap, rep_bytes ? rep_bytes : 4))
        return -1;
    return 0;
}

/* ------------------------------------------------------------------ create_fec_schemes */

/* create_rlc_fec_scheme_gf256.c:46-59: outputs [0] receiver scheme, [1] sender scheme
 * (the same object); returns 0 or PICOQUIC_ERROR_MEMORY.  The 64 KiB multiplication and
 * inverse tables of the reference are not needed: the device derives products from
 * GF(2^8) bit planes. */
protoop_arg_t pquic_fec_rlc_create_fec_schemes(picoquic_cnx_t *cnx) {
    if (!g_fec_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_scheme_t *fs = g_fec_api.my_malloc(cnx, sizeof *fs);
    if (!fs) return PQUIC_ERROR_MEMORY;
    fs->magic = RLC_MAGIC;
    fs->device = (uint32_t)g_device;
    g_fec_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 0, (protoop_arg_t)(uintptr_t)fs);
    g_fec_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 1, (protoop_arg_t)(uintptr_t)fs);
    return 0;
}

/* create_xor_fec_scheme.c:4-9: both outputs NULL */
protoop_arg_t pquic_fec_xor_create_fec_schemes(picoquic_cnx_t *cnx) {
    if (!g_fec_bound) return PQUIC_FEC_ERR_UNBOUND;
    g_fec_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 0, 0);
    g_fec_api.set_cnx(cnx, PQUIC_AK_CNX_OUTPUT, 1, 0);
    return 0;
}

/* ------------------------------------------------------------------ generate */

static protoop_arg_t generate(picoquic_cnx_t *cnx, int xor_scheme) {
    if (!g_fec_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_block_t *fb = (pquic_fec_block_t *)(uintptr_t)g_fec_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 0);
    uint16_t maxl = 0;
    const int chk = fec_generate_check(fb, xor_scheme, &maxl);
    if (chk == FEC_STAGE_REJECT) {
        FEC_STAT_ADD(errors, 1);
        return PQUIC_FEC_ERR_UNBOUND;
    }
    if (chk) return 1;
    const int k = fb->total_source_symbols, r = fb->total_repair_symbols;
    const uint32_t fbn = fb->fec_block_number & 0xffffffu;
    pthread_mutex_lock(&g_mu);
    FEC_STAT_ADD(generate_calls, 1);
    const uint32_t L = fec_pad4(maxl ? maxl : 1);
    int rc = stage((size_t)k * L, (size_t)r * L);
    fecgpu_host_ctx_t *c = rc ? NULL : ctx();
    if (c) {
        fec_generate_stage(fb, g_src, L);
        fecgpu_block_svc_t *v = xor_scheme ? NULL : svc();
        rc = v ? fecgpu_block_svc_rlc_encode(v, g_src, g_rep, (uint32_t)k, (uint32_t)r, L, fbn) : FECGPU_ERR_INVALID;
        if (rc == FECGPU_ERR_INVALID)
            rc = xor_scheme ? fecgpu_xor_encode_host(c, g_src, g_rep, 1, (uint32_t)k, L)
                            : fecgpu_rlc_encode_host(c, g_src, g_rep, 1, (uint32_t)k, (uint32_t)r, L, fbn, NULL);
    } else {
        rc = -1;
    }
    protoop_arg_t ret;
    if (rc) {
        FEC_STAT_ADD(errors, 1);
        ret = PQUIC_FEC_ERR_UNBOUND;
    } else {
        ret = fec_generate_finish(cnx, fb, g_rep, L, maxl);
    }
    pthread_mutex_unlock(&g_mu);
    return ret;
}

protoop_arg_t pquic_fec_rlc_generate_repair_symbols(picoquic_cnx_t *cnx) { return generate(cnx, 0); }
protoop_arg_t pquic_fec_xor_generate_repair_symbols(picoquic_cnx_t *cnx) { return generate(cnx, 1); }

/* ------------------------------------------------------------------ recover */

/* rlc_fec_scheme_gf256.c:134-251 and xor_fec_scheme.c:41-74.  The RLC equations are seeded by each
 * received repair's own FPID (:200), so blocks of the block framework ((fbn << 8) | i) and of the
 * sliding-window framework (block numbered by its window start, repairs (0 << 8) | i) both recover
 * as the reference does. */
static protoop_arg_t recover(picoquic_cnx_t *cnx, int xor_scheme) {
    if (!g_fec_bound) return PQUIC_FEC_ERR_UNBOUND;
    pquic_fec_block_t *fb = (pquic_fec_block_t *)(uintptr_t)g_fec_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 0);
    uint16_t maxl = 0;
    const int chk = fec_recover_check(fb, xor_scheme, &maxl);
    if (chk == FEC_STAGE_REJECT) {
        FEC_STAT_ADD(errors, 1);
        return PQUIC_FEC_ERR_UNBOUND;
    }
    if (chk != FEC_STAGE_OK) return (protoop_arg_t)chk;
    const int k = fb->total_source_symbols, r = xor_scheme ? 1 : fb->total_repair_symbols;
    pthread_mutex_lock(&g_mu);
    FEC_STAT_ADD(recover_calls, 1);
    const uint32_t L = fec_pad4(maxl ? maxl : 1);
    int rc = stage((size_t)k * L, (size_t)r * L);
    fecgpu_host_ctx_t *c = rc ? NULL : ctx();
    if (c) {
        aux_t *a = g_aux;
        a->st = FECGPU_BLOCK_NOTHING;
        a->rec[0] = a->rec[1] = 0;
        fec_recover_stage(fb, xor_scheme, maxl, g_src, g_rep, L, a->sp, a->rp, a->seeds);
        fecgpu_block_svc_t *v = xor_scheme ? NULL : svc();
        rc = v ? fecgpu_block_svc_rlc_decode_seeded(v, g_src, g_rep, g_src, (uint32_t)k, (uint32_t)r, L, a->seeds,
                                                    a->sp, a->rp, &a->st, a->rec)
               : FECGPU_ERR_INVALID;
        if (rc == FECGPU_ERR_INVALID)
            rc = xor_scheme ? fecgpu_xor_decode_host(c, g_src, g_rep, 1, (uint32_t)k, L, a->sp, a->rp, &a->st, a->rec)
                            : fecgpu_rlc_decode_host_seeded(c, g_src, g_rep, 1, (uint32_t)k, (uint32_t)r, L, a->seeds,
                                                            a->sp, a->rp, &a->st, a->rec);
    } else {
        rc = -1;
    }
    protoop_arg_t ret;
    if (rc) {
        FEC_STAT_ADD(errors, 1);
        ret = PQUIC_FEC_ERR_UNBOUND;
    } else {
        ret = fec_recover_finish(cnx, fb, xor_scheme, g_aux->st, g_aux->rec, g_src, L, maxl, NULL);
    }
    pthread_mutex_unlock(&g_mu);
    return ret;
}

protoop_arg_t pquic_fec_rlc_recover(picoquic_cnx_t *cnx) { return recover(cnx, 0); }
protoop_arg_t pquic_fec_xor_recover(picoquic_cnx_t *cnx) { return recover(cnx, 1); }

/* ---- source-symbol capture ---- */
static int skip_via_host(void *cnx, const uint8_t *bytes, size_t bytes_max, size_t *consumed, int *pure_ack) {
    return g_fec_api.skip_frame((picoquic_cnx_t *)cnx, (uint8_t *)bytes, bytes_max, consumed, pure_ack);
}

protoop_arg_t pquic_fec_packet_payload_to_source_symbol(picoquic_cnx_t *cnx) {
    if (!g_fec_bound || !g_fec_api.skip_frame) return PQUIC_FEC_ERR_UNBOUND;
    const uint8_t *payload = (const uint8_t *)g_fec_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 0);
    uint8_t *buffer = (uint8_t *)g_fec_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 1);
    const uint32_t length = (uint32_t)g_fec_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 2);
    const uint64_t pn = (uint64_t)g_fec_api.get_cnx(cnx, PQUIC_AK_CNX_INPUT, 3);
    if (!buffer) return PQUIC_ERROR_MEMORY;                                /* :14-16 */
    return pquic_fec_payload_to_source_symbol(payload, length, pn, buffer, skip_via_host, cnx);
}
