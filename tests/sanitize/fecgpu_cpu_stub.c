/*
 * tests/sanitize/fecgpu_cpu_stub.c -- TEST INFRASTRUCTURE ONLY, never linked into the product.
 *
 * A CPU stand-in for the engine entry points (include/fecgpu.h) that the host C of the adapter layer
 * calls -- protoops.c, fec_core.c and batch.c -- so that layer can be built with AddressSanitizer /
 * UndefinedBehaviorSanitizer / ThreadSanitizer and driven by the CPU-only tests (tests/host/mini_host.c
 * and the Python suites over it) on a machine without a GPU.  Sanitizers cannot instrument the HIP
 * engine; what they check here is the host logic around it: allocation, attach and free of symbols,
 * the batcher's stagers, engine threads, arena registry and ordered completions.
 *
 * Every computation is the oracle's (oracle/fec_oracle.c).  "Device" memory is host memory: a
 * page-locked range is one returned by fecgpu_host_alloc or registered with fecgpu_host_register, and
 * its device address is its host address.  The resident block service is reported unavailable, so the
 * adapters take their launch path (fecgpu_*_host).  tests/sanitize/Makefile builds it; the product's
 * libpquic_fec.so never contains it (tests/test_abi.py checks the exported symbols).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fecgpu.h"
#include "fec_oracle.h"

/* ---- page-locked ranges: host_alloc'd blocks and registered ranges (sorted by nothing: few) ---- */
typedef struct { uintptr_t base; size_t bytes; int owned; } range_t;
static range_t *g_ranges;
static int g_nranges, g_cap;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static int range_add(void *p, size_t bytes, int owned) {
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nranges; i++)
        if ((uintptr_t)p < g_ranges[i].base + g_ranges[i].bytes && g_ranges[i].base < (uintptr_t)p + bytes) {
            pthread_mutex_unlock(&g_mu);
            return FECGPU_ERR_INVALID;  /* overlap, as hipHostRegister refuses */
        }
    if (g_nranges == g_cap) {
        g_cap = g_cap ? 2 * g_cap : 64;
        g_ranges = realloc(g_ranges, sizeof *g_ranges * (size_t)g_cap);
    }
    g_ranges[g_nranges++] = (range_t){(uintptr_t)p, bytes, owned};
    pthread_mutex_unlock(&g_mu);
    return FECGPU_OK;
}
static int range_del(void *p, int owned) {
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nranges; i++)
        if (g_ranges[i].base == (uintptr_t)p && g_ranges[i].owned == owned) {
            g_ranges[i] = g_ranges[--g_nranges];
            pthread_mutex_unlock(&g_mu);
            return FECGPU_OK;
        }
    pthread_mutex_unlock(&g_mu);
    return FECGPU_ERR_INVALID;
}

void *fecgpu_host_alloc(size_t bytes) {
    void *p = NULL;
    if (posix_memalign(&p, 4096, bytes ? bytes : 1)) return NULL;
    if (range_add(p, bytes ? bytes : 1, 1)) { free(p); return NULL; }
    return p;
}
void fecgpu_host_free(void *p) {
    if (p && range_del(p, 1) == FECGPU_OK) free(p);
}
int fecgpu_host_register(void *p, size_t bytes) {
    if (!p || !bytes) return FECGPU_ERR_INVALID;
    return range_add(p, bytes, 0);
}
int fecgpu_host_unregister(void *p) { return range_del(p, 0); }
int fecgpu_host_device_address(const void *p, size_t bytes, uint64_t *dev) {
    if (!p || !dev) return FECGPU_ERR_INVALID;
    pthread_mutex_lock(&g_mu);
    int ok = 0;
    for (int i = 0; i < g_nranges && !ok; i++)
        ok = (uintptr_t)p >= g_ranges[i].base && (uintptr_t)p + bytes <= g_ranges[i].base + g_ranges[i].bytes;
    pthread_mutex_unlock(&g_mu);
    if (!ok) return FECGPU_ERR_INVALID;
    *dev = (uint64_t)(uintptr_t)p;
    return FECGPU_OK;
}
int fecgpu_device_local_cpus(int device, char *buf, size_t len) {
    (void)device; (void)buf; (void)len;
    return FECGPU_ERR_NO_DEVICE;  /* the batcher then leaves its threads unpinned */
}

/* ---- host contexts: nothing to hold; a distinct object per create for the callers' bookkeeping ---- */
struct fecgpu_host_ctx { int device; };
fecgpu_host_ctx_t *fecgpu_host_ctx_create(int device, int nstreams, size_t chunk_bytes) {
    (void)nstreams; (void)chunk_bytes;
    fecgpu_host_ctx_t *c = malloc(sizeof *c);
    if (c) c->device = device;
    return c;
}
void fecgpu_host_ctx_destroy(fecgpu_host_ctx_t *ctx) { free(ctx); }

/* the resident block service is not available here: the adapters take the launch path */
fecgpu_block_svc_t *fecgpu_block_svc_create(int device) { (void)device; return NULL; }
void fecgpu_block_svc_destroy(fecgpu_block_svc_t *svc) { (void)svc; }
int fecgpu_block_svc_rlc_encode(fecgpu_block_svc_t *svc, const void *src, void *rep, uint32_t k, uint32_t r,
                                uint32_t symbol_size, uint32_t fbn) {
    (void)svc; (void)src; (void)rep; (void)k; (void)r; (void)symbol_size; (void)fbn;
    return FECGPU_ERR_INVALID;
}
int fecgpu_block_svc_rlc_decode_seeded(fecgpu_block_svc_t *svc, const void *src, const void *rep, void *dst,
                                       uint32_t k, uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed,
                                       const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                                       uint64_t *recovered) {
    (void)svc; (void)src; (void)rep; (void)dst; (void)k; (void)r; (void)symbol_size; (void)rep_seed;
    (void)src_present; (void)rep_present; (void)status; (void)recovered;
    return FECGPU_ERR_INVALID;
}
uint64_t fecgpu_block_svc_deadline_misses(fecgpu_block_svc_t *svc) { (void)svc; return 0; }
int fecgpu_block_svc_worker_running(fecgpu_block_svc_t *svc) { return svc ? 0 : FECGPU_ERR_INVALID; }
int fecgpu_block_svc_last_stamps(fecgpu_block_svc_t *svc, uint64_t out[6]) {
    (void)svc;
    for (int i = 0; i < 6; i++) out[i] = 0;
    return FECGPU_ERR_INVALID;
}

/* ---- the operations, block by block through the oracle ---- */
#define MAXS 256
static int bad_shape(uint32_t k, uint32_t r, uint32_t L) { return !k || k > 128 || r > 128 || !L || L % 4; }
static uint32_t fbn_of(uint32_t fbn_base, const uint32_t *fbn, uint64_t b) {
    return (fbn ? fbn[b] : fbn_base + (uint32_t)b) & 0xffffffu;
}
static int present(const uint64_t *m, uint64_t b, uint32_t j) { return (int)((m[2 * b + (j >> 6)] >> (j & 63)) & 1); }

/* one RLC block from row pointers; rows are all L bytes */
static void enc_rows(uint32_t fbn, uint32_t k, uint32_t r, uint32_t L, const uint8_t *const *s, uint8_t *const *o) {
#ifdef STUB_NULL_ENGINE  /* host-cost profiling only (tools/sender_cpu_probe.py): the repairs are not computed */
    (void)fbn; (void)k; (void)r; (void)L; (void)s; (void)o;
#else
    uint16_t sl[MAXS], rl[MAXS];
    for (uint32_t j = 0; j < k; j++) sl[j] = (uint16_t)L;
    oracle_rlc_encode_block(fbn, (int)k, (int)r, s, sl, o, rl);
#endif
}
/* one RLC decode from row pointers: missing sources' rows receive the recovered bytes */
static void dec_rows(uint32_t k, uint32_t r, uint32_t L, uint8_t *const *s, const uint8_t *const *p,
                     const uint32_t *seed, const uint64_t *sp, const uint64_t *rp, uint64_t b, uint8_t *status,
                     uint64_t *recovered) {
    const uint8_t *src[MAXS], *rep[MAXS];
    uint16_t sl[MAXS], rl[MAXS], ol[MAXS];
    uint8_t *out[MAXS], rec[MAXS];
    for (uint32_t j = 0; j < k; j++) {
        src[j] = present(sp, b, j) ? s[j] : NULL;
        sl[j] = (uint16_t)L;
        out[j] = s[j];  /* a missing source's row is where its recovered bytes go */
    }
    for (uint32_t i = 0; i < r; i++) {
        rep[i] = present(rp, b, i) ? p[i] : NULL;
        rl[i] = (uint16_t)L;
    }
    memset(rec, 0, sizeof rec);
    status[b] = (uint8_t)oracle_rlc_decode_block(0, (int)k, (int)r, src, sl, rep, rl, seed, out, ol, rec);
    recovered[2 * b] = recovered[2 * b + 1] = 0;
    for (uint32_t j = 0; j < k; j++)
        if (rec[j]) recovered[2 * b + (j >> 6)] |= 1ull << (j & 63);
}

int fecgpu_rlc_encode_host(fecgpu_host_ctx_t *ctx, const void *src, void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn) {
    if (!ctx || !src || !rep || bad_shape(k, r, symbol_size)) return FECGPU_ERR_INVALID;
    const uint8_t *s[MAXS];
    uint8_t *o[MAXS];
    for (uint64_t b = 0; b < nblocks; b++) {
        for (uint32_t j = 0; j < k; j++) s[j] = (const uint8_t *)src + (b * k + j) * symbol_size;
        for (uint32_t i = 0; i < r; i++) o[i] = (uint8_t *)rep + (b * r + i) * symbol_size;
        enc_rows(fbn_of(fbn_base, fbn, b), k, r, symbol_size, s, o);
    }
    return FECGPU_OK;
}

int fecgpu_rlc_encode_rows_host(fecgpu_host_ctx_t *ctx, const uint64_t *src_rows, const uint64_t *rep_rows,
                                uint64_t nblocks, uint32_t k, uint32_t r, uint32_t symbol_size, const uint32_t *fbn) {
    if (!ctx || !src_rows || !rep_rows || bad_shape(k, r, symbol_size)) return FECGPU_ERR_INVALID;
    const uint8_t *s[MAXS];
    uint8_t *o[MAXS];
    for (uint64_t b = 0; b < nblocks; b++) {
        for (uint32_t j = 0; j < k; j++) s[j] = (const uint8_t *)(uintptr_t)src_rows[b * k + j];
        for (uint32_t i = 0; i < r; i++) o[i] = (uint8_t *)(uintptr_t)rep_rows[b * r + i];
        enc_rows(fbn_of(0, fbn, b), k, r, symbol_size, s, o);
    }
    return FECGPU_OK;
}

int fecgpu_rlc_decode_host_seeded(fecgpu_host_ctx_t *ctx, void *src, const void *rep, uint64_t nblocks, uint32_t k,
                                  uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed,
                                  const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                                  uint64_t *recovered) {
    if (!ctx || !src || !rep || !rep_seed || !src_present || !rep_present || !status || !recovered || !r ||
        bad_shape(k, r, symbol_size))
        return FECGPU_ERR_INVALID;
    uint8_t *s[MAXS];
    const uint8_t *p[MAXS];
    for (uint64_t b = 0; b < nblocks; b++) {
        for (uint32_t j = 0; j < k; j++) s[j] = (uint8_t *)src + (b * k + j) * symbol_size;
        for (uint32_t i = 0; i < r; i++) p[i] = (const uint8_t *)rep + (b * r + i) * symbol_size;
        dec_rows(k, r, symbol_size, s, p, rep_seed + b * r, src_present, rep_present, b, status, recovered);
    }
    return FECGPU_OK;
}

int fecgpu_rlc_decode_rows_host(fecgpu_host_ctx_t *ctx, const uint64_t *src_rows, const uint64_t *rep_rows,
                                uint64_t nblocks, uint32_t k, uint32_t r, uint32_t symbol_size,
                                const uint32_t *rep_seed, const uint64_t *src_present, const uint64_t *rep_present,
                                uint8_t *status, uint64_t *recovered) {
    if (!ctx || !src_rows || !rep_seed || !src_present || !rep_present || !status || !recovered ||
        bad_shape(k, r, symbol_size) || (r && !rep_rows))
        return FECGPU_ERR_INVALID;
    uint8_t *s[MAXS];
    const uint8_t *p[MAXS];
    for (uint64_t b = 0; b < nblocks; b++) {
        for (uint32_t j = 0; j < k; j++) s[j] = (uint8_t *)(uintptr_t)src_rows[b * k + j];
        for (uint32_t i = 0; i < r; i++) p[i] = (const uint8_t *)(uintptr_t)rep_rows[b * r + i];
        dec_rows(k, r, symbol_size, s, p, rep_seed + b * r, src_present, rep_present, b, status, recovered);
    }
    return FECGPU_OK;
}

int fecgpu_rlc_window_encode_host(fecgpu_host_ctx_t *ctx, const void *symbols, uint64_t nrows, const uint32_t *wrow,
                                  uint64_t nwindows, uint32_t k, uint32_t r, uint32_t symbol_size, void *rep) {
    if (!ctx || !symbols || !wrow || !rep || bad_shape(k, r, symbol_size)) return FECGPU_ERR_INVALID;
    for (uint64_t w = 0; w < nwindows; w++)
        if ((uint64_t)wrow[w] + k > nrows) return FECGPU_ERR_INVALID;
    const uint8_t *s[MAXS];
    uint8_t *o[MAXS];
    for (uint64_t w = 0; w < nwindows; w++) {
        for (uint32_t j = 0; j < k; j++) s[j] = (const uint8_t *)symbols + ((uint64_t)wrow[w] + j) * symbol_size;
        for (uint32_t i = 0; i < r; i++) o[i] = (uint8_t *)rep + (w * r + i) * symbol_size;
        enc_rows(0, k, r, symbol_size, s, o);  /* window blocks are block number 0 */
    }
    return FECGPU_OK;
}

int fecgpu_xor_encode_host(fecgpu_host_ctx_t *ctx, const void *src, void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t symbol_size) {
    if (!ctx || !src || !rep || bad_shape(k, 1, symbol_size)) return FECGPU_ERR_INVALID;
    return oracle_xor_encode_batch(src, rep, nblocks, (int)k, (int)symbol_size, 1) < 0 ? FECGPU_ERR_INVALID : FECGPU_OK;
}

int fecgpu_xor_decode_host(fecgpu_host_ctx_t *ctx, void *src, const void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t symbol_size, const uint64_t *src_present, const uint64_t *rep_present,
                           uint8_t *status, uint64_t *recovered) {
    if (!ctx || !src || !rep || !src_present || !rep_present || !status || !recovered || bad_shape(k, 1, symbol_size))
        return FECGPU_ERR_INVALID;
    return oracle_xor_decode_batch(src, rep, nblocks, (int)k, (int)symbol_size, src_present, rep_present, status,
                                   recovered, 1) < 0 ? FECGPU_ERR_INVALID : FECGPU_OK;
}

/* knobs select among kernels that give identical bytes; the stand-in has one path, so they are only
 * remembered (the batching tests set window_sc to run both window paths) */
static struct { char name[32]; int value; } g_knobs[32];
static int g_nknobs;
int fecgpu_set_knob(const char *name, int value) {
    if (!name || strlen(name) >= sizeof g_knobs[0].name) return FECGPU_ERR_INVALID;
    pthread_mutex_lock(&g_mu);
    int i = 0;
    while (i < g_nknobs && strcmp(g_knobs[i].name, name)) i++;
    if (i == g_nknobs && g_nknobs < 32) strcpy(g_knobs[g_nknobs++].name, name);
    if (i < 32) g_knobs[i].value = value;
    pthread_mutex_unlock(&g_mu);
    return i < 32 ? FECGPU_OK : FECGPU_ERR_INVALID;
}
int fecgpu_get_knob(const char *name, int *value) {
    if (!name || !value) return FECGPU_ERR_INVALID;
    pthread_mutex_lock(&g_mu);
    *value = 1;  /* the engine's defaults for the knobs the suites read (window_sc) */
    for (int i = 0; i < g_nknobs; i++)
        if (!strcmp(g_knobs[i].name, name)) *value = g_knobs[i].value;
    pthread_mutex_unlock(&g_mu);
    return FECGPU_OK;
}

/* Deliberate defects, called only by tests/test_sanitize.py to show each build's sanitizer is live:
 * kind 1 reads one byte past a heap block (AddressSanitizer), kind 2 races two threads on a plain int
 * (ThreadSanitizer).  Never called by the suites. */
static int g_racy;
static void *canary_thread(void *p) {
    (void)p;
    for (int i = 0; i < 1000; i++) g_racy++;
    return NULL;
}
int san_canary(int kind) {
    if (kind == 1) {
        volatile char *p = malloc(16);
        const int v = p[16];
        free((void *)p);
        return v;
    }
    pthread_t a, b;
    pthread_create(&a, NULL, canary_thread, NULL);
    pthread_create(&b, NULL, canary_thread, NULL);
    pthread_join(a, NULL);
    pthread_join(b, NULL);
    return g_racy;
}
