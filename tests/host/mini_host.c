/*
 * tests/host/mini_host.c -- TEST INFRASTRUCTURE: a minimal stand-in for the picoquic plugin
 * runtime, enough to drive the FEC scheme protocol operations the way the reference does.
 *
 *   - picoquic_cnx_t carries protoop_inputv / protoop_outputv like the real connection
 *     (picoquic/picoquic_internal.h), read and written by get_cnx / set_cnx
 *     (picoquic/getset.c:137-142, 370-379);
 *   - my_malloc hands out fixed 2100-byte slots for requests <= 2092 bytes and falls back
 *     to the heap above that, like a plugin with dynamic_memory (picoquic/memory.c:72-95,
 *     181-191; plugin.c:409-424); live allocations are counted for leak checks;
 *   - run_protoop mirrors plugin_run_protoop_internal's argument passing
 *     (picoquic/plugin.c:1279-1450): set inputs, call the operation, collect outputs.
 * Blocks are assembled as the block framework does (block_framework_sender.h:175-203,
 * block_framework_receiver.h:29-80, fec.h:292-308).
 */
#define _GNU_SOURCE  /* MAP_ANONYMOUS */
#include <stdint.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <string.h>

#include "pquic_fec_protoops.h"

struct mh_arena;

struct st_picoquic_cnx_t {
    protoop_arg_t inputv[16];
    protoop_arg_t outputv[16];
    int inputc, outputc;
    struct mh_arena *arena;  /* the connection's plugin memory (NULL: the default arena, if any) */
};

static long g_live;

static protoop_arg_t mh_get_cnx(picoquic_cnx_t *cnx, access_key_t ak, uint16_t param) {
    if (ak == PQUIC_AK_CNX_INPUT) return param < cnx->inputc ? cnx->inputv[param] : 0;
    if (ak == PQUIC_AK_CNX_OUTPUT) return cnx->outputv[param];
    return 0;
}

static void mh_set_cnx(picoquic_cnx_t *cnx, access_key_t ak, uint16_t param, protoop_arg_t val) {
    if (ak == PQUIC_AK_CNX_OUTPUT && param < 16) {
        cnx->outputv[param] = val;
        if (param + 1 > cnx->outputc) cnx->outputc = param + 1;
    }
}

static long g_fail_after = -1;  /* allocation-failure injection: the n-th allocation from now fails */
static long g_fail_count = 1;   /* ... and this many in a row from there */
static int g_arena_strict;      /* a full arena fails the allocation instead of falling back to the heap */

void mh_fail_alloc_after(long n) { g_fail_after = n; g_fail_count = 1; }
void mh_fail_alloc_range(long n, long count) { g_fail_after = n; g_fail_count = count > 0 ? count : 1; }
/* mh_arena_strict(1): a plugin without dynamic memory -- my_malloc_block returns NULL once its arena is
 * full (picoquic/memory.c:72-110) */
void mh_arena_strict(int on) { g_arena_strict = on; }

/* Plugin-style memory arenas (picoquic_internal.h:576 memory[PLUGIN_MEMORY], carved into 2100-B
 * slots, picoquic/memory.c:181-191): allocations up to 2092 B come from the arena of the connection
 * that asks (every connection owns its plugin instances and their memory, plugin.c:835, 946-950), or
 * from the default arena (mh_arena_enable) for connections without one; a full arena falls back to the
 * heap, as a plugin with dynamic_memory would (plugin.c:409-424).  The batching adapter can be given
 * the arenas (pquic_fec_batch_register_heap) and gather rows in place. */
enum { MH_SLOT = 2112 };
typedef struct mh_arena {
    uint8_t *base;
    size_t size, used;
    void *free_list;
    long live;
} mh_arena_t;
static mh_arena_t **g_arenas;  /* every arena made, for frees (a symbol outlives nothing but its arena) */
static int g_narenas, g_arenas_cap;
static mh_arena_t *g_default_arena;

static mh_arena_t *arena_new(size_t bytes) {
    mh_arena_t *a = calloc(1, sizeof *a);
    if (!a) return NULL;
    a->size = (bytes + 4095) & ~(size_t)4095;
    void *p = mmap(NULL, a->size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
        free(a);
        return NULL;
    }
    a->base = p;
    if (g_narenas == g_arenas_cap) {
        g_arenas_cap = g_arenas_cap ? 2 * g_arenas_cap : 64;
        g_arenas = realloc(g_arenas, sizeof *g_arenas * (size_t)g_arenas_cap);
    }
    g_arenas[g_narenas++] = a;
    return a;
}

static void arena_drop(mh_arena_t *a) {  /* an arena nothing lives in any more */
    for (int i = 0; i < g_narenas; i++)
        if (g_arenas[i] == a) {
            g_arenas[i] = g_arenas[--g_narenas];
            break;
        }
    munmap(a->base, a->size);
    free(a);
}

/* A fresh default arena of `bytes` (the previous one is dropped once nothing lives in it). */
int mh_arena_enable(size_t bytes) {
    mh_arena_t *old = g_default_arena;
    g_default_arena = arena_new(bytes);
    if (old && !old->live) arena_drop(old);
    return g_default_arena ? 0 : -1;
}

static mh_arena_t *arena_of(picoquic_cnx_t *cnx, const void *p) {
    const uintptr_t a = (uintptr_t)p;
    if (cnx && cnx->arena && a - (uintptr_t)cnx->arena->base < cnx->arena->size) return cnx->arena;
    for (int i = 0; i < g_narenas; i++)
        if (a - (uintptr_t)g_arenas[i]->base < g_arenas[i]->size) return g_arenas[i];
    return NULL;
}

static void *mh_malloc(picoquic_cnx_t *cnx, unsigned int size) {
    if (g_fail_after == 0) {
        if (--g_fail_count <= 0) {
            g_fail_after = -1;
            g_fail_count = 1;
        }
        return NULL;
    }
    if (g_fail_after > 0) g_fail_after--;
    void *p = NULL;
    mh_arena_t *ar = cnx && cnx->arena ? cnx->arena : g_default_arena;
    if (ar && size <= 2092) {
        if (ar->free_list) {
            p = ar->free_list;
            ar->free_list = *(void **)p;
        } else if (ar->used + MH_SLOT <= ar->size) {
            p = ar->base + ar->used;
            ar->used += MH_SLOT;
        }
        if (p) ar->live++;
        else if (g_arena_strict) return NULL;
    }
    if (!p) p = malloc(size <= 2092 ? 2100 : size);
    if (p) g_live++;
    return p;
}

static void mh_free(picoquic_cnx_t *cnx, void *p) {
    if (!p) return;
    g_live--;
    mh_arena_t *ar = arena_of(cnx, p);
    if (ar) {
        *(void **)p = ar->free_list;
        ar->free_list = p;
        ar->live--;
    } else {
        free(p);
    }
}

typedef protoop_arg_t (*op_t)(picoquic_cnx_t *);

static protoop_arg_t run_protoop(picoquic_cnx_t *cnx, op_t op, int inputc, const protoop_arg_t *inputv,
                                 protoop_arg_t *outputv) {
    memset(cnx, 0, sizeof *cnx);
    cnx->inputc = inputc;
    for (int i = 0; i < inputc; i++) cnx->inputv[i] = inputv[i];
    protoop_arg_t ret = op(cnx);
    if (outputv)
        for (int i = 0; i < cnx->outputc; i++) outputv[i] = cnx->outputv[i];
    return ret;
}

/* skip_frame stand-in: the synthetic frame grammar of oracle/ref/ref_driver.c
 * (ref_skip_frame_synthetic): PADDING runs of 0x00, every other type [type][len][len bytes]. */
static int mh_skip_frame(picoquic_cnx_t *cnx, uint8_t *bytes, size_t bytes_max, size_t *consumed, int *pure_ack) {
    (void)cnx;
    *pure_ack = 0;
    if (bytes_max == 0) { *consumed = 0; return -1; }
    size_t n;
    if (bytes[0] == 0x00) {
        n = 1;
        while (n < bytes_max && bytes[n] == 0x00) n++;
    } else {
        n = bytes_max < 2 ? bytes_max : 2 + (size_t)bytes[1];
        if (n > bytes_max) n = bytes_max;
    }
    *consumed = n;
    return 0;
}

int mh_bind(int device) {
    pquic_fec_host_api_t api = {mh_get_cnx, mh_set_cnx, mh_malloc, mh_free, mh_skip_frame};
    return pquic_fec_bind_host(&api, device);
}

/* the packet_payload_to_source_symbol protoop with the reference's four inputs */
long mh_payload_to_source_symbol(const uint8_t *payload, uint32_t len, uint64_t pn, uint8_t *buffer) {
    picoquic_cnx_t cnx;
    protoop_arg_t in[4] = {(protoop_arg_t)payload, (protoop_arg_t)buffer, len, pn};
    return (long)run_protoop(&cnx, pquic_fec_packet_payload_to_source_symbol, 4, in, NULL);
}

int mh_unbind(void) { return pquic_fec_bind_host(NULL, 0); }

long mh_live_allocations(void) { return g_live; }

static op_t op_create(int xor_scheme) {
    return xor_scheme ? pquic_fec_xor_create_fec_schemes : pquic_fec_rlc_create_fec_schemes;
}

static pquic_source_symbol_t *mk_source_in(picoquic_cnx_t *c, uint32_t fbn, int j, const uint8_t *data, uint16_t len) {
    pquic_source_symbol_t *s = mh_malloc(c, sizeof *s);
    memset(s, 0, sizeof *s);
    s->fpid.raw = (fbn << 8) | (uint32_t)j;
    s->data = mh_malloc(c, len);
    memcpy(s->data, data, len);
    s->data_length = len;
    return s;
}

static pquic_source_symbol_t *mk_source(uint32_t fbn, int j, const uint8_t *data, uint16_t len) {
    picoquic_cnx_t c = {0};
    return mk_source_in(&c, fbn, j, data, len);
}

static void free_block(pquic_fec_block_t *fb) {
    picoquic_cnx_t c = {0};
    for (int j = 0; j < PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK; j++) {
        if (fb->source_symbols[j]) { mh_free(&c, fb->source_symbols[j]->data); mh_free(&c, fb->source_symbols[j]); }
        if (fb->repair_symbols[j]) { mh_free(&c, fb->repair_symbols[j]->data); mh_free(&c, fb->repair_symbols[j]); }
    }
    free(fb);
}

static long g_fail_next_op = -1;
/* the next mh_generate's operation fails its n-th allocation (the block is built before) */
void mh_fail_next_generate(long n) { g_fail_next_op = n; }

/* Sender side: k sources -> fec_generate_repair_symbols.  Returns the protoop's code;
 * repairs copied to rep_out[i * stride], lengths / raw FPIDs per repair. */
long mh_generate(int xor_scheme, uint32_t fbn, int k, int r, const uint8_t *src, const uint16_t *src_len,
                 int src_stride, uint8_t *rep_out, uint16_t *rep_len, uint64_t *rep_fpid, int rep_stride,
                 uint64_t *scheme_out) {
    picoquic_cnx_t cnx;
    protoop_arg_t schemes[2] = {0, 0};
    protoop_arg_t ret = run_protoop(&cnx, op_create(xor_scheme), 0, NULL, schemes);
    if (ret) return (long)ret;
    scheme_out[0] = schemes[0];
    scheme_out[1] = schemes[1];
    pquic_fec_block_t *fb = calloc(1, sizeof *fb);
    fb->fec_block_number = fbn;
    for (int j = 0; j < k; j++) fb->source_symbols[j] = mk_source(fbn, j, src + (size_t)j * src_stride, src_len[j]);
    fb->current_source_symbols = (uint8_t)k;
    fb->total_source_symbols = (uint8_t)k;      /* block_framework_sender.h:184-185 */
    fb->total_repair_symbols = (uint8_t)r;
    protoop_arg_t in[2] = {(protoop_arg_t)(uintptr_t)fb, schemes[1]};
    g_fail_after = g_fail_next_op;  /* armed for the operation only (mh_fail_next_generate) */
    g_fail_next_op = -1;
    ret = run_protoop(&cnx, xor_scheme ? pquic_fec_xor_generate_repair_symbols : pquic_fec_rlc_generate_repair_symbols,
                      2, in, NULL);
    g_fail_after = -1;
    for (int i = 0; i < r; i++) {
        pquic_repair_symbol_t *rs = fb->repair_symbols[i];
        rep_len[i] = rs ? rs->data_length : 0;
        rep_fpid[i] = rs ? rs->fpid.raw : 0;
        if (rs) memcpy(rep_out + (size_t)i * rep_stride, rs->data, rs->data_length);
    }
    if (schemes[1] && !xor_scheme) mh_free(&cnx, (void *)(uintptr_t)schemes[1]);
    free_block(fb);
    return (long)ret;
}

/* Receiver side: a block with the given sources / repairs present -> fec_recover.
 * recovered[j] = 1 for every source inserted by the operation; its bytes, length and source FPID in
 * out[j * stride] / out_len[j] / out_fpid[j] (out_fpid may be NULL); *cur_ss =
 * current_source_symbols afterwards.  fbn is the block's own number: the block framework's block
 * number, or the window framework's first source id (window_framework_receiver.h:60-86); repair
 * FPIDs are taken as given (rep_fpid). */
long mh_recover(int xor_scheme, uint32_t fbn, int k, int r, const uint8_t *src, const uint16_t *src_len,
                const uint8_t *src_present, int src_stride, const uint8_t *rep, const uint16_t *rep_len,
                const uint8_t *rep_present, const uint64_t *rep_fpid, int rep_stride, uint8_t *out,
                uint16_t *out_len, uint8_t *recovered, int out_stride, int *cur_ss, uint32_t *out_fpid) {
    picoquic_cnx_t cnx;
    protoop_arg_t schemes[2] = {0, 0};
    protoop_arg_t ret = run_protoop(&cnx, op_create(xor_scheme), 0, NULL, schemes);
    if (ret) return (long)ret;
    pquic_fec_block_t *fb = calloc(1, sizeof *fb);
    fb->fec_block_number = fbn;
    fb->total_source_symbols = (uint8_t)k;       /* block_framework_receiver.h:42-43 */
    fb->total_repair_symbols = (uint8_t)r;
    for (int j = 0; j < k; j++)
        if (src_present[j]) {
            fb->source_symbols[j] = mk_source(fbn, j, src + (size_t)j * src_stride, src_len[j]);
            fb->current_source_symbols++;
        }
    for (int i = 0; i < r; i++)
        if (rep_present[i]) {
            pquic_repair_symbol_t *rs = mh_malloc(&cnx, sizeof *rs);
            memset(rs, 0, sizeof *rs);
            rs->fpid.raw = rep_fpid[i];
            rs->data = mh_malloc(&cnx, rep_len[i]);
            memcpy(rs->data, rep + (size_t)i * rep_stride, rep_len[i]);
            rs->data_length = rep_len[i];
            fb->repair_symbols[i] = rs;
            fb->current_repair_symbols++;
        }
    pquic_source_symbol_t *before[PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK];
    memcpy(before, fb->source_symbols, sizeof before);
    protoop_arg_t in[2] = {(protoop_arg_t)(uintptr_t)fb, schemes[0]};
    ret = run_protoop(&cnx, xor_scheme ? pquic_fec_xor_recover : pquic_fec_rlc_recover, 2, in, NULL);
    for (int j = 0; j < k; j++) {
        pquic_source_symbol_t *ss = fb->source_symbols[j];
        recovered[j] = ss && ss != before[j];
        out_len[j] = recovered[j] ? ss->data_length : 0;
        if (out_fpid) out_fpid[j] = recovered[j] ? ss->fpid.raw : 0;
        if (recovered[j]) memcpy(out + (size_t)j * out_stride, ss->data, ss->data_length);
    }
    *cur_ss = fb->current_source_symbols;
    if (schemes[0] && !xor_scheme) mh_free(&cnx, (void *)(uintptr_t)schemes[0]);
    free_block(fb);
    return (long)ret;
}

/* A block whose totals exceed its 100 symbol slots (nss / nrs are u8 fields the peer sets,
 * block_framework_receiver.h:44-45): only the first 100 slots are populated.  Runs generate
 * (op 0) or recover (op 1) and returns the operation's value; the adapter must refuse the block
 * before touching the device (the reference reads past fec_block_t here). */
long mh_oversized(int xor_scheme, int op, int k_total, int r_total) {
    picoquic_cnx_t cnx;
    protoop_arg_t schemes[2] = {0, 0};
    protoop_arg_t ret = run_protoop(&cnx, op_create(xor_scheme), 0, NULL, schemes);
    if (ret) return (long)ret;
    pquic_fec_block_t *fb = calloc(1, sizeof *fb);
    uint8_t data[64];
    memset(data, 7, sizeof data);
    fb->fec_block_number = 9;
    fb->total_source_symbols = (uint8_t)k_total;
    fb->total_repair_symbols = (uint8_t)r_total;
    const int ns = op ? 90 : (k_total < PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK ? k_total : PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK);
    for (int j = 0; j < ns; j++) fb->source_symbols[j] = mk_source(9, j, data, sizeof data);
    fb->current_source_symbols = (uint8_t)k_total;
    if (op) {  /* counters that pass the reference's preconditions, so only the slot guard stops it */
        fb->current_source_symbols = (uint8_t)(k_total - (r_total < 10 ? r_total : 10));
        for (int i = 0; i < 10 && i < r_total; i++) {
            pquic_repair_symbol_t *rs = mh_malloc(&cnx, sizeof *rs);
            memset(rs, 0, sizeof *rs);
            rs->fpid.raw = (9u << 8) | (uint32_t)i;
            rs->data = mh_malloc(&cnx, sizeof data);
            memcpy(rs->data, data, sizeof data);
            rs->data_length = sizeof data;
            fb->repair_symbols[i] = rs;
            fb->current_repair_symbols++;
        }
    }
    protoop_arg_t in[2] = {(protoop_arg_t)(uintptr_t)fb, schemes[op ? 0 : 1]};
    op_t f = op ? (xor_scheme ? pquic_fec_xor_recover : pquic_fec_rlc_recover)
                : (xor_scheme ? pquic_fec_xor_generate_repair_symbols : pquic_fec_rlc_generate_repair_symbols);
    ret = run_protoop(&cnx, f, 2, in, NULL);
    if (schemes[0] && !xor_scheme) mh_free(&cnx, (void *)(uintptr_t)schemes[0]);
    free_block(fb);
    return (long)ret;
}

void mh_protoop_stats(uint64_t out[5]) {
    pquic_fec_protoop_stats_t s;
    pquic_fec_protoop_stats(&s);
    out[0] = s.generate_calls; out[1] = s.recover_calls; out[2] = s.recovered_symbols;
    out[3] = s.ref_ub_blocks; out[4] = s.errors;
}

/* ------------------------------------------------------------------------------------------
 * Batching adapter (include/pquic_fec_batch.h): blocks built exactly as above, submitted to
 * one batcher, completed through its callback; results read back per ticket.
 * ------------------------------------------------------------------------------------------ */
#include "pquic_fec_batch.h"

typedef struct {
    pquic_fec_block_t *fb;
    pquic_source_symbol_t *before[PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK];
    long ret;
    long order;  /* position among all completions */
    int done, calls, k, r;
    int shared;  /* window block: its source symbols belong to a stream */
} ticket_t;

static pquic_fec_batcher_t *g_batcher;
static ticket_t *g_tickets;
static long g_nt, g_capt;
static picoquic_cnx_t g_bcnx;
static long g_ndone;
/* connections with arenas of their own (mh_batch_connections); mh_batch_use_connection picks the one
 * the next blocks are built and submitted on (-1: g_bcnx, the default arena) */
static picoquic_cnx_t *g_cnxs;
static int g_ncnx;
static picoquic_cnx_t *g_cur = &g_bcnx;

/* n connections, each with an arena of `bytes` registered with the open batcher */
int mh_batch_connections(int n, size_t bytes) {
    g_cnxs = calloc((size_t)n, sizeof *g_cnxs);
    if (!g_cnxs) return -1;
    for (int i = 0; i < n; i++) {
        if (!(g_cnxs[i].arena = arena_new(bytes))) return -1;
        g_ncnx = i + 1;
        if (pquic_fec_batch_register_heap(g_batcher, g_cnxs[i].arena->base, g_cnxs[i].arena->size)) return -1;
    }
    return 0;
}

/* connection i closes: its arena leaves the batcher's registry (its rows are staged from then on) */
int mh_batch_unregister_connection(int i) {
    if (i < 0 || i >= g_ncnx) return -1;
    return pquic_fec_batch_unregister_heap(g_batcher, g_cnxs[i].arena->base);
}

int mh_batch_use_connection(int i) {
    if (i >= g_ncnx) return -1;
    g_cur = i < 0 ? &g_bcnx : &g_cnxs[i];
    return 0;
}

/* arena slots in use of connection i (-1: the default arena) */
long mh_arena_live(int i) {
    const mh_arena_t *a = i < 0 ? g_default_arena : (i < g_ncnx ? g_cnxs[i].arena : NULL);
    return a ? a->live : -1;
}

static void on_done(void *user, pquic_fec_block_t *fb, protoop_arg_t ret) {
    ticket_t *t = &g_tickets[(long)(intptr_t)user];
    (void)fb;
    t->ret = (long)ret;
    t->done = 1;
    t->calls++;
    t->order = g_ndone++;
}

/* completion position of ticket t (-1 before its completion) */
long mh_batch_order(long t) { return g_tickets[t].done ? g_tickets[t].order : -1; }

int mh_batch_open(int device, unsigned batch_blocks, unsigned max_delay_us, unsigned max_symbol, int nstreams,
                  unsigned poll_blocks) {
    pquic_fec_batch_cfg_t cfg = {device, batch_blocks, max_delay_us, max_symbol, nstreams, poll_blocks};
    g_batcher = pquic_fec_batcher_create(&cfg);
    return g_batcher ? 0 : -1;
}

/* registers the default arena (mh_arena_enable) with the open batcher */
int mh_batch_register_arena(void) {
    return g_default_arena ? pquic_fec_batch_register_heap(g_batcher, g_default_arena->base, g_default_arena->size) : -1;
}

static long new_ticket(pquic_fec_block_t *fb, int k, int r) {
    if (g_nt == g_capt) {
        g_capt = g_capt ? 2 * g_capt : 1024;
        g_tickets = realloc(g_tickets, g_capt * sizeof *g_tickets);
    }
    ticket_t *t = &g_tickets[g_nt];
    memset(t, 0, sizeof *t);
    t->fb = fb;
    t->k = k;
    t->r = r;
    return g_nt++;
}

/* returns the ticket (>= 0) or -1 when the batcher refused the block */
long mh_batch_generate(int xor_scheme, uint32_t fbn, int k, int r, const uint8_t *src, const uint16_t *src_len,
                       int src_stride, uint64_t now_us) {
    pquic_fec_block_t *fb = calloc(1, sizeof *fb);
    fb->fec_block_number = fbn;
    for (int j = 0; j < k; j++) fb->source_symbols[j] = mk_source_in(g_cur, fbn, j, src + (size_t)j * src_stride, src_len[j]);
    fb->current_source_symbols = (uint8_t)k;
    fb->total_source_symbols = (uint8_t)k;
    fb->total_repair_symbols = (uint8_t)r;
    long t = new_ticket(fb, k, r);
    g_fail_after = g_fail_next_op;  /* armed from here on: the caller disarms after the completion */
    g_fail_next_op = -1;
    if (pquic_fec_batch_generate(g_batcher, g_cur, fb, xor_scheme, now_us, on_done, (void *)(intptr_t)t)) {
        free_block(fb);
        g_nt--;
        return -1;
    }
    return t;
}

long mh_batch_recover(int xor_scheme, uint32_t fbn, int k, int r, const uint8_t *src, const uint16_t *src_len,
                      const uint8_t *src_present, int src_stride, const uint8_t *rep, const uint16_t *rep_len,
                      const uint8_t *rep_present, const uint64_t *rep_fpid, int rep_stride, uint64_t now_us) {
    picoquic_cnx_t *c = g_cur;
    pquic_fec_block_t *fb = calloc(1, sizeof *fb);
    fb->fec_block_number = fbn;
    fb->total_source_symbols = (uint8_t)k;
    fb->total_repair_symbols = (uint8_t)r;
    for (int j = 0; j < k; j++)
        if (src_present[j]) {
            fb->source_symbols[j] = mk_source_in(c, fbn, j, src + (size_t)j * src_stride, src_len[j]);
            fb->current_source_symbols++;
        }
    for (int i = 0; i < r; i++)
        if (rep_present[i]) {
            pquic_repair_symbol_t *rs = mh_malloc(c, sizeof *rs);
            memset(rs, 0, sizeof *rs);
            rs->fpid.raw = rep_fpid[i];
            rs->data = mh_malloc(c, rep_len[i]);
            memcpy(rs->data, rep + (size_t)i * rep_stride, rep_len[i]);
            rs->data_length = rep_len[i];
            fb->repair_symbols[i] = rs;
            fb->current_repair_symbols++;
        }
    long t = new_ticket(fb, k, r);
    memcpy(g_tickets[t].before, fb->source_symbols, sizeof g_tickets[t].before);
    if (pquic_fec_batch_recover(g_batcher, c, fb, xor_scheme, now_us, on_done, (void *)(intptr_t)t)) {
        free_block(fb);
        g_nt--;
        return -1;
    }
    return t;
}

/* Sliding-window sender streams: each stream owns its source symbols (the framework's window,
 * window_framework_sender.h), and window blocks point into it, so consecutive windows share symbols.
 * Each stream is its own connection.  Streams live until mh_batch_close. */
enum { MH_MAX_STREAMS = 256 };
static pquic_source_symbol_t **g_stream[MH_MAX_STREAMS];
static int g_stream_len[MH_MAX_STREAMS], g_nstreams;
static picoquic_cnx_t g_stream_cnx[MH_MAX_STREAMS];

/* returns the stream id or -1; symbol x carries source FPID first_fpid + x */
int mh_stream_open(int nsym, const uint8_t *data, const uint16_t *len, int stride, uint32_t first_fpid) {
    if (g_nstreams >= MH_MAX_STREAMS || nsym < 1) return -1;
    pquic_source_symbol_t **v = calloc((size_t)nsym, sizeof *v);
    if (!v) return -1;
    for (int x = 0; x < nsym; x++) {
        v[x] = mk_source(0, 0, data + (size_t)x * stride, len[x]);
        v[x]->fpid.raw = first_fpid + (uint32_t)x;
    }
    g_stream[g_nstreams] = v;
    g_stream_len[g_nstreams] = nsym;
    return g_nstreams++;
}

/* window block over symbols [start, start + k) of a stream, submitted as the window sender would
 * (block number 0); returns the ticket or -1 */
long mh_batch_generate_window(int stream, int start, int k, int r, uint64_t now_us) {
    if (stream < 0 || stream >= g_nstreams || start < 0 || start + k > g_stream_len[stream]) return -1;
    pquic_fec_block_t *fb = calloc(1, sizeof *fb);
    for (int j = 0; j < k; j++) fb->source_symbols[j] = g_stream[stream][start + j];
    fb->current_source_symbols = fb->total_source_symbols = (uint8_t)k;
    fb->total_repair_symbols = (uint8_t)r;
    long t = new_ticket(fb, k, r);
    g_tickets[t].shared = 1;
    if (pquic_fec_batch_generate_window(g_batcher, &g_stream_cnx[stream], fb, now_us, on_done, (void *)(intptr_t)t)) {
        memset(fb->source_symbols, 0, sizeof fb->source_symbols);
        free_block(fb);
        g_nt--;
        return -1;
    }
    return t;
}

int mh_batch_poll(uint64_t now_us) { return pquic_fec_batch_poll(g_batcher, now_us); }
int mh_batch_drain(void) { return pquic_fec_batch_drain(g_batcher); }

/* ticket state: -1 not done; else the operation's value.  calls = number of done() calls */
long mh_batch_status(long t, int *calls) {
    *calls = g_tickets[t].calls;
    return g_tickets[t].done ? g_tickets[t].ret : -1;
}

/* generate result: repairs of ticket t */
void mh_batch_repairs(long t, uint8_t *rep_out, uint16_t *rep_len, uint64_t *rep_fpid, int rep_stride) {
    ticket_t *tk = &g_tickets[t];
    for (int i = 0; i < tk->r; i++) {
        pquic_repair_symbol_t *rs = tk->fb->repair_symbols[i];
        rep_len[i] = rs ? rs->data_length : 0;
        rep_fpid[i] = rs ? rs->fpid.raw : 0;
        if (rs) memcpy(rep_out + (size_t)i * rep_stride, rs->data, rs->data_length);
    }
}

/* recover result: inserted sources of ticket t (as mh_recover reports them) */
void mh_batch_recovered(long t, uint8_t *out, uint16_t *out_len, uint8_t *recovered, int out_stride, int *cur_ss,
                        uint32_t *out_fpid) {
    ticket_t *tk = &g_tickets[t];
    for (int j = 0; j < tk->k; j++) {
        pquic_source_symbol_t *ss = tk->fb->source_symbols[j];
        recovered[j] = ss && ss != tk->before[j];
        out_len[j] = recovered[j] ? ss->data_length : 0;
        if (out_fpid) out_fpid[j] = recovered[j] ? ss->fpid.raw : 0;
        if (recovered[j]) memcpy(out + (size_t)j * out_stride, ss->data, ss->data_length);
    }
    *cur_ss = tk->fb->current_source_symbols;
}

void mh_batch_get_stats(uint64_t out[15]) {
    pquic_fec_batch_stats_t s;
    pquic_fec_batch_get_stats(g_batcher, &s);
    out[0] = s.submitted; out[1] = s.completed; out[2] = s.batches; out[3] = s.flushed_full;
    out[4] = s.flushed_deadline; out[5] = s.flushed_drain; out[6] = s.immediate; out[7] = s.engine_errors;
    out[8] = s.windows; out[9] = s.window_rows; out[10] = s.rows_in_place; out[11] = s.rows_staged;
    out[12] = s.jobs_allocated; out[13] = s.job_alloc_us; out[14] = s.deadline_holds;
}

/* frees every ticket's block and the batcher */
void mh_batch_close(void) {
    pquic_fec_batcher_destroy(g_batcher);
    g_batcher = NULL;
    for (long t = 0; t < g_nt; t++) {
        if (g_tickets[t].shared) memset(g_tickets[t].fb->source_symbols, 0, sizeof g_tickets[t].fb->source_symbols);
        free_block(g_tickets[t].fb);
    }
    picoquic_cnx_t c = {0};
    for (int i = 0; i < g_nstreams; i++) {
        for (int x = 0; x < g_stream_len[i]; x++) { mh_free(&c, g_stream[i][x]->data); mh_free(&c, g_stream[i][x]); }
        free(g_stream[i]);
        g_stream[i] = NULL;
    }
    g_nstreams = 0;
    free(g_tickets);
    g_tickets = NULL;
    g_nt = g_capt = 0;
    g_ndone = 0;
    for (int i = 0; i < g_ncnx; i++)  /* the batcher unregistered them; nothing lives in them any more */
        if (g_cnxs[i].arena && !g_cnxs[i].arena->live) arena_drop(g_cnxs[i].arena);
    free(g_cnxs);
    g_cnxs = NULL;
    g_ncnx = 0;
    g_cur = &g_bcnx;
}

/* ------------------------------------------------------------------------------------------
 * Recovered packets -> congestion control (include/pquic_fec_cc.h): the same scripted transport
 * as oracle/ref/ref_driver.c's ref_cc_scenario, bound through pquic_fec_transport_api_t, with the
 * same event log, so the product's calls can be compared with the reference pluglet's.
 * ------------------------------------------------------------------------------------------ */
#include "pquic_fec_cc.h"

typedef struct { uint64_t pn; int pure_ack, needed; } cc_pkt_t;
static cc_pkt_t *g_ccp;
static int g_ccn;
static uint64_t g_srtt, g_latest, *g_ev;
static int g_nev, g_maxev;
static int g_path_obj, g_ctx_obj;

static void ev(uint64_t k, uint64_t a, uint64_t b, uint64_t c) {
    if (g_nev < g_maxev) { uint64_t *e = g_ev + 4 * g_nev; e[0] = k; e[1] = a; e[2] = b; e[3] = c; }
    g_nev++;
}
static void *t_path(picoquic_cnx_t *cnx) { (void)cnx; return &g_path_obj; }
static void *t_ctx(void *path) { (void)path; return &g_ctx_obj; }
static void *t_oldest(void *ctx) { (void)ctx; return g_ccn ? &g_ccp[0] : NULL; }
static void *t_next(void *p) { cc_pkt_t *q = p; return q + 1 < g_ccp + g_ccn ? q + 1 : NULL; }
static uint64_t t_pn(void *p) { return ((cc_pkt_t *)p)->pn; }
static int t_pure(void *p) { return ((cc_pkt_t *)p)->pure_ack; }
static uint64_t t_latest(void *ctx) { (void)ctx; return g_latest; }
static void t_set_latest(void *ctx, uint64_t v) { (void)ctx; g_latest = v; ev(5, v, 0, 0); }
static uint64_t t_srtt(void *path) { (void)path; return g_srtt; }
static int t_needed(picoquic_cnx_t *cnx, void *p, uint64_t now, int *tb) {
    (void)cnx;
    ev(1, ((cc_pkt_t *)p)->pn, now, (uint64_t)*tb);
    *tb = 0;
    return ((cc_pkt_t *)p)->needed;
}
static void t_lost(picoquic_cnx_t *cnx, void *p, void *path) { (void)cnx; ev(2, ((cc_pkt_t *)p)->pn, path == &g_path_obj, 0); }
static void t_deq(picoquic_cnx_t *cnx, void *p, int f) { (void)cnx; ev(3, ((cc_pkt_t *)p)->pn, (uint64_t)f, 0); }
static void t_notify(picoquic_cnx_t *cnx, void *path, int n, uint64_t rtt, uint64_t nb, uint64_t lost, uint64_t now) {
    (void)cnx; (void)path; (void)rtt; (void)nb;
    ev(4, (uint64_t)n, lost, now);
}

int mh_cc_scenario(int n, const uint64_t *pns, const uint8_t *pure, const uint8_t *needed, uint64_t srtt,
                   uint64_t latest, uint64_t now, uint32_t *buf_start, uint32_t *buf_size, uint64_t *buf_pns,
                   uint64_t *events, int maxev, uint64_t *latest_out) {
    static const pquic_fec_transport_api_t t = {t_path, t_ctx, t_oldest, t_next, t_pn, t_pure, t_latest,
                                                t_set_latest, t_srtt, t_needed, t_lost, t_deq, t_notify};
    cc_pkt_t *pk = calloc((size_t)(n ? n : 1), sizeof *pk);
    for (int i = 0; i < n; i++) { pk[i].pn = pns[i]; pk[i].pure_ack = pure[i]; pk[i].needed = needed[i]; }
    g_ccp = pk; g_ccn = n; g_srtt = srtt; g_latest = latest; g_ev = events; g_nev = 0; g_maxev = maxev;
    pquic_fec_recovered_packets_buffer_t b;
    b.start = *buf_start;
    b.size = *buf_size;
    memcpy(b.packet_numbers, buf_pns, sizeof b.packet_numbers);
    picoquic_cnx_t cnx;
    pquic_fec_maybe_notify_recovered_packets_to_cc(&cnx, &t, &b, now);
    *buf_start = b.start;
    *buf_size = b.size;
    memcpy(buf_pns, b.packet_numbers, sizeof b.packet_numbers);
    *latest_out = g_latest;
    free(pk);
    return g_nev;
}

void mh_process_recovered(const uint64_t *pns, int n, uint32_t *buf_start, uint32_t *buf_size, uint64_t *buf_pns) {
    pquic_fec_recovered_packets_buffer_t b;
    b.start = *buf_start;
    b.size = *buf_size;
    memcpy(b.packet_numbers, buf_pns, sizeof b.packet_numbers);
    pquic_fec_enqueue_recovered_packets(&b, pns, (uint8_t)n);
    *buf_start = b.start;
    *buf_size = b.size;
    memcpy(buf_pns, b.packet_numbers, sizeof b.packet_numbers);
}
