/*
 * oracle/ref/ref_driver.c -- TEST INFRASTRUCTURE ONLY (this container).
 *
 * Links the reference's own FEC scheme pluglets, compiled in place from
 * /root/reference/plugins/fec/fec_scheme_protoops/*.c by oracle/Makefile, into
 * oracle/_ref/libfecref.so, and drives them the way plugin_run_protoop_internal
 * (picoquic/plugin.c:1279-1450) does: a picoquic_cnx_t whose protoop_inputv / protoop_outputv
 * carry the arguments, read and written by the reference's own accessors -- picoquic/getset.c,
 * compiled in place and linked (get_cnx at :137-148, set_cnx at :370-379; the CC scenario's
 * path, packet context and packets through its get_path / get_pkt_ctx / set_pkt_ctx / get_pkt).
 *
 * Stand-ins, only for what the accessors and pluglets import and the tree cannot provide here:
 *   get_plugin_metadata / set_plugin_metadata (plugin.c, uthash-based) -> the one FEC state slot
 *   picoquic_set_cnx_state (quicctx.c) -> never reached by these pluglets, aborts if it is
 *   my_malloc           -> malloc of max(size, 2100): the plugin allocator hands out
 *                          fixed 2100-B slots (picoquic/memory.c:72-95,181-191) and the
 *                          RLC encoder relies on it (knowns[] is under-allocated,
 *                          rlc_fec_scheme_generate_gf256.c:50); memory.c itself includes the
 *                          absent michelfralloc submodule
 *   my_free / my_memcpy / my_memset -> libc
 *   plugin_run_protoop -> the transport protoops the pluglets call (skip_frame, the CC hooks)
 * Recover runs in a fork()ed child because the reference decoder dereferences x[-1]
 * on some erasure patterns (rlc_fec_scheme_gf256.c:74-77).
 */
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <stddef.h>
#include <stdio.h>
#include "picoquic_internal.h"   /* picoquic_cnx_t / path / packet context as getset.c sees them */
#include "fec/fec_protoops.h"     /* fec.h + frame helpers; resolved with -I$(REF)/plugins */
#include "fec/prng/tinymt32.c"

/* ---- the connection the pluglets run on ---- */
static protoop_arg_t g_in[PROTOOPARGS_MAX];
static protoop_arg_t g_out[PROTOOPARGS_MAX];
static picoquic_cnx_t g_cnx;
static protoop_plugin_t g_plugin;       /* the FEC plugin "running" (get_cnx_metadata needs one) */
static picoquic_path_t g_cc_path;       /* the CC scenario's path (below) */
static picoquic_path_t *g_paths[1] = {&g_cc_path};
static int g_cc_active;

/* The connection as plugin_run_protoop_internal hands it to a pluglet (plugin.c:1300-1390): the
 * arguments in protoop_inputv, no outputs yet, the plugin current. */
static picoquic_cnx_t *call_cnx(void) {
    g_cnx.protoop_inputv = g_in;
    g_cnx.protoop_inputc = PROTOOPARGS_MAX;
    g_cnx.protoop_outputv = g_out;
    g_cnx.protoop_outputc_callee = 0;
    g_cnx.current_plugin = &g_plugin;
    g_cnx.path = g_paths;
    g_cnx.nb_paths = 1;
    return &g_cnx;
}

static bpf_state g_state;  /* the FEC plugin's per-connection state (metadata slot FEC_OPAQUE_ID) */
int get_plugin_metadata(protoop_plugin_t *plugin, plugin_struct_metadata_t **metadata, int idx, uint64_t *out) {
    (void)plugin; (void)metadata;
    *out = idx == FEC_OPAQUE_ID ? (uint64_t)(uintptr_t)&g_state : 0;
    return 0;
}
int set_plugin_metadata(protoop_plugin_t *plugin, plugin_struct_metadata_t **metadata, int idx, uint64_t val) {
    (void)plugin; (void)metadata; (void)idx; (void)val;
    return 0;
}
void picoquic_set_cnx_state(picoquic_cnx_t *cnx, picoquic_state_enum state) {
    (void)cnx; (void)state;
    fprintf(stderr, "ref_driver: picoquic_set_cnx_state reached\n");
    abort();
}
void *my_malloc(picoquic_cnx_t *cnx, unsigned int size) {
    (void)cnx;
    return malloc(size < 2100 ? 2100 : size);
}
void my_free(picoquic_cnx_t *cnx, void *ptr) { (void)cnx; free(ptr); }
void *my_memcpy(void *d, const void *s, size_t n) { return memcpy(d, s, n); }
void *my_memset(void *d, int c, size_t n) { return memset(d, c, n); }

/* ---- the reference pluglets, renamed per TU by the Makefile ---- */
protoop_arg_t rlc_create(picoquic_cnx_t *cnx);
protoop_arg_t rlc_encode(picoquic_cnx_t *cnx);
protoop_arg_t rlc_decode(picoquic_cnx_t *cnx);
protoop_arg_t xor_create(picoquic_cnx_t *cnx);
protoop_arg_t xor_encode(picoquic_cnx_t *cnx);
protoop_arg_t xor_decode(picoquic_cnx_t *cnx);

typedef struct { uint8_t **table_mul; uint8_t *table_inv; } ref_rlc_scheme_t;
static ref_rlc_scheme_t *g_scheme;

static ref_rlc_scheme_t *scheme(void) {
    if (!g_scheme) {
        memset(g_out, 0, sizeof g_out);
        if (rlc_create(call_cnx()) == 0) g_scheme = (ref_rlc_scheme_t *)g_out[0];
    }
    return g_scheme;
}

int ref_gf_tables(uint8_t *mul, uint8_t *inv) {
    ref_rlc_scheme_t *s = scheme();
    if (!s) return -1;
    for (int a = 0; a < 256; a++) memcpy(mul + 256 * a, s->table_mul[a], 256);
    memcpy(inv, s->table_inv, 256);
    return 0;
}

int ref_create_outputs(int xor_scheme, uint64_t *out0, uint64_t *out1) {
    memset(g_out, 0, sizeof g_out);
    int ret = (int)(xor_scheme ? xor_create(call_cnx()) : rlc_create(call_cnx()));
    *out0 = g_out[0]; *out1 = g_out[1];
    return ret;
}

void ref_tinymt32(uint32_t seed, int n, uint32_t *out) {
    tinymt32_t t;
    t.mat1 = 0x8f7011ee; t.mat2 = 0xfc78ff1f; t.tmat = 0x3793fdff;
    tinymt32_init(&t, seed);
    for (int i = 0; i < n; i++) out[i] = tinymt32_generate_uint32(&t);
}

static source_symbol_t *mk_source(uint32_t fbn, int j, const uint8_t *data, uint16_t len) {
    source_symbol_t *s = my_malloc(NULL, sizeof *s);
    memset(s, 0, sizeof *s);
    s->fec_block_offset = (uint8_t)j;
    s->fec_block_number = fbn;
    s->data = my_malloc(NULL, len);
    memcpy(s->data, data, len);
    s->data_length = len;
    return s;
}

/* Encode one block.  rep_out receives r * max_len bytes; meta_out per repair:
 * [raw fpid u64, data_length].  Returns the pluglet's return code. */
int ref_encode(int xor_scheme, uint32_t fbn, int k, int r, const uint8_t *src,
               const uint16_t *src_len, int src_stride, uint8_t *rep_out, int rep_stride,
               uint64_t *fpid_out, uint16_t *len_out) {
    fec_block_t *fb = calloc(1, sizeof *fb);
    fb->fec_block_number = fbn;
    fb->total_source_symbols = (uint8_t)k;
    fb->total_repair_symbols = (uint8_t)r;
    for (int j = 0; j < k; j++)
        fb->source_symbols[j] = mk_source(fbn, j, src + (size_t)j * src_stride, src_len[j]);
    fb->current_source_symbols = (uint8_t)k;
    g_in[0] = (protoop_arg_t)fb;
    g_in[1] = (protoop_arg_t)scheme();
    int ret = (int)(xor_scheme ? xor_encode(call_cnx()) : rlc_encode(call_cnx()));
    if (ret == 0) {
        for (int i = 0; i < r; i++) {
            repair_symbol_t *rs = fb->repair_symbols[i];
            if (!rs) { len_out[i] = 0; fpid_out[i] = 0; continue; }
            memcpy(rep_out + (size_t)i * rep_stride, rs->data, rs->data_length);
            len_out[i] = rs->data_length;
            fpid_out[i] = rs->repair_fec_payload_id.raw;
        }
    }
    return ret;
}

/* Recover one block in a child process.
 * src / rep: dense [k][stride] / [r][stride]; presence bytes per symbol.
 * rep_fpid: raw repair FPIDs (the seed is its low 32 bits, rlc_fec_scheme_gf256.c:200).
 * out: [k][out_stride]; recovered[j] = 1 when the pluglet inserted source j, out_fpid[j] (may
 * be NULL) its source FPID raw value.
 * Returns the pluglet's return code, or -1000 - signal when the child died. */
int ref_decode(int xor_scheme, uint32_t fbn, int k, int r, const uint8_t *src,
               const uint16_t *src_len, const uint8_t *src_present, int src_stride,
               const uint8_t *rep, const uint16_t *rep_len, const uint8_t *rep_present,
               const uint64_t *rep_fpid, int rep_stride, uint8_t *out, uint16_t *out_len,
               uint8_t *recovered, int out_stride, uint32_t *out_fpid) {
    size_t shm_len = (size_t)k * out_stride + (size_t)k * 7 + 64;
    uint8_t *shm = mmap(NULL, shm_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (shm == MAP_FAILED) return -2000;
    memset(shm, 0, shm_len);
    pid_t pid = fork();
    if (pid == 0) {
        fec_block_t *fb = calloc(1, sizeof *fb);
        fb->fec_block_number = fbn;
        fb->total_source_symbols = (uint8_t)k;
        fb->total_repair_symbols = (uint8_t)r;
        for (int j = 0; j < k; j++)
            if (src_present[j]) {
                fb->source_symbols[j] = mk_source(fbn, j, src + (size_t)j * src_stride, src_len[j]);
                fb->current_source_symbols++;
            }
        for (int i = 0; i < r; i++)
            if (rep_present[i]) {
                repair_symbol_t *rs = my_malloc(NULL, sizeof *rs);
                memset(rs, 0, sizeof *rs);
                rs->repair_fec_payload_id.raw = rep_fpid[i];
                rs->data = my_malloc(NULL, rep_len[i]);
                memcpy(rs->data, rep + (size_t)i * rep_stride, rep_len[i]);
                rs->data_length = rep_len[i];
                fb->repair_symbols[i] = rs;
                fb->current_repair_symbols++;
            }
        source_symbol_t *before[MAX_SYMBOLS_PER_FEC_BLOCK];
        memcpy(before, fb->source_symbols, sizeof before);
        g_in[0] = (protoop_arg_t)fb;
        g_in[1] = (protoop_arg_t)scheme();
        int ret = (int)(xor_scheme ? xor_decode(call_cnx()) : rlc_decode(call_cnx()));
        int32_t *hdr = (int32_t *)shm;
        hdr[0] = ret;
        uint8_t *rec = shm + 64, *lens = rec + k, *data = lens + 2 * (size_t)k;
        uint8_t *fps = data + (size_t)k * out_stride;
        for (int j = 0; j < k; j++) {
            source_symbol_t *ss = fb->source_symbols[j];
            if (ss && ss != before[j]) {
                rec[j] = 1;
                uint16_t L = ss->data_length;
                memcpy(lens + 2 * j, &L, 2);
                memcpy(fps + 4 * j, &ss->source_fec_payload_id.raw, 4);
                memcpy(data + (size_t)j * out_stride, ss->data, L > out_stride ? out_stride : L);
            }
        }
        _exit(0);
    }
    int status = 0;
    waitpid(pid, &status, 0);
    int ret;
    if (WIFEXITED(status) && WEXITSTATUS(status) == 0) {
        ret = ((int32_t *)shm)[0];
        uint8_t *rec = shm + 64, *lens = rec + k, *data = lens + 2 * (size_t)k;
        uint8_t *fps = data + (size_t)k * out_stride;
        for (int j = 0; j < k; j++) {
            recovered[j] = rec[j];
            memcpy(&out_len[j], lens + 2 * j, 2);
            if (out_fpid) memcpy(&out_fpid[j], fps + 4 * j, 4);
            if (rec[j]) memcpy(out + (size_t)j * out_stride, data + (size_t)j * out_stride, out_len[j]);
        }
    } else {
        ret = WIFSIGNALED(status) ? -1000 - WTERMSIG(status) : -1000;
        memset(recovered, 0, (size_t)k);
    }
    munmap(shm, shm_len);
    return ret;
}

/* Batched encode for the calibration leg (no fork): same layout as the device engine. */
int ref_rlc_encode_batch(const uint8_t *src, uint8_t *rep, uint64_t nblocks, int k, int r,
                         int L, uint32_t fbn_base) {
    uint16_t lens[256], rl[256];
    uint64_t fp[256];
    for (int j = 0; j < k; j++) lens[j] = (uint16_t)L;
    for (uint64_t b = 0; b < nblocks; b++) {
        fec_block_t fb;
        memset(&fb, 0, sizeof fb);
        fb.fec_block_number = (uint32_t)((fbn_base + b) & 0xffffff);
        fb.total_source_symbols = (uint8_t)k;
        fb.total_repair_symbols = (uint8_t)r;
        fb.current_source_symbols = (uint8_t)k;
        source_symbol_t ss[256];
        for (int j = 0; j < k; j++) {
            memset(&ss[j], 0, sizeof ss[j]);
            ss[j].data = (uint8_t *)src + (b * k + j) * L;
            ss[j].data_length = (uint16_t)L;
            fb.source_symbols[j] = &ss[j];
        }
        g_in[0] = (protoop_arg_t)&fb;
        g_in[1] = (protoop_arg_t)scheme();
        if (rlc_encode(call_cnx()) != 0) return -1;
        for (int i = 0; i < r; i++) {
            memcpy(rep + (b * r + i) * L, fb.repair_symbols[i]->data, L);
            my_free(NULL, fb.repair_symbols[i]->data);
            my_free(NULL, fb.repair_symbols[i]);
        }
    }
    (void)lens; (void)rl; (void)fp;
    return 0;
}

/* Layout facts the product's layout-compatible header must match (fec.h:44-130). */
int ref_layout(uint64_t *out) {
    out[0] = sizeof(fec_block_t);
    out[1] = sizeof(source_symbol_t);
    out[2] = sizeof(repair_symbol_t);
    out[3] = offsetof(fec_block_t, source_symbols);
    out[4] = offsetof(fec_block_t, repair_symbols);
    out[5] = offsetof(source_symbol_t, data);
    out[6] = offsetof(repair_symbol_t, data);
    out[7] = sizeof(repair_fpid_t);
    return 8;
}

/* ---- frame codecs ---------------------------------------------------
 * FEC frame header and SFPID frame: the reference's own inline helpers (fec.h:175-194,
 * fec_protoops.h:92-100).  RECOVERED frame: the reference pluglets write_simple_recovered_frame.c
 * and parse_simple_recovered_frame.c, compiled in place and run through the stubs above. */
int ref_write_fec_frame_header(int fin, int data_length, int offset, uint64_t fpid_raw, int nss, int nrs,
                               uint8_t *out) {
    fec_frame_header_t h;
    memset(&h, 0, sizeof h);
    h.fin_bit = fin;
    h.data_length = data_length;
    h.offset = offset;
    h.repair_fec_payload_id.raw = fpid_raw;
    h.nss = nss;
    h.nrs = nrs;
    write_fec_frame_header(&h, out);
    return 1 + (int)sizeof(fec_frame_header_t);
}

void ref_parse_fec_frame_header(const uint8_t *in, uint64_t *fields) {
    fec_frame_header_t h;
    memset(&h, 0, sizeof h);
    parse_fec_frame_header(&h, (uint8_t *)in + 1);
    fields[0] = h.fin_bit;
    fields[1] = h.data_length;
    fields[2] = h.offset;
    fields[3] = h.repair_fec_payload_id.raw;
    fields[4] = h.nss;
    fields[5] = h.nrs;
}

int ref_write_sfpid_frame(uint32_t raw, uint8_t *out, size_t bytes_max) {
    source_fpid_frame_t f;
    size_t consumed = 0;
    f.source_fpid.raw = raw;
    int ret = helper_write_source_fpid_frame(NULL, &f, out, bytes_max, &consumed);
    return ret ? -ret : (int)consumed;
}

uint32_t ref_parse_sfpid_frame(const uint8_t *in) {
    source_fpid_frame_t f;
    parse_sfpid_frame(&f, (uint8_t *)in + 1);
    return f.source_fpid.raw;
}

protoop_arg_t ref_write_recovered_frame(picoquic_cnx_t *cnx);
protoop_arg_t ref_parse_recovered_frame(picoquic_cnx_t *cnx);

/* returns the pluglet's value; *consumed = output[0] */
long ref_write_recovered(const uint64_t *packets, int n, uint8_t *bytes, long bytes_len, long *consumed) {
    recovered_packets_t *rp = malloc(sizeof *rp);
    rp->packets = malloc(sizeof(uint64_t) * (n ? n : 1));
    memcpy(rp->packets, packets, sizeof(uint64_t) * n);
    rp->number_of_packets = (uint8_t)n;
    memset(g_in, 0, sizeof g_in);
    memset(g_out, 0, sizeof g_out);
    g_in[0] = (protoop_arg_t)bytes;
    g_in[1] = (protoop_arg_t)(bytes + bytes_len);
    g_in[2] = (protoop_arg_t)rp;
    long ret = (long)ref_write_recovered_frame(call_cnx());  /* frees rp */
    *consumed = (long)g_out[0];
    return ret;
}

/* returns bytes consumed (parse return - bytes) or -1 for NULL; packets/n from output[0] */
long ref_parse_recovered(const uint8_t *bytes, long bytes_len, uint64_t *packets, int *n) {
    memset(g_in, 0, sizeof g_in);
    memset(g_out, 0, sizeof g_out);
    g_in[0] = (protoop_arg_t)bytes;
    g_in[1] = (protoop_arg_t)(bytes + bytes_len);
    protoop_arg_t end = ref_parse_recovered_frame(call_cnx());
    uint8_t *sp = (uint8_t *)g_out[0];
    *n = 0;
    if (sp) {
        *n = sp[0];
        memcpy(packets, sp + 1, sizeof(uint64_t) * sp[0]);
        free(sp);
    }
    return end ? (long)((const uint8_t *)end - bytes) : -1;
}

/* ---- source-symbol capture: protoops/packet_payload_to_source_symbol.c ----
 * The pluglet walks the packet payload with the transport's skip_frame protoop
 * (helper_skip_frame, plugins/helpers.h:234-245).  The transport's frame parser is not part of
 * this path, so the driver answers skip_frame with a synthetic grammar shared with
 * tests/test_frames.py: PADDING (0x00) consumes its run of zero bytes (as picoquic's
 * skip_frame does); every other type is [type][len][len bytes], capped at the payload end.
 * The pluglet's bpf_state write (state->current_symbol_length) goes to a local state that
 * get_cnx_metadata hands out. */
int ref_skip_frame_synthetic(const uint8_t *bytes, size_t bytes_max, size_t *consumed) {
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

static protoop_arg_t cc_protoop(const char *pid, protoop_params_t *pp);
protoop_arg_t plugin_run_protoop(picoquic_cnx_t *cnx, protoop_params_t *pp, char *pid_str, protoop_id_t *pid) {
    (void)cnx; (void)pid;
    if (g_cc_active) return cc_protoop(pid_str, pp);
    if (strcmp(pid_str, PROTOOPID_NOPARAM_SKIP_FRAME) == 0) {
        size_t consumed = 0;
        int ret = ref_skip_frame_synthetic((const uint8_t *)pp->inputv[0], (size_t)pp->inputv[1], &consumed);
        pp->outputv[0] = (protoop_arg_t)consumed;
        pp->outputv[1] = 0;
        return (protoop_arg_t)ret;
    }
    return 0;
}

protoop_arg_t ref_packet_payload_to_source_symbol(picoquic_cnx_t *cnx);

/* returns the pluglet's value (symbol length); the symbol is written to buffer */
long ref_payload_to_source_symbol(const uint8_t *payload, uint32_t len, uint64_t pn, uint8_t *buffer,
                                  uint32_t *state_len) {
    memset(g_in, 0, sizeof g_in);
    memset(g_out, 0, sizeof g_out);
    g_in[0] = (protoop_arg_t)payload;
    g_in[1] = (protoop_arg_t)buffer;
    g_in[2] = (protoop_arg_t)len;
    g_in[3] = (protoop_arg_t)pn;
    long ret = (long)ref_packet_payload_to_source_symbol(call_cnx());
    *state_len = g_state.current_symbol_length;
    return ret;
}

/* ---- CPU baseline: the reference pluglets themselves on every host core --------------------------
 * bench.py's cpu_baseline leg ("kind": "reference").  The driver keeps its protoop arguments in
 * globals (g_in / g_out above), so the workers are fork()ed processes, one per core, each running
 * a contiguous share of the sample: RLC encode of its blocks (rlc_fec_scheme_generate_gf256.c:24-77,
 * block numbers fbn_base + b), then RLC decode of the same blocks with the erasures of sp[]
 * (rlc_fec_scheme_gf256.c:134-251; recovered symbols are allocated by the pluglet and freed here,
 * as the framework frees them).  Blocks flagged in skip[] are patterns on which the reference
 * dereferences x[-1] (flagged by the caller's screen): they are encoded but not
 * decoded.  The workers start together on a shared flag; out[0] = wall seconds from the start to
 * the last worker's exit, out[1] = the slowest worker's own compute seconds, out[2] = blocks
 * decoded.  Returns 0, or -1 if a worker failed. */
#include <time.h>

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static long ref_work_range(const uint8_t *src, uint8_t *rep, uint64_t b0, uint64_t b1, int k, int r, int L,
                           uint32_t fbn_base, const uint64_t *sp, const uint8_t *skip) {
    source_symbol_t ss[256];
    repair_symbol_t rs[256];
    long decoded = 0;
    for (uint64_t b = b0; b < b1; b++) {  /* encode */
        fec_block_t fb;
        memset(&fb, 0, sizeof fb);
        fb.fec_block_number = (uint32_t)((fbn_base + b) & 0xffffff);
        fb.total_source_symbols = (uint8_t)k;
        fb.total_repair_symbols = (uint8_t)r;
        fb.current_source_symbols = (uint8_t)k;
        for (int j = 0; j < k; j++) {
            memset(&ss[j], 0, sizeof ss[j]);
            ss[j].data = (uint8_t *)src + (b * k + j) * (size_t)L;
            ss[j].data_length = (uint16_t)L;
            fb.source_symbols[j] = &ss[j];
        }
        g_in[0] = (protoop_arg_t)&fb;
        g_in[1] = (protoop_arg_t)scheme();
        if (rlc_encode(call_cnx()) != 0) return -1;
        for (int i = 0; i < r; i++) {
            memcpy(rep + ((b - b0) * r + i) * (size_t)L, fb.repair_symbols[i]->data, L);
            my_free(NULL, fb.repair_symbols[i]->data);
            my_free(NULL, fb.repair_symbols[i]);
        }
    }
    for (uint64_t b = b0; b < b1; b++) {  /* decode */
        if (skip[b]) continue;
        fec_block_t fb;
        memset(&fb, 0, sizeof fb);
        const uint32_t fbn = (uint32_t)((fbn_base + b) & 0xffffff);
        fb.fec_block_number = fbn;
        fb.total_source_symbols = (uint8_t)k;
        fb.total_repair_symbols = (uint8_t)r;
        for (int j = 0; j < k; j++)
            if ((sp[2 * b + (j >> 6)] >> (j & 63)) & 1) {
                memset(&ss[j], 0, sizeof ss[j]);
                ss[j].data = (uint8_t *)src + (b * k + j) * (size_t)L;
                ss[j].data_length = (uint16_t)L;
                fb.source_symbols[j] = &ss[j];
                fb.current_source_symbols++;
            }
        for (int i = 0; i < r; i++) {
            memset(&rs[i], 0, sizeof rs[i]);
            rs[i].repair_fec_payload_id.raw = ((uint64_t)fbn << 8) | (uint64_t)i;
            rs[i].data = rep + ((b - b0) * r + i) * (size_t)L;
            rs[i].data_length = (uint16_t)L;
            fb.repair_symbols[i] = &rs[i];
            fb.current_repair_symbols++;
        }
        source_symbol_t *before[MAX_SYMBOLS_PER_FEC_BLOCK];
        memcpy(before, fb.source_symbols, sizeof before);
        g_in[0] = (protoop_arg_t)&fb;
        g_in[1] = (protoop_arg_t)scheme();
        if (rlc_decode(call_cnx()) != 0) return -1;
        for (int j = 0; j < k; j++)
            if (fb.source_symbols[j] && fb.source_symbols[j] != before[j]) {
                my_free(NULL, fb.source_symbols[j]->data);
                my_free(NULL, fb.source_symbols[j]);
            }
        decoded++;
    }
    return decoded;
}

int ref_cpu_baseline(int nworkers, const uint8_t *src, uint64_t nblocks, int k, int r, int L, uint32_t fbn_base,
                     const uint64_t *sp, const uint8_t *skip, int passes, double *out) {
    if (nworkers < 1 || nworkers > 4096 || !scheme()) return -1;
    size_t shm_len = 64 + (size_t)nworkers * 16;
    uint8_t *shm = mmap(NULL, shm_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (shm == MAP_FAILED) return -1;
    memset(shm, 0, shm_len);
    volatile int *go = (volatile int *)shm;
    double *wt = (double *)(shm + 64);
    long *wd = (long *)(shm + 64 + (size_t)nworkers * 8);
    pid_t *pids = calloc((size_t)nworkers, sizeof *pids);
    int started = 0;
    for (; started < nworkers; started++) {
        pid_t pid = fork();
        if (pid < 0) break;
        if (pid == 0) {
            const uint64_t b0 = nblocks * (uint64_t)started / (uint64_t)nworkers;
            const uint64_t b1 = nblocks * (uint64_t)(started + 1) / (uint64_t)nworkers;
            uint8_t *rep = malloc((b1 - b0 + 1) * (size_t)r * L);
            while (!*go) { }
            const double t0 = now_s();
            long dec = 0;
            for (int p = 0; p < passes && dec >= 0; p++) {
                const long d = ref_work_range(src, rep, b0, b1, k, r, L, fbn_base, sp, skip);
                dec = d < 0 ? -1 : dec + d;
            }
            wt[started] = now_s() - t0;
            wd[started] = dec;
            _exit(dec < 0 ? 1 : 0);
        }
        pids[started] = pid;
    }
    __sync_synchronize();
    const double t0 = now_s();
    *go = 1;
    int ok = started == nworkers;
    for (int i = 0; i < started; i++) {
        int status = 0;
        waitpid(pids[i], &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) ok = 0;
    }
    const double wall = now_s() - t0;
    double mx = 0;
    long dec = 0;
    for (int i = 0; i < started; i++) {
        if (wt[i] > mx) mx = wt[i];
        dec += wd[i];
    }
    out[0] = wall;
    out[1] = mx;
    out[2] = (double)dec;
    free(pids);
    munmap(shm, shm_len);
    return ok ? 0 : -1;
}

/* In-process, one core (no fork): the same work as one ref_cpu_baseline worker; returns the
 * number of blocks decoded, or -1.  bench.py's hook-latency leg divides by it for the reference
 * pluglets' own time per block.  The caller screens out the crash patterns (skip[]). */
long ref_work_serial(const uint8_t *src, uint64_t nblocks, int k, int r, int L, uint32_t fbn_base,
                     const uint64_t *sp, const uint8_t *skip, double *enc_s, double *dec_s) {
    uint8_t *rep = malloc(nblocks * (size_t)r * L + 1);
    if (!rep || !scheme()) return -1;
    uint8_t *none = calloc(nblocks + 1, 1);
    uint8_t *all = malloc(nblocks + 1);
    memset(all, 1, nblocks + 1);
    double t0 = now_s();  /* encode only: every block skipped in the decode half */
    long d = ref_work_range(src, rep, 0, nblocks, k, r, L, fbn_base, sp, all);
    double t1 = now_s();
    /* decode only: re-encode untimed is not possible through ref_work_range, so time both and
     * subtract the encode time measured just before */
    long d2 = ref_work_range(src, rep, 0, nblocks, k, r, L, fbn_base, sp, skip);
    double t2 = now_s();
    *enc_s = t1 - t0;
    *dec_s = (t2 - t1) - (t1 - t0);
    free(rep); free(none); free(all);
    return d < 0 || d2 < 0 ? -1 : d2;
}

/* ---- recovered packets -> congestion control -----------------------------------
 * The reference pluglet protoops/maybe_notify_recovered_packets_to_cc.c (prepare_packet_ready pre-hook,
 * fec_protoops.h:151-184), compiled in place, run against a scripted transport: a retransmit queue of
 * packets (number, pure-ACK flag, "retransmit needed" verdict), one path (smoothed RTT) and its
 * application packet context (latest CC notification time).  Every transport call the pluglet makes
 * is logged as 4 u64: {kind, a, b, c}:
 *   1 retransmit_needed_by_packet(pn, now, timer_based_in)   2 packet_was_lost(pn)
 *   3 dequeue_retransmit_packet(pn, should_free)             4 congestion_algorithm_notify(notification,
 *   5 set latest CC notification time(t)                        lost pn, now) [rtt / bytes are 0] */
static picoquic_packet_t *g_cc_pkts;  /* the retransmit queue, linked through next_packet */
static uint8_t *g_cc_needed;          /* retransmit_needed_by_packet's verdict per packet */
static int g_cc_n;
static uint64_t *g_cc_ev;
static int g_cc_nev, g_cc_maxev;

static picoquic_packet_context_t *cc_ctx(void) { return &g_cc_path.pkt_ctx[picoquic_packet_context_application]; }

static void cc_log(uint64_t k, uint64_t a, uint64_t b, uint64_t c) {
    if (g_cc_nev < g_cc_maxev) {
        uint64_t *e = g_cc_ev + 4 * g_cc_nev;
        e[0] = k; e[1] = a; e[2] = b; e[3] = c;
    }
    g_cc_nev++;
}

/* The transport protoops the pluglet calls.  Event 5 (the pluglet's set_pkt_ctx of the latest CC
 * notification time, which getset.c performs without telling anyone) is logged from the field itself
 * right before the notification it always precedes (fec_protoops.h:171-174: set, then notify, in
 * one branch and nowhere else). */
static protoop_arg_t cc_protoop(const char *pid, protoop_params_t *pp) {
    if (strcmp(pid, PROTOOPID_NOPARAM_RETRANSMIT_NEEDED_BY_PACKET) == 0) {
        picoquic_packet_t *p = (picoquic_packet_t *)pp->inputv[0];
        cc_log(1, p->sequence_number, pp->inputv[1], pp->inputv[2]);
        if (pp->outputv) { pp->outputv[0] = 0; pp->outputv[1] = 0; pp->outputv[2] = 0; }
        return (protoop_arg_t)g_cc_needed[p - g_cc_pkts];
    }
    if (strcmp(pid, PROTOOPID_NOPARAM_PACKET_WAS_LOST) == 0) {
        cc_log(2, ((picoquic_packet_t *)pp->inputv[0])->sequence_number, pp->inputv[1] == (protoop_arg_t)&g_cc_path, 0);
        return 0;
    }
    if (strcmp(pid, PROTOOPID_NOPARAM_DEQUEUE_RETRANSMIT_PACKET) == 0) {
        cc_log(3, ((picoquic_packet_t *)pp->inputv[0])->sequence_number, pp->inputv[1], 0);
        return 0;
    }
    if (strcmp(pid, PROTOOPID_NOPARAM_CONGESTION_ALGORITHM_NOTIFY) == 0) {
        cc_log(5, cc_ctx()->latest_retransmit_cc_notification_time, 0, 0);
        cc_log(4, pp->inputv[1], pp->inputv[4], pp->inputv[5]);
        return 0;
    }
    return (protoop_arg_t)-1;
}

protoop_arg_t ref_prepare_packet_ready(picoquic_cnx_t *cnx);

/* One scenario.  pkts: n x {pn, pure_ack, needed}; buf: {start, size, 50 packet numbers} in/out.
 * Returns the number of events (log holds min(that, maxev)); *latest_out = the final time. */
int ref_cc_scenario(int n, const uint64_t *pns, const uint8_t *pure, const uint8_t *needed, uint64_t srtt,
                    uint64_t latest, uint64_t now, uint32_t *buf_start, uint32_t *buf_size, uint64_t *buf_pns,
                    uint64_t *events, int maxev, uint64_t *latest_out) {
    picoquic_packet_t *pk = calloc((size_t)(n ? n : 1), sizeof *pk);
    uint8_t *nd = calloc((size_t)(n ? n : 1), 1);
    for (int i = 0; i < n; i++) {
        pk[i].sequence_number = pns[i];
        pk[i].is_pure_ack = pure[i] ? 1 : 0;
        pk[i].next_packet = i + 1 < n ? &pk[i + 1] : NULL;
        pk[i].previous_packet = i ? &pk[i - 1] : NULL;
        nd[i] = needed[i];
    }
    memset(&g_cc_path, 0, sizeof g_cc_path);
    g_cc_path.smoothed_rtt = srtt;
    cc_ctx()->retransmit_oldest = n ? &pk[0] : NULL;
    cc_ctx()->retransmit_newest = n ? &pk[n - 1] : NULL;
    cc_ctx()->latest_retransmit_cc_notification_time = latest;
    g_cc_pkts = pk; g_cc_needed = nd; g_cc_n = n;
    g_cc_ev = events; g_cc_nev = 0; g_cc_maxev = maxev;
    memset(&g_state, 0, sizeof g_state);
    g_state.recovered_packets.start = *buf_start;
    g_state.recovered_packets.size = *buf_size;
    memcpy(g_state.recovered_packets.packet_numbers, buf_pns, sizeof g_state.recovered_packets.packet_numbers);
    memset(g_in, 0, sizeof g_in);
    g_in[2] = now;
    g_cc_active = 1;
    ref_prepare_packet_ready(call_cnx());
    g_cc_active = 0;
    *buf_start = g_state.recovered_packets.start;
    *buf_size = g_state.recovered_packets.size;
    memcpy(buf_pns, g_state.recovered_packets.packet_numbers, sizeof g_state.recovered_packets.packet_numbers);
    *latest_out = cc_ctx()->latest_retransmit_cc_notification_time;
    free(pk);
    free(nd);
    return g_cc_nev;
}

protoop_arg_t ref_process_recovered_frame(picoquic_cnx_t *cnx);

/* process_recovered_frame (protoops/process_simple_recovered_frame.c): enqueue a parsed frame's
 * packet numbers ([n][n x u64], as parse_recovered_frame hands them over) into the ring
 * {start, size, 50 pns} (in/out). */
void ref_process_recovered(const uint64_t *pns, int n, uint32_t *buf_start, uint32_t *buf_size, uint64_t *buf_pns) {
    uint8_t *sp = malloc(1 + 8 * (size_t)(n ? n : 1));
    sp[0] = (uint8_t)n;
    memcpy(sp + 1, pns, 8 * (size_t)n);
    memset(&g_state, 0, sizeof g_state);
    g_state.recovered_packets.start = *buf_start;
    g_state.recovered_packets.size = *buf_size;
    memcpy(g_state.recovered_packets.packet_numbers, buf_pns, sizeof g_state.recovered_packets.packet_numbers);
    memset(g_in, 0, sizeof g_in);
    g_in[0] = (protoop_arg_t)sp;
    ref_process_recovered_frame(call_cnx());
    *buf_start = g_state.recovered_packets.start;
    *buf_size = g_state.recovered_packets.size;
    memcpy(buf_pns, g_state.recovered_packets.packet_numbers, sizeof g_state.recovered_packets.packet_numbers);
    free(sp);
}
