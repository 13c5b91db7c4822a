/*
 * pquic_amd/csrc/fec_core.c -- the block <-> row-layout halves of the FEC scheme operations
 * (see fec_core.h).  Host C, like the reference pluglets whose behaviour each function cites.
 */
#include "fec_core.h"

#include <string.h>

#include "fecgpu.h"

/* malloc_repair_symbol (plugins/fec/fec.h:231-244): zeroed struct, fpid, data */
static pquic_repair_symbol_t *new_repair(picoquic_cnx_t *cnx, uint64_t fpid_raw, uint16_t len) {
    pquic_repair_symbol_t *s = g_fec_api.my_malloc(cnx, sizeof *s);
    uint8_t *d = g_fec_api.my_malloc(cnx, len);
    if (!s || !d) {
        if (s) g_fec_api.my_free(cnx, s);
        if (d) g_fec_api.my_free(cnx, d);
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
    pquic_source_symbol_t *s = g_fec_api.my_malloc(cnx, sizeof *s);
    uint8_t *d = g_fec_api.my_malloc(cnx, len);
    if (!s || !d) {
        if (s) g_fec_api.my_free(cnx, s);
        if (d) g_fec_api.my_free(cnx, d);
        return NULL;
    }
    memset(s, 0, sizeof *s);
    s->fpid.raw = fpid_raw;
    s->data = d;
    s->data_length = len;
    return s;
}

int fec_generate_check(const pquic_fec_block_t *fb, int xor_scheme, uint16_t *maxl) {
    const int k = fb->total_source_symbols, r = fb->total_repair_symbols;
    /* rlc_fec_scheme_generate_gf256.c:34-39 / xor_fec_scheme_generate.c:45-50 */
    if ((xor_scheme ? r != 1 : r == 0) || k < 1 || fb->current_source_symbols != fb->total_source_symbols)
        return 1;
    /* fec_block_t holds 100 source and 100 repair pointers (fec.h:8,128-129); the reference would
     * index past them for larger totals (they are u8 fields the peer controls on the receive side) */
    if (k > PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK || r > PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK) return FEC_STAGE_REJECT;
    uint16_t m = 0;
    for (int j = 0; j < k; j++)
        if (fb->source_symbols[j] && fb->source_symbols[j]->data_length > m) m = fb->source_symbols[j]->data_length;
    *maxl = m;
    return 0;
}

void fec_generate_stage(const pquic_fec_block_t *fb, uint8_t *src_rows, uint32_t stride) {
    for (int j = 0; j < fb->total_source_symbols; j++) {  /* zero-padded to max_length (:41-55) */
        uint8_t *row = src_rows + (size_t)j * stride;
        const pquic_source_symbol_t *ss = fb->source_symbols[j];
        const uint16_t n = ss ? ss->data_length : 0;
        if (n) memcpy(row, ss->data, n);
        memset(row + n, 0, stride - n);
    }
}

int fec_generate_alloc(picoquic_cnx_t *cnx, const pquic_fec_block_t *fb, uint16_t maxl,
                       pquic_repair_symbol_t **reps) {
    const uint32_t fbn = fb->fec_block_number & 0xffffffu;
    for (int i = 0; i < fb->total_repair_symbols; i++) {
        /* repair fpid: raw 0, fec_block_number, symbol_number = i, fec_scheme_specific 0
         * (rlc_fec_scheme_generate_gf256.c:57-61; xor_fec_scheme_generate.c:71-75) */
        reps[i] = new_repair(cnx, ((uint64_t)fbn << 8) | (uint64_t)(i & 0xff), maxl);
        if (!reps[i]) return i;
    }
    return fb->total_repair_symbols;
}

protoop_arg_t fec_generate_attach(pquic_fec_block_t *fb, pquic_repair_symbol_t *const *reps, int nalloc) {
    for (int i = 0; i < nalloc; i++) fb->repair_symbols[i] = reps[i];
    return nalloc < fb->total_repair_symbols ? PQUIC_ERROR_MEMORY : 0;
}

protoop_arg_t fec_generate_finish(picoquic_cnx_t *cnx, pquic_fec_block_t *fb, const uint8_t *rep_rows,
                                  uint32_t stride, uint16_t maxl) {
    pquic_repair_symbol_t *reps[PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK];
    const int n = fec_generate_alloc(cnx, fb, maxl, reps);
    for (int i = 0; i < n; i++) memcpy(reps[i]->data, rep_rows + (size_t)i * stride, maxl);
    return fec_generate_attach(fb, reps, n);
}

int fec_recover_check(const pquic_fec_block_t *fb, int xor_scheme, uint16_t *maxl) {
    const int k = fb->total_source_symbols, r = fb->total_repair_symbols;
    if (xor_scheme) {
        if (r != 1 || fb->current_source_symbols + fb->current_repair_symbols != fb->total_source_symbols)
            return 1;  /* xor_fec_scheme.c:45-49 */
        if (k > PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK) return FEC_STAGE_REJECT;
        if (!fb->repair_symbols[0]) return 1;  /* the reference dereferences NULL here (:50-51) */
        *maxl = fb->repair_symbols[0]->data_length;
        return FEC_STAGE_OK;
    }
    if (r == 0 || fb->current_source_symbols == fb->total_source_symbols ||
        fb->current_source_symbols + fb->current_repair_symbols < fb->total_source_symbols)
        return 0;  /* rlc_fec_scheme_gf256.c:140-144 */
    /* totals beyond the block's 100 symbol slots (fec.h:8): the reference reads past them */
    if (k > PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK || r > PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK) return FEC_STAGE_REJECT;
    int first = -1;
    for (int i = 0; i < r && first < 0; i++)
        if (fb->repair_symbols[i]) first = i;
    if (first < 0) return 0;
    *maxl = fb->repair_symbols[first]->data_length;  /* :186 */
    return FEC_STAGE_OK;
}

void fec_recover_stage(const pquic_fec_block_t *fb, int xor_scheme, uint16_t maxl, uint8_t *src_rows,
                       uint8_t *rep_rows, uint32_t stride, uint64_t sp[2], uint64_t rp[2], uint32_t *seeds) {
    const int k = fb->total_source_symbols, r = xor_scheme ? 1 : fb->total_repair_symbols;
    sp[0] = sp[1] = rp[0] = rp[1] = 0;
    for (int j = 0; j < k; j++) {
        uint8_t *row = src_rows + (size_t)j * stride;
        const pquic_source_symbol_t *ss = fb->source_symbols[j];
        uint16_t n = 0;
        if (ss) {  /* bytes past max_length are never read back (:205): truncate */
            n = ss->data_length < maxl ? ss->data_length : maxl;
            memcpy(row, ss->data, n);
            sp[j >> 6] |= 1ull << (j & 63);
        }
        memset(row + n, 0, stride - n);
    }
    for (int i = 0; i < r; i++) {
        uint8_t *row = rep_rows + (size_t)i * stride;
        const pquic_repair_symbol_t *rs = fb->repair_symbols[i];
        uint16_t n = 0;
        if (rs) {
            n = rs->data_length < maxl ? rs->data_length : maxl;
            memcpy(row, rs->data, n);
            rp[i >> 6] |= 1ull << (i & 63);
        }
        memset(row + n, 0, stride - n);
        /* every equation is seeded by its repair's own FPID (rlc_fec_scheme_gf256.c:200), which the
         * block framework sets to (fbn << 8) | i and the window framework to (0 << 8) | i in a block
         * numbered by its window start (window_framework_sender.h:239-243) */
        if (seeds) seeds[i] = rs ? rs->fpid.f.source_fpid.raw : 0;
    }
}

protoop_arg_t fec_recover_finish(picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int xor_scheme, uint8_t status,
                                 const uint64_t rec[2], const uint8_t *src_rows, uint32_t stride, uint16_t maxl,
                                 uint64_t *nrec_acc) {
    const int k = fb->total_source_symbols;
    if (status == FECGPU_BLOCK_REF_UB) FEC_STAT_ADD(ref_ub_blocks, 1);
    if (!xor_scheme) {
        const uint32_t fbn = fb->fec_block_number & 0xffffffu;
        uint64_t nrec = 0;
        for (int j = 0; j < k && status == FECGPU_BLOCK_RECOVERED; j++) {  /* :218-236 */
            if (!((rec[j >> 6] >> (j & 63)) & 1)) continue;
            pquic_source_symbol_t *ss = new_source(cnx, (fbn << 8) + (uint8_t)j, maxl);
            if (!ss) continue;  /* the reference skips an unallocatable symbol (:222-226) */
            memcpy(ss->data, src_rows + (size_t)j * stride, maxl);
            fb->source_symbols[j] = ss;
            fb->current_source_symbols++;
            nrec++;
        }
        if (nrec_acc) *nrec_acc += nrec;
        else if (nrec) FEC_STAT_ADD(recovered_symbols, nrec);
        return 0;
    }
    protoop_arg_t ret = 1;
    for (int j = 0; j < k && status == FECGPU_BLOCK_RECOVERED; j++) {
        if (!((rec[j >> 6] >> (j & 63)) & 1)) continue;
        pquic_source_symbol_t *ss = new_source(cnx, (fb->fec_block_number << 8) | (uint32_t)j, maxl);
        if (!ss) return PQUIC_ERROR_MEMORY;
        memcpy(ss->data, src_rows + (size_t)j * stride, maxl);
        fb->source_symbols[j] = ss;  /* current_source_symbols is NOT incremented (:72) */
        if (nrec_acc) ++*nrec_acc;
        else FEC_STAT_ADD(recovered_symbols, 1);
        ret = 0;
    }
    return ret;
}

int fec_recover_alloc(picoquic_cnx_t *cnx, const pquic_fec_block_t *fb, uint16_t maxl, pquic_source_symbol_t **pre) {
    const uint32_t fbn = fb->fec_block_number & 0xffffffu;
    int n = 0;
    for (int j = 0; j < fb->total_source_symbols; j++) {
        pre[j] = NULL;
        if (fb->source_symbols[j]) continue;
        if ((pre[j] = new_source(cnx, (fbn << 8) + (uint8_t)j, maxl))) n++;
    }
    return n;
}

protoop_arg_t fec_recover_finish_pre(picoquic_cnx_t *cnx, pquic_fec_block_t *fb, uint8_t status, const uint64_t rec[2],
                                     pquic_source_symbol_t *const *pre, const uint64_t copy[2], const uint8_t *src_rows,
                                     uint32_t stride, uint16_t maxl, uint64_t *nrec_acc) {
    const int k = fb->total_source_symbols;
    const uint32_t fbn = fb->fec_block_number & 0xffffffu;
    if (status == FECGPU_BLOCK_REF_UB) FEC_STAT_ADD(ref_ub_blocks, 1);
    /* first the symbols allocated for sources the reference leaves unrecovered go back to the arena, so
     * an allocation retried below for a recovered one (its pre-allocation had failed) finds their room,
     * as the reference's allocations after decoding would (it allocates only what it recovers).  The
     * reference's own loop (:219-236) frees unknowns[] in source order, so at its malloc for source j
     * the unknowns after j are still live -- but those are its elimination scratch, which here lives on
     * the device, not in the plugin arena; a pre-allocation for an unrecovered source has no counterpart
     * in the reference at all, so it must not take room from a recovered one
     * (test_batch_recover_frees_unrecovered_preallocations_first: recovered 5 before unrecovered 6) */
    for (int j = 0; j < k; j++) {
        const int got = status == FECGPU_BLOCK_RECOVERED && ((rec[j >> 6] >> (j & 63)) & 1);
        if (!got && pre[j]) {
            g_fec_api.my_free(cnx, pre[j]->data);
            g_fec_api.my_free(cnx, pre[j]);
        }
    }
    uint64_t nrec = 0;
    for (int j = 0; j < k; j++) {  /* :218-236, in source order as the reference inserts them */
        const int got = status == FECGPU_BLOCK_RECOVERED && ((rec[j >> 6] >> (j & 63)) & 1);
        if (!got) continue;  /* (freed above) */
        pquic_source_symbol_t *ss = pre[j];
        if (!ss) {
            if (!(ss = new_source(cnx, (fbn << 8) + (uint8_t)j, maxl))) continue;
            memcpy(ss->data, src_rows + (size_t)j * stride, maxl);
        } else if ((copy[j >> 6] >> (j & 63)) & 1) {
            memcpy(ss->data, src_rows + (size_t)j * stride, maxl);
        }
        fb->source_symbols[j] = ss;
        fb->current_source_symbols++;
        nrec++;
    }
    *nrec_acc += nrec;
    return 0;
}
