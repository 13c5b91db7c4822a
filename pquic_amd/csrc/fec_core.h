/*
 * pquic_amd/csrc/fec_core.h -- internal: the block <-> row-layout halves of the FEC scheme
 * operations, shared by the synchronous protocol operations (protoops.c) and the batching
 * adapter (batch.c).
 *
 * A block is staged into k source rows (and r repair rows for recover) of `stride` bytes,
 * zero-padded, exactly as the reference pads symbols to max_length; the device engine runs
 * on the rows; the finish half writes repair / recovered symbols back into the block with
 * the bound host allocator, with the reference's FPIDs, lengths and counters.
 */
#ifndef PQUIC_AMD_FEC_CORE_H
#define PQUIC_AMD_FEC_CORE_H

#include <stdint.h>

#include "pquic_fec_protoops.h"

#ifdef __cplusplus
extern "C" {
#endif

#pragma GCC visibility push(hidden)  /* library-internal: not part of the C ABI */

extern pquic_fec_host_api_t g_fec_api;   /* bound by pquic_fec_bind_host */
extern int g_fec_bound;
extern pquic_fec_protoop_stats_t g_fec_stats;

static inline uint32_t fec_pad4(uint32_t x) { return (x + 3u) & ~3u; }

/* The adapter counters are shared by the synchronous operations and the batching adapter's
 * completion path, which may run on different threads. */
#define FEC_STAT_ADD(field, n) __atomic_fetch_add(&g_fec_stats.field, (uint64_t)(n), __ATOMIC_RELAXED)

/* Generate, before the engine: preconditions of rlc_fec_scheme_generate_gf256.c:34-39 /
 * xor_fec_scheme_generate.c:45-50.  Returns 1 (the reference's "nothing done") when they
 * fail, else 0 with *maxl = max_length (:41-45) and, if src_rows is non-NULL, the k sources
 * copied into rows of `stride` bytes zero-padded to the stride (stride >= *maxl). */
int fec_generate_check(const pquic_fec_block_t *fb, int xor_scheme, uint16_t *maxl);
void fec_generate_stage(const pquic_fec_block_t *fb, uint8_t *src_rows, uint32_t stride);
/* Generate, after the engine: r repair symbols of max_length bytes from rep_rows into
 * fb->repair_symbols with FPID (fbn << 8 | i) (:57-61).  Returns 0 or PQUIC_ERROR_MEMORY. */
protoop_arg_t fec_generate_finish(picoquic_cnx_t *cnx, pquic_fec_block_t *fb, const uint8_t *rep_rows,
                                  uint32_t stride, uint16_t maxl);
/* The same in three steps, so the copy can run off the allocator's thread (batch.c):
 * fec_generate_alloc allocates the r repair symbols (FPIDs and lengths set, data unwritten) into
 * reps[0..r) and returns how many it got (r, or the index of the first failed allocation);
 * after their data is written, fec_generate_attach stores them in the block and returns the
 * operation's value (0, or PQUIC_ERROR_MEMORY when an allocation failed). */
int fec_generate_alloc(picoquic_cnx_t *cnx, const pquic_fec_block_t *fb, uint16_t maxl,
                       pquic_repair_symbol_t **reps);
protoop_arg_t fec_generate_attach(pquic_fec_block_t *fb, pquic_repair_symbol_t *const *reps, int nalloc);

/* Recover, before the engine.  Returns FEC_STAGE_OK when the block goes to the engine;
 * otherwise the value the reference operation returns without doing anything
 * (rlc_fec_scheme_gf256.c:140-144 -> 0; xor_fec_scheme.c:45-51 -> 1), or FEC_STAGE_REJECT for
 * totals past the block's 100 symbol slots (fec.h:8; the reference reads out of bounds there).
 * *maxl = the first present repair's length (:186).  fec_generate_check returns FEC_STAGE_REJECT
 * for the same totals. */
#define FEC_STAGE_OK (-1)
#define FEC_STAGE_REJECT (-2)
int fec_recover_check(const pquic_fec_block_t *fb, int xor_scheme, uint16_t *maxl);
/* Rows of `stride` bytes, sources truncated to maxl, zero-padded; presence masks; seeds[i] (r
 * entries, may be NULL) = the TinyMT32 seed of the repair in slot i, its own FPID (:200). */
void fec_recover_stage(const pquic_fec_block_t *fb, int xor_scheme, uint16_t maxl, uint8_t *src_rows,
                       uint8_t *rep_rows, uint32_t stride, uint64_t sp[2], uint64_t rp[2], uint32_t *seeds);
/* Recover, after the engine: inserts every source the engine marked recovered (maxl bytes
 * from src_rows) with the reference's FPID and counter behaviour (RLC increments
 * current_source_symbols, :230; XOR does not, xor_fec_scheme.c:72).  Returns the
 * operation's value (RLC 0; XOR 0 after an insertion, else 1).  The recovered-symbol counter is added to
 * atomically, or -- nrec_acc non-NULL, the batcher's completions -- into *nrec_acc, which the caller adds
 * once per poll (a locked add per block waited for the completion's outstanding stores). */
protoop_arg_t fec_recover_finish(picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int xor_scheme, uint8_t status,
                                 const uint64_t rec[2], const uint8_t *src_rows, uint32_t stride, uint16_t maxl,
                                 uint64_t *nrec_acc);

/* RLC recover with the recovered symbols allocated before the engine (the batching adapter's gather
 * path, batch.c): fec_recover_alloc allocates one source symbol of maxl bytes, FPID (fbn << 8) + j, for
 * every missing source j into pre[j] (pre[j] = NULL for received sources and failed allocations) and
 * returns how many it got; the engine then writes the recovered bytes into their data.  After it,
 * fec_recover_finish_pre inserts pre[j] for every recovered source (first copying maxl bytes from
 * src_rows row j when bit j of `copy` is set: the engine wrote that row into the staging rows), allocates
 * anew for a recovered source without a pre-allocated symbol (skipped when that fails, :222-226), and
 * frees the pre-allocated symbols of sources left unrecovered -- the block ends as fec_recover_finish
 * leaves it.  pre[] is only read (the caller drops it: every pre[j] is inserted or freed; not writing it
 * back keeps the array's lines shared with the stager threads that read them).  Returns 0
 * (rlc_fec_scheme_gf256.c:250).  Recovered symbols are counted into *nrec_acc (see fec_recover_finish). */
int fec_recover_alloc(picoquic_cnx_t *cnx, const pquic_fec_block_t *fb, uint16_t maxl, pquic_source_symbol_t **pre);
protoop_arg_t fec_recover_finish_pre(picoquic_cnx_t *cnx, pquic_fec_block_t *fb, uint8_t status, const uint64_t rec[2],
                                     pquic_source_symbol_t *const *pre, const uint64_t copy[2], const uint8_t *src_rows,
                                     uint32_t stride, uint16_t maxl, uint64_t *nrec_acc);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif
