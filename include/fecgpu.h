/*
 * include/fecgpu.h -- C ABI of the MI355X FEC engine (libpquic_fec.so).
 *
 * Batched, device-resident replacement for the arithmetic inside PQUIC's FEC scheme
 * pluglets (plugins/fec/fec_scheme_protoops/):
 *   fecgpu_rlc_encode  <- fec_generate_repair_symbols, RLC-GF(256)
 *                         (rlc_fec_scheme_generate_gf256.c:24-77)
 *   fecgpu_rlc_decode  <- fec_recover, RLC-GF(256) Gaussian elimination
 *                         (rlc_fec_scheme_gf256.c:134-251)
 *   fecgpu_xor_encode  <- fec_generate_repair_symbols, XOR (xor_fec_scheme_generate.c:41-78)
 *   fecgpu_xor_decode  <- fec_recover, XOR (xor_fec_scheme.c:41-74)
 * The per-block protoop adapters that keep the reference's hook surface are declared in
 * include/pquic_fec_protoops.h and call these entry points.
 *
 * Layout (all device pointers, HBM-resident, 4-byte aligned):
 *   src  [nblocks][k][symbol_size]   source symbols of consecutive FEC blocks
 *   rep  [nblocks][r][symbol_size]   repair symbols
 * Equal-length symbols; symbol_size % 4 == 0 (callers with ragged payloads zero-pad to a
 * common length, which is what the reference does internally: every symbol of a block is
 * treated as zero-padded to max(data_length)).
 * FEC block number of block b: fbn[b] if fbn != NULL, else (fbn_base + b) mod 2^24.
 * RLC coefficients of repair i of block fbn come from TinyMT32 seeded with
 * (fbn << 8) | i, exactly as the reference (fec.h:44-75).
 *
 * `stream` is a hipStream_t (NULL = the null stream).  Every call is asynchronous and
 * graph-capturable: no allocation, no synchronisation inside.
 */
#ifndef PQUIC_FECGPU_H
#define PQUIC_FECGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Call status. */
#define FECGPU_OK              0
#define FECGPU_ERR_INVALID    -1   /* argument out of range / NULL / misaligned          */
#define FECGPU_ERR_HIP        -2   /* a HIP runtime call failed: fecgpu_last_error()     */
#define FECGPU_ERR_NO_DEVICE  -3   /* no gfx950 device visible                           */
#define FECGPU_ERR_NOMEM      -4   /* workspace too small / allocation failed            */

/* Per-block decode outcome written to status[b]. */
#define FECGPU_BLOCK_RECOVERED 0   /* recovery ran (reference fec_recover returned 0 after
                                      solving); recovered[] lists the inserted sources     */
#define FECGPU_BLOCK_NOTHING   1   /* a precondition failed; nothing to recover          */
#define FECGPU_BLOCK_REF_UB    2   /* erasure pattern on which the reference dereferences
                                      x[-1] (rlc_fec_scheme_gf256.c:74-77) or a NULL repair
                                      (xor_fec_scheme.c:50-51): no output, flagged          */

#define FECGPU_MAX_K 128           /* presence masks are 2 x u64 per block               */
#define FECGPU_MAX_R 128

/* Engine version / device check.  Returns FECGPU_OK when a gfx950 device is usable. */
int fecgpu_init(int device);
const char *fecgpu_version(void);
const char *fecgpu_last_error(void);

/* RLC-GF(256) encode: rep[b][i] = sum_j coef(fbn_b, i)[j] * src[b][j] over GF(2^8)/0x11D. */
int fecgpu_rlc_encode(const void *src, void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                      uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn,
                      void *stream);

/* Sliding-window RLC encode (window_framework_sender.h:214-250): window w protects the k
 * consecutive symbols starting at symbol w * step of one symbol stream (windows overlap when
 * step < k; symbols[] holds (nwindows - 1) * step + k rows of symbol_size bytes).  Window
 * blocks carry fec_block_number 0 (malloc_fec_block(cnx, 0), :218), so every window's
 * coefficients are seeded by the repair index alone:
 *   rep[w][i] = sum_j coef(0, i)[j] * symbols[w * step + j]. */
int fecgpu_rlc_window_encode(const void *symbols, uint64_t nwindows, uint32_t step, uint32_t k, uint32_t r,
                             uint32_t symbol_size, void *rep, void *stream);

/* Window encode over de-duplicated symbol streams (the batching adapter's window jobs): symbols[] holds
 * nrows rows of symbol_size bytes -- each connection's symbols once, in order -- and window w protects
 * the k rows starting at row wrow[w] (a device array), with block number 0 like every window:
 *   rep[w][i] = sum_j coef(0, i)[j] * symbols[wrow[w] + j].
 * symbol_size % 16 == 0, 16-B aligned buffers, nrows * symbol_size < 2 GiB; knob window_sc != 0.
 * Every window must lie in the stream: wrow[w] + k <= nrows for all w.  wrow[] is device memory, so
 * this entry point cannot check it and the kernel reads the rows it names unchecked (the host form,
 * fecgpu_rlc_window_encode_host, checks it before any launch). */
int fecgpu_rlc_window_encode_table(const void *symbols, uint64_t nrows, const uint32_t *wrow, uint64_t nwindows,
                                   uint32_t k, uint32_t r, uint32_t symbol_size, void *rep, void *stream);

/* RLC encode with every row given by its address: src_rows[b * k + j] / rep_rows[b * r + i] are the
 * device addresses (4-byte aligned; device memory or mapped page-locked host memory, e.g. a registered
 * plugin arena) of source row j / repair row i of block b, each symbol_size bytes.  The tables and
 * fbn[] must themselves be device-accessible.  Same result as fecgpu_rlc_encode on packed rows. */
int fecgpu_rlc_encode_rows(const uint64_t *src_rows, const uint64_t *rep_rows, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn, void *stream);

/* RLC decode with every row given by its address (the batching adapter's received symbols where they
 * lie in registered plugin arenas): src_rows[b * k + j] is the device address of source row j of block b
 * -- for a received source the row read, for a missing one the row its recovered bytes are written to --
 * and rep_rows[b * r + i] that of repair row i (entries of repairs not present are not read).  Every
 * equation is seeded by rep_seed[b * r + i] (the repair's own FPID, as fecgpu_rlc_decode_seeded); masks,
 * status, recovered and workspace as fecgpu_rlc_decode.  Rows are symbol_size bytes, 4-byte aligned;
 * the tables and arrays must be device-accessible.  Same bytes, status and masks as
 * fecgpu_rlc_decode_seeded on packed rows. */
int fecgpu_rlc_decode_rows(const uint64_t *src_rows, const uint64_t *rep_rows, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed, const uint64_t *src_present,
                           const uint64_t *rep_present, uint8_t *status, uint64_t *recovered, void *workspace,
                           size_t workspace_bytes, void *stream);

/* XOR encode (r == 1): rep[b][0] = XOR_j src[b][j]. */
int fecgpu_xor_encode(const void *src, void *rep, uint64_t nblocks, uint32_t k,
                      uint32_t symbol_size, void *stream);

/* RLC decode.  Presence masks: bit j of src_present[2*b + j/64] set <=> source j of
 * block b was received; same for rep_present.  Recovered sources are written IN PLACE
 * into src[b][j]; bit j of recovered[2*b + j/64] is set for every source the reference
 * would insert (determined and non-zero, rlc_fec_scheme_gf256.c:218-236).  Bytes of a
 * missing slot whose bit stays clear are unspecified.  `workspace` must hold
 * fecgpu_rlc_decode_workspace(nblocks, k, r) bytes of device memory. */
size_t fecgpu_rlc_decode_workspace(uint64_t nblocks, uint32_t k, uint32_t r);
int fecgpu_rlc_decode(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                      uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn,
                      const uint64_t *src_present, const uint64_t *rep_present,
                      uint8_t *status, uint64_t *recovered, void *workspace,
                      size_t workspace_bytes, void *stream);

/* The two stages fecgpu_rlc_decode runs, for callers that schedule or time them apart:
 * plan  -- coefficient-only replay of the reference elimination per block (workspace);
 * apply -- the data pass (e recovered symbols from k received ones, written in place) and the
 *          reference's zero/undetermined rule, writing status[] and recovered[].  When
 *          min(k, r) <= 16 the rule runs inside the data kernel; otherwise apply launches one
 *          more small kernel after the data passes. */
int fecgpu_rlc_decode_plan(uint64_t nblocks, uint32_t k, uint32_t r, uint32_t fbn_base,
                           const uint32_t *fbn, const uint64_t *src_present,
                           const uint64_t *rep_present, void *workspace, size_t workspace_bytes,
                           void *stream);
int fecgpu_rlc_decode_apply(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                            uint32_t symbol_size, uint8_t *status, uint64_t *recovered,
                            void *workspace, size_t workspace_bytes, void *stream);
/* apply with the recovered symbols written to dst instead of in place: dst has src's layout
 * ([block][k][symbol_size]) and receives only the recovered rows (every other byte of dst is left
 * untouched); src is only read.  dst may be any memory the device can write -- e.g. page-locked
 * host packet buffers, so recovered symbols cross PCIe once and nothing else comes back
 * (fecgpu_rlc_decode_host uses this for pinned buffers). */
int fecgpu_rlc_decode_apply_to(const void *src, const void *rep, void *dst, uint64_t nblocks,
                               uint32_t k, uint32_t r, uint32_t symbol_size, uint8_t *status,
                               uint64_t *recovered, void *workspace, size_t workspace_bytes,
                               void *stream);
/* apply with the recovered symbols packed: dst is [nblocks][min(k, r)][symbol_size] and row u of
 * block b receives the u-th missing source of b in ascending source order (the u-th clear bit of
 * src_present below k); rows past the block's erasures and rows whose recovered[] bit stays clear are
 * unspecified.  The reference's fec_recover allocates every recovered symbol anew
 * (rlc_fec_scheme_gf256.c:218-236), so a packed row per recovered symbol is as faithful as src's
 * layout, and a block's rows are contiguous: no written row shares a cache line with bytes the pass
 * does not write (recovered rows at their src-layout slots leave two half-written 128-B lines each,
 * which the memory system fetches to merge). */
int fecgpu_rlc_decode_apply_packed(const void *src, const void *rep, void *dst, uint64_t nblocks,
                                   uint32_t k, uint32_t r, uint32_t symbol_size, uint8_t *status,
                                   uint64_t *recovered, void *workspace, size_t workspace_bytes,
                                   void *stream);

/* RLC decode with the coefficients of every received repair seeded by its own FPID, as the
 * reference does (get_coefs(..., rs->repair_fec_payload_id.source_fpid.raw, ...),
 * rlc_fec_scheme_gf256.c:200): rep_seed[b * r + i] is the low 32 bits of the FPID of the repair
 * in slot i of block b (entries of absent repairs are ignored).  This is the general form: the
 * block framework's repairs carry (fbn << 8) | i, which is what fecgpu_rlc_decode assumes, but
 * the sliding-window framework's blocks are numbered by their window start while their repairs
 * carry block number 0 (window_framework_receiver.h:60-86, window_framework_sender.h:239-243).
 * Recovered FPIDs are the caller's business (the host adapters stamp (fec_block_number << 8) + j,
 * :222). */
int fecgpu_rlc_decode_plan_seeded(uint64_t nblocks, uint32_t k, uint32_t r, const uint32_t *rep_seed,
                                  const uint64_t *src_present, const uint64_t *rep_present, void *workspace,
                                  size_t workspace_bytes, void *stream);
int fecgpu_rlc_decode_seeded(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                             uint32_t symbol_size, const uint32_t *rep_seed, const uint64_t *src_present,
                             const uint64_t *rep_present, uint8_t *status, uint64_t *recovered, void *workspace,
                             size_t workspace_bytes, void *stream);

/* XOR decode (r == 1), same conventions. */
int fecgpu_xor_decode(void *src, const void *rep, uint64_t nblocks, uint32_t k,
                      uint32_t symbol_size, const uint64_t *src_present,
                      const uint64_t *rep_present, uint8_t *status, uint64_t *recovered,
                      void *stream);
/* fecgpu_xor_decode with the recovered symbol of block b written to dst + b * symbol_size (one row per
 * block, as fec_recover allocates the recovered symbol anew, xor_fec_scheme.c:54-58) instead of into
 * src; src is not written.  Rows of blocks with nothing recovered are left as they were. */
int fecgpu_xor_decode_to(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k,
                         uint32_t symbol_size, const uint64_t *src_present,
                         const uint64_t *rep_present, uint8_t *status, uint64_t *recovered,
                         void *stream);

/* ---- Host-resident path --------------------------------------------------------------------
 * The same operations on HOST buffers (pageable or pinned): H2D copy, kernels, D2H copy,
 * pipelined over sub-batches of about `chunk_bytes` of payload on `nstreams` HIP streams so
 * that PCIe transfers overlap the kernels.  Synchronous: results are in host memory on
 * return.  Used by the protoop adapters (one block per call) and by the PCIe-inclusive
 * measurement.  Page-locked buffers (fecgpu_host_alloc, hipHostMalloc, registered) are zero-copy:
 * the kernels read the blocks and write repairs / recovered rows directly over PCIe, so only the
 * bytes the operation needs cross the bus.  Pageable buffers are staged by copies (decode then
 * copies whole source rows back). */
typedef struct fecgpu_host_ctx fecgpu_host_ctx_t;
fecgpu_host_ctx_t *fecgpu_host_ctx_create(int device, int nstreams, size_t chunk_bytes);
void fecgpu_host_ctx_destroy(fecgpu_host_ctx_t *ctx);
int fecgpu_rlc_encode_host(fecgpu_host_ctx_t *ctx, const void *src, void *rep, uint64_t nblocks,
                           uint32_t k, uint32_t r, uint32_t symbol_size, uint32_t fbn_base,
                           const uint32_t *fbn);
int fecgpu_rlc_decode_host(fecgpu_host_ctx_t *ctx, void *src, const void *rep, uint64_t nblocks,
                           uint32_t k, uint32_t r, uint32_t symbol_size, uint32_t fbn_base,
                           const uint32_t *fbn, const uint64_t *src_present,
                           const uint64_t *rep_present, uint8_t *status, uint64_t *recovered);
/* host-resident fecgpu_rlc_decode_seeded: rep_seed is a host array [nblocks][r] */
int fecgpu_rlc_decode_host_seeded(fecgpu_host_ctx_t *ctx, void *src, const void *rep, uint64_t nblocks,
                                  uint32_t k, uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed,
                                  const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                                  uint64_t *recovered);
/* fecgpu_rlc_encode_rows from the host: the row tables and fbn[] are host arrays (page-locked arrays
 * are read in place, others are copied), the rows themselves must be device-accessible. */
int fecgpu_rlc_encode_rows_host(fecgpu_host_ctx_t *ctx, const uint64_t *src_rows, const uint64_t *rep_rows,
                                uint64_t nblocks, uint32_t k, uint32_t r, uint32_t symbol_size, const uint32_t *fbn);
/* fecgpu_rlc_decode_rows from the host: the row tables, seeds, masks, status and recovered are host
 * arrays (page-locked ones are used in place, others copied); the rows must be device-accessible.  With
 * r == 0 the repair table and the seeds have no entries and are not read (NULL is accepted). */
int fecgpu_rlc_decode_rows_host(fecgpu_host_ctx_t *ctx, const uint64_t *src_rows, const uint64_t *rep_rows,
                                uint64_t nblocks, uint32_t k, uint32_t r, uint32_t symbol_size,
                                const uint32_t *rep_seed, const uint64_t *src_present, const uint64_t *rep_present,
                                uint8_t *status, uint64_t *recovered);
/* fecgpu_rlc_window_encode_table from the host: the stream (host rows) crosses PCIe once, by one copy,
 * before the windows are coded from device memory -- a symbol serves up to k windows, so reading it in
 * place would cross the bus that many times; wrow[] is a host array; repairs go to page-locked `rep` in
 * place, others by a copy.  With knob window_sc 0 the windows run through the row-table kernel. */
int fecgpu_rlc_window_encode_host(fecgpu_host_ctx_t *ctx, const void *symbols, uint64_t nrows, const uint32_t *wrow,
                                  uint64_t nwindows, uint32_t k, uint32_t r, uint32_t symbol_size, void *rep);
int fecgpu_xor_encode_host(fecgpu_host_ctx_t *ctx, const void *src, void *rep, uint64_t nblocks,
                           uint32_t k, uint32_t symbol_size);
int fecgpu_xor_decode_host(fecgpu_host_ctx_t *ctx, void *src, const void *rep, uint64_t nblocks,
                           uint32_t k, uint32_t symbol_size, const uint64_t *src_present,
                           const uint64_t *rep_present, uint8_t *status, uint64_t *recovered);

/* ---- Resident single-block service (the synchronous hooks) ------------------------------------
 * One block per call, as the block framework calls fec_generate_repair_symbols / fec_recover
 * (block_framework_sender.h:187, fec_protoops.h:246): a worker workgroup stays resident on the device
 * and polls a page-locked mailbox, so a call costs a mailbox round trip over PCIe instead of a
 * kernel launch.  The worker ends by itself after 20 ms without a request (and after 50 ms in all);
 * the next call relaunches it.  It runs on a stream of the greatest priority (its own hardware queue
 * unless the process creates other such streams), so the process's other kernels do not queue behind it.  Every buffer must be page-locked (fecgpu_host_alloc, registered
 * ranges); the rows are zero-copy.  Returns FECGPU_ERR_INVALID when the block does not fit the
 * worker (e > 16 unknowns, rows beyond its LDS), a buffer is not page-locked, knob block_svc is 0, or
 * the request was withdrawn at its deadline (below) -- the caller then takes the host path.
 * Thread-safe (one request at a time per service). */
typedef struct fecgpu_block_svc fecgpu_block_svc_t;
fecgpu_block_svc_t *fecgpu_block_svc_create(int device);
void fecgpu_block_svc_destroy(fecgpu_block_svc_t *svc);
/* rep[i] = sum_j coef((fbn << 8) | i)[j] * src[j] for one block (k rows of symbol_size bytes) */
int fecgpu_block_svc_rlc_encode(fecgpu_block_svc_t *svc, const void *src, void *rep, uint32_t k, uint32_t r,
                                uint32_t symbol_size, uint32_t fbn);
/* fecgpu_rlc_decode_seeded for one block; recovered rows go to dst (src's layout), src is only read */
int fecgpu_block_svc_rlc_decode_seeded(fecgpu_block_svc_t *svc, const void *src, const void *rep, void *dst,
                                       uint32_t k, uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed,
                                       const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                                       uint64_t *recovered);
/* worker generations launched so far (diagnostics: one per idle gap) */
uint64_t fecgpu_block_svc_launches(const fecgpu_block_svc_t *svc);
/* A call waits at most `deadline_us` (default 2000) for a worker to take its request.  Past it the
 * request is withdrawn on the spot unless a worker has claimed it (compare-and-swap on the request
 * number, against the worker's own claim): a withdrawn request is never served later, and the call
 * returns FECGPU_ERR_INVALID without waiting for the worker (it may be queued behind a long kernel),
 * so the caller takes the host path; for the next 50 ms every call returns FECGPU_ERR_INVALID at once.
 * A request a worker claimed before the deadline is being served and is waited for (the call
 * succeeds).  0: withdraw whatever is not done at the first check (tests). */
int fecgpu_block_svc_set_deadline(fecgpu_block_svc_t *svc, uint64_t deadline_us);
/* requests withdrawn at the deadline so far */
uint64_t fecgpu_block_svc_deadline_misses(fecgpu_block_svc_t *svc);
/* Diagnostics: the phases of the last served request.  out[0..3]: the worker's clock (s_memrealtime,
 * 100 MHz ticks) when it claimed the request, when the request was in LDS, when its rows were coded, and
 * just before it published `done`; out[4], out[5]: the host's clock (CLOCK_MONOTONIC, us) when the request
 * was posted and when the call saw it done.  Returns FECGPU_OK, or FECGPU_ERR_INVALID for NULL. */
int fecgpu_block_svc_last_stamps(fecgpu_block_svc_t *svc, uint64_t out[6]);
/* Whether a worker is running now (it ends by itself after 20 ms without a request, 50 ms in all):
 * 1 running, 0 not (or never launched), FECGPU_ERR_HIP if the last one ended in an error,
 * FECGPU_ERR_INVALID for NULL.  Lets a caller (a test) wait for the idle state instead of a time. */
int fecgpu_block_svc_worker_running(fecgpu_block_svc_t *svc);

/* FEC frames for a batch of repair symbols, ready for packet buffers (the block framework's
 * get_repair_payload_from_queue + write_fec_frame, block_framework_sender.h:100-133,
 * protoops/write_fec_frame.c; wire format in pquic_fec_frames.h).  Frame b*r + i, at
 * frames + (b*r + i) * frame_stride, is the 14-byte header {fin 1, data_length, offset 1,
 * repair FPID (fbn_b << 8) | i, nss, nrs} followed by the first data_length bytes of rep[b][i];
 * the rest of the slot is zeroed.  Device buffers; symbol_size and frame_stride multiples of 4,
 * frame_stride >= 14 + data_length. */
int fecgpu_write_repair_frames(const void *rep, uint64_t nblocks, uint32_t r, uint32_t symbol_size,
                               uint16_t data_length, uint32_t fbn_base, const uint32_t *fbn, uint8_t nss, uint8_t nrs,
                               void *frames, uint32_t frame_stride, void *stream);

/* Page-locked host memory for staging buffers (hipHostMalloc / hipHostFree), so callers in
 * C need no HIP headers.  NULL on failure. */
void *fecgpu_host_alloc(size_t bytes);
void fecgpu_host_free(void *p);
/* The host CPUs nearest the device ("local_cpulist" of its PCI function, e.g. "0-63,128-191"), for
 * placing the threads that feed it: page-locked rows read over PCIe from the device's own socket
 * avoid the cross-socket hop.  FECGPU_OK or an error. */
int fecgpu_device_local_cpus(int device, char *buf, size_t len);
/* Page-lock and map an existing host range (hipHostRegister, mapped) so the kernels read and write
 * it in place -- e.g. a FEC plugin instance's memory arena (picoquic_internal.h:576, char
 * memory[PLUGIN_MEMORY], carved into 2100-B slots by picoquic/memory.c:181-191), which holds every
 * symbol the framework hands over.  Unregister before the range is freed.  fecgpu_host_device_address
 * gives the device address of [p, p + bytes) when all of it lies in page-locked memory. */
int fecgpu_host_register(void *p, size_t bytes);
int fecgpu_host_unregister(void *p);
int fecgpu_host_device_address(const void *p, size_t bytes, uint64_t *dev);

/* Synthetic payload generator (bench/tests): byte o of dst = byte (o mod 8) of
 * splitmix64(seed + (o/8 + 1) * 0x9e3779b97f4a7c15), o counted from `offset`. */
int fecgpu_synth_fill(void *dst, uint64_t nbytes, uint64_t seed, uint64_t offset, void *stream);

/* Experiment knobs (A/B runs, cross-checks of alternative kernels in the tests).  Every knob has
 * a measured default and only these calls change it (the library reads no environment variables;
 * tools/ab_inproc.py maps the FECGPU_* names of earlier rounds onto them).  Names and accepted values:
 * "plan" (0 auto, 1 wave in LDS, 2 lane, 3 reg, 4 tile, 5 wave in registers where it fits),
 * "interleave" (0/1), "group" (0 = defaults, else a cap on blocks per group), "enc_tile_rt" (0 =
 * default tiling, else 1/2/4/8/16) / "enc_tile_waves" (0..4), "zc_read" (0/1), "ring" (the LDS-ring
 * data path of 16-repair / 16-unknown tiles: 2 = default, 0 off), "window_sc" (window encode on the
 * shared-coefficient kernel: 0 never, 1 = default for overlapping windows, 2 wherever it applies),
 * "min_groups" (batches with fewer block groups than this stream fewer blocks per wave; default
 * 1024, 0 = the per-shape group sizes at any batch size), "chunk_waves" (symbols wider than one column
 * chunk coded by 4-wave workgroups over (block, chunk) items: 1 = default, 0 one wave per group),
 * "small_lds" (batches of <= 64 blocks with their rows staged in LDS: 1 = default, 0 the bitsliced
 * kernels), "block_svc" (the resident single-block service: 1 = default, 0 refused), "ws_lds" (the
 * recover data pass copies a group's plan records into LDS in one round trip: 1 = default, 0 reads
 * them in place), "dec_waves" (0 = default, n = at most n waves per SIMD for the register-prefetch
 * recover tiles).  Returns FECGPU_OK, or FECGPU_ERR_INVALID
 * for an unknown name or a value outside its range. */
int fecgpu_set_knob(const char *name, int value);
int fecgpu_get_knob(const char *name, int *value);

/* Per-process counters, the analogue of the reference's per-pluglet count/time
 * (picoquic/ubpf.c:302-319 under DEBUG_PLUGIN_EXECUTION_TIME). */
typedef struct {
    uint64_t encode_calls, encode_blocks;
    uint64_t decode_calls, decode_blocks;
    /* host path: page-locked buffers found in the library's registry of its own fecgpu_host_alloc /
     * fecgpu_host_register ranges, and those that needed a hipPointerGetAttributes query instead */
    uint64_t pinned_registry_hits, pinned_registry_misses;
    /* zero-copy bulk calls while the synchronous hooks are in use: slices launched, and slices held back
     * until a pending hook request had finished (host_path.hip, Pacer) */
    uint64_t yield_slices, yield_waits;
} fecgpu_stats_t;
void fecgpu_get_stats(fecgpu_stats_t *out);

#ifdef __cplusplus
}
#endif
#endif
