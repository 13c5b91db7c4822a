/*
 * pquic_fec_batch.h -- batching adapter for PQUIC's block FEC framework.
 *
 * The reference runs fec_generate_repair_symbols / fec_recover synchronously, one block per
 * protocol-operation call (block_framework_sender.h:175-203 generate_and_queue_repair_symbols;
 * block_framework_receiver.h:29-80 via fec_protoops.h:215-246 recover_block).  On a GPU a
 * single block is pure launch and PCIe latency, so this adapter queues blocks from any number
 * of connections into per-(operation, scheme, k, r) batches in page-locked memory and runs a
 * batch through the device engine when it is full or when its oldest block has waited
 * `max_delay_us` (the latency cap).  A worker thread runs the engine (H2D, kernels, D2H
 * overlapped on HIP streams) while the caller keeps queueing.
 *
 * Completion has exactly the synchronous operation's effect: the repair symbols (or
 * recovered source symbols) are allocated with the bound host allocator
 * (pquic_fec_bind_host), written into the caller's fec_block_t with the reference's FPIDs,
 * lengths and counters, and `done(user, fb, ret)` receives the value the protocol operation
 * would have returned.  Completions run on the caller's thread inside pquic_fec_batch_poll /
 * pquic_fec_batch_drain, never on the worker, because picoquic's allocator and connection
 * state are single-threaded (picoquic/memory.c, plugin.c:1357-1360).
 *
 * The caller keeps `fb` (and its symbols) alive and unmodified until `done` runs for it.
 */
#ifndef PQUIC_FEC_BATCH_H
#define PQUIC_FEC_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "pquic_fec_protoops.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pquic_fec_batcher pquic_fec_batcher_t;

typedef struct {
    int device;              /* HIP device */
    uint32_t batch_blocks;   /* a queue is flushed when it holds this many blocks (>= 1) */
    uint32_t max_delay_us;   /* ... or when its oldest block has waited this long (poll) */
    uint32_t max_symbol;     /* largest symbol length accepted (<= 32767, fec.h:95,109) */
    int nstreams;            /* HIP streams the engine pipelines a batch over (>= 1) */
    uint32_t poll_blocks;    /* poll completes at most this many blocks per call (0: every finished one);
                              * a sender's event loop that polls between submissions then frees and
                              * reallocates symbols in small interleaved runs, so its allocator's free
                              * list stays in cache */
} pquic_fec_batch_cfg_t;

/* Called once per submitted block, on the caller's thread (see above). */
typedef void (*pquic_fec_block_done_fn)(void *user, pquic_fec_block_t *fb, protoop_arg_t ret);

typedef struct {
    uint64_t submitted, completed;  /* blocks */
    uint64_t batches;               /* engine calls */
    uint64_t flushed_full, flushed_deadline, flushed_drain;
    uint64_t immediate;             /* blocks completed at submit (preconditions failed) */
    uint64_t engine_errors;
    uint64_t windows, window_rows;  /* window blocks coded from shared streams; stream rows staged for them */
    uint64_t engine_us, stage_us;   /* thread time in engine calls / in stager work items (all threads) */
    uint64_t complete_us;           /* caller-thread time in completions (poll / drain) */
    uint64_t rows_in_place;         /* symbol rows the kernels read or wrote where they lie (registered arenas) */
    uint64_t rows_staged;           /* symbol rows copied through the page-locked staging rows instead */
    uint64_t jobs_allocated;        /* batch jobs (page-locked queue buffers) allocated on the caller's thread */
    uint64_t job_alloc_us;          /* caller-thread time in those allocations */
    uint64_t deadline_holds;        /* polls that kept an overdue queue open: no idle job for its successor while
                                     * two or more were in flight (flushed at the first poll with one back) */
} pquic_fec_batch_stats_t;

/* NULL on failure (bad configuration, no device, out of pinned memory). */
pquic_fec_batcher_t *pquic_fec_batcher_create(const pquic_fec_batch_cfg_t *cfg);
/* Drains (completing every queued block) and frees. */
void pquic_fec_batcher_destroy(pquic_fec_batcher_t *b);

/* Register a host memory range that holds symbols -- a FEC plugin instance's memory arena
 * (picoquic_internal.h:576, char memory[PLUGIN_MEMORY], carved into 2100-B slots by
 * picoquic/memory.c:181-191, registered once after init_memory_management, memory.c:254).  Every
 * connection owns its plugin instances (plugin.c:835, 946-950), so a process registers one arena per
 * connection: any number of them, kept sorted and looked up by binary search, registered and
 * unregistered while batches run (call from the thread that submits).  It is page-locked and mapped
 * (fecgpu_host_register) until unregistered or the batcher is destroyed.  RLC generate batches then
 * read source symbols and write repair symbols in it directly, and RLC recover batches read the received
 * sources and repairs in it and write each recovered source into a symbol allocated for it at submission
 * (through the bound allocator, so in the connection's arena), instead of copying rows through staging
 * rows.  Returns 0, or -1 (NULL / empty range, overlap with a registered range, registration failure). */
int pquic_fec_batch_register_heap(pquic_fec_batcher_t *b, void *base, size_t bytes);
/* Unregister the range registered at `base` (a connection closing).  No block whose symbols lie in it
 * may still be queued: the caller has had every done() for them.  Returns 0 or -1. */
int pquic_fec_batch_unregister_heap(pquic_fec_batcher_t *b, void *base);

/* Queue fec_generate_repair_symbols (xor_scheme = 0: RLC-GF(256), 1: XOR) for `fb`, whose
 * totals are set as the block framework sets them before the call
 * (block_framework_sender.h:184-185).  `now_us` starts the block's latency clock.
 * Returns 0 when accepted -- `done` is then called exactly once, possibly before this returns
 * when the reference's preconditions fail -- or -1 (NULL argument, symbol longer than
 * max_symbol, allocation failure), in which case `done` is never called. */
int pquic_fec_batch_generate(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int xor_scheme,
                             uint64_t now_us, pquic_fec_block_done_fn done, void *user);
/* Queue fec_generate_repair_symbols (RLC-GF(256)) for a window block of the sliding-window sender
 * (window_framework_sender.h:209-260: malloc_fec_block(cnx, 0) at :215, the symbols in flight chosen by
 * window_select_symbols_to_protect, the generate call at :235).  Same contract and result as
 * pquic_fec_batch_generate; in addition the batch stages each connection's symbols once for all the
 * windows that share them and codes the windows together (every window is block number 0, so they share
 * their coefficients).  Windows from one connection should arrive in sending order, as the sender
 * produces them; a block with a non-zero block number is queued as an ordinary block. */
int pquic_fec_batch_generate_window(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb,
                                    uint64_t now_us, pquic_fec_block_done_fn done, void *user);
/* Queue fec_recover for `fb` (the receiver's block copy, fec_protoops.h:220-222). */
int pquic_fec_batch_recover(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int xor_scheme,
                            uint64_t now_us, pquic_fec_block_done_fn done, void *user);

/* Flushes every queue that is full or past its deadline at `now_us`, then runs `done` for
 * the blocks whose batch has finished: all of them, or at most cfg.poll_blocks.  Batches complete
 * in the order they were flushed (a finished batch waits for the ones flushed before it), and the
 * blocks of a batch in submission order, so the blocks of one queue -- one (operation, scheme, k, r)
 * -- complete in submission order, as the synchronous operation completes them one by one; a block
 * whose preconditions fail completes inside its submission call.  Non-blocking.  Returns the number
 * of completions. */
int pquic_fec_batch_poll(pquic_fec_batcher_t *b, uint64_t now_us);
/* Flushes everything and waits until every queued block has completed.  Returns the number
 * of completions. */
int pquic_fec_batch_drain(pquic_fec_batcher_t *b);

void pquic_fec_batch_get_stats(const pquic_fec_batcher_t *b, pquic_fec_batch_stats_t *out);

#ifdef __cplusplus
}
#endif
#endif
