/*
 * pquic_amd/csrc/batch.c -- batching adapter for the block FEC framework
 * (include/pquic_fec_batch.h).  Host C, like the framework it serves.
 *
 * Submission checks the reference's preconditions and records the block in the open "job"
 * (one per operation, scheme, k and r); a generate submission also allocates the block's r
 * repair symbols there, on the caller's thread like every allocator call.  A full or overdue
 * job goes through a pipeline off the caller's thread:
 *   - stager threads (several jobs at once) copy each block into the job's page-locked rows: k
 *     source rows (+ r repair rows for recover) of `stride` bytes, zero-padded like the
 *     reference pads to max_length, plus presence masks;
 *   - the engine thread runs staged jobs through the host-resident entry points (zero-copy
 *     kernels on the page-locked rows);
 *   - for generate, the stager threads copy the repair rows into the symbols allocated at
 *     submission (the caller's thread was the bound when it copied them itself).
 * Gather (pquic_fec_batch_register_heap): once the FEC plugin's memory arena is registered, a
 * generate job's stagers copy nothing for rows that lie in it -- they write the rows' device
 * addresses into page-locked tables and the kernel (fecgpu_rlc_encode_rows) reads the sources and
 * writes the repairs where the symbols are.  Rows outside a registered arena, or shorter than the
 * block's length (the reference zero-pads them), are staged as before.
 * Windows (pquic_fec_batch_generate_window): the sliding-window sender protects the symbols in flight
 * once per window, so consecutive windows of a connection share most of their symbols, and every window
 * is block number 0, so all windows share their coefficients.  A window job therefore stages each
 * connection's symbols once, as one run of rows (a stager lays the runs out at flush: windows grouped
 * by connection, each window matched against the run's tail by symbol identity), records where each
 * window starts, and the engine codes all windows from that stream with the shared-coefficient kernel
 * (fecgpu_rlc_window_encode_host) after one copy of the stream to the device.
 * Finished jobs are completed on the caller's thread in poll / drain with the same finish
 * halves the synchronous operations use (fec_core.c), so a batched block ends in exactly the
 * state the protocol operation would leave it in.  The caller keeps a block unmodified until
 * its completion (pquic_fec_batch.h), which is what lets the copy happen late.
 */
#define _GNU_SOURCE  /* sched_getaffinity / CPU_COUNT */
#include "pquic_fec_batch.h"

#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "fec_core.h"
#include "fecgpu.h"

enum { OP_GENERATE = 0, OP_RECOVER = 1, OP_WINDOW = 2 /* generate, window blocks */ };
#define GENERATES(op) ((op) != OP_RECOVER)
enum { MAX_OPEN = 32, MAX_STAGERS = 16, MAX_ENGINES = 4, STAGE_CHUNK = 256 /* blocks per staging work item */ };

typedef struct {
    uintptr_t base;
    size_t size;
    uint64_t dev;  /* device address of base */
} heap_t;

typedef struct {
    picoquic_cnx_t *cnx;
    pquic_fec_block_t *fb;
    pquic_fec_block_done_fn done;
    void *user;
    uint16_t maxl;
    int16_t nalloc;                /* generate: repair symbols allocated at submission */
} entry_t;

typedef struct job {
    struct job *next;
    int op, xor_scheme;
    uint32_t k, r, n, cap, stride;
    uint32_t cap_alloc;            /* blocks its per-block buffers hold: batch_blocks, or small_cap (job_get) */
    size_t src_bytes, rep_bytes;   /* allocated pinned sizes */
    uint8_t *src, *rep, *st;       /* pinned */
    uint32_t *fbn;                 /* pinned: block numbers (generate) */
    uint32_t *seeds;               /* pinned: [cap][r] repair FPID seeds (recover) */
    size_t seed_bytes;
    uint64_t *sp, *rp, *rec;       /* pinned, 2 words per block */
    entry_t *ent;
    pquic_repair_symbol_t **reps;  /* generate: [cap][r] symbols allocated at submission */
    size_t reps_cap;
    uint64_t t_first;
    int rc;
    int post;                      /* 1 once the engine ran: work items copy repairs out */
    uint32_t next_chunk, chunks_done;  /* staging work items claimed / finished (under the batcher lock) */
    int gather;                    /* generate with row tables (fecgpu_rlc_encode_rows) */
    uint64_t *srow, *rrow;         /* pinned: [cap][k] source / [cap][r] repair row device addresses (recover:
                                    * a missing source's entry is the row its recovered bytes go to) */
    pquic_source_symbol_t **pre;   /* recover gather: [cap][k] symbols allocated at submission for the missing
                                    * sources (written in place by the kernel), NULL where none */
    uint64_t *cpm;                 /* recover gather: [cap][2] missing sources whose recovered row is staged
                                    * (copied into its symbol at completion), set by the stagers */
    size_t pre_cap;
    uint64_t seq;                  /* flush order: completions are handed out in it */
    size_t srow_cap, rrow_cap;
    uint64_t src_dev, rep_dev;     /* device addresses of the staging rows */
    uint8_t *copy;                 /* gather: block needs its repairs copied out of the staging rows */
    uint32_t ncopy;                /* blocks flagged in copy[] (atomic while staging) */
    uint32_t *wrow;                /* window: pinned [cap] start row of each window in the stream */
    const pquic_source_symbol_t **rowsym;  /* window: [cap * k] the symbol of each stream row */
    uint32_t *order;               /* window: [cap] entries grouped by connection */
    size_t rowsym_cap;
    uint64_t nrows;                /* window: stream rows */
} job_t;

struct pquic_fec_batcher {
    pquic_fec_batch_cfg_t cfg;
    uint32_t stride;
    fecgpu_host_ctx_t *ctx[MAX_ENGINES];  /* one per engine thread: its own streams and device buffers */
    job_t *open[MAX_OPEN];
    job_t *free_jobs;
    pthread_t worker[MAX_ENGINES];
    int nengines;
    struct engine_arg { struct pquic_fec_batcher *b; int idx; } earg[MAX_ENGINES];
    pthread_t stager[MAX_STAGERS];
    int nstagers;
    pthread_mutex_t mu;
    pthread_cond_t cv_todo, cv_staged, cv_done;
    job_t *todo_head, *todo_tail, *staged_head, *staged_tail, *post_head, *post_tail, *done_head, *done_tail;
    int inflight, stop, stagers_done;
    uint32_t pf;                   /* completion prefetch distance in blocks (prefetch_syms; 0: off) */
    int done_ready;                /* atomic: the next job in flush order is finished (set under mu), so a
                                    * poll with nothing to complete takes no lock */
    uint64_t next_due;             /* caller thread: the oldest first-submission time of the open jobs
                                    * (UINT64_MAX: none), so a poll scans them only when one may be overdue */
    int last_slot;                 /* open[] slot of the last submission (caller thread) */
    job_t *completing;             /* finished job whose completions a bounded poll left part-done */
    uint32_t completing_i;         /* its next entry */
    pquic_fec_batch_stats_t stats;
    /* the provisioner (prov_main): one request at a time, under mu; the spares it made, under mu */
    pthread_t prov;
    int prov_started, prov_want, prov_op, prov_xor;
    uint32_t prov_k, prov_r;
    pthread_cond_t cv_prov;
    job_t *spares;
    uint64_t stats_spares;         /* spares made (under mu) */
    int reserve;                   /* idle jobs of a shape to keep, free + spare (PQUIC_FEC_BATCH_RESERVE, default 1) */
    uint32_t small_cap;            /* blocks of a job the caller allocates itself (0: full size; job_get) */
    int hold;                      /* deadline_hold on (PQUIC_FEC_BATCH_HOLD=0 turns it off, A/B) */
    uint64_t next_seq;             /* caller thread: sequence number of the next flushed job */
    uint64_t collect_seq;          /* caller thread: the job whose completions come next */
    uint64_t jobs_back;            /* caller thread: flushed jobs completed and back in free_jobs */
    /* registered arenas, sorted by base and disjoint; stagers look rows up under the read lock (one
     * lock per work item), registration takes the write lock, so connections may come and go while
     * batches run */
    heap_t *heaps;
    int nheaps, heaps_cap;
    pthread_rwlock_t heaps_mu;
};

/* Index of the last registered heap whose base is <= a, or -1 (caller holds heaps_mu). */
static int heap_floor(const pquic_fec_batcher_t *b, uintptr_t a) {
    int lo = 0, hi = b->nheaps - 1, f = -1;
    while (lo <= hi) {
        const int m = (lo + hi) >> 1;
        if (b->heaps[m].base <= a) {
            f = m;
            lo = m + 1;
        } else {
            hi = m - 1;
        }
    }
    return f;
}

/* Device address of [p, p + n) when it lies in one registered heap, else 0 (caller holds heaps_mu for
 * reading).  *hint: the heap the previous row was found in -- a block's rows, and a connection's
 * blocks, come from one arena -- tried before the binary search. */
static uint64_t heap_dev(const pquic_fec_batcher_t *b, const void *p, size_t n, int *hint) {
    const uintptr_t a = (uintptr_t)p;
    if ((a & 3) || !b->nheaps) return 0;
    int i = *hint;
    if (i < 0 || i >= b->nheaps || a - b->heaps[i].base >= b->heaps[i].size) i = heap_floor(b, a);
    if (i < 0) return 0;
    const heap_t *h = &b->heaps[i];
    if (a - h->base >= h->size || n > h->size - (a - h->base)) return 0;
    *hint = i;
    return h->dev + (a - h->base);
}

/* Page-locking a 16 MiB arena takes milliseconds: it happens outside heaps_mu, so stagers keep looking rows
 * up meanwhile; only the insertion into the sorted registry takes the lock (and re-checks for overlap). */
int pquic_fec_batch_register_heap(pquic_fec_batcher_t *b, void *base, size_t bytes) {
    if (!b || !base || !bytes) return -1;
    const uintptr_t a = (uintptr_t)base;
    if (fecgpu_host_register(base, bytes) != FECGPU_OK) return -1;
    uint64_t dev = 0;
    if (fecgpu_host_device_address(base, bytes, &dev) != FECGPU_OK) {
        fecgpu_host_unregister(base);
        return -1;
    }
    pthread_rwlock_wrlock(&b->heaps_mu);
    const int f = heap_floor(b, a);
    const int overlap = (f >= 0 && a - b->heaps[f].base < b->heaps[f].size) ||
                        (f + 1 < b->nheaps && b->heaps[f + 1].base - a < bytes);
    int rc = -1;
    if (!overlap) {
        if (b->nheaps == b->heaps_cap) {
            const int nc = b->heaps_cap ? 2 * b->heaps_cap : 64;
            heap_t *nh = realloc(b->heaps, sizeof *nh * (size_t)nc);
            if (!nh) goto out;
            b->heaps = nh;
            b->heaps_cap = nc;
        }
        memmove(&b->heaps[f + 2], &b->heaps[f + 1], sizeof *b->heaps * (size_t)(b->nheaps - f - 1));
        b->heaps[f + 1] = (heap_t){a, bytes, dev};
        b->nheaps++;
        rc = 0;
    }
out:
    pthread_rwlock_unlock(&b->heaps_mu);
    if (rc) fecgpu_host_unregister(base);
    return rc;
}

/* The arena leaves the registry under heaps_mu (no stager is between a lookup and its use of it) and is
 * unpinned after the lock is released: nothing queued refers to it (the caller's contract) and no later
 * lookup can find it. */
int pquic_fec_batch_unregister_heap(pquic_fec_batcher_t *b, void *base) {
    if (!b || !base) return -1;
    pthread_rwlock_wrlock(&b->heaps_mu);
    const int f = heap_floor(b, (uintptr_t)base);
    int found = 0;
    if (f >= 0 && b->heaps[f].base == (uintptr_t)base) {
        memmove(&b->heaps[f], &b->heaps[f + 1], sizeof *b->heaps * (size_t)(b->nheaps - f - 1));
        b->nheaps--;
        found = 1;
    }
    pthread_rwlock_unlock(&b->heaps_mu);
    return found && fecgpu_host_unregister(base) == FECGPU_OK ? 0 : -1;
}

static void job_free(job_t *j) {
    if (!j) return;
    fecgpu_host_free(j->wrow);
    free(j->rowsym);
    free(j->order);
    fecgpu_host_free(j->srow);
    fecgpu_host_free(j->rrow);
    free(j->pre);
    free(j->cpm);
    free(j->copy);
    fecgpu_host_free(j->src);
    fecgpu_host_free(j->rep);
    fecgpu_host_free(j->st);
    fecgpu_host_free(j->fbn);
    fecgpu_host_free(j->seeds);
    fecgpu_host_free(j->sp);
    free(j->ent);
    free(j->reps);
    free(j);
}

static uint64_t mono_us(void);
static uint32_t window_stride(const pquic_fec_batcher_t *b) { return (b->stride + 15u) & ~15u; }

/* A job's page-locked queue buffers for `cap` blocks of sb / rb bytes of rows (NULL on failure). */
static job_t *job_alloc(uint32_t cap, size_t sb, size_t rb) {
    job_t *j = calloc(1, sizeof *j);
    if (!j) return NULL;
    j->cap_alloc = cap;
    j->src_bytes = sb;
    j->rep_bytes = rb;
    j->src = fecgpu_host_alloc(sb);
    j->rep = fecgpu_host_alloc(rb ? rb : 4);
    j->st = fecgpu_host_alloc(cap);
    j->fbn = fecgpu_host_alloc((size_t)cap * 4);
    j->sp = fecgpu_host_alloc((size_t)cap * 48);  /* sp | rp | rec, 2 words each per block */
    j->ent = calloc(cap, sizeof *j->ent);
    if (!j->src || !j->rep || !j->st || !j->fbn || !j->sp || !j->ent) {
        job_free(j);
        return NULL;
    }
    return j;
}

/* Grows what a job needs for (op, scheme, k, r) beyond its row buffers -- seeds, gather tables, window tables,
 * repair pointers -- and sets it up for that use.  Touches nothing of the batcher but its configuration and
 * the heap count, so the provisioner thread may run it on a job no one else sees.  Returns 0, or -1 when an
 * allocation failed (the job stays valid for another use). */
static int job_prepare(pquic_fec_batcher_t *b, job_t *j, int op, int xor_scheme, uint32_t k, uint32_t r) {
    const uint32_t S = op == OP_WINDOW ? window_stride(b) : b->stride;
    /* the blocks of this shape its row buffers hold: a job allocated for a narrower shape (or a small one,
     * job_get) may hold fewer than its per-block arrays */
    uint32_t cap = j->cap_alloc;
    if (k && j->src_bytes / ((size_t)k * S) < cap) cap = (uint32_t)(j->src_bytes / ((size_t)k * S));
    if (r && j->rep_bytes / ((size_t)r * S) < cap) cap = (uint32_t)(j->rep_bytes / ((size_t)r * S));
    if (!cap) return -1;
    const size_t sb = (size_t)cap * k * S, rb = (size_t)cap * r * S;
    /* recover only: the repairs' FPID seeds, [cap][r] (grown on reuse like the repair table) */
    const size_t eb = (size_t)cap * (r ? r : 1) * 4;
    if (op == OP_RECOVER && j->seed_bytes < eb) {
        fecgpu_host_free(j->seeds);
        j->seed_bytes = 0;
        if (!(j->seeds = fecgpu_host_alloc(eb))) return -1;
        j->seed_bytes = eb;
    }
    /* gather tables (RLC generate or recover with a registered heap): grown on reuse like the repair table */
    j->gather = (op == OP_GENERATE || op == OP_RECOVER) && !xor_scheme && __atomic_load_n(&b->nheaps, __ATOMIC_RELAXED) > 0;
    if (j->gather && op == OP_RECOVER && j->pre_cap < (size_t)cap * k) {
        free(j->pre);
        j->pre_cap = (j->pre = calloc((size_t)cap * k, sizeof *j->pre)) ? (size_t)cap * k : 0;
        if (!j->pre) j->gather = 0;
    }
    if (j->gather && op == OP_RECOVER && !j->cpm && !(j->cpm = malloc(sizeof *j->cpm * 2 * (size_t)cap)))
        j->gather = 0;
    if (j->gather && (j->srow_cap < (size_t)cap * k || j->rrow_cap < (size_t)cap * r || !j->copy)) {
        if (j->srow_cap < (size_t)cap * k) {
            fecgpu_host_free(j->srow);
            j->srow_cap = (j->srow = fecgpu_host_alloc((size_t)cap * k * 8)) ? (size_t)cap * k : 0;
        }
        if (j->rrow_cap < (size_t)cap * r) {
            fecgpu_host_free(j->rrow);
            j->rrow_cap = (j->rrow = fecgpu_host_alloc((size_t)cap * r * 8)) ? (size_t)cap * r : 0;
        }
        if (!j->copy) j->copy = malloc(cap);
        if (!j->srow || !j->rrow || !j->copy) j->gather = 0;  /* staged instead */
    }
    if (j->gather && (fecgpu_host_device_address(j->src, sb, &j->src_dev) != FECGPU_OK ||
                      fecgpu_host_device_address(j->rep, rb ? rb : 4, &j->rep_dev) != FECGPU_OK))
        j->gather = 0;
    j->ncopy = 0;
    if (op == OP_WINDOW) {  /* window tables: start rows (page-locked), the stream's symbols, the grouping */
        if (!j->wrow) j->wrow = fecgpu_host_alloc((size_t)cap * 4);
        if (!j->order) j->order = malloc((size_t)cap * 4);
        if (j->rowsym_cap < (size_t)cap * k) {
            const pquic_source_symbol_t **rs = realloc((void *)j->rowsym, sizeof *rs * (size_t)cap * k);
            if (rs) {
                j->rowsym = rs;
                j->rowsym_cap = (size_t)cap * k;
            }
        }
        if (!j->wrow || !j->order || j->rowsym_cap < (size_t)cap * k) return -1;
    }
    j->nrows = 0;
    if (GENERATES(op) && j->reps_cap < (size_t)cap * r) {
        pquic_repair_symbol_t **nr = realloc(j->reps, sizeof *nr * (size_t)cap * r);
        if (!nr) return -1;
        j->reps = nr;
        j->reps_cap = (size_t)cap * r;
    }
    j->rp = j->sp + 2 * (size_t)cap;
    j->rec = j->rp + 2 * (size_t)cap;
    j->next = NULL;
    j->op = op;
    j->xor_scheme = xor_scheme;
    j->k = k;
    j->r = r;
    j->n = 0;
    j->cap = cap;
    j->stride = S;
    j->rc = 0;
    j->post = 0;
    j->next_chunk = j->chunks_done = 0;
    return 0;
}

/* Unlinks and returns the first job of *pp with rows for at least sb / rb bytes, or NULL. */
static job_t *take_fit(job_t **pp, size_t sb, size_t rb) {
    for (; *pp; pp = &(*pp)->next)
        if ((*pp)->src_bytes >= sb && (*pp)->rep_bytes >= rb) {
            job_t *j = *pp;
            *pp = j->next;
            j->next = NULL;
            return j;
        }
    return NULL;
}

static int count_fit(const job_t *j, size_t sb, size_t rb) {
    int n = 0;
    for (; j; j = j->next)
        if (j->src_bytes >= sb && j->rep_bytes >= rb) n++;
    return n;
}

/* Spare jobs.  Allocating a job's page-locked buffers takes milliseconds (6.3 ms for a 2048-block k16 r4 job,
 * profiles/r06_conn512_probe.log), and on the caller's thread it stalls every block queued meanwhile: the run
 * whose pipeline went one job deeper than ever before had its p99 at 8.7 ms against 2.3-3.8 in the others.  So
 * whenever the caller takes the last job that fits a shape, the provisioner thread allocates the next one
 * (same shape, prepared for the same use) and leaves it in b->spares, where job_get finds it.  One spare
 * covers one job more in flight per allocation time (about 20 ms for a 4096-block k16 r4 job); a stall that
 * deepens the pipeline faster (the paced leg under a kernel trace: 1-2 caller allocations of 20-45 ms in 3 of
 * 12 runs, profiles/r06_paced_probe.log) makes the caller allocate.  That allocation is a small job (job_get);
 * PQUIC_FEC_BATCH_RESERVE > 1 has the provisioner keep more idle full-size jobs of the shape (free or spare). */
static void *prov_main(void *arg) {
    pquic_fec_batcher_t *b = arg;
    pthread_mutex_lock(&b->mu);
    for (;;) {
        while (!b->stop && !b->prov_want) pthread_cond_wait(&b->cv_prov, &b->mu);
        if (b->stop) break;
        const int op = b->prov_op, xs = b->prov_xor;
        const uint32_t k = b->prov_k, r = b->prov_r;
        pthread_mutex_unlock(&b->mu);
        const uint32_t cap = b->cfg.batch_blocks, S = op == OP_WINDOW ? window_stride(b) : b->stride;
        job_t *j = job_alloc(cap, (size_t)cap * k * S, (size_t)cap * r * S);
        if (j && job_prepare(b, j, op, xs, k, r)) {
            job_free(j);
            j = NULL;
        }
        pthread_mutex_lock(&b->mu);
        if (j) {
            j->next = b->spares;
            b->spares = j;
            b->stats_spares++;
        }
        b->prov_want = 0;
    }
    pthread_mutex_unlock(&b->mu);
    return NULL;
}

/* A job for (op, scheme, k, r): from the free list, else a spare, else a small job from the free list, else
 * allocated here (counted).  What the caller allocates itself is small (b->small_cap blocks, a sixteenth of
 * batch_blocks when that is at least 1024, window jobs excepted): page-locking a full 4096-block k16 r4 job
 * takes about 20 ms, a 256-block one about 1, and a small job only flushes sooner (at its own capacity).
 * The provisioner makes the full-size ones. */
static job_t *job_get(pquic_fec_batcher_t *b, int op, int xor_scheme, uint32_t k, uint32_t r) {
    const uint32_t cap = b->cfg.batch_blocks, S = op == OP_WINDOW ? window_stride(b) : b->stride;
    const size_t sb = (size_t)cap * k * S, rb = (size_t)cap * r * S;
    job_t *j = take_fit(&b->free_jobs, sb, rb);
    if (!j && b->prov_started) {
        pthread_mutex_lock(&b->mu);
        j = take_fit(&b->spares, sb, rb);
        pthread_mutex_unlock(&b->mu);
    }
    const uint32_t small = b->prov_started && op != OP_WINDOW ? b->small_cap : 0;
    if (!j && small) j = take_fit(&b->free_jobs, (size_t)small * k * S, (size_t)small * r * S);
    if (!j) {
        const uint32_t c = small ? small : cap;
        const uint64_t t_alloc = mono_us();
        if (!(j = job_alloc(c, (size_t)c * k * S, (size_t)c * r * S))) return NULL;
        b->stats.jobs_allocated++;
        b->stats.job_alloc_us += mono_us() - t_alloc;
    }
    if (job_prepare(b, j, op, xor_scheme, k, r)) {
        j->next = b->free_jobs;
        b->free_jobs = j;
        return NULL;
    }
    /* fewer idle jobs of this shape than the reserve: have the next one made off this thread */
    const int idle = count_fit(b->free_jobs, sb, rb);
    if (b->prov_started && idle < b->reserve) {
        pthread_mutex_lock(&b->mu);
        if (!b->prov_want && idle + count_fit(b->spares, sb, rb) < b->reserve) {
            b->prov_want = 1;
            b->prov_op = op;
            b->prov_xor = xor_scheme;
            b->prov_k = k;
            b->prov_r = r;
            pthread_cond_signal(&b->cv_prov);
        }
        pthread_mutex_unlock(&b->mu);
    }
    return j;
}

static void run_engine(fecgpu_host_ctx_t *c, job_t *j) {
    const uint32_t S = j->stride;
    if (j->op == OP_WINDOW)
        j->rc = fecgpu_rlc_window_encode_host(c, j->src, j->nrows, j->wrow, j->n, j->k, j->r, S, j->rep);
    else if (j->gather && j->op == OP_RECOVER)
        j->rc = fecgpu_rlc_decode_rows_host(c, j->srow, j->rrow, j->n, j->k, j->r, S, j->seeds, j->sp, j->rp, j->st,
                                            j->rec);
    else if (j->gather)
        j->rc = fecgpu_rlc_encode_rows_host(c, j->srow, j->rrow, j->n, j->k, j->r, S, j->fbn);
    else if (j->op == OP_GENERATE)
        j->rc = j->xor_scheme ? fecgpu_xor_encode_host(c, j->src, j->rep, j->n, j->k, S)
                              : fecgpu_rlc_encode_host(c, j->src, j->rep, j->n, j->k, j->r, S, 0, j->fbn);
    else
        j->rc = j->xor_scheme
                    ? fecgpu_xor_decode_host(c, j->src, j->rep, j->n, j->k, S, j->sp, j->rp, j->st, j->rec)
                    : fecgpu_rlc_decode_host_seeded(c, j->src, j->rep, j->n, j->k, j->r, S, j->seeds, j->sp, j->rp,
                                                    j->st, j->rec);
}

/* Gather: the row tables of blocks [i0, i1).  A source row is read in place when it lies in a
 * registered heap and is as long as the block (shorter ones are zero-padded, :41-55, so they are
 * staged); a repair row is written in place when its symbol is in a heap and as long as the stride
 * (the kernel writes `stride` bytes), else into the staging rows and copied out after the engine. */
static void gather_recover_blocks(pquic_fec_batcher_t *b, job_t *j, uint32_t i0, uint32_t i1);

static void gather_blocks(pquic_fec_batcher_t *b, job_t *j, uint32_t i0, uint32_t i1) {
    if (j->op == OP_RECOVER) {
        gather_recover_blocks(b, j, i0, i1);
        return;
    }
    const uint32_t S = j->stride, k = j->k, r = j->r;
    uint32_t ncopy = 0;
    uint64_t inplace = 0, staged = 0;
    int hint = -1;
    pthread_rwlock_rdlock(&b->heaps_mu);
    for (uint32_t i = i0; i < i1; i++) {
        const entry_t *e = &j->ent[i];
        const pquic_fec_block_t *fb = e->fb;
        for (uint32_t x = 0; x < k; x++) {
            const pquic_source_symbol_t *ss = fb->source_symbols[x];
            const size_t o = ((size_t)i * k + x) * S;
            uint64_t d = ss && ss->data_length == e->maxl ? heap_dev(b, ss->data, S, &hint) : 0;
            if (!d) {  /* staged, zero-padded to the stride */
                const uint16_t n = ss ? ss->data_length : 0;
                if (n) memcpy(j->src + o, ss->data, n);
                memset(j->src + o + n, 0, S - n);
                d = j->src_dev + o;
                staged++;
            } else {
                inplace++;
            }
            j->srow[(size_t)i * k + x] = d;
        }
        uint8_t cp = 0;
        for (uint32_t x = 0; x < r; x++) {
            pquic_repair_symbol_t *rs = (int)x < e->nalloc ? j->reps[(size_t)i * r + x] : NULL;
            uint64_t d = rs && e->maxl == S ? heap_dev(b, rs->data, S, &hint) : 0;
            if (!d) {
                d = j->rep_dev + ((size_t)i * r + x) * S;
                cp |= rs != NULL;
                staged += rs != NULL;
            } else {
                inplace++;
            }
            j->rrow[(size_t)i * r + x] = d;
        }
        j->copy[i] = cp;
        ncopy += cp;
    }
    pthread_rwlock_unlock(&b->heaps_mu);
    if (ncopy) __atomic_fetch_add(&j->ncopy, ncopy, __ATOMIC_RELAXED);
    __atomic_fetch_add(&b->stats.rows_in_place, inplace, __ATOMIC_RELAXED);
    __atomic_fetch_add(&b->stats.rows_staged, staged, __ATOMIC_RELAXED);
}

/* Recover gather: the tables of blocks [i0, i1).  A block is read in place only when its length (the
 * first present repair's, rlc_fec_scheme_gf256.c:186) is the stride -- the kernel reads and writes
 * `stride` bytes per row and its zero rule looks at all of them (:98-101), so no byte past max_length may
 * reach it -- and then a received source or repair row is read where it lies when it is in a registered
 * heap and at least that long (longer ones are read up to max_length, the reference's truncation, :205);
 * a missing source's row is the symbol allocated for it at submission.  Everything else is staged as
 * fec_recover_stage stages it (truncated, zero-padded), recovered bytes into the staging row. */
static void gather_recover_blocks(pquic_fec_batcher_t *b, job_t *j, uint32_t i0, uint32_t i1) {
    const uint32_t S = j->stride, k = j->k, r = j->r;
    uint64_t inplace = 0, staged = 0;
    int hint = -1;
    pthread_rwlock_rdlock(&b->heaps_mu);
    for (uint32_t i = i0; i < i1; i++) {
        const entry_t *e = &j->ent[i];
        const pquic_fec_block_t *fb = e->fb;
        const int whole = e->maxl == S;
        uint64_t *sp = j->sp + 2 * (size_t)i, *rp = j->rp + 2 * (size_t)i, *cpm = j->cpm + 2 * (size_t)i;
        sp[0] = sp[1] = rp[0] = rp[1] = cpm[0] = cpm[1] = 0;
        for (uint32_t x = 0; x < k; x++) {
            const pquic_source_symbol_t *ss = fb->source_symbols[x];
            const size_t o = ((size_t)i * k + x) * S;
            uint64_t d = 0;
            if (ss) {
                sp[x >> 6] |= 1ull << (x & 63);
                d = whole && ss->data_length >= S ? heap_dev(b, ss->data, S, &hint) : 0;
                if (!d) {
                    const uint16_t n = ss->data_length < e->maxl ? ss->data_length : e->maxl;
                    memcpy(j->src + o, ss->data, n);
                    memset(j->src + o + n, 0, S - n);
                    staged++;
                } else {
                    inplace++;
                }
            } else {
                const pquic_source_symbol_t *pre = j->pre[(size_t)i * k + x];
                d = whole && pre ? heap_dev(b, pre->data, S, &hint) : 0;
                inplace += d != 0;
                if (!d) cpm[x >> 6] |= 1ull << (x & 63);  /* recovered into the staging row */
            }
            j->srow[(size_t)i * k + x] = d ? d : j->src_dev + o;
        }
        for (uint32_t x = 0; x < r; x++) {
            const pquic_repair_symbol_t *rs = fb->repair_symbols[x];
            const size_t o = ((size_t)i * r + x) * S;
            uint64_t d = 0;
            if (rs) {
                rp[x >> 6] |= 1ull << (x & 63);
                d = whole && rs->data_length >= S ? heap_dev(b, rs->data, S, &hint) : 0;
                if (!d) {
                    const uint16_t n = rs->data_length < e->maxl ? rs->data_length : e->maxl;
                    memcpy(j->rep + o, rs->data, n);
                    memset(j->rep + o + n, 0, S - n);
                    staged++;
                } else {
                    inplace++;
                }
            }
            j->rrow[(size_t)i * r + x] = d ? d : j->rep_dev + o;  /* absent repairs: never read */
            /* every equation is seeded by its repair's own FPID (rlc_fec_scheme_gf256.c:200) */
            j->seeds[(size_t)i * r + x] = rs ? rs->fpid.f.source_fpid.raw : 0;
        }
    }
    pthread_rwlock_unlock(&b->heaps_mu);
    __atomic_fetch_add(&b->stats.rows_in_place, inplace, __ATOMIC_RELAXED);
    __atomic_fetch_add(&b->stats.rows_staged, staged, __ATOMIC_RELAXED);
}

/* Copies blocks [i0, i1) of a job into its page-locked rows (the stage halves of fec_core.c). */
static void stage_blocks(job_t *j, uint32_t i0, uint32_t i1) {
    const uint32_t S = j->stride, k = j->k, r = j->r;
    for (uint32_t i = i0; i < i1; i++) {
        const entry_t *e = &j->ent[i];
        uint8_t *src = j->src + (size_t)i * k * S;
        if (j->op == OP_GENERATE)
            fec_generate_stage(e->fb, src, S);
        else
            fec_recover_stage(e->fb, j->xor_scheme, e->maxl, src, j->rep + (size_t)i * r * S, S, j->sp + 2 * (size_t)i,
                              j->rp + 2 * (size_t)i, j->seeds + (size_t)i * r);
    }
}

/* Window job: the stream layout, then its rows.  Entries are grouped by connection (stable), and a
 * connection's windows extend one run of rows: a window whose first symbol is among the run's last
 * rows, and whose symbols continue the run as far as it goes, starts there and appends only its new
 * symbols; any other window starts a fresh run of its k symbols.  Rows are zero-padded to the stride
 * (the reference pads each window's symbols to its max_length, which the copy-out then keeps). */
static int cmp_cnx(const void *a, const void *b, void *arg) {
    const job_t *j = arg;
    const uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    const uintptr_t cx = (uintptr_t)j->ent[x].cnx, cy = (uintptr_t)j->ent[y].cnx;
    return cx != cy ? (cx < cy ? -1 : 1) : (x > y) - (x < y);
}

static void stage_windows(job_t *j) {
    const uint32_t S = j->stride, k = j->k;
    for (uint32_t i = 0; i < j->n; i++) j->order[i] = i;
    qsort_r(j->order, j->n, sizeof *j->order, cmp_cnx, j);
    uint64_t nrows = 0, run = 0;  /* run: first row of the current connection's run */
    const picoquic_cnx_t *cur = NULL;
    for (uint32_t o = 0; o < j->n; o++) {
        const uint32_t i = j->order[o];
        pquic_source_symbol_t *const *ss = j->ent[i].fb->source_symbols;
        if (o == 0 || j->ent[i].cnx != cur) {
            cur = j->ent[i].cnx;
            run = nrows;
        }
        uint64_t start = nrows;
        const uint64_t lo = nrows - run > k ? nrows - k : run;
        for (uint64_t q = nrows; q-- > lo;) {  /* the newest row holding the window's first symbol */
            if (!ss[0] || j->rowsym[q] != ss[0]) continue;
            uint32_t x = 0;
            while (x < k && q + x < nrows && ss[x] && j->rowsym[q + x] == ss[x]) x++;
            if (q + x == nrows || x == k) start = q;  /* continues the run to its end, or lies within it */
            break;
        }
        j->wrow[i] = (uint32_t)start;
        for (uint64_t x = nrows - start; x < k; x++) j->rowsym[nrows++] = ss[x];
    }
    j->nrows = nrows;
    for (uint64_t q = 0; q < nrows; q++) {
        const pquic_source_symbol_t *sym = j->rowsym[q];
        const uint16_t n = sym ? sym->data_length : 0;
        if (n) memcpy(j->src + q * S, sym->data, n);
        memset(j->src + q * S + n, 0, S - n);
    }
}

/* Generate, after the engine: repair rows of blocks [i0, i1) into the symbols allocated at
 * submission (the copy half of fec_generate_finish). */
static void copy_out_blocks(job_t *j, uint32_t i0, uint32_t i1) {
    const uint32_t S = j->stride, r = j->r;
    for (uint32_t i = i0; i < i1; i++) {
        const entry_t *e = &j->ent[i];
        if (j->gather && !j->copy[i]) continue;  /* every row written in place by the kernel */
        for (int x = 0; x < e->nalloc; x++) {
            const size_t q = (size_t)i * r + x;
            /* a block's repairs may be split between the arena and other memory (an arena filled part
             * way through the block): only the rows the kernel wrote into the staging area are copied */
            if (j->gather && j->rrow[q] != j->rep_dev + q * S) continue;
            memcpy(j->reps[q]->data, j->rep + q * S, e->maxl);
        }
    }
}

static uint64_t mono_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

static void push(job_t **head, job_t **tail, job_t *j) {
    j->next = NULL;
    if (*tail) (*tail)->next = j; else *head = j;
    *tail = j;
}

/* Finished jobs wait in flush order (two engine threads, and generate jobs that take a copy-out pass,
 * can finish out of it), so completions reach the caller in the order its blocks were submitted, across
 * batches too, as the synchronous operations complete (caller holds b->mu). */
static void push_done(pquic_fec_batcher_t *b, job_t *j) {
    if (!b->done_tail || b->done_tail->seq < j->seq) {
        push(&b->done_head, &b->done_tail, j);
    } else {
        job_t **pp = &b->done_head;
        while (*pp && (*pp)->seq < j->seq) pp = &(*pp)->next;
        j->next = *pp;
        *pp = j;
    }
    __atomic_store_n(&b->done_ready, b->done_head->seq == b->collect_seq, __ATOMIC_RELEASE);
}

/* Stager threads split every job into work items of STAGE_CHUNK blocks, so several threads copy
 * one job at once (a 4096-block k16 job is 79 MB of rows: one thread alone bounded the saturated
 * rate); the thread finishing a job's last item hands it on: a staged job to the engine thread,
 * a copied-out one to the caller.  Copy-out items go first (they finish jobs). */
static void *stager_main(void *arg) {
    pquic_fec_batcher_t *b = arg;
    pthread_mutex_lock(&b->mu);
    for (;;) {
        while (!b->todo_head && !b->post_head && !b->stop) pthread_cond_wait(&b->cv_todo, &b->mu);
        job_t **head = b->post_head ? &b->post_head : &b->todo_head;
        job_t **tail = b->post_head ? &b->post_tail : &b->todo_tail;
        if (!*head) break;  /* stop requested and nothing left */
        job_t *j = *head;
        /* a window job's layout is one item (it is sequential); its copy-out splits like any other */
        const uint32_t nchunks = j->op == OP_WINDOW && !j->post ? 1 : (j->n + STAGE_CHUNK - 1) / STAGE_CHUNK;
        const uint32_t c = j->next_chunk++;
        if (j->next_chunk >= nchunks) {  /* every item of this job is claimed: the next job is up */
            *head = j->next;
            if (!*head) *tail = NULL;
        }
        pthread_mutex_unlock(&b->mu);
        const uint64_t t0 = mono_us();
        const uint32_t i0 = c * STAGE_CHUNK, i1 = i0 + STAGE_CHUNK < j->n ? i0 + STAGE_CHUNK : j->n;
        if (j->post) copy_out_blocks(j, i0, i1);
        else if (j->op == OP_WINDOW) stage_windows(j);
        else if (j->gather) gather_blocks(b, j, i0, i1);
        else stage_blocks(j, i0, i1);
        const uint64_t dt = mono_us() - t0;
        pthread_mutex_lock(&b->mu);
        b->stats.stage_us += dt;
        if (++j->chunks_done == nchunks) {
            if (j->post) {
                push_done(b, j);
                b->inflight--;
                pthread_cond_broadcast(&b->cv_done);
            } else {
                push(&b->staged_head, &b->staged_tail, j);
                pthread_cond_signal(&b->cv_staged);
            }
        }
    }
    b->stagers_done++;
    pthread_cond_broadcast(&b->cv_staged);
    pthread_mutex_unlock(&b->mu);
    return NULL;
}

/* CPUs this process may use: the affinity mask bounded by a cgroup v2 CPU quota when one is set
 * (a shared host can list every CPU in the mask and grant a slice of them). */
static int host_cpus(void) {
    cpu_set_t cs;
    int n = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : 2;
    FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r");
    if (f) {
        char q[32] = {0};
        long per = 0;
        if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
            const long quota = (atol(q) + per / 2) / per;
            if (quota >= 1 && quota < n) n = (int)quota;
        }
        fclose(f);
    }
    return n < 1 ? 1 : n;
}

/* The CPUs nearest the device within this process's affinity mask: the engine and stager threads run
 * there, so the page-locked rows they fill and the registered symbols the kernels read sit on the
 * device's socket (a GPU box's second socket reaches the device over the inter-socket link).  Empty
 * when unknown or disjoint from the mask. */
static void local_cpus(int device, cpu_set_t *out) {
    CPU_ZERO(out);
    char list[512];
    cpu_set_t aff;
    if (fecgpu_device_local_cpus(device, list, sizeof list) != FECGPU_OK || sched_getaffinity(0, sizeof aff, &aff))
        return;
    for (char *p = list; *p;) {
        char *end;
        long a = strtol(p, &end, 10), b = a;
        if (end == p) break;
        if (*end == '-') b = strtol(end + 1, &end, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            if (c >= 0 && CPU_ISSET(c, &aff)) CPU_SET(c, out);
        p = *end == ',' ? end + 1 : end;
        if (*end != ',') break;
    }
}

/* Engine threads (PQUIC_FEC_BATCH_ENGINES, default 2): each runs staged jobs through its own host
 * context, so one job's kernels (reading and writing page-locked rows over PCIe) overlap the next job's
 * launch and the previous one's synchronisation instead of leaving the bus idle between jobs. */
static void *worker_main(void *arg) {
    const struct engine_arg *ea = arg;
    pquic_fec_batcher_t *b = ea->b;
    pthread_mutex_lock(&b->mu);
    for (;;) {
        while (!b->staged_head && b->stagers_done < b->nstagers) pthread_cond_wait(&b->cv_staged, &b->mu);
        if (!b->staged_head) break;  /* every stager has stopped and nothing is left */
        job_t *j = b->staged_head;
        b->staged_head = j->next;
        if (!b->staged_head) b->staged_tail = NULL;
        pthread_mutex_unlock(&b->mu);
        const uint64_t t0 = mono_us();
        run_engine(b->ctx[ea->idx], j);
        const uint64_t dt = mono_us() - t0;
        pthread_mutex_lock(&b->mu);
        b->stats.engine_us += dt;
        if (GENERATES(j->op) && !j->rc && (!j->gather || j->ncopy)) {  /* repair rows to their symbols */
            j->post = 1;
            j->next_chunk = j->chunks_done = 0;
            push(&b->post_head, &b->post_tail, j);
            pthread_cond_broadcast(&b->cv_todo);
        } else {
            push_done(b, j);
            b->inflight--;
            pthread_cond_broadcast(&b->cv_done);
        }
    }
    pthread_mutex_unlock(&b->mu);
    return NULL;
}

pquic_fec_batcher_t *pquic_fec_batcher_create(const pquic_fec_batch_cfg_t *cfg) {
    if (!cfg || cfg->batch_blocks < 1 || cfg->max_symbol < 1 || cfg->max_symbol > 32767 || cfg->nstreams < 1)
        return NULL;
    pquic_fec_batcher_t *b = calloc(1, sizeof *b);
    if (!b) return NULL;
    b->cfg = *cfg;
    b->stride = fec_pad4(cfg->max_symbol);
    b->next_due = UINT64_MAX;
    const char *pfs = getenv("PQUIC_FEC_BATCH_PREFETCH");  /* read once per batcher, like the thread counts */
    b->pf = pfs && atoi(pfs) >= 0 ? (uint32_t)atoi(pfs) : 8;
    if (b->pf > 64) b->pf = 64;
    const size_t chunk = (size_t)cfg->batch_blocks * 20 * b->stride / (size_t)cfg->nstreams;
    const char *ne = getenv("PQUIC_FEC_BATCH_ENGINES");
    b->nengines = ne && atoi(ne) > 0 ? atoi(ne) : 2;
    if (b->nengines > MAX_ENGINES) b->nengines = MAX_ENGINES;
    for (int e = 0; e < b->nengines; e++) {
        b->ctx[e] = fecgpu_host_ctx_create(cfg->device, cfg->nstreams, chunk < (1u << 20) ? (1u << 20) : chunk);
        if (!b->ctx[e]) {
            for (int x = 0; x < e; x++) fecgpu_host_ctx_destroy(b->ctx[x]);
            free(b);
            return NULL;
        }
    }
    pthread_mutex_init(&b->mu, NULL);
    pthread_rwlock_init(&b->heaps_mu, NULL);
    pthread_cond_init(&b->cv_todo, NULL);
    pthread_cond_init(&b->cv_staged, NULL);
    pthread_cond_init(&b->cv_done, NULL);
    pthread_cond_init(&b->cv_prov, NULL);
    /* copy threads: half the CPUs of the process's share (the caller and the engine thread keep the
     * rest), at least 2; PQUIC_FEC_BATCH_STAGERS overrides, read once per batcher */
    const char *ns = getenv("PQUIC_FEC_BATCH_STAGERS");
    const int half = host_cpus() / 2;
    b->nstagers = ns && atoi(ns) > 0 ? atoi(ns) : (half > 2 ? half : 2);
    if (b->nstagers > MAX_STAGERS) b->nstagers = MAX_STAGERS;
    int started = 0;
    cpu_set_t near;
    local_cpus(cfg->device, &near);
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    if (CPU_COUNT(&near)) pthread_attr_setaffinity_np(&attr, sizeof near, &near);
    for (; started < b->nstagers; started++)
        if (pthread_create(&b->stager[started], &attr, stager_main, b)) break;
    int engines = 0;
    if (started == b->nstagers)
        for (; engines < b->nengines; engines++) {
            b->earg[engines] = (struct engine_arg){b, engines};
            if (pthread_create(&b->worker[engines], &attr, worker_main, &b->earg[engines])) break;
        }
    pthread_attr_destroy(&attr);
    if (engines < b->nengines) {
        pthread_mutex_lock(&b->mu);
        b->stop = 1;
        b->nstagers = started;
        pthread_cond_broadcast(&b->cv_todo);
        pthread_mutex_unlock(&b->mu);
        for (int i = 0; i < started; i++) pthread_join(b->stager[i], NULL);
        for (int i = 0; i < engines; i++) pthread_join(b->worker[i], NULL);
        pthread_cond_destroy(&b->cv_todo);
        pthread_cond_destroy(&b->cv_staged);
        pthread_cond_destroy(&b->cv_done);
        pthread_cond_destroy(&b->cv_prov);
        pthread_mutex_destroy(&b->mu);
        pthread_rwlock_destroy(&b->heaps_mu);
        for (int e = 0; e < b->nengines; e++) fecgpu_host_ctx_destroy(b->ctx[e]);
        free(b);
        return NULL;
    }
    /* the provisioner (spare jobs); without it every job is allocated on the caller's thread.
     * PQUIC_FEC_BATCH_SPARES=0 turns it off (A/B), read once per batcher like the thread counts */
    const char *sp = getenv("PQUIC_FEC_BATCH_SPARES");
    b->prov_started = !(sp && atoi(sp) == 0) && pthread_create(&b->prov, NULL, prov_main, b) == 0;
    const char *rs = getenv("PQUIC_FEC_BATCH_RESERVE");  /* idle jobs per shape the provisioner keeps (A/B) */
    b->reserve = rs && atoi(rs) > 0 ? (atoi(rs) < 8 ? atoi(rs) : 8) : 1;
    const char *sm = getenv("PQUIC_FEC_BATCH_SMALL");  /* 0: the caller allocates full-size jobs (A/B) */
    b->small_cap = cfg->batch_blocks >= 1024 && !(sm && atoi(sm) == 0) ? cfg->batch_blocks / 16 : 0;
    const char *ho = getenv("PQUIC_FEC_BATCH_HOLD");
    b->hold = !(ho && atoi(ho) == 0);
    return b;
}

static void flush_job(pquic_fec_batcher_t *b, int slot, uint64_t *counter) {
    job_t *j = b->open[slot];
    b->open[slot] = NULL;
    if (!j) return;
    if (j->n && j->t_first == b->next_due) {  /* the oldest open job leaves: the next oldest */
        b->next_due = UINT64_MAX;
        for (int s = 0; s < MAX_OPEN; s++)
            if (b->open[s] && b->open[s]->n && b->open[s]->t_first < b->next_due) b->next_due = b->open[s]->t_first;
    }
    if (!j->n) {  /* nothing queued: back to the free list */
        j->next = b->free_jobs;
        b->free_jobs = j;
        return;
    }
    (*counter)++;
    b->stats.batches++;
    j->seq = b->next_seq++;
    pthread_mutex_lock(&b->mu);
    j->next = NULL;
    if (b->todo_tail) b->todo_tail->next = j; else b->todo_head = j;
    b->todo_tail = j;
    b->inflight++;
    pthread_cond_signal(&b->cv_todo);
    pthread_mutex_unlock(&b->mu);
}

/* The open job for a key, opening one (and if every slot is taken, flushing the oldest). */
static job_t *open_job(pquic_fec_batcher_t *b, int op, int xor_scheme, uint32_t k, uint32_t r, int *slot_out) {
    job_t *hit = b->open[b->last_slot];  /* consecutive blocks of one sender share a key */
    if (hit && hit->op == op && hit->xor_scheme == xor_scheme && hit->k == k && hit->r == r) {
        *slot_out = b->last_slot;
        return hit;
    }
    int free_slot = -1, oldest = -1;
    for (int s = 0; s < MAX_OPEN; s++) {
        job_t *j = b->open[s];
        if (!j) {
            if (free_slot < 0) free_slot = s;
            continue;
        }
        if (j->op == op && j->xor_scheme == xor_scheme && j->k == k && j->r == r) {
            *slot_out = b->last_slot = s;
            return j;
        }
        if (oldest < 0 || j->t_first < b->open[oldest]->t_first) oldest = s;
    }
    if (free_slot < 0) {
        flush_job(b, oldest, &b->stats.flushed_full);
        free_slot = oldest;
    }
    job_t *j = job_get(b, op, xor_scheme, k, r);
    if (!j) return NULL;
    b->open[free_slot] = j;
    *slot_out = b->last_slot = free_slot;
    return j;
}

static int submit(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int op, int xor_scheme,
                  uint64_t now_us, pquic_fec_block_done_fn done, void *user) {
    if (!b || !fb || !done) return -1;
    if (!g_fec_bound) {
        b->stats.immediate++;
        done(user, fb, PQUIC_FEC_ERR_UNBOUND);
        return 0;
    }
    uint16_t maxl = 0;
    const uint32_t k = fb->total_source_symbols;
    uint32_t r = fb->total_repair_symbols;
    if (GENERATES(op)) {
        const int chk = fec_generate_check(fb, xor_scheme, &maxl);
        if (chk) {  /* the reference returns 1, nothing done; totals past 100 slots are an error */
            b->stats.immediate++;
            if (chk == FEC_STAGE_REJECT) FEC_STAT_ADD(errors, 1);
            done(user, fb, chk == FEC_STAGE_REJECT ? PQUIC_FEC_ERR_UNBOUND : 1);
            return 0;
        }
    } else {
        const int chk = fec_recover_check(fb, xor_scheme, &maxl);
        if (chk != FEC_STAGE_OK) {
            b->stats.immediate++;
            if (chk == FEC_STAGE_REJECT) FEC_STAT_ADD(errors, 1);
            done(user, fb, chk == FEC_STAGE_REJECT ? PQUIC_FEC_ERR_UNBOUND : (protoop_arg_t)chk);
            return 0;
        }
        if (xor_scheme) r = 1;
    }
    if (maxl > b->cfg.max_symbol) return -1;
    int slot;
    job_t *j = open_job(b, op, xor_scheme, k, r, &slot);
    if (!j) return -1;
    const uint32_t i = j->n;
    j->fbn[i] = fb->fec_block_number & 0xffffffu;  /* rows are copied later, by a stager */
    j->ent[i] = (entry_t){cnx, fb, done, user, maxl, -1};
    if (GENERATES(op))  /* the protocol operation's allocations, in its order, on this thread */
        j->ent[i].nalloc = (int16_t)fec_generate_alloc(cnx, fb, maxl, j->reps + (size_t)i * r);
    else if (j->gather)  /* the recovered symbols, so the kernel writes them where they will stay */
        fec_recover_alloc(cnx, fb, maxl, j->pre + (size_t)i * k);
    if (!i) {
        j->t_first = now_us;
        if (now_us < b->next_due) b->next_due = now_us;
    }
    j->n = i + 1;
    b->stats.submitted++;
    if (j->n == j->cap) flush_job(b, slot, &b->stats.flushed_full);
    return 0;
}

int pquic_fec_batch_generate(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int xor_scheme,
                             uint64_t now_us, pquic_fec_block_done_fn done, void *user) {
    return submit(b, cnx, fb, OP_GENERATE, xor_scheme ? 1 : 0, now_us, done, user);
}

int pquic_fec_batch_generate_window(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb,
                                    uint64_t now_us, pquic_fec_block_done_fn done, void *user) {
    /* window jobs need block number 0 (shared coefficients) and a stream the kernel's 32-bit offsets
     * reach; anything else is an ordinary block */
    if (!b || !fb) return -1;
    const size_t worst = ((size_t)b->cfg.batch_blocks + 1) * fb->total_source_symbols * window_stride(b);
    if (fb->fec_block_number != 0 || worst >= ((size_t)1 << 31))
        return submit(b, cnx, fb, OP_GENERATE, 0, now_us, done, user);
    return submit(b, cnx, fb, OP_WINDOW, 0, now_us, done, user);
}

int pquic_fec_batch_recover(pquic_fec_batcher_t *b, picoquic_cnx_t *cnx, pquic_fec_block_t *fb, int xor_scheme,
                            uint64_t now_us, pquic_fec_block_done_fn done, void *user) {
    return submit(b, cnx, fb, OP_RECOVER, xor_scheme ? 1 : 0, now_us, done, user);
}

/* The symbols a completion hands to the framework -- a generate's repairs, a gathered recover's
 * recovered sources -- are what the framework touches next (it sends their bytes, then frees them; the
 * plugin allocator reads the slot header just before the data, picoquic/memory.c:123-127).  The kernel
 * wrote their data over PCIe, so those lines are in no CPU cache.  Entry i + 2P's symbol structs and
 * entry i + P's data lines are prefetched while entry i completes (P = b->pf, 0: off), so the misses
 * overlap instead of stalling the caller one block at a time. */
/* the lines of [p, p + n) */
static void prefetch_range(const void *p, size_t n) {
    const uintptr_t a = (uintptr_t)p & ~(uintptr_t)63, e = (uintptr_t)p + n;
    for (uintptr_t x = a; x < e; x += 64) __builtin_prefetch((const void *)x, 1);
}

static void prefetch_syms(const job_t *j, uint32_t i, int data) {
    if (data) {  /* the block's symbol pointers the completion writes (and the framework then reads) */
        pquic_fec_block_t *fb = j->ent[i].fb;
        if (GENERATES(j->op))
            prefetch_range(&fb->repair_symbols[0], sizeof fb->repair_symbols[0] * (j->ent[i].nalloc > 0 ? j->ent[i].nalloc : 1));
        else
            prefetch_range(&fb->source_symbols[0], sizeof fb->source_symbols[0] * j->k);
    }
    if (GENERATES(j->op)) {
        const entry_t *e = &j->ent[i];
        pquic_repair_symbol_t *const *reps = j->reps + (size_t)i * j->r;
        for (int x = 0; x < e->nalloc; x++) {
            if (!data) {
                __builtin_prefetch(reps[x], 0);
            } else {
                const uint8_t *d = reps[x]->data;
                __builtin_prefetch(d - 8, 1);
                __builtin_prefetch(d, 1);
            }
        }
    } else {
        if (data) {  /* the status and masks the kernel wrote, the stagers' copy masks */
            __builtin_prefetch(j->st + i, 0);
            __builtin_prefetch(j->rec + 2 * (size_t)i, 0);
            if (j->gather) __builtin_prefetch(j->cpm + 2 * (size_t)i, 0);
        }
        if (!j->gather) return;
        pquic_source_symbol_t *const *pre = j->pre + (size_t)i * j->k;
        for (uint32_t x = 0; x < j->k; x++) {
            if (!pre[x]) continue;
            if (!data) {
                __builtin_prefetch(pre[x], 0);
            } else {
                const uint8_t *d = pre[x]->data;
                __builtin_prefetch(d - 8, 1);
                __builtin_prefetch(d, 1);
            }
        }
    }
}

/* Completes finished jobs, at most `budget` blocks (0: all): the finish halves of the protocol
 * operations, then done().  A job left part-done continues at the next call. */
static int collect(pquic_fec_batcher_t *b, uint32_t budget) {
    job_t *j = b->completing;
    if (__atomic_load_n(&b->done_ready, __ATOMIC_ACQUIRE)) {  /* the finished jobs that come next */
        pthread_mutex_lock(&b->mu);
        /* the finished jobs that continue the flush order; a later job waits for the ones before it */
        job_t *more = NULL, **tail = &more;
        while (b->done_head && b->done_head->seq == b->collect_seq) {
            job_t *x = b->done_head;
            b->done_head = x->next;
            x->next = NULL;
            *tail = x;
            tail = &x->next;
            b->collect_seq++;
        }
        if (!b->done_head) b->done_tail = NULL;
        __atomic_store_n(&b->done_ready, b->done_head && b->done_head->seq == b->collect_seq, __ATOMIC_RELAXED);
        pthread_mutex_unlock(&b->mu);
        if (!j) {
            j = more;
        } else if (more) {
            job_t *t = j;
            while (t->next) t = t->next;
            t->next = more;
        }
    }
    if (!j) return 0;
    const uint64_t t0 = mono_us();
    uint32_t i = b->completing_i;
    uint64_t nrec = 0;  /* recovered symbols, added to the protoop counters once per call */
    int n = 0;
    while (j) {
        const uint32_t S = j->stride;
        if (i == 0) {  /* per-job accounting, once */
            if (j->rc) b->stats.engine_errors++;
            if (GENERATES(j->op)) FEC_STAT_ADD(generate_calls, j->n); else FEC_STAT_ADD(recover_calls, j->n);
        }
        const uint32_t end = budget && j->n - i > budget - (uint32_t)n ? i + (budget - (uint32_t)n) : j->n;
        const uint32_t pf = j->rc ? 0 : b->pf;
        if (pf && i == 0) {  /* the job's first entries: their structs, then their data */
            for (uint32_t x = 0; x < 2 * pf && x < j->n; x++) prefetch_syms(j, x, 0);
            for (uint32_t x = 0; x < pf && x < j->n; x++) prefetch_syms(j, x, 1);
        }
        for (; i < end; i++) {
            entry_t *e = &j->ent[i];
            if (i + 4 < j->n) __builtin_prefetch(j->ent[i + 4].fb, 1);  /* the blocks were last touched at submission */
            if (pf) {
                if (i + 2 * pf < j->n) prefetch_syms(j, i + 2 * pf, 0);
                if (i + pf < j->n) prefetch_syms(j, i + pf, 1);
            }
            protoop_arg_t ret;
            pquic_repair_symbol_t **reps = GENERATES(j->op) ? j->reps + (size_t)i * j->r : NULL;
            pquic_source_symbol_t **pre = j->op == OP_RECOVER && j->gather ? j->pre + (size_t)i * j->k : NULL;
            if (j->rc) {
                FEC_STAT_ADD(errors, 1);
                ret = PQUIC_FEC_ERR_UNBOUND;
                for (int x = 0; reps && x < e->nalloc; x++) {  /* nothing reaches the block */
                    g_fec_api.my_free(e->cnx, reps[x]->data);
                    g_fec_api.my_free(e->cnx, reps[x]);
                }
                for (uint32_t x = 0; pre && x < j->k; x++)
                    if (pre[x]) {
                        g_fec_api.my_free(e->cnx, pre[x]->data);
                        g_fec_api.my_free(e->cnx, pre[x]);
                        pre[x] = NULL;
                    }
            } else if (GENERATES(j->op)) {
                ret = fec_generate_attach(e->fb, reps, e->nalloc);
            } else if (pre) {
                /* rows the kernel wrote into the staging area (no in-place row for them) are copied */
                ret = fec_recover_finish_pre(e->cnx, e->fb, j->st[i], j->rec + 2 * (size_t)i, pre,
                                             j->cpm + 2 * (size_t)i, j->src + (size_t)i * j->k * S, S, e->maxl,
                                             &nrec);
            } else {
                ret = fec_recover_finish(e->cnx, e->fb, j->xor_scheme, j->st[i], j->rec + 2 * (size_t)i,
                                         j->src + (size_t)i * j->k * S, S, e->maxl, &nrec);
            }
            e->done(e->user, e->fb, ret);
            n++;
        }
        if (i < j->n) break;  /* budget spent inside this job */
        b->stats.completed += j->n;
        if (j->op == OP_WINDOW && !j->rc) {
            b->stats.windows += j->n;
            b->stats.window_rows += j->nrows;
        }
        job_t *next = j->next;
        j->n = 0;
        j->next = b->free_jobs;
        b->free_jobs = j;
        b->jobs_back++;
        j = next;
        i = 0;
        if (budget && (uint32_t)n >= budget) break;
    }
    b->completing = j;
    b->completing_i = i;
    if (nrec) FEC_STAT_ADD(recovered_symbols, nrec);
    b->stats.complete_us += mono_us() - t0;  /* caller-thread field: only the caller reads it */
    return n;
}

/* Whether an overdue queue stays open for now: its successor would find no idle job (none free, no spare)
 * while at least two jobs are in flight, so the next submission would page-lock a new one on the caller's
 * thread -- and under a GPU stall that allocation waits out the stall itself (17-48 ms beside a 10-30 ms one,
 * profiles/r06_paced_stall.log) while a batch flushed every deadline needs a new job each time.  The queue
 * keeps filling instead, up to its capacity, and is flushed at the first poll that has a job back; the
 * provisioner is asked for one meanwhile. */
static int deadline_hold(pquic_fec_batcher_t *b, const job_t *j) {
    if (!b->hold || !b->prov_started || b->next_seq - b->jobs_back < 2) return 0;
    const uint32_t cap = b->cfg.batch_blocks, S = j->op == OP_WINDOW ? window_stride(b) : b->stride;
    const size_t sb = (size_t)cap * j->k * S, rb = (size_t)cap * j->r * S;
    const uint32_t sm = j->op == OP_WINDOW ? 0 : b->small_cap;
    if (count_fit(b->free_jobs, sm ? (size_t)sm * j->k * S : sb, sm ? (size_t)sm * j->r * S : rb)) return 0;
    pthread_mutex_lock(&b->mu);
    const int hold = !count_fit(b->spares, sb, rb);
    if (hold && !b->prov_want) {
        b->prov_want = 1;
        b->prov_op = j->op;
        b->prov_xor = j->xor_scheme;
        b->prov_k = j->k;
        b->prov_r = j->r;
        pthread_cond_signal(&b->cv_prov);
    }
    pthread_mutex_unlock(&b->mu);
    return hold;
}

/* Flushes the overdue queues (deadline_hold aside); returns 1 if one was held. */
static int deadline_pass(pquic_fec_batcher_t *b, uint64_t now_us) {
    int held = 0;
    for (int s = 0; s < MAX_OPEN; s++) {
        job_t *j = b->open[s];
        if (b->next_due == UINT64_MAX || now_us - b->next_due < b->cfg.max_delay_us) break;  /* none overdue */
        if (!j || !j->n || now_us - j->t_first < b->cfg.max_delay_us) continue;
        if (deadline_hold(b, j)) held = 1;
        else flush_job(b, s, &b->stats.flushed_deadline);
    }
    b->stats.deadline_holds += (uint64_t)held;
    return held;
}

int pquic_fec_batch_poll(pquic_fec_batcher_t *b, uint64_t now_us) {
    if (!b) return 0;
    const int held = deadline_pass(b, now_us);
    const int n = collect(b, b->cfg.poll_blocks);
    if (held && n) deadline_pass(b, now_us);  /* a job came back: the held queue goes now */
    return n;
}

int pquic_fec_batch_drain(pquic_fec_batcher_t *b) {
    if (!b) return 0;
    for (int s = 0; s < MAX_OPEN; s++)
        if (b->open[s]) flush_job(b, s, &b->stats.flushed_drain);
    pthread_mutex_lock(&b->mu);
    while (b->inflight) pthread_cond_wait(&b->cv_done, &b->mu);
    pthread_mutex_unlock(&b->mu);
    return collect(b, 0);
}

void pquic_fec_batch_get_stats(const pquic_fec_batcher_t *b, pquic_fec_batch_stats_t *out) {
    if (!b || !out) return;
    pthread_mutex_t *mu = (pthread_mutex_t *)&b->mu;  /* the worker threads add their times under it */
    pthread_mutex_lock(mu);
    *out = b->stats;
    pthread_mutex_unlock(mu);
}

void pquic_fec_batcher_destroy(pquic_fec_batcher_t *b) {
    if (!b) return;
    pquic_fec_batch_drain(b);
    pthread_mutex_lock(&b->mu);
    b->stop = 1;
    pthread_cond_broadcast(&b->cv_todo);
    pthread_mutex_unlock(&b->mu);
    pthread_cond_broadcast(&b->cv_prov);
    for (int i = 0; i < b->nstagers; i++) pthread_join(b->stager[i], NULL);
    for (int e = 0; e < b->nengines; e++) pthread_join(b->worker[e], NULL);
    if (b->prov_started) pthread_join(b->prov, NULL);
    while (b->free_jobs) {
        job_t *j = b->free_jobs;
        b->free_jobs = j->next;
        job_free(j);
    }
    while (b->spares) {
        job_t *j = b->spares;
        b->spares = j->next;
        job_free(j);
    }
    for (int i = 0; i < b->nheaps; i++) fecgpu_host_unregister((void *)b->heaps[i].base);
    free(b->heaps);
    pthread_rwlock_destroy(&b->heaps_mu);
    for (int e = 0; e < b->nengines; e++) fecgpu_host_ctx_destroy(b->ctx[e]);
    pthread_mutex_destroy(&b->mu);
    pthread_cond_destroy(&b->cv_todo);
    pthread_cond_destroy(&b->cv_staged);
    pthread_cond_destroy(&b->cv_done);
    pthread_cond_destroy(&b->cv_prov);
    free(b);
}
