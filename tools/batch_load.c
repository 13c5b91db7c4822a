/*
 * tools/batch_load.c -- load generator for the batching adapter (include/pquic_fec_batch.h),
 * used by bench.py's batching leg.  Plays a single-threaded picoquic sender: `nconn`
 * connections each fill FEC blocks of k source symbols (L bytes, from a synthetic payload
 * pool) and hand every full block to the batcher, optionally paced to an offered load; the
 * completion callback stamps the block's latency and frees the repair symbols as the framework
 * does after sending them (block_framework_sender.h:125-133).  Reports end-to-end throughput
 * (host staging + PCIe + kernels) and the submit -> completion latency distribution.
 */
#define _GNU_SOURCE  /* MAP_ANONYMOUS */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>
#include <x86intrin.h>

#include "fecgpu.h"
#include "pquic_fec_batch.h"

struct bl_arena;
struct st_picoquic_cnx_t { int id; protoop_arg_t in[16], out[16]; struct bl_arena *arena; };

static protoop_arg_t bl_get(picoquic_cnx_t *c, access_key_t ak, uint16_t p) {
    return ak == PQUIC_AK_CNX_INPUT ? c->in[p & 15] : c->out[p & 15];
}
static void bl_set(picoquic_cnx_t *c, access_key_t ak, uint16_t p, protoop_arg_t v) {
    if (ak == PQUIC_AK_CNX_OUTPUT) c->out[p & 15] = v;
}
/* The plugin allocator hands out fixed 2100-byte slots from a free list carved out of the plugin's
 * memory arena (picoquic/memory.c:72-95, 181-191; picoquic_internal.h:576); this load generator does
 * the same, so completions cost what they cost in PQUIC rather than glibc malloc's price.  Every
 * connection owns its plugin instances and their 16 MiB arena (PLUGIN_MEMORY, picoquic_internal.h:523;
 * init_memory_management per inserted plugin, plugin.c:835; cached plugins consumed one per connection,
 * plugin.c:946-950): with per-connection arenas each connection allocates from its own, registered with
 * the batcher one by one.  A connection without one uses the sender thread's arena.  Larger requests
 * (and an exhausted arena) fall back to the heap, tagged. */
enum { SLOT = 2112 };  /* 2100 B rounded to 64, plus room for the tag */
#define PLUGIN_MEMORY ((size_t)16 << 20)
typedef union slot_u { union slot_u *next; uint8_t bytes[SLOT]; } slot_u;
typedef struct bl_arena {
    uint8_t *base;
    size_t bytes, used;
    slot_u *free_slots;
} bl_arena_t;
/* per sender thread (bl_run_senders runs several, each a PQUIC process's single thread with its own heap) */
static __thread bl_arena_t g_thread_arena;
/* out of line: a thread-local in a dlopen()ed library costs a __tls_get_addr call, which the
 * per-connection allocations (the bench legs) then never make */
__attribute__((noinline)) static bl_arena_t *thread_arena(void) { return &g_thread_arena; }
static void *bl_malloc(picoquic_cnx_t *c, unsigned int n) {
    if (n > SLOT - 16) {
        uint8_t *p = malloc((size_t)n + 16);
        if (!p) return NULL;
        p[0] = 1;
        return p + 16;
    }
    bl_arena_t *a = c ? c->arena : NULL;
    if (!a) a = thread_arena();
    slot_u *s = a->free_slots;
    if (s) {
        a->free_slots = s->next;
    } else if (a->base && a->used + SLOT <= a->bytes) {
        s = (slot_u *)(a->base + a->used);
        a->used += SLOT;
    } else if (!(s = malloc(sizeof *s))) {
        return NULL;
    } else {
        s->bytes[0] = 2;  /* heap slot: freed to the heap */
        return s->bytes + 16;
    }
    s->bytes[0] = 0;
    return s->bytes + 16;
}
static void bl_free(picoquic_cnx_t *c, void *p) {
    if (!p) return;
    uint8_t *b = (uint8_t *)p - 16;
    if (b[0]) { free(b); return; }
    bl_arena_t *a = c ? c->arena : NULL;
    if (!a) a = thread_arena();
    slot_u *s = (slot_u *)b;
    s->next = a->free_slots;
    a->free_slots = s;
}

static int arena_map(bl_arena_t *a, size_t bytes, int hugepages) {
    memset(a, 0, sizeof *a);
    a->bytes = (bytes + 4095) & ~(size_t)4095;
    void *p = mmap(NULL, a->bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return -1;
    if (hugepages) madvise(p, a->bytes, MADV_HUGEPAGE);  /* before first touch */
    a->base = p;
    return 0;
}

static void arena_unmap(bl_arena_t *a) {
    if (a->base) munmap(a->base, a->bytes);
    memset(a, 0, sizeof *a);
}

/* the device's local CPUs (fecgpu_device_local_cpus) within `aff`; 0 when non-empty */
static int near_cpus(int device, const cpu_set_t *aff, cpu_set_t *out) {
    char list[512];
    CPU_ZERO(out);
    if (fecgpu_device_local_cpus(device, list, sizeof list) != FECGPU_OK) return -1;
    for (char *p = list; *p;) {
        char *end;
        long a = strtol(p, &end, 10), b = a;
        if (end == p) break;
        if (*end == '-') b = strtol(end + 1, &end, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            if (c >= 0 && CPU_ISSET(c, aff)) CPU_SET(c, out);
        if (*end != ',') break;
        p = end + 1;
    }
    return CPU_COUNT(out) ? 0 : -1;
}

static uint64_t now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

/* bl_run's per-block stamps (submission, completion, the clock handed to the batcher) read the TSC when
 * it is invariant and cheaper than the vDSO clock (on the GPU boxes clock_gettime took about a fifth of
 * the sender thread's time), calibrated against CLOCK_MONOTONIC once; wall times stay on now_us(). */
static double g_tsc_us;  /* microseconds per tick; 0: stamps use now_us() */
static uint64_t g_tsc_base, g_tsc_base_us;
static pthread_once_t g_tsc_once = PTHREAD_ONCE_INIT;
static void tsc_init(void) {
    FILE *f = fopen("/proc/cpuinfo", "r");
    char line[8192];
    int inv = 0;
    while (f && fgets(line, sizeof line, f))
        if (!strncmp(line, "flags", 5)) {
            inv = strstr(line, " constant_tsc") && strstr(line, " nonstop_tsc");
            break;
        }
    if (f) fclose(f);
    if (!inv) return;
    volatile uint64_t sink = 0;
    const uint64_t c0 = __rdtsc(), u0 = now_us();
    for (int i = 0; i < 20000; i++) sink += now_us();
    const uint64_t c1 = __rdtsc();
    for (int i = 0; i < 20000; i++) sink += __rdtsc();
    const uint64_t c2 = __rdtsc();
    if (c2 - c1 >= c1 - c0) return;  /* the TSC is not the cheaper clock here */
    while (now_us() - u0 < 30000) {}  /* 30 ms or more of calibration */
    const uint64_t c3 = __rdtsc(), u3 = now_us();
    g_tsc_base = c3;
    g_tsc_base_us = u3;
    g_tsc_us = (double)(u3 - u0) / (double)(c3 - c0);
}
static __thread uint64_t t_stamp_last;  /* per thread: stamps never go back */
static inline uint64_t stamp_us(void) {
    if (g_tsc_us <= 0) return now_us();
    /* signed: a core whose TSC reads a little behind the calibrating one gives a small negative offset.
     * A thread that migrates onto such a core would see its stamps go back a little: held at the last
     * stamp, so a latency (stamp - t_submit) never wraps and the batcher never sees a poll time earlier
     * than a submit time */
    uint64_t t = (uint64_t)((int64_t)g_tsc_base_us + (int64_t)((double)(int64_t)(__rdtsc() - g_tsc_base) * g_tsc_us));
    if (t < t_stamp_last) t = t_stamp_last;
    t_stamp_last = t;
    return t;
}
static inline uint64_t since_us(uint64_t t0) {
    const uint64_t t = stamp_us();
    return t > t0 ? t - t0 : 0;  /* a stamp taken on another thread may lie a little ahead */
}

/* PC sampler for the sender thread's measured pass (bl_set_sampling; tools/sender_phase_probe.py
 * --profile): a per-thread timer delivers SIGPROF to the sender thread alone every 1/hz s of wall time,
 * and the handler records the interrupted instruction address.  Profiling aid only. */
static int g_sample_hz;
static uint64_t *g_samples;
static volatile long g_nsamples;
static long g_max_samples;
static timer_t g_timer;
static void on_sigprof(int sig, siginfo_t *si, void *uc) {
    (void)sig; (void)si;
    const long n = g_nsamples;
    if (n < g_max_samples) {
        g_samples[n] = (uint64_t)((ucontext_t *)uc)->uc_mcontext.gregs[REG_RIP];
        g_nsamples = n + 1;
    }
}
void bl_set_sampling(int hz, long max_samples) {
    g_sample_hz = hz;
    free(g_samples);
    g_samples = hz > 0 ? calloc((size_t)max_samples, sizeof *g_samples) : NULL;
    g_max_samples = g_samples ? max_samples : 0;
    g_nsamples = 0;
}
long bl_samples(uint64_t *out, long max) {
    const long n = g_nsamples < max ? g_nsamples : max;
    if (n > 0) memcpy(out, g_samples, sizeof *out * (size_t)n);
    return n;
}
static void sampling_start(void) {
    if (g_sample_hz <= 0 || !g_samples) return;
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_sigprof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGPROF, &sa, NULL);
    struct sigevent ev;
    memset(&ev, 0, sizeof ev);
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev.sigev_signo = SIGPROF;
    ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
    if (timer_create(CLOCK_MONOTONIC, &ev, &g_timer)) return;
    const long ns = 1000000000L / g_sample_hz;
    struct itimerspec it = {{ns / 1000000000L, ns % 1000000000L}, {ns / 1000000000L, ns % 1000000000L}};
    timer_settime(g_timer, 0, &it, NULL);
}
static void sampling_stop(void) {
    if (g_sample_hz <= 0 || !g_samples) return;
    timer_delete(g_timer);
    signal(SIGPROF, SIG_IGN);
}

/* a sender's completion tallies; the callbacks reach them through their slot (no thread-local access
 * per block) */
typedef struct {
    uint64_t *lat;
    long nlat, recovered;
    const pquic_source_symbol_t *recv_lo, *recv_hi;  /* the received symbols' descriptors (receiver) */
} bl_tally_t;
static __thread bl_tally_t g_tally;
#define g_lat (g_tally.lat)
#define g_nlat (g_tally.nlat)
#define g_recovered (g_tally.recovered)
#define g_recv_lo (g_tally.recv_lo)
#define g_recv_hi (g_tally.recv_hi)

typedef struct {
    pquic_fec_block_t fb;
    uint64_t t_submit;
    picoquic_cnx_t *cnx;
    bl_tally_t *tally;
    int busy;
} slot_t;
static unsigned g_poll_blocks;  /* pquic_fec_batch_cfg_t.poll_blocks of the next runs (0: all) */
static int g_hugepages;         /* the next runs' arena on transparent huge pages */
static int g_detail;            /* time every submission (one more clock read per block) */
static long g_pool_blocks = 32768;  /* blocks of distinct source payload (bl_run) */
static int g_inflight = 4;          /* batches a sender keeps in flight at most (its block slots) */

void bl_set_options(unsigned poll_blocks, int hugepages, int detail, long pool_blocks) {
    g_poll_blocks = poll_blocks;
    g_hugepages = hugepages;
    g_detail = detail;
    if (pool_blocks > 0) g_pool_blocks = pool_blocks;
}

/* batches in flight per sender (1..16; default 4): the back-pressure that bounds queueing latency */
void bl_set_inflight(int batches) { g_inflight = batches < 1 ? 1 : batches > 16 ? 16 : batches; }

/* nanoseconds per now_us() call (the load generator stamps every block at submission and completion) */
double bl_clock_cost(void) {
    const uint64_t t0 = now_us();
    uint64_t acc = 0;
    for (int i = 0; i < 1000000; i++) acc += now_us();
    return (double)(now_us() - t0) * 1e3 / 1e6 + (double)(acc & 0);
}

static pthread_barrier_t *g_sync;  /* bl_run_senders: the senders' pass barrier */
static __thread uint64_t g_span[2];  /* the last measured pass: start, end (us) */
static __thread double g_jobs[3];   /* the last measured pass: batch jobs allocated, caller us in those allocations,
                                     * polls that held an overdue queue (no idle job) */
static __thread double g_lat_q[8];  /* the last measured pass's latency: p50 p90 p95 p99 p99.9 max mean, count */
static __thread double g_rows[2];   /* the last bl_run's measured pass: rows in place, rows staged */
static __thread double g_phases[6];  /* the last bl_run's measured pass: engine, stager, completion thread-us; wall us;
                             * caller us waiting for a free slot; caller us inside pquic_fec_batch_generate */

static void on_done(void *user, pquic_fec_block_t *fb, protoop_arg_t ret) {
    slot_t *s = user;
    bl_tally_t *t = s->tally;
    (void)ret;
    t->lat[t->nlat++] = since_us(s->t_submit);
    for (int i = 0; i < fb->total_repair_symbols; i++) {
        pquic_repair_symbol_t *rs = fb->repair_symbols[i];
        if (rs) { bl_free(s->cnx, rs->data); bl_free(s->cnx, rs); fb->repair_symbols[i] = NULL; }
    }
    s->busy = 0;
}

/* receiver: the framework decodes the recovered symbols' frames and frees them (fec_protoops.h:252-275) */
static void on_recovered(void *user, pquic_fec_block_t *fb, protoop_arg_t ret) {
    slot_t *s = user;
    bl_tally_t *t = s->tally;
    (void)ret;
    t->lat[t->nlat++] = since_us(s->t_submit);
    for (int j = 0; j < fb->total_source_symbols; j++) {
        pquic_source_symbol_t *ss = fb->source_symbols[j];
        if (ss && (ss < t->recv_lo || ss >= t->recv_hi)) {  /* inserted by the recover (allocated by the adapter) */
            t->recovered++;
            bl_free(s->cnx, ss->data);
            bl_free(s->cnx, ss);
        }
        fb->source_symbols[j] = NULL;
    }
    s->busy = 0;
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* out: [0] payload GiB/s, [1] p50 us, [2] p99 us, [3] max us, [4] batches, [5] wall s,
 *      [6] blocks completed, [7] mean blocks per batch.  register_heap: bit 0 -- the symbols' arenas are
 * registered with the batcher, which then reads and writes rows in place; bit 1 -- one 16 MiB arena per
 * connection (PQUIC's topology, each registered on its own) instead of one arena for the sender.
 * recover_e > 0: the receiver side instead -- every block arrives with recover_e sources lost and all r
 * repairs, and goes through pquic_fec_batch_recover.  Returns 0 or -1. */
static int run_sender(int device, int k, int r, int L, int nconn, long nblocks, unsigned batch_blocks,
                      unsigned max_delay_us, int nstreams, double offered_gib_s, int register_heap, int recover_e,
                      double out[8]);

int bl_run(int device, int k, int r, int L, int nconn, long nblocks, unsigned batch_blocks, unsigned max_delay_us,
           int nstreams, double offered_gib_s, int register_heap, double out[8]) {
    pquic_fec_host_api_t api = {bl_get, bl_set, bl_malloc, bl_free, NULL};
    if (pquic_fec_bind_host(&api, device)) return -1;
    return run_sender(device, k, r, L, nconn, nblocks, batch_blocks, max_delay_us, nstreams, offered_gib_s,
                      register_heap, 0, out);
}

/* The receiver: `nblocks` blocks, each with `e` of its k sources lost (a rotating run) and its r repairs,
 * recovered through the batcher (out as bl_run; [6] counts recovered symbols, not blocks). */
int bl_run_recover(int device, int k, int r, int L, int e, int nconn, long nblocks, unsigned batch_blocks,
                   unsigned max_delay_us, int nstreams, int register_heap, double out[8]) {
    pquic_fec_host_api_t api = {bl_get, bl_set, bl_malloc, bl_free, NULL};
    if (e < 1 || e > r || e > k || pquic_fec_bind_host(&api, device)) return -1;
    return run_sender(device, k, r, L, nconn, nblocks, batch_blocks, max_delay_us, nstreams, 0.0, register_heap, e,
                      out);
}

/* `nsenders` bl_run senders at once, one thread each with its own batcher, arena and connections -- a
 * server running one PQUIC process per core (each process single-threaded, plugin.c:1357-1360) on one
 * GPU.  out: [0] the senders' payload GiB/s summed, [1] / [2] / [3] the largest p50 / p99 / max of any
 * sender, [4] batches summed, [5] the longest wall s, [6] blocks summed, [7] mean blocks per batch. */
struct sender_arg {
    int device, k, r, L, nconn, nstreams, reg, rc;
    long nblocks;
    unsigned batch, delay;
    double out[8];
    uint64_t span[2];
};
static void *sender_main(void *p) {
    struct sender_arg *a = p;
    a->rc = run_sender(a->device, a->k, a->r, a->L, a->nconn, a->nblocks, a->batch, a->delay, a->nstreams, 0.0,
                       a->reg, 0, a->out);
    a->span[0] = g_span[0];
    a->span[1] = g_span[1];
    return NULL;
}
int bl_run_senders(int nsenders, int device, int k, int r, int L, int nconn, long nblocks, unsigned batch_blocks,
                   unsigned max_delay_us, int nstreams, int register_heap, double out[8]) {
    if (nsenders < 1 || nsenders > 16) return -1;
    pquic_fec_host_api_t api = {bl_get, bl_set, bl_malloc, bl_free, NULL};
    if (pquic_fec_bind_host(&api, device)) return -1;
    struct sender_arg a[16];
    pthread_t th[16];
    pthread_barrier_t bar;
    if (pthread_barrier_init(&bar, NULL, (unsigned)nsenders)) return -1;
    g_sync = nsenders > 1 ? &bar : NULL;
    int started = 0, rc = 0;
    for (; started < nsenders; started++) {
        a[started] = (struct sender_arg){device, k, r, L, nconn, nstreams, register_heap, -1, nblocks, batch_blocks,
                                         max_delay_us, {0}, {0, 0}};
        if (pthread_create(&th[started], NULL, sender_main, &a[started])) break;
    }
    if (started < nsenders) abort();  /* the started senders would wait at the barrier for ever */
    for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
    g_sync = NULL;
    pthread_barrier_destroy(&bar);
    /* every sender's measured pass starts at the barrier: the job's rate is all their blocks over the
     * span from the first start to the last drain */
    memset(out, 0, 8 * sizeof *out);
    uint64_t t_first = UINT64_MAX, t_last = 0;
    for (int i = 0; i < nsenders; i++) {
        if (a[i].rc) rc = -1;
        t_first = a[i].span[0] < t_first ? a[i].span[0] : t_first;
        t_last = a[i].span[1] > t_last ? a[i].span[1] : t_last;
        for (int x = 1; x <= 3; x++) out[x] = a[i].out[x] > out[x] ? a[i].out[x] : out[x];
        out[4] += a[i].out[4];
        out[6] += a[i].out[6];
    }
    out[5] = (t_last - t_first) * 1e-6;
    out[0] = out[5] > 0 ? (double)nsenders * nblocks * k * L / out[5] / 1073741824.0 : 0;
    out[7] = out[4] > 0 ? out[6] / out[4] : 0;
    return rc;
}

/* A sender that fails still meets the other senders at the pass barriers it has not reached. */
static int sender_fail(int waits) {
    for (; g_sync && waits < 2; waits++) pthread_barrier_wait(g_sync);
    return -1;
}

static void xorshift_fill(uint8_t *p, size_t n, uint64_t x) {
    for (size_t o = 0; o < n; o += 8) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        memcpy(p + o, &x, n - o < 8 ? n - o : 8);
    }
}

static int run_sender(int device, int k, int r, int L, int nconn, long nblocks, unsigned batch_blocks,
                      unsigned max_delay_us, int nstreams, double offered_gib_s, int register_heap, int recover_e,
                      double out[8]) {
    int waits = 0;  /* pass barriers this sender has passed (bl_run_senders) */
    const int reg = register_heap & 1, per_conn = (register_heap >> 1) & 1;
    /* the sender runs on the device's socket, like the batcher's threads, so the arenas it first
     * touches are local to the device */
    cpu_set_t saved, near;
    const int pinned = !sched_getaffinity(0, sizeof saved, &saved) && !near_cpus(device, &saved, &near) &&
                       !sched_setaffinity(0, sizeof near, &near);
    pquic_fec_batch_cfg_t cfg = {device, batch_blocks, max_delay_us, (uint32_t)L, nstreams, g_poll_blocks};
    pquic_fec_batcher_t *b = pquic_fec_batcher_create(&cfg);
    if (!b) return sender_fail(waits);
    /* blocks in flight at most: every queued batch plus one being filled, per connection slot */
    const long nslots = (long)batch_blocks * g_inflight + nconn + 64;
    slot_t *slots = calloc(nslots, sizeof *slots);
    /* Distinct payload for g_pool_blocks blocks, reused in turn, spread over the connections: connection c
     * sends pool blocks c, c + nconn, ... (its own arena's, with per-connection arenas).  The default pool
     * (32768 blocks, 629 MB at k16 L1200) is well past the device's caches, so every source row the
     * kernels read in place crosses PCIe; a small pool stays cached on the device and overstates the
     * gathered read rate.  The receiver's pool carries each block's r repairs too. */
    const long ppc = (g_pool_blocks + nconn - 1) / nconn;  /* pool blocks per connection */
    const size_t blk_bytes = (size_t)(k + (recover_e ? r : 0)) * L;
    const size_t pool_conn = (size_t)ppc * blk_bytes;
    /* allocator slots: 2 per repair (generate) or recovered source (recover) of every block in flight */
    const size_t slots_total = ((size_t)nslots * (recover_e ? recover_e : r) * 2 + 1024);
    picoquic_cnx_t *cnx = calloc(nconn, sizeof *cnx);
    bl_arena_t *ar = per_conn ? calloc(nconn, sizeof *ar) : NULL;
    if (!slots || !cnx || (per_conn && !ar)) return sender_fail(waits);
    uint8_t **pool = calloc(nconn, sizeof *pool);  /* connection c's payload */
    if (!pool) return sender_fail(waits);
    if (per_conn) {
        /* PLUGIN_MEMORY per connection, larger only when a connection's share of the payload and its
         * slots would not fit (few connections, big pools) */
        size_t need = ((pool_conn + 63) & ~(size_t)63) + (slots_total / nconn + 64) * SLOT;
        if (need < PLUGIN_MEMORY) need = PLUGIN_MEMORY;
        for (int c = 0; c < nconn; c++) {
            if (arena_map(&ar[c], need, g_hugepages)) return sender_fail(waits);
            cnx[c].arena = &ar[c];
            pool[c] = ar[c].base;
            ar[c].used = (pool_conn + 63) & ~(size_t)63;
        }
    } else {
        bl_arena_t *a = &g_thread_arena;
        if (arena_map(a, slots_total * SLOT + pool_conn * nconn + 64, g_hugepages)) return sender_fail(waits);
        for (int c = 0; c < nconn; c++) pool[c] = a->base + (size_t)c * pool_conn;
        a->used = (pool_conn * nconn + 63) & ~(size_t)63;
    }
    for (int c = 0; c < nconn; c++) {
        cnx[c].id = c;
        xorshift_fill(pool[c], (size_t)ppc * k * L, 0x5EEDF3C0 + (uint64_t)c * 0x9E3779B97F4A7C15ull);
    }
    if (recover_e) {  /* the pool's repairs: each pool block q of connection c is block number c * ppc + q */
        fecgpu_host_ctx_t *hc = fecgpu_host_ctx_create(device, 2, (size_t)64 << 20);
        uint32_t *fbn = malloc(sizeof *fbn * (size_t)ppc);
        uint8_t *rep = malloc((size_t)ppc * r * L);
        if (!hc || !fbn || !rep) return sender_fail(waits);
        for (int c = 0; c < nconn; c++) {
            for (long q = 0; q < ppc; q++) fbn[q] = (uint32_t)(c * ppc + q) & 0xffffffu;
            if (fecgpu_rlc_encode_host(hc, pool[c], rep, ppc, k, r, L, 0, fbn)) return sender_fail(waits);
            memcpy(pool[c] + (size_t)ppc * k * L, rep, (size_t)ppc * r * L);
        }
        free(fbn);
        free(rep);
        fecgpu_host_ctx_destroy(hc);
    }
    if (reg) {
        if (per_conn) {
            for (int c = 0; c < nconn; c++)
                if (pquic_fec_batch_register_heap(b, ar[c].base, ar[c].bytes)) return sender_fail(waits);
        } else if (pquic_fec_batch_register_heap(b, g_thread_arena.base, g_thread_arena.bytes)) {
            return sender_fail(waits);
        }
    }
    pquic_source_symbol_t *ss = calloc((size_t)nslots * k, sizeof *ss);
    pquic_repair_symbol_t *rsy = recover_e ? calloc((size_t)nslots * r, sizeof *rsy) : NULL;
    g_lat = malloc(sizeof *g_lat * (size_t)(nblocks + nblocks / 5 + 1));
    g_nlat = 0;
    g_recovered = 0;
    g_recv_lo = ss;
    g_recv_hi = ss + (size_t)nslots * k;
    if (!ss || !g_lat || (recover_e && !rsy)) return sender_fail(waits);
    bl_tally_t *const tally = &g_tally;
    pthread_once(&g_tsc_once, tsc_init);
    const double bytes_per_block = (double)k * L;
    long next_slot = 0;
    /* pass 0 warms up (pinned queue buffers allocated, device buffers grown), pass 1 is measured */
    uint64_t t0 = 0, t_wait = 0, t_submit = 0;
    long rec0 = 0;
    pquic_fec_batch_stats_t st0;
    memset(&st0, 0, sizeof st0);
    for (int pass = 0; pass < 2; pass++) {
        const long nb = pass ? nblocks : nblocks / 5 + 1;
        if (pass) {
            pquic_fec_batch_drain(b);
            pquic_fec_batch_get_stats(b, &st0);
            g_nlat = 0;
            rec0 = g_recovered;
        }
        if (g_sync) pthread_barrier_wait(g_sync), waits++;  /* bl_run_senders: every sender starts each pass together */
        if (pass) sampling_start();
        t0 = now_us();
        const uint64_t t0s = stamp_us();
        t_wait = t_submit = 0;
        int cur_c = 0, cur_lost = 0;
        long cur_q = 0, cur_round = 0;
        for (long blk = 0; blk < nb; blk++) {
            if (offered_gib_s > 0) {  /* pace: block blk is due at t0 + blk * bytes / rate */
                const uint64_t due = t0s + (uint64_t)(blk * bytes_per_block / (offered_gib_s * 1073741824.0) * 1e6);
                while (stamp_us() < due) pquic_fec_batch_poll(b, stamp_us());
            }
            slot_t *s = &slots[next_slot];
            if (s->busy) {
                const uint64_t w0 = stamp_us();
                while (s->busy) pquic_fec_batch_poll(b, stamp_us());  /* back-pressure: slot still in flight */
                t_wait += stamp_us() - w0;
            }
            const long si = next_slot;
            if (++next_slot == nslots) next_slot = 0;
            /* block blk: connection c = blk % nconn, round blk / nconn, pool block q = round % ppc, kept as
             * counters (no divisions per block) */
            const int c = cur_c;
            const long q = cur_q;
            const uint8_t *pb = pool[c] + (size_t)q * k * L;
            memset(&s->fb, 0, sizeof s->fb);
            const uint32_t fbn = recover_e ? (uint32_t)(c * ppc + q) & 0xffffffu : (uint32_t)cur_round & 0xffffffu;
            if (++cur_c == nconn) {
                cur_c = 0;
                cur_round++;
                if (++cur_q == ppc) cur_q = 0;
            }
            s->fb.fec_block_number = fbn;
            s->cnx = &cnx[c];
            s->tally = tally;
            const int lost0 = recover_e ? cur_lost : k;  /* sources lost0 .. +e-1, lost0 = blk % (k - e + 1) */
            if (recover_e && ++cur_lost == k - recover_e + 1) cur_lost = 0;
            for (int j = 0; j < k; j++) {
                if (j >= lost0 && j < lost0 + recover_e) continue;
                pquic_source_symbol_t *sym = &ss[si * k + j];
                sym->fpid.raw = (fbn << 8) | (uint32_t)j;
                sym->data = (uint8_t *)pb + (size_t)j * L;
                sym->data_length = (uint16_t)L;
                s->fb.source_symbols[j] = sym;
                s->fb.current_source_symbols++;
            }
            s->fb.total_source_symbols = (uint8_t)k;
            s->fb.total_repair_symbols = (uint8_t)r;
            if (recover_e) {
                const uint8_t *pr = pool[c] + (size_t)ppc * k * L + (size_t)q * r * L;
                for (int i = 0; i < r; i++) {
                    pquic_repair_symbol_t *rs = &rsy[si * r + i];
                    memset(rs, 0, sizeof *rs);
                    rs->fpid.raw = ((uint64_t)fbn << 8) | (uint64_t)i;
                    rs->data = (uint8_t *)pr + (size_t)i * L;
                    rs->data_length = (uint16_t)L;
                    s->fb.repair_symbols[i] = rs;
                }
                s->fb.current_repair_symbols = (uint8_t)r;
            }
            s->busy = 1;
            s->t_submit = stamp_us();
            const int rc = recover_e ? pquic_fec_batch_recover(b, &cnx[c], &s->fb, 0, s->t_submit, on_recovered, s)
                                     : pquic_fec_batch_generate(b, &cnx[c], &s->fb, 0, s->t_submit, on_done, s);
            if (rc) return sender_fail(waits);
            if (g_detail) t_submit += stamp_us() - s->t_submit;
            if ((blk & 15) == 0) pquic_fec_batch_poll(b, stamp_us());
        }
    }
    pquic_fec_batch_drain(b);
    const uint64_t t_end = now_us();
    sampling_stop();
    const double wall = (t_end - t0) * 1e-6;
    g_span[0] = t0;
    g_span[1] = t_end;
    pquic_fec_batch_stats_t st;
    pquic_fec_batch_get_stats(b, &st);
    pquic_fec_batcher_destroy(b);  /* unregisters the arenas */
    qsort(g_lat, g_nlat, sizeof *g_lat, cmp_u64);
    {
        static const double qs[6] = {0.5, 0.9, 0.95, 0.99, 0.999, 1.0};
        for (int i = 0; i < 6; i++)
            g_lat_q[i] = g_nlat ? (double)g_lat[qs[i] >= 1.0 ? g_nlat - 1 : (long)(g_nlat * qs[i])] : 0;
        double sum = 0;
        for (long i = 0; i < g_nlat; i++) sum += (double)g_lat[i];
        g_lat_q[6] = g_nlat ? sum / g_nlat : 0;
        g_lat_q[7] = (double)g_nlat;
    }
    out[0] = nblocks * bytes_per_block / wall / 1073741824.0;
    out[1] = g_nlat ? (double)g_lat[g_nlat / 2] : 0;
    out[2] = g_nlat ? (double)g_lat[(long)(g_nlat * 0.99)] : 0;
    out[3] = g_nlat ? (double)g_lat[g_nlat - 1] : 0;
    out[4] = (double)(st.batches - st0.batches);
    out[5] = wall;
    out[6] = recover_e ? (double)(g_recovered - rec0) : (double)(st.completed - st0.completed);
    out[7] = out[4] > 0 ? (double)(st.completed - st0.completed) / out[4] : 0;
    g_phases[0] = (double)(st.engine_us - st0.engine_us);
    g_phases[1] = (double)(st.stage_us - st0.stage_us);
    g_phases[2] = (double)(st.complete_us - st0.complete_us);
    g_phases[3] = wall * 1e6;
    g_phases[4] = (double)t_wait;
    g_phases[5] = (double)t_submit;
    g_rows[0] = (double)(st.rows_in_place - st0.rows_in_place);
    g_rows[1] = (double)(st.rows_staged - st0.rows_staged);
    g_jobs[0] = (double)(st.jobs_allocated - st0.jobs_allocated);
    g_jobs[1] = (double)(st.job_alloc_us - st0.job_alloc_us);
    g_jobs[2] = (double)(st.deadline_holds - st0.deadline_holds);
    free(slots); free(ss); free(rsy); free(g_lat); free(cnx); free(pool);
    g_lat = NULL;
    if (pinned) sched_setaffinity(0, sizeof saved, &saved);
    /* every slot lives in an arena or was malloc'd and leaks here (tool only) */
    if (per_conn) {
        for (int c = 0; c < nconn; c++) arena_unmap(&ar[c]);
        free(ar);
    } else {
        arena_unmap(&g_thread_arena);
    }
    return 0;
}

/* Sliding-window sender load (window_framework_sender.h:209-260): `nconn` connections each send a
 * stream of L-byte source symbols and, after every `step` new symbols, generate repairs for a window of
 * the last k (block number 0, as malloc_fec_block(cnx, 0) at :215), through
 * pquic_fec_batch_generate_window (window_api 1: each connection's symbols staged once per batch,
 * windows coded on the shared-coefficient kernel) or pquic_fec_batch_generate (0: every window a block
 * of its own).  Symbols live in per-connection rings sized past the windows that can be in flight.
 * out: [0] stream GiB/s (new symbols protected), [1] p50 us, [2] p99 us, [3] max us, [4] batches,
 *      [5] wall s, [6] windows completed, [7] window GiB/s (k symbols per window).  Returns 0 or -1. */
int bl_run_window(int device, int k, int r, int L, int step, int nconn, long nwindows, unsigned batch_blocks,
                  unsigned max_delay_us, int nstreams, int window_api, double out[8]) {
    if (k < 1 || k > 64 || r < 1 || step < 1 || nconn < 1 || L < 1 || L > 2048) return -1;
    pquic_fec_host_api_t api = {bl_get, bl_set, bl_malloc, bl_free, NULL};
    if (pquic_fec_bind_host(&api, device)) return -1;
    cpu_set_t saved, near;
    const int pinned = !sched_getaffinity(0, sizeof saved, &saved) && !near_cpus(device, &saved, &near) &&
                       !sched_setaffinity(0, sizeof near, &near);
    pquic_fec_batch_cfg_t cfg = {device, batch_blocks, max_delay_us, (uint32_t)L, nstreams, g_poll_blocks};
    pquic_fec_batcher_t *b = pquic_fec_batcher_create(&cfg);
    if (!b) return -1;
    const long nslots = (long)batch_blocks * 4 + nconn + 64;
    const long ring = ((nslots / nconn + 4) * step + k) * 2;  /* symbols per connection ring */
    const size_t pool_syms = 4096, pool_bytes = pool_syms * (size_t)L;
    if (arena_map(&g_thread_arena, ((size_t)nslots * r * 2 + 1024) * SLOT + pool_bytes, 0)) return -1;
    uint8_t *pool = g_thread_arena.base;
    g_thread_arena.used = (pool_bytes + 63) & ~(size_t)63;
    slot_t *slots = calloc(nslots, sizeof *slots);
    pquic_source_symbol_t *rings = calloc((size_t)nconn * ring, sizeof *rings);
    long *sent = calloc(nconn, sizeof *sent);
    g_lat = malloc(sizeof *g_lat * (size_t)(nwindows + nwindows / 5 + 1));
    g_nlat = 0;
    picoquic_cnx_t *cnx = calloc(nconn, sizeof *cnx);
    if (!slots || !rings || !sent || !g_lat || !cnx) return -1;
    uint64_t x = 0x5EEDF3C0;
    for (size_t o = 0; o < pool_bytes; o++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; pool[o] = (uint8_t)x; }
    for (int c = 0; c < nconn; c++) {
        cnx[c].id = c;
        sent[c] = k > step ? k - step : 0;  /* symbols already sent: the first window then ends at k */
    }
    pthread_once(&g_tsc_once, tsc_init);
    long next_slot = 0;
    uint64_t t0 = 0;
    pquic_fec_batch_stats_t st0;
    memset(&st0, 0, sizeof st0);
    for (int pass = 0; pass < 2; pass++) {
        const long nw = pass ? nwindows : nwindows / 5 + 1;
        if (pass) {
            pquic_fec_batch_drain(b);
            pquic_fec_batch_get_stats(b, &st0);
            g_nlat = 0;
        }
        t0 = now_us();
        for (long w = 0; w < nw; w++) {
            slot_t *s = &slots[next_slot];
            while (s->busy) pquic_fec_batch_poll(b, stamp_us());
            next_slot = (next_slot + 1) % nslots;
            const int c = (int)(w % nconn);
            pquic_source_symbol_t *rc = rings + (size_t)c * ring;
            for (long q = w < nconn ? 0 : sent[c]; q < sent[c] + step; q++) {  /* new symbols (all, at first) */
                pquic_source_symbol_t *sym = &rc[q % ring];
                sym->fpid.raw = (uint32_t)q;
                sym->data = pool + (size_t)((q * 31 + c * 977) % (long)pool_syms) * L;
                sym->data_length = (uint16_t)L;
            }
            sent[c] += step;
            memset(&s->fb, 0, sizeof s->fb);
            for (int j = 0; j < k; j++) s->fb.source_symbols[j] = &rc[(sent[c] - k + j) % ring];
            s->fb.current_source_symbols = s->fb.total_source_symbols = (uint8_t)k;
            s->fb.total_repair_symbols = (uint8_t)r;
            s->busy = 1;
            s->cnx = NULL;  /* the repairs come from the thread arena */
            s->tally = &g_tally;
            s->t_submit = stamp_us();
            const int rc2 = window_api ? pquic_fec_batch_generate_window(b, &cnx[c], &s->fb, s->t_submit, on_done, s)
                                       : pquic_fec_batch_generate(b, &cnx[c], &s->fb, 0, s->t_submit, on_done, s);
            if (rc2) return -1;
            if ((w & 15) == 0) pquic_fec_batch_poll(b, stamp_us());
        }
    }
    pquic_fec_batch_drain(b);
    const double wall = (now_us() - t0) * 1e-6;
    pquic_fec_batch_stats_t st;
    pquic_fec_batch_get_stats(b, &st);
    pquic_fec_batcher_destroy(b);
    qsort(g_lat, g_nlat, sizeof *g_lat, cmp_u64);
    out[0] = (double)nwindows * step * L / wall / 1073741824.0;
    out[1] = g_nlat ? (double)g_lat[g_nlat / 2] : 0;
    out[2] = g_nlat ? (double)g_lat[(long)(g_nlat * 0.99)] : 0;
    out[3] = g_nlat ? (double)g_lat[g_nlat - 1] : 0;
    out[4] = (double)(st.batches - st0.batches);
    out[5] = wall;
    out[6] = (double)(st.completed - st0.completed);
    out[7] = (double)nwindows * k * L / wall / 1073741824.0;
    free(slots); free(rings); free(sent); free(g_lat); free(cnx);
    g_lat = NULL;
    if (pinned) sched_setaffinity(0, sizeof saved, &saved);
    arena_unmap(&g_thread_arena);
    return 0;
}

/* Latency of the synchronous drop-in hooks: one block per call, exactly as the block framework
 * calls fec_generate_repair_symbols (block_framework_sender.h:187) and fec_recover
 * (fec_protoops.h:246), through pquic_fec_rlc_generate_repair_symbols / pquic_fec_rlc_recover.
 * Each call stages the block, runs the device and writes the repairs / recovered symbols back
 * with the bound allocator.  `e` sources are erased for recover (all r repairs present).
 * out: [0] generate p50 us, [1] p99, [2] mean, [3] recover p50, [4] p99, [5] mean,
 *      [6] recovered symbols per recover call (check).  Returns 0 or -1. */
/* Every timed hook call of the last bl_hook_latency: op (0 generate, 1 recover), start (CLOCK_MONOTONIC
 * us) and duration (us), for lining calls up with a kernel trace (bl_hook_calls). */
static uint64_t *g_hook_calls;
static long g_hook_ncalls;

long bl_hook_calls(uint64_t *out, long max) {
    const long n = g_hook_ncalls < max ? g_hook_ncalls : max;
    if (out && g_hook_calls) memcpy(out, g_hook_calls, sizeof *out * 3 * (size_t)n);
    return n;
}

int bl_hook_latency(int device, int k, int r, int L, int e, long ncalls, double out[7]) {
    pquic_fec_host_api_t api = {bl_get, bl_set, bl_malloc, bl_free, NULL};
    if (pquic_fec_bind_host(&api, device) || k > 100 || r > 100 || e > r || e > k) return -1;
    picoquic_cnx_t cnx;
    memset(&cnx, 0, sizeof cnx);
    if (pquic_fec_rlc_create_fec_schemes(&cnx)) return -1;
    const protoop_arg_t scheme = cnx.out[0];
    uint8_t *pool = malloc((size_t)k * L);
    pquic_source_symbol_t *ss = calloc((size_t)k, sizeof *ss);
    uint64_t *lat = malloc(sizeof *lat * (size_t)ncalls);
    if (!pool || !ss || !lat) return -1;
    free(g_hook_calls);
    g_hook_ncalls = 0;
    g_hook_calls = malloc(sizeof *g_hook_calls * 3 * 2 * (size_t)ncalls);
    uint64_t x = 0x5EEDF3C0;
    for (size_t o = 0; o < (size_t)k * L; o++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; pool[o] = (uint8_t)x; }
    pquic_fec_block_t fb;
    long recovered = 0;
    for (int op = 0; op < 2; op++) {
        for (long c = -ncalls / 10 - 1; c < ncalls; c++) {  /* the first tenth warms up */
            const uint32_t fbn = (uint32_t)(c & 0xffffff);
            memset(&fb, 0, sizeof fb);
            fb.fec_block_number = fbn;
            fb.total_source_symbols = (uint8_t)k;
            fb.total_repair_symbols = (uint8_t)r;
            for (int j = 0; j < k; j++) {
                ss[j].fpid.raw = (fbn << 8) | (uint32_t)j;
                ss[j].data = pool + (size_t)j * L;
                ss[j].data_length = (uint16_t)L;
                fb.source_symbols[j] = &ss[j];
            }
            fb.current_source_symbols = (uint8_t)k;
            cnx.in[0] = (protoop_arg_t)(uintptr_t)&fb;
            cnx.in[1] = scheme;
            /* repairs for this block (untimed when measuring recover) */
            uint64_t t0 = now_us();
            if (pquic_fec_rlc_generate_repair_symbols(&cnx)) return -1;
            uint64_t t1 = now_us();
            if (op == 1) {
                fb.current_repair_symbols = (uint8_t)r;
                const int first = (int)(c % (k - e + 1) + k - e + 1) % (k - e + 1);
                for (int j = first; j < first + e; j++) fb.source_symbols[j] = NULL;
                fb.current_source_symbols = (uint8_t)(k - e);
                t0 = now_us();
                if (pquic_fec_rlc_recover(&cnx)) return -1;
                t1 = now_us();
                for (int j = first; j < first + e; j++)
                    if (fb.source_symbols[j]) {
                        if (c >= 0) recovered++;
                        bl_free(NULL, fb.source_symbols[j]->data);
                        bl_free(NULL, fb.source_symbols[j]);
                    }
            }
            for (int i = 0; i < r; i++)
                if (fb.repair_symbols[i]) { bl_free(NULL, fb.repair_symbols[i]->data); bl_free(NULL, fb.repair_symbols[i]); }
            if (c >= 0) {
                lat[c] = t1 - t0;
                if (g_hook_calls) {
                    uint64_t *h = g_hook_calls + 3 * g_hook_ncalls++;
                    h[0] = (uint64_t)op; h[1] = t0; h[2] = t1 - t0;
                }
            }
        }
        double sum = 0;
        for (long c = 0; c < ncalls; c++) sum += (double)lat[c];
        qsort(lat, ncalls, sizeof *lat, cmp_u64);
        out[3 * op + 0] = (double)lat[ncalls / 2];
        out[3 * op + 1] = (double)lat[(long)(ncalls * 0.99)];
        out[3 * op + 2] = sum / ncalls;
    }
    out[6] = (double)recovered / ncalls;
    bl_free(NULL, (void *)(uintptr_t)scheme);
    free(pool); free(ss); free(lat);
    return 0;
}

/* The synchronous hooks while a bulk job occupies the same GPU: a background thread runs back-to-back
 * fecgpu_rlc_encode_host calls of `bulk_blocks` k16 r4 L1200 blocks in page-locked host memory (the
 * batching adapter's kind of job: kernels reading their rows over PCIe, ~2 ms per 4096 blocks) while
 * this thread times `ncalls` generate and recover hooks exactly as bl_hook_latency does.
 * out: [0..6] as bl_hook_latency, [7] bulk calls started while the hooks ran, [8] hook requests the
 * resident block service withdrew at its deadline (those calls took the launch path), [9] / [10] mean /
 * max ms of those bulk calls (how long the hooks' worker held the bulk job up).  Returns 0 or -1. */
struct bulk_arg {
    int device, blocks;
    volatile int stop, window;  /* window: the hooks are being timed */
    volatile long calls;
    long in_window;
    double sum_ms, max_ms;
    int rc;
};
static void *bulk_main(void *p) {
    struct bulk_arg *a = p;
    const size_t sb = (size_t)a->blocks * 16 * 1200, rb = (size_t)a->blocks * 4 * 1200;
    fecgpu_host_ctx_t *c = fecgpu_host_ctx_create(a->device, 4, (size_t)64 << 20);
    uint8_t *src = fecgpu_host_alloc(sb), *rep = fecgpu_host_alloc(rb);
    if (!c || !src || !rep) {
        a->rc = -1;
    } else {
        xorshift_fill(src, sb, 0x5EEDF3C0);
        while (!a->stop) {
            const int w = a->window;
            const uint64_t t0 = now_us();
            if (fecgpu_rlc_encode_host(c, src, rep, (uint64_t)a->blocks, 16, 4, 1200, 0, NULL)) { a->rc = -1; break; }
            const double ms = (now_us() - t0) * 1e-3;
            if (w) {  /* a call started while the hooks were timed (one held up past the window included) */
                a->in_window++;
                a->sum_ms += ms;
                if (ms > a->max_ms) a->max_ms = ms;
            }
            a->calls++;
        }
    }
    fecgpu_host_free(src);
    fecgpu_host_free(rep);
    if (c) fecgpu_host_ctx_destroy(c);
    return NULL;
}

int bl_hook_latency_loaded(int device, int bulk_blocks, long ncalls, double out[11]) {
    struct bulk_arg a = {device, bulk_blocks, 0, 0, 0, 0, 0.0, 0.0, 0};
    pthread_t th;
    pquic_fec_protoop_stats_t s0, s1;
    pquic_fec_protoop_stats(&s0);
    if (pthread_create(&th, NULL, bulk_main, &a)) return -1;
    while (a.calls < 2 && !a.rc) {  /* the bulk job is running */
        struct timespec ts = {0, 1000000};
        nanosleep(&ts, NULL);
    }
    a.window = 1;
    const int rc = a.rc ? -1 : bl_hook_latency(device, 16, 4, 1200, 4, ncalls, out);
    a.window = 0;
    a.stop = 1;
    pthread_join(th, NULL);
    pquic_fec_protoop_stats(&s1);
    out[7] = (double)a.in_window;
    out[8] = (double)(s1.svc_deadline_misses - s0.svc_deadline_misses);
    out[9] = a.in_window ? a.sum_ms / a.in_window : 0;
    out[10] = a.max_ms;
    return rc || a.rc ? -1 : 0;
}

/* Where the last bl_run's measured pass spent its time: out[0] engine-thread us (all engines, inside
 * the engine calls), [1] stager-thread us, [2] caller-thread us in completions, [3] wall us, [4] caller
 * us waiting for a free block slot (completions inside it included), [5] caller us in submissions. */
void bl_last_phases(double out[6]) {
    for (int i = 0; i < 6; i++) out[i] = g_phases[i];
}

/* The last bl_run's measured pass: batch jobs the batcher allocated on the sender's thread, the us spent, and
 * the polls that held an overdue queue for want of an idle job (pquic_fec_batch_stats_t deadline_holds). */
void bl_last_jobs(double out[3]) {
    out[0] = g_jobs[0];
    out[1] = g_jobs[1];
    out[2] = g_jobs[2];
}

/* The last bl_run's measured pass, block latency (us): p50, p90, p95, p99, p99.9, max, mean; [7] blocks. */
void bl_last_latency(double out[8]) {
    for (int i = 0; i < 8; i++) out[i] = g_lat_q[i];
}

/* Rows the last bl_run's measured pass coded where they lie ([0]) and through the staging rows ([1]). */
void bl_last_rows(double out[2]) {
    out[0] = g_rows[0];
    out[1] = g_rows[1];
}

/* The gathered generate path without the batcher: `ncalls` calls of fecgpu_rlc_encode_rows_host on
 * `nblocks` blocks whose rows lie in a registered arena the way bl_run lays them out (sources in
 * distinct L-byte rows, repairs in 2112-B slots), row tables page-locked.  mode 0: as bl_run (the
 * sources of 64 blocks reused); 1: every block's sources distinct.  For comparison, [2] is the same
 * blocks staged in page-locked rows through fecgpu_rlc_encode_host (H2D, kernel, D2H).
 * out: [0] gathered payload GiB/s, [1] gathered ms per call, [2] staged GiB/s, [3] staged ms per call. */
int bl_rows_probe(int device, int k, int r, int L, long nblocks, int ncalls, int mode, double out[4]) {
    if (k < 1 || r < 1 || L < 4 || nblocks < 1 || ncalls < 1) return -1;
    const long src_blocks = mode ? nblocks : (nblocks < 64 ? nblocks : 64);
    const size_t pool = (size_t)src_blocks * k * L, slots = (size_t)nblocks * r * SLOT;
    const size_t bytes = ((pool + 4095) & ~(size_t)4095) + slots;
    uint8_t *arena = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (arena == MAP_FAILED) return -1;
    uint64_t x = 0x5EEDF3C0;
    for (size_t o = 0; o < pool; o++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; arena[o] = (uint8_t)x; }
    memset(arena + pool, 0, bytes - pool);
    uint64_t dev = 0;
    fecgpu_host_ctx_t *c = fecgpu_host_ctx_create(device, 2, (size_t)64 << 20);
    uint64_t *srow = fecgpu_host_alloc((size_t)nblocks * k * 8), *rrow = fecgpu_host_alloc((size_t)nblocks * r * 8);
    uint32_t *fbn = fecgpu_host_alloc((size_t)nblocks * 4);
    uint8_t *ssrc = fecgpu_host_alloc((size_t)nblocks * k * L), *srep = fecgpu_host_alloc((size_t)nblocks * r * L);
    int rc = -1;
    if (!c || !srow || !rrow || !fbn || !ssrc || !srep) goto out;
    if (fecgpu_host_register(arena, bytes) != FECGPU_OK) goto out;
    if (fecgpu_host_device_address(arena, bytes, &dev) != FECGPU_OK) goto unreg;
    const size_t rep0 = (pool + 4095) & ~(size_t)4095;
    for (long b = 0; b < nblocks; b++) {
        fbn[b] = (uint32_t)b & 0xffffffu;
        for (int j = 0; j < k; j++) srow[(size_t)b * k + j] = dev + ((size_t)(b % src_blocks) * k + j) * L;
        for (int i = 0; i < r; i++) rrow[(size_t)b * r + i] = dev + rep0 + ((size_t)b * r + i) * SLOT + 16;
    }
    for (long b = 0; b < nblocks; b++) memcpy(ssrc + (size_t)b * k * L, arena + (size_t)(b % src_blocks) * k * L, (size_t)k * L);
    for (int pass = 0; pass < 2; pass++) {
        if (pass ? fecgpu_rlc_encode_host(c, ssrc, srep, nblocks, k, r, L, 0, fbn)
                 : fecgpu_rlc_encode_rows_host(c, srow, rrow, nblocks, k, r, L, fbn))
            goto unreg;  /* warm-up call */
        const uint64_t t0 = now_us();
        for (int n = 0; n < ncalls; n++)
            if (pass ? fecgpu_rlc_encode_host(c, ssrc, srep, nblocks, k, r, L, 0, fbn)
                     : fecgpu_rlc_encode_rows_host(c, srow, rrow, nblocks, k, r, L, fbn))
                goto unreg;
        const double s = (now_us() - t0) * 1e-6;
        out[2 * pass] = (double)ncalls * nblocks * k * L / s / 1073741824.0;
        out[2 * pass + 1] = s * 1e3 / ncalls;
    }
    rc = 0;
unreg:
    fecgpu_host_unregister(arena);
out:
    fecgpu_host_free(srow); fecgpu_host_free(rrow); fecgpu_host_free(fbn); fecgpu_host_free(ssrc); fecgpu_host_free(srep);
    if (c) fecgpu_host_ctx_destroy(c);
    munmap(arena, bytes);
    return rc;
}

/* The bulk job of bl_hook_latency_loaded alone: `ncalls` back-to-back fecgpu_rlc_encode_host calls of
 * `blocks` k16 r4 L1200 blocks in page-locked memory.  out: [0] ms per call, [1] GiB/s of sources. */
int bl_bulk_rate(int device, int blocks, int ncalls, double out[2]) {
    const size_t sb = (size_t)blocks * 16 * 1200, rb = (size_t)blocks * 4 * 1200;
    fecgpu_host_ctx_t *c = fecgpu_host_ctx_create(device, 4, (size_t)64 << 20);
    uint8_t *src = fecgpu_host_alloc(sb), *rep = fecgpu_host_alloc(rb);
    int rc = -1;
    if (c && src && rep) {
        xorshift_fill(src, sb, 0x5EEDF3C0);
        rc = fecgpu_rlc_encode_host(c, src, rep, (uint64_t)blocks, 16, 4, 1200, 0, NULL);  /* warm-up */
        const uint64_t t0 = now_us();
        for (int n = 0; n < ncalls && !rc; n++) rc = fecgpu_rlc_encode_host(c, src, rep, (uint64_t)blocks, 16, 4, 1200, 0, NULL);
        const double s = (now_us() - t0) * 1e-6;
        out[0] = s * 1e3 / ncalls;
        out[1] = (double)ncalls * sb / s / 1073741824.0;
    }
    fecgpu_host_free(src);
    fecgpu_host_free(rep);
    if (c) fecgpu_host_ctx_destroy(c);
    return rc ? -1 : 0;
}
