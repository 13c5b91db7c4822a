// pquic_amd/csrc/host_path.hip -- host-resident entry points of include/fecgpu.h.
//
// The reference path starts and ends in host packet buffers (picoquic/packet.c:1468 on
// receive, sender.c:1084 on send).  These entry points move a batch of FEC blocks through
// the device: per sub-batch, H2D copy -> fecgpu_* kernels -> D2H copy on one of `nstreams`
// streams, so the copies of one sub-batch overlap the kernels of the next.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <shared_mutex>
#include <vector>

#include "../../include/fecgpu.h"

namespace {
constexpr int kMaxStreams = 4;
constexpr int kMaxYieldDepth = 16;

struct Slot {
  hipStream_t st = nullptr;
  void *d_src = nullptr, *d_rep = nullptr, *d_aux = nullptr, *d_ws = nullptr;
  size_t cap_src = 0, cap_rep = 0, cap_aux = 0, cap_ws = 0;
};

hipError_t grow(void **p, size_t *cap, size_t need) {
  if (need <= *cap) return hipSuccess;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipMalloc(p, need);
  if (e == hipSuccess) *cap = need;
  return e;
}
}  // namespace

struct fecgpu_host_ctx {
  int device = 0;
  int ns = 1;
  size_t chunk_bytes = 64u << 20;
  Slot slot[kMaxStreams];
  hipEvent_t yev[16] = {};  // the Pacer's slice completions (created on first use)
  std::mutex mu;
};

#define HCHK(x)                        \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return FECGPU_ERR_HIP; \
  } while (0)

extern "C" {

int fecgpu_svc_cu_mask(int device, int worker, uint32_t *mask, int max_words);  // fec_engine.hip (internal)

fecgpu_host_ctx_t *fecgpu_host_ctx_create(int device, int nstreams, size_t chunk_bytes) {
  if (fecgpu_init(device) != FECGPU_OK) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  auto *c = new fecgpu_host_ctx;
  c->device = device;
  c->ns = nstreams < 1 ? 1 : (nstreams > kMaxStreams ? kMaxStreams : nstreams);
  c->chunk_bytes = chunk_bytes ? chunk_bytes : (64u << 20);
  uint32_t cu_mask[16];
  const int mw = fecgpu_svc_cu_mask(device, 0, cu_mask, 16);  // off the block service's CUs (if reserved)
  for (int i = 0; i < c->ns; i++) {
    if ((mw ? hipExtStreamCreateWithCUMask(&c->slot[i].st, (uint32_t)mw, cu_mask)
            : hipStreamCreateWithFlags(&c->slot[i].st, hipStreamNonBlocking)) != hipSuccess) {
      fecgpu_host_ctx_destroy(c);
      return nullptr;
    }
  }
  return c;
}

void fecgpu_host_ctx_destroy(fecgpu_host_ctx_t *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (int i = 0; i < kMaxStreams; i++) {
    Slot &s = c->slot[i];
    if (s.st) { (void)hipStreamSynchronize(s.st); (void)hipStreamDestroy(s.st); }
    if (s.d_src) (void)hipFree(s.d_src);
    if (s.d_rep) (void)hipFree(s.d_rep);
    if (s.d_aux) (void)hipFree(s.d_aux);
    if (s.d_ws) (void)hipFree(s.d_ws);
  }
  for (hipEvent_t e : c->yev)
    if (e) (void)hipEventDestroy(e);
  delete c;
}

// Page-locked ranges the library made itself (fecgpu_host_alloc) or registered for a caller
// (fecgpu_host_register: e.g. a plugin's memory arena), with their device addresses, so the per-call
// lookups (the synchronous hooks pass seven pointers per recover, the batcher one table per job) skip
// hipPointerGetAttributes.  Sorted by base, read under a shared lock; an entry is removed before its
// memory stops being page-locked, so a stale entry can never describe unpinned memory.
namespace {
struct PinnedRange { uintptr_t base; size_t size; uint8_t *dev; bool registered; };
std::vector<PinnedRange> g_pinned;  // sorted by base, disjoint
std::shared_mutex g_pinned_mu;
std::atomic<uint64_t> g_pin_hits{0}, g_pin_misses{0};

void pinned_add(uintptr_t base, size_t size, uint8_t *dev, bool registered) {
  std::unique_lock<std::shared_mutex> g(g_pinned_mu);
  auto it = std::lower_bound(g_pinned.begin(), g_pinned.end(), base,
                             [](const PinnedRange &r, uintptr_t b) { return r.base < b; });
  g_pinned.insert(it, PinnedRange{base, size, dev, registered});
}

// removes the range starting at base; returns whether it was there (and whether it was registered)
bool pinned_remove(uintptr_t base, bool *registered) {
  std::unique_lock<std::shared_mutex> g(g_pinned_mu);
  auto it = std::lower_bound(g_pinned.begin(), g_pinned.end(), base,
                             [](const PinnedRange &r, uintptr_t b) { return r.base < b; });
  if (it == g_pinned.end() || it->base != base) return false;
  if (registered) *registered = it->registered;
  g_pinned.erase(it);
  return true;
}
}  // namespace

extern "C" __attribute__((visibility("hidden"))) void fecgpu_host_registry_stats(uint64_t *hits, uint64_t *misses) {
  *hits = g_pin_hits.load();
  *misses = g_pin_misses.load();
}


// Device address of [p, p + len) when ALL of it is page-locked host memory (hipHostMalloc'd or
// registered), else nullptr: the kernels then read and write the caller's memory directly, so an
// array that starts inside a pinned buffer but runs past its end must take the staged copies.
static uint8_t *mapped_host(const void *p, size_t len) {
  if (!p) return nullptr;
  const uintptr_t a = (uintptr_t)p;
  {
    std::shared_lock<std::shared_mutex> g(g_pinned_mu);
    auto it = std::upper_bound(g_pinned.begin(), g_pinned.end(), a,
                               [](uintptr_t x, const PinnedRange &r) { return x < r.base; });
    if (it != g_pinned.begin()) {
      --it;
      if (a - it->base < it->size) {
        g_pin_hits++;
        return len <= it->size - (a - it->base) ? it->dev + (a - it->base) : nullptr;
      }
    }
  }
  g_pin_misses++;
  hipPointerAttribute_t pa;
  if (hipPointerGetAttributes(&pa, p) != hipSuccess || pa.type != hipMemoryTypeHost || !pa.devicePointer) {
    (void)hipGetLastError();  // pageable memory: clear the query error
    return nullptr;
  }
  uint8_t *d = (uint8_t *)pa.devicePointer;
  if (len > 1) {  // the last byte must map into the same allocation, at the same offset
    hipPointerAttribute_t pe;
    if (hipPointerGetAttributes(&pe, (const uint8_t *)p + len - 1) != hipSuccess || pe.type != hipMemoryTypeHost ||
        (uint8_t *)pe.devicePointer != d + len - 1) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  return d;
}

// Page-locked host buffers are read (and written) by the kernels directly over PCIe instead of
// being staged by copies: measured 49.2 -> 51.0 GiB/s encode, 39.2 -> 50.3 GiB/s decode
// (k16 r4, 2^18 blocks).  Knob zc_read = 0 (FECGPU_ZC_READ=0) restores the staged copies (A/B).
int fecgpu_knob_zc_read(void);  // fec_engine.hip (library-internal, C linkage)
int fecgpu_rlc_decode_to_internal(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k,
                                  uint32_t r, uint32_t L, uint32_t fbn_base, const uint32_t *fbn,
                                  const uint32_t *seeds, const uint64_t *sp, const uint64_t *rp, uint8_t *status,
                                  uint64_t *recovered, void *ws, size_t wsb, void *stream);  // fec_engine.hip
int fecgpu_knob_window_sc(void);  // fec_engine.hip (library-internal)
static bool zc_read() { return fecgpu_knob_zc_read() != 0; }

// ---- zero-copy bulk calls yield to the synchronous hooks ----
// A hook's rows cross the same PCIe link as a zero-copy bulk call's, and the hook's reads complete only
// once the bulk kernel running at that moment ends: beside back-to-back bulk calls of 4096 / 1024 / 512 /
// 256 blocks (1.58 / 0.47 / 0.30 / 0.17 ms each) the hooks' p99 was 1471 / 417 / 271 / 138 us
// (profiles/r05_hook_sweep.log; rocprofv3 trace in profiles/r05_hook_trace_summary.txt: the slow calls
// spend no time in HIP calls and involve no worker launch -- the resident worker's reads wait).  So
// while the block service is in use (a hook request within the last yield_window_ms, 100 ms), a zero-copy launch
// is cut into slices of about yield_slice_kb of payload, alternating over yield_streams of the context's
// streams (consecutive slices overlap, so the cut costs less), at most yield_depth in flight (knobs;
// defaults and their measurement in fec_engine.hip knobs_default).  Optionally (yield_gate_us) no
// slice starts while a hook request is pending.  Without hooks nothing changes (one launch).  The
// hooks still wait for the slices running when they arrive; the slice size trades their p99 against
// the bulk call's time (about 55-80 us of PCIe transfer per 2.25-2.5 MiB slice).
int fecgpu_svc_hooks_pending(void);                                  // fec_engine.hip (library-internal)
uint64_t fecgpu_svc_last_request_us(void);                           // fec_engine.hip (library-internal)
void fecgpu_knob_yield(int *slice_kb, int *depth, int *gate_us, int *streams, int *always,
                       int *window_ms);  // fec_engine.hip
namespace {
std::atomic<uint64_t> g_yield_slices{0}, g_yield_waits{0};

uint64_t mono_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

struct Pacer {
  fecgpu_host_ctx_t *c;
  uint64_t slice = 0;  // blocks per slice; 0: hooks idle or the call is small, launch it whole
  int n = 0;           // slices launched
  int depth = 4, gate_us = 0, streams = 1;
  Pacer(fecgpu_host_ctx_t *c_, uint64_t nblocks, size_t bytes_per_block) : c(c_) {
    int kb = 0, always = 0, window_ms = 100;
    fecgpu_knob_yield(&kb, &depth, &gate_us, &streams, &always, &window_ms);
    const uint64_t last = fecgpu_svc_last_request_us();
    if (!always && (!last || mono_us() - last > (uint64_t)window_ms * 1000u)) return;
    if (streams > c->ns) streams = c->ns;
    if (!kb || depth > kMaxYieldDepth) return;
    uint64_t per = ((uint64_t)kb << 10) / (bytes_per_block ? bytes_per_block : 1);
    if (per < 32) per = 32;
    if (per >= nblocks) return;
    for (int i = 0; i < depth; i++)
      if (!c->yev[i] && hipEventCreateWithFlags(&c->yev[i], hipEventDisableTiming) != hipSuccess) return;
    slice = per;
  }
  // the stream of the next slice (slices alternate over `streams` of the context's streams)
  hipStream_t stream(hipStream_t whole) const { return slice ? c->slot[n % streams].st : whole; }
  // before slice n: at most `depth` in flight, and (gate) none started while a hook request is pending
  hipError_t before() {
    if (!slice) return hipSuccess;
    if (n >= depth)
      if (hipError_t e = hipEventSynchronize(c->yev[n % depth])) return e;
    if (gate_us && fecgpu_svc_hooks_pending() > 0) {
      g_yield_waits++;
      const uint64_t t0 = mono_us();
      while (fecgpu_svc_hooks_pending() > 0 && mono_us() - t0 < (uint64_t)gate_us) __builtin_ia32_pause();
    }
    return hipSuccess;
  }
  hipError_t after() {
    if (!slice) return hipSuccess;
    g_yield_slices++;
    const hipError_t e = hipEventRecord(c->yev[n % depth], c->slot[n % streams].st);
    n++;
    return e;
  }
};
}  // namespace

__attribute__((visibility("hidden"))) void fecgpu_host_yield_stats(uint64_t *slices, uint64_t *waits) {
  *slices = g_yield_slices.load();
  *waits = g_yield_waits.load();
}

static uint64_t sub_batch(const fecgpu_host_ctx_t *c, uint64_t nblocks, size_t per_block) {
  uint64_t n = c->chunk_bytes / (per_block ? per_block : 1);
  if (n < 1) n = 1;
  return n < nblocks ? n : nblocks;
}

// Every stream drains before a call returns -- also after an error part-way through a batch: work
// already queued (copies, and with page-locked buffers kernels writing repairs / recovered rows
// straight into host memory) must not outlive the call, or it could overwrite buffers the caller
// reuses (the batching adapter recycles its page-locked rows as soon as a job completes).
static int finish(fecgpu_host_ctx_t *c, int rc) {
  for (int i = 0; i < c->ns; i++) {
    const hipError_t e = hipStreamSynchronize(c->slot[i].st);
    if (e != hipSuccess && rc == FECGPU_OK) rc = FECGPU_ERR_HIP;
  }
  return rc;
}

// HCHK inside a sub-batch loop: record the error and leave the loop (finish() then drains).
#define LCHK(x)                               \
  if ((x) != hipSuccess) {                    \
    rc = FECGPU_ERR_HIP;                      \
    break;                                    \
  }

int fecgpu_rlc_encode_host(fecgpu_host_ctx_t *c, const void *src, void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t L, uint32_t fbn_base, const uint32_t *fbn) {
  if (!c || !src || !rep) return FECGPU_ERR_INVALID;
  if (!nblocks || !r) return FECGPU_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HCHK(hipSetDevice(c->device));
  const size_t sb = (size_t)k * L, rb = (size_t)r * L;
  const uint64_t n = sub_batch(c, nblocks, sb);
  uint8_t *zs = zc_read() ? mapped_host(src, nblocks * sb) : nullptr, *zr = zs ? mapped_host(rep, nblocks * rb) : nullptr;
  int si = 0, rc = FECGPU_OK;
  if (zs && zr) {  // page-locked, hooks in use: slices that yield to them (Pacer)
    Slot &s = c->slot[0];
    Pacer pc(c, nblocks, sb + rb);
    if (pc.slice) {
      const uint32_t *df = nullptr;
      do {
        if (fbn) {
          LCHK(grow(&s.d_aux, &s.cap_aux, nblocks * 4));
          LCHK(hipMemcpyAsync(s.d_aux, fbn, nblocks * 4, hipMemcpyHostToDevice, s.st));
          if (pc.streams > 1) LCHK(hipStreamSynchronize(s.st));  // slices on the other streams read it
          df = (const uint32_t *)s.d_aux;
        }
        for (uint64_t b0 = 0; b0 < nblocks; b0 += pc.slice) {
          const uint64_t m = nblocks - b0 < pc.slice ? nblocks - b0 : pc.slice;
          LCHK(pc.before());
          if ((rc = fecgpu_rlc_encode(zs + b0 * sb, zr + b0 * rb, m, k, r, L, (uint32_t)((fbn_base + b0) & 0xffffffu),
                                      df ? df + b0 : nullptr, pc.stream(s.st))))
            break;
          LCHK(pc.after());
        }
      } while (0);
      return finish(c, rc);
    }
  }
  for (uint64_t b0 = 0; b0 < nblocks; b0 += n, si = (si + 1) % c->ns) {
    Slot &s = c->slot[si];
    const uint64_t m = nblocks - b0 < n ? nblocks - b0 : n;
    const uint32_t *df = nullptr;
    if (fbn) {
      LCHK(grow(&s.d_aux, &s.cap_aux, n * 4));
      LCHK(hipMemcpyAsync(s.d_aux, fbn + b0, m * 4, hipMemcpyHostToDevice, s.st));
      df = (const uint32_t *)s.d_aux;
    }
    const uint32_t fb0 = (uint32_t)((fbn_base + b0) & 0xffffffu);
    if (zs && zr) {  // page-locked buffers: the kernel reads sources from / writes repairs to host memory
      if ((rc = fecgpu_rlc_encode(zs + b0 * sb, zr + b0 * rb, m, k, r, L, fb0, df, s.st))) break;
      continue;
    }
    LCHK(grow(&s.d_src, &s.cap_src, n * sb));
    LCHK(grow(&s.d_rep, &s.cap_rep, n * rb));
    LCHK(hipMemcpyAsync(s.d_src, (const uint8_t *)src + b0 * sb, m * sb, hipMemcpyHostToDevice, s.st));
    if ((rc = fecgpu_rlc_encode(s.d_src, s.d_rep, m, k, r, L, fb0, df, s.st))) break;
    LCHK(hipMemcpyAsync((uint8_t *)rep + b0 * rb, s.d_rep, m * rb, hipMemcpyDeviceToHost, s.st));
  }
  return finish(c, rc);
}

int fecgpu_rlc_encode_rows_host(fecgpu_host_ctx_t *c, const uint64_t *src_rows, const uint64_t *rep_rows,
                                uint64_t nblocks, uint32_t k, uint32_t r, uint32_t L, const uint32_t *fbn) {
  if (!c || !src_rows || !rep_rows) return FECGPU_ERR_INVALID;
  if (!nblocks || !r) return FECGPU_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HCHK(hipSetDevice(c->device));
  Slot &s = c->slot[0];
  const uint64_t *ds = (const uint64_t *)mapped_host(src_rows, nblocks * k * 8);
  const uint64_t *dr = (const uint64_t *)mapped_host(rep_rows, nblocks * r * 8);
  const uint32_t *df = fbn ? (const uint32_t *)mapped_host(fbn, nblocks * 4) : nullptr;
  int rc = FECGPU_OK;
  do {
    if (!ds || !dr || (fbn && !df)) {  // pageable tables: one device copy
      const size_t need = nblocks * (k + r) * 8 + (fbn ? nblocks * 4 : 0);
      LCHK(grow(&s.d_aux, &s.cap_aux, need));
      uint8_t *a = (uint8_t *)s.d_aux;
      LCHK(hipMemcpyAsync(a, src_rows, nblocks * k * 8, hipMemcpyHostToDevice, s.st));
      LCHK(hipMemcpyAsync(a + nblocks * k * 8, rep_rows, nblocks * r * 8, hipMemcpyHostToDevice, s.st));
      if (fbn) LCHK(hipMemcpyAsync(a + nblocks * (k + r) * 8, fbn, nblocks * 4, hipMemcpyHostToDevice, s.st));
      ds = (const uint64_t *)a;
      dr = (const uint64_t *)(a + nblocks * k * 8);
      df = fbn ? (const uint32_t *)(a + nblocks * (k + r) * 8) : nullptr;
    }
    Pacer pc(c, nblocks, (size_t)(k + r) * L);  // hooks in use: slices that yield to them
    if (pc.slice && pc.streams > 1) LCHK(hipStreamSynchronize(s.st));  // copied tables, read from other streams
    for (uint64_t b0 = 0, step = pc.slice ? pc.slice : nblocks; b0 < nblocks; b0 += step) {
      const uint64_t m = nblocks - b0 < step ? nblocks - b0 : step;
      LCHK(pc.before());
      // without fbn[] block b is block number b (fecgpu.h:21): slice b0 starts at b0, not 0
      if ((rc = fecgpu_rlc_encode_rows(ds + b0 * k, dr + b0 * r, m, k, r, L, df ? 0u : (uint32_t)(b0 & 0xffffffu),
                                       df ? df + b0 : nullptr, pc.stream(s.st))))
        break;
      LCHK(pc.after());
    }
  } while (0);
  return finish(c, rc);
}

int fecgpu_rlc_window_encode_host(fecgpu_host_ctx_t *c, const void *symbols, uint64_t nrows, const uint32_t *wrow,
                                  uint64_t nwin, uint32_t k, uint32_t r, uint32_t L, void *rep) {
  if (!c || !symbols || !wrow || !rep || !k) return FECGPU_ERR_INVALID;
  if (!nwin || !r) return FECGPU_OK;
  for (uint64_t w = 0; w < nwin; w++)  // the rows every window names exist (the kernel reads them unchecked)
    if ((uint64_t)wrow[w] + k > nrows) return FECGPU_ERR_INVALID;
  std::lock_guard<std::mutex> g(c->mu);
  HCHK(hipSetDevice(c->device));
  Slot &s = c->slot[0];
  const size_t sb = nrows * (size_t)L, rb = nwin * (size_t)r * L;
  uint8_t *zr = zc_read() ? mapped_host(rep, rb) : nullptr;
  const bool table = fecgpu_knob_window_sc() != 0;
  int rc = FECGPU_OK;
  do {
    LCHK(grow(&s.d_src, &s.cap_src, sb));
    LCHK(hipMemcpyAsync(s.d_src, symbols, sb, hipMemcpyHostToDevice, s.st));
    uint8_t *dr = zr;
    if (!dr) {
      LCHK(grow(&s.d_rep, &s.cap_rep, rb));
      dr = (uint8_t *)s.d_rep;
    }
    if (table) {
      LCHK(grow(&s.d_aux, &s.cap_aux, nwin * 4));
      LCHK(hipMemcpyAsync(s.d_aux, wrow, nwin * 4, hipMemcpyHostToDevice, s.st));
      if ((rc = fecgpu_rlc_window_encode_table(s.d_src, nrows, (const uint32_t *)s.d_aux, nwin, k, r, L, dr, s.st)))
        break;
    } else {  // row tables: window w's rows and repairs by address, block number 0
      std::vector<uint64_t> rows(nwin * (size_t)(k + r));
      const uint64_t sd = (uint64_t)(uintptr_t)s.d_src, rd = (uint64_t)(uintptr_t)dr;
      for (uint64_t w = 0; w < nwin; w++) {
        for (uint32_t j = 0; j < k; j++) rows[w * k + j] = sd + ((uint64_t)wrow[w] + j) * L;
        for (uint32_t i = 0; i < r; i++) rows[nwin * k + w * r + i] = rd + (w * r + i) * (uint64_t)L;
      }
      LCHK(grow(&s.d_aux, &s.cap_aux, rows.size() * 8 + nwin * 4));
      LCHK(hipMemcpyAsync(s.d_aux, rows.data(), rows.size() * 8, hipMemcpyHostToDevice, s.st));
      const uint64_t *t = (const uint64_t *)s.d_aux;
      uint32_t *zero_fbn = (uint32_t *)(t + rows.size());  // every window is block number 0
      LCHK(hipMemsetAsync(zero_fbn, 0, nwin * 4, s.st));
      if ((rc = fecgpu_rlc_encode_rows(t, t + nwin * k, nwin, k, r, L, 0, zero_fbn, s.st))) break;
      LCHK(hipStreamSynchronize(s.st));  // `rows` is pageable and leaves scope
    }
    if (!zr) LCHK(hipMemcpyAsync(rep, dr, rb, hipMemcpyDeviceToHost, s.st));
  } while (0);
  return finish(c, rc);
}

int fecgpu_xor_encode_host(fecgpu_host_ctx_t *c, const void *src, void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t L) {
  if (!c || !src || !rep) return FECGPU_ERR_INVALID;
  if (!nblocks) return FECGPU_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HCHK(hipSetDevice(c->device));
  const size_t sb = (size_t)k * L, rb = L;
  const uint64_t n = sub_batch(c, nblocks, sb);
  int si = 0, rc = FECGPU_OK;
  for (uint64_t b0 = 0; b0 < nblocks; b0 += n, si = (si + 1) % c->ns) {
    Slot &s = c->slot[si];
    const uint64_t m = nblocks - b0 < n ? nblocks - b0 : n;
    LCHK(grow(&s.d_src, &s.cap_src, n * sb));
    LCHK(grow(&s.d_rep, &s.cap_rep, n * rb));
    LCHK(hipMemcpyAsync(s.d_src, (const uint8_t *)src + b0 * sb, m * sb, hipMemcpyHostToDevice, s.st));
    if ((rc = fecgpu_xor_encode(s.d_src, s.d_rep, m, k, L, s.st))) break;
    LCHK(hipMemcpyAsync((uint8_t *)rep + b0 * rb, s.d_rep, m * rb, hipMemcpyDeviceToHost, s.st));
  }
  return finish(c, rc);
}

// aux layout per sub-batch: fbn[n] or rep_seed[n][r] (u32, padded to 16), src_present[n][2],
// rep_present[n][2], recovered[n][2] (u64), status[n] (u8)
static size_t aux_bytes(uint64_t n, uint32_t nseed) { return ((n * 4 * nseed + 15) & ~(size_t)15) + n * 16 * 3 + n; }

// seeds: rep_seed[nblocks][r] (per-repair FPID seeds) or nullptr (block numbers from fbn / fbn_base)
static int decode_host(fecgpu_host_ctx_t *c, bool xr, void *src, const void *rep, uint64_t nblocks, uint32_t k,
                       uint32_t r, uint32_t L, uint32_t fbn_base, const uint32_t *fbn, const uint32_t *seeds,
                       const uint64_t *sp, const uint64_t *rp, uint8_t *status, uint64_t *recovered) {
  if (!c || !src || !rep || !sp || !rp || !status || !recovered) return FECGPU_ERR_INVALID;
  if (!nblocks) return FECGPU_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HCHK(hipSetDevice(c->device));
  const size_t sb = (size_t)k * L, rb = (size_t)r * L;
  const uint32_t nseed = seeds ? (r ? r : 1) : 1;
  const uint64_t n = sub_batch(c, nblocks, sb + rb);
  // page-locked src (hipHostMalloc / registered): the apply kernel writes the recovered rows
  // straight into it over PCIe, so nothing but status comes back by copy
  uint8_t *zdst = xr ? nullptr : mapped_host(src, nblocks * sb);
  const uint8_t *zrep = zdst && zc_read() ? mapped_host(rep, nblocks * rb) : nullptr;
  // page-locked masks / seeds / outputs as well (the synchronous protoops keep theirs so): the
  // kernels read and write them in place, and a call is two launches and one synchronisation with
  // no copies at all -- the latency of one-block calls is launch + PCIe round trips
  const uint32_t *zseed = nullptr;
  const uint64_t *zsp = nullptr, *zrp = nullptr;
  uint8_t *zst = nullptr;
  uint64_t *zrec = nullptr;
  if (zrep) {
    zsp = (const uint64_t *)mapped_host(sp, nblocks * 16);
    zrp = zsp ? (const uint64_t *)mapped_host(rp, nblocks * 16) : nullptr;
    zst = zrp ? mapped_host(status, nblocks) : nullptr;
    zrec = zst ? (uint64_t *)mapped_host(recovered, nblocks * 16) : nullptr;
    const uint32_t *sf = seeds ? seeds : fbn;
    zseed = zrec && sf ? (const uint32_t *)mapped_host(sf, nblocks * 4 * (seeds ? (r ? r : 1) : 1)) : nullptr;
    if (!zrec || (sf && !zseed)) zsp = nullptr;  // all or nothing
  }
  int si = 0, rc = FECGPU_OK;
  for (uint64_t b0 = 0; b0 < nblocks; b0 += n, si = (si + 1) % c->ns) {
    Slot &s = c->slot[si];
    const uint64_t m = nblocks - b0 < n ? nblocks - b0 : n;
    LCHK(grow(&s.d_aux, &s.cap_aux, aux_bytes(n, nseed)));
    uint8_t *aux = (uint8_t *)s.d_aux;
    uint32_t *d_fbn = (uint32_t *)aux;  // fbn[] or rep_seed[][]
    uint64_t *d_sp = (uint64_t *)(aux + ((n * 4 * nseed + 15) & ~(size_t)15));
    uint64_t *d_rp = d_sp + 2 * n, *d_rec = d_rp + 2 * n;
    uint8_t *d_st = (uint8_t *)(d_rec + 2 * n);
    if (zsp) {  // everything page-locked: the kernels use the caller's arrays in place
      d_sp = const_cast<uint64_t *>(zsp) + 2 * b0;
      d_rp = const_cast<uint64_t *>(zrp) + 2 * b0;
      d_rec = zrec + 2 * b0;
      d_st = zst + b0;
      if (zseed) d_fbn = const_cast<uint32_t *>(zseed) + (seeds ? b0 * r : b0);
    } else {
      LCHK(hipMemcpyAsync(d_sp, sp + 2 * b0, m * 16, hipMemcpyHostToDevice, s.st));
      LCHK(hipMemcpyAsync(d_rp, rp + 2 * b0, m * 16, hipMemcpyHostToDevice, s.st));
      if (seeds && r) {
        LCHK(hipMemcpyAsync(d_fbn, seeds + b0 * r, m * 4 * r, hipMemcpyHostToDevice, s.st));
      } else if (fbn) {
        LCHK(hipMemcpyAsync(d_fbn, fbn + b0, m * 4, hipMemcpyHostToDevice, s.st));
      }
    }
    const uint8_t *in_src, *in_rep;
    if (zrep) {
      in_src = zdst + b0 * sb;
      in_rep = zrep + b0 * rb;
    } else {
      LCHK(grow(&s.d_src, &s.cap_src, n * sb));
      LCHK(grow(&s.d_rep, &s.cap_rep, n * rb));
      in_src = (const uint8_t *)s.d_src;
      in_rep = (const uint8_t *)s.d_rep;
      LCHK(hipMemcpyAsync(s.d_src, (const uint8_t *)src + b0 * sb, m * sb, hipMemcpyHostToDevice, s.st));
      LCHK(hipMemcpyAsync(s.d_rep, (const uint8_t *)rep + b0 * rb, m * rb, hipMemcpyHostToDevice, s.st));
    }
    if (xr) {
      rc = fecgpu_xor_decode(s.d_src, s.d_rep, m, k, L, d_sp, d_rp, d_st, d_rec, s.st);
    } else {
      const size_t wsb = fecgpu_rlc_decode_workspace(n, k, r);
      LCHK(grow(&s.d_ws, &s.cap_ws, wsb));
      // plan + data pass (one launch for a few blocks, e.g. the synchronous hook's one)
      rc = fecgpu_rlc_decode_to_internal(in_src, in_rep, zdst ? zdst + b0 * sb : s.d_src, m, k, r, L,
                                         seeds ? 0u : (uint32_t)((fbn_base + b0) & 0xffffffu),
                                         (!seeds && fbn) ? d_fbn : nullptr, seeds ? d_fbn : nullptr, d_sp, d_rp,
                                         d_st, d_rec, s.d_ws, s.cap_ws, s.st);
    }
    if (rc) break;
    if (!zdst) LCHK(hipMemcpyAsync((uint8_t *)src + b0 * sb, s.d_src, m * sb, hipMemcpyDeviceToHost, s.st));
    if (!zsp) {
      LCHK(hipMemcpyAsync(status + b0, d_st, m, hipMemcpyDeviceToHost, s.st));
      LCHK(hipMemcpyAsync(recovered + 2 * b0, d_rec, m * 16, hipMemcpyDeviceToHost, s.st));
    }
  }
  return finish(c, rc);
}

int fecgpu_rlc_decode_host(fecgpu_host_ctx_t *c, void *src, const void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t L, uint32_t fbn_base, const uint32_t *fbn,
                           const uint64_t *sp, const uint64_t *rp, uint8_t *status, uint64_t *recovered) {
  return decode_host(c, false, src, rep, nblocks, k, r, L, fbn_base, fbn, nullptr, sp, rp, status, recovered);
}

int fecgpu_rlc_decode_host_seeded(fecgpu_host_ctx_t *c, void *src, const void *rep, uint64_t nblocks, uint32_t k,
                                  uint32_t r, uint32_t L, const uint32_t *rep_seed, const uint64_t *sp,
                                  const uint64_t *rp, uint8_t *status, uint64_t *recovered) {
  if (nblocks && r && !rep_seed) return FECGPU_ERR_INVALID;
  return decode_host(c, false, src, rep, nblocks, k, r, L, 0, nullptr, rep_seed, sp, rp, status, recovered);
}

int fecgpu_rlc_decode_rows_host(fecgpu_host_ctx_t *c, const uint64_t *src_rows, const uint64_t *rep_rows,
                                uint64_t nblocks, uint32_t k, uint32_t r, uint32_t L, const uint32_t *seeds,
                                const uint64_t *sp, const uint64_t *rp, uint8_t *status, uint64_t *recovered) {
  if (!c || !src_rows || (r && (!rep_rows || !seeds)) || !sp || !rp || !status || !recovered) return FECGPU_ERR_INVALID;
  if (!nblocks) return FECGPU_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HCHK(hipSetDevice(c->device));
  Slot &s = c->slot[0];
  const uint32_t nseed = r ? r : 1;
  // every array page-locked (the batching adapter's job tables): the kernels use them in place.  With
  // r == 0 the repair table and seeds have no entries and are never read: the source table stands in
  const uint64_t *ds = (const uint64_t *)mapped_host(src_rows, nblocks * k * 8);
  const uint64_t *dr = !ds ? nullptr : r ? (const uint64_t *)mapped_host(rep_rows, nblocks * r * 8) : ds;
  const uint32_t *dseed = !dr ? nullptr : r ? (const uint32_t *)mapped_host(seeds, nblocks * r * 4)
                                            : (const uint32_t *)ds;
  const uint64_t *dsp = dseed ? (const uint64_t *)mapped_host(sp, nblocks * 16) : nullptr;
  const uint64_t *drp = dsp ? (const uint64_t *)mapped_host(rp, nblocks * 16) : nullptr;
  uint8_t *dst = drp ? mapped_host(status, nblocks) : nullptr;
  uint64_t *drec = dst ? (uint64_t *)mapped_host(recovered, nblocks * 16) : nullptr;
  int rc = FECGPU_OK;
  do {
    const size_t wsb = fecgpu_rlc_decode_workspace(nblocks, k, r);
    LCHK(grow(&s.d_ws, &s.cap_ws, wsb));
    if (!drec) {  // pageable: one device copy of the tables and masks, status and masks copied back
      const size_t tb = nblocks * (k + nseed) * 8, sdb = (nblocks * nseed * 4 + 15) & ~(size_t)15;
      LCHK(grow(&s.d_aux, &s.cap_aux, tb + sdb + nblocks * 48 + nblocks));
      uint8_t *a = (uint8_t *)s.d_aux;
      ds = (const uint64_t *)a;
      dr = (const uint64_t *)(a + nblocks * k * 8);
      dseed = (const uint32_t *)(a + tb);
      uint64_t *m = (uint64_t *)(a + tb + sdb);
      dsp = m;
      drp = m + 2 * nblocks;
      drec = m + 4 * nblocks;
      dst = (uint8_t *)(m + 6 * nblocks);
      LCHK(hipMemcpyAsync((void *)ds, src_rows, nblocks * k * 8, hipMemcpyHostToDevice, s.st));
      if (r) LCHK(hipMemcpyAsync((void *)dr, rep_rows, nblocks * r * 8, hipMemcpyHostToDevice, s.st));
      if (r) LCHK(hipMemcpyAsync((void *)dseed, seeds, nblocks * r * 4, hipMemcpyHostToDevice, s.st));
      LCHK(hipMemcpyAsync((void *)dsp, sp, nblocks * 16, hipMemcpyHostToDevice, s.st));
      LCHK(hipMemcpyAsync((void *)drp, rp, nblocks * 16, hipMemcpyHostToDevice, s.st));
      if ((rc = fecgpu_rlc_decode_rows(ds, dr, nblocks, k, r, L, dseed, dsp, drp, dst, drec, s.d_ws, s.cap_ws, s.st)))
        break;
      LCHK(hipMemcpyAsync(status, dst, nblocks, hipMemcpyDeviceToHost, s.st));
      LCHK(hipMemcpyAsync(recovered, drec, nblocks * 16, hipMemcpyDeviceToHost, s.st));
      break;
    }
    Pacer pc(c, nblocks, (size_t)(k + r) * L);  // hooks in use: slices that yield to them
    for (uint64_t b0 = 0, step = pc.slice ? pc.slice : nblocks; b0 < nblocks; b0 += step) {
      const uint64_t m = nblocks - b0 < step ? nblocks - b0 : step;
      LCHK(pc.before());
      // one workspace per stream the slices alternate over
      Slot &ws = c->slot[pc.slice ? pc.n % pc.streams : 0];
      if (&ws != &s) LCHK(grow(&ws.d_ws, &ws.cap_ws, fecgpu_rlc_decode_workspace(m, k, r)));
      if ((rc = fecgpu_rlc_decode_rows(ds + b0 * k, dr + b0 * nseed, m, k, r, L, dseed + b0 * nseed, dsp + 2 * b0,
                                       drp + 2 * b0, dst + b0, drec + 2 * b0, ws.d_ws, ws.cap_ws, pc.stream(s.st))))
        break;
      LCHK(pc.after());
    }
  } while (0);
  return finish(c, rc);
}

int fecgpu_xor_decode_host(fecgpu_host_ctx_t *c, void *src, const void *rep, uint64_t nblocks, uint32_t k,
                           uint32_t L, const uint64_t *sp, const uint64_t *rp, uint8_t *status,
                           uint64_t *recovered) {
  return decode_host(c, true, src, rep, nblocks, k, 1, L, 0, nullptr, nullptr, sp, rp, status, recovered);
}

}  // extern "C"

extern "C" {
int fecgpu_knob_host_alloc(void);  // fec_engine.hip (library-internal)

void *fecgpu_host_alloc(size_t bytes) {
  void *p = nullptr;
  const int mode = fecgpu_knob_host_alloc();
  const unsigned flags = mode == 1 ? hipHostMallocMapped | hipHostMallocCoherent
                       : mode == 2 ? hipHostMallocMapped | hipHostMallocNonCoherent : hipHostMallocDefault;
  if (hipHostMalloc(&p, bytes ? bytes : 1, flags) != hipSuccess) return nullptr;
  hipPointerAttribute_t pa;
  if (hipPointerGetAttributes(&pa, p) == hipSuccess && pa.devicePointer)
    pinned_add((uintptr_t)p, bytes ? bytes : 1, (uint8_t *)pa.devicePointer, false);
  else
    (void)hipGetLastError();
  return p;
}

void fecgpu_host_free(void *p) {
  if (!p) return;
  pinned_remove((uintptr_t)p, nullptr);
  (void)hipHostFree(p);
}

int fecgpu_device_local_cpus(int device, char *buf, size_t len) {
  if (!buf || len < 2) return FECGPU_ERR_INVALID;
  char bus[64];
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return FECGPU_ERR_NO_DEVICE;
  }
  for (char *c = bus; *c; c++)
    if (*c >= 'A' && *c <= 'F') *c = (char)(*c - 'A' + 'a');  // sysfs names are lower case
  char path[128];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/local_cpulist", bus);
  FILE *f = fopen(path, "r");
  if (!f) return FECGPU_ERR_INVALID;
  const bool ok = fgets(buf, (int)len, f) != nullptr;
  fclose(f);
  if (!ok) return FECGPU_ERR_INVALID;
  for (char *c = buf; *c; c++)
    if (*c == '\n') *c = 0;
  return FECGPU_OK;
}

int fecgpu_host_register(void *p, size_t bytes) {
  if (!p || !bytes) return FECGPU_ERR_INVALID;
  if (hipHostRegister(p, bytes, hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    return FECGPU_ERR_HIP;
  }
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    (void)hipHostUnregister(p);
    return FECGPU_ERR_HIP;
  }
  pinned_add((uintptr_t)p, bytes, (uint8_t *)d, true);
  return FECGPU_OK;
}

int fecgpu_host_unregister(void *p) {
  bool reg = false;
  if (!p || !pinned_remove((uintptr_t)p, &reg) || !reg) return FECGPU_ERR_INVALID;
  return hipHostUnregister(p) == hipSuccess ? FECGPU_OK : FECGPU_ERR_HIP;
}

int fecgpu_host_device_address(const void *p, size_t bytes, uint64_t *dev) {
  if (!dev) return FECGPU_ERR_INVALID;
  uint8_t *d = mapped_host(p, bytes);
  *dev = (uint64_t)(uintptr_t)d;
  return d ? FECGPU_OK : FECGPU_ERR_INVALID;
}
}  // extern "C"
