// pquic_amd/csrc/fec_engine.hip -- MI355X (gfx950) FEC engine: kernels + C ABI (include/fecgpu.h).
//
// Data path (HBM-bound byte arithmetic over GF(2^8), no MFMA):
//   k_rlc_encode_bs / _bs2 / _rows   a wave streams a group of blocks (one column chunk of <= 2 KiB
//                  at a time, a lane owning 32 B of a row).  Each source row is loaded once and
//                  bit-sliced in registers (three shift-exchange rounds -> 8 bit planes), its
//                  Four-Russians XOR combinations are built once, and every coefficient then costs
//                  one 3-input XOR per output plane, dispatched by the wave-uniform coefficient
//                  through a chain of generated case blocks (bitslice_gen.h, from gen_bitslice.py).
//                  Coefficients come from TinyMT32 run per (block, repair) in the group setup (seed
//                  (fbn << 8) | i) and wait in LDS as 16-bit case offsets.  Sources wait in VGPRs
//                  (register prefetch, tiles of 1-8 repairs) or in a per-wave LDS ring fed by LDS-DMA
//                  (16-repair tiles).
//   k_rlc_plan*    the decode plan: replays the reference's fec_recover on the coefficients only
//                  (repair selection, sort_system, elimination without re-pivoting, back
//                  substitution) and emits the e x k matrix that maps the k received symbols to the e
//                  unknowns, plus the dependency pattern of the "all-zero unknown" rule.
//   k_rlc_recover_bs / _bs2   the data pass of decode: the encode's bodies with the plan's rows as
//                  coefficients and the inputs gathered by the plan's slot map (or row tables); the
//                  zero/undetermined rule fused for e <= 16, k_rlc_finalize beyond.
//   k_rlc_encode_lds / k_rlc_decode_lds / k_block_svc   one block per workgroup (the synchronous hooks):
//                  rows staged in LDS, a packed v_perm multiply (fec_device.h gf_mac) per dword.
//   k_xor_*        XOR scheme, streaming 16-B lanes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <atomic>
#include <mutex>
#include <stdlib.h>

#include "fec_device.h"
#ifdef FEC_BS_GEN_HEADER  // A/B experiments: an alternative generated body set
#include FEC_BS_GEN_HEADER
#else
#ifdef FEC_GEN_HDR  // A/B builds of a generator variant (tools/gen_variant.py)
#include FEC_GEN_HDR
#else
#include "bitslice_gen.h"
#endif
#endif
#include "../../include/fecgpu.h"

using namespace fecdev;

#define FECGPU_VERSION "pquic_amd fecgpu 0.2 (gfx950, bitsliced GF(256) data path)"

static thread_local char g_err[256];
static std::atomic<uint64_t> g_stats[4];

// ---------------------------------------------------------------------------------------------
// Experiment knobs (A/B runs; the tests cross-check alternative kernels).  The defaults are the
// measured best, and only fecgpu_set_knob changes one (include/fecgpu.h): the library reads no
// environment variables, so nothing outside the caller's own calls can change which kernels run.
// ---------------------------------------------------------------------------------------------
enum KnobId { K_PLAN, K_INTERLEAVE, K_GROUP, K_ENC_RT, K_ENC_W, K_ZC_READ, K_RING, K_WINDOW_SC, K_MIN_GROUPS,
              K_ENC_BW,
              K_CHUNK_WAVES, K_SMALL_LDS, K_BLOCK_SVC, K_WS_LDS, K_DEC_WAVES, K_YIELD_SLICE_KB, K_YIELD_DEPTH,
              K_YIELD_GATE_US, K_YIELD_STREAMS, K_YIELD_ALWAYS, K_YIELD_WINDOW_MS, K_SVC_RESERVE_CUS, K_HOST_ALLOC, K_ZC_CUS, K_N };
static const char *const kKnobName[K_N] = {"plan", "interleave", "group", "enc_tile_rt", "enc_tile_waves",
                                           "zc_read", "ring", "window_sc", "min_groups", "enc_block_waves", "chunk_waves",
                                           "small_lds", "block_svc", "ws_lds", "dec_waves", "yield_slice_kb",
                                           "yield_depth", "yield_gate_us", "yield_streams", "yield_always",
                                           "yield_window_ms", "svc_reserve_cus", "host_alloc", "zc_cus"};
enum { PLAN_AUTO = 0, PLAN_WAVE = 1, PLAN_LANE = 2, PLAN_REG = 3, PLAN_TILE = 4, PLAN_WREG = 5 };
static std::atomic<int> g_knob[K_N];
static std::once_flag g_knob_once;

static void knobs_default() {
  g_knob[K_PLAN] = PLAN_AUTO;  // plan kernel by batch size and shape
  g_knob[K_INTERLEAVE] = 1;    // bit 0: interleaved block groups; bit 1: XCD-aware group order (grp_index)
  g_knob[K_GROUP] = 0;         // 0: the measured per-shape group sizes
  g_knob[K_ENC_RT] = 0;        // encode tiles by r (0), one wave per group (enc_tile_waves 0)
  g_knob[K_ENC_W] = 0;
  // register-prefetch encode: waves per workgroup, each on its own block group (adjacent groups share a CU;
  // §5.6 probe acol); 1 = one wave per workgroup
  g_knob[K_ENC_BW] = 1;
  g_knob[K_ZC_READ] = 1;       // page-locked host buffers read by the kernels in place
  // LDS-ring data path (bs2 bodies) for 16-repair / 16-unknown tiles: 2 (default) on, 0 off
  g_knob[K_RING] = 2;
  // window encode on the shared-coefficient kernel (k_rlc_encode_sc): 0 never, 1 (default) for
  // overlapping windows, 2 wherever it applies (tests)
  g_knob[K_WINDOW_SC] = 1;
  // batches too small to fill the chip stream fewer blocks per wave: groups of blocks shrink until
  // there are at least this many groups (0: the per-shape group sizes at every batch size)
  g_knob[K_MIN_GROUPS] = 1024;
  // ring tiles of symbols wider than one column chunk: one wave per chunk of a block at once (1) or
  // one wave coding the chunks in turn (0)
  g_knob[K_CHUNK_WAVES] = 1;
  // batches of <= kSmallLdsMaxBlocks blocks: rows staged in LDS by a workgroup per block (1) or the
  // bitsliced one-wave-per-block kernels (0)
  g_knob[K_SMALL_LDS] = 1;
  // fecgpu_block_svc_*: the resident worker serves requests (1) or every call returns
  // FECGPU_ERR_INVALID so the caller takes the launch path (0)
  g_knob[K_BLOCK_SVC] = 1;
  // recover data pass: a group's workspace records copied into LDS in one round trip (1) or read
  // where they lie during the setup (0)
  g_knob[K_WS_LDS] = 1;
  // recover data pass (register-prefetch bodies): 0 = the occupancy its registers allow, n = at most
  // n waves per SIMD
  g_knob[K_DEC_WAVES] = 0;
  // zero-copy bulk calls while the hooks are in use (host_path.hip, Pacer): slices of this many KiB of
  // payload (0: never slice), at most yield_depth in flight, alternating over yield_streams of the
  // context's streams, and a slice held back at most yield_gate_us while a hook request is pending (0:
  // not held).  Beside back-to-back 4096-block zero-copy encodes (profiles/r05_pacer_sweep.log): 2560 KiB,
  // 16, 2 streams -> hooks p99 174 / 184 us (generate / recover; unsliced 1473 / 1486) for bulk calls
  // 9 % longer (1.725 against 1.582 ms); 2048 KiB -> p99 142-152 us, +12 %; 3072 KiB -> 207-218 us, +7 %.
  // 2304 KiB (profiles/r05_pacer_sweep2.log, one box, twice): p99 158 / 170 us against 2560's 175 / 187 for
  // bulk calls 0.9 % longer -- the margin under 200 us the bench's runs needed (one read recover p99 202)
  g_knob[K_YIELD_SLICE_KB] = 2304;
  g_knob[K_YIELD_DEPTH] = 16;
  g_knob[K_YIELD_GATE_US] = 0;
  g_knob[K_YIELD_STREAMS] = 2;
  g_knob[K_YIELD_ALWAYS] = 0;   // A/B: slice even when no hook has run lately
  // the hooks count as in use for this long after a request (tests lengthen it so that slicing does
  // not depend on how quickly the call follows the hook)
  g_knob[K_YIELD_WINDOW_MS] = 100;
  // CUs kept for the block service's worker (0: none): its stream runs on the last n CUs only and the
  // host-path contexts' streams (the zero-copy bulk calls) on the others; read when a service or a
  // context is created
  g_knob[K_SVC_RESERVE_CUS] = 0;
  // fecgpu_host_alloc's page-locked memory: 0 the runtime's default, 1 fine-grained (coherent), 2
  // coarse-grained (non-coherent), mapped either way (A/B of how zero-copy kernels' host lines sit in L2)
  g_knob[K_HOST_ALLOC] = 0;
  // host-path context streams on only n CUs spread over the chip (0: all): caps how many waves a zero-copy
  // bulk call keeps reading host memory at once (A/B of the hooks' wait behind it)
  g_knob[K_ZC_CUS] = 0;
}

static inline int knob(KnobId id) {
  std::call_once(g_knob_once, knobs_default);
  return g_knob[id].load(std::memory_order_relaxed);
}

// host_path.hip reads the zero-copy knob through this (library-internal)
extern "C" __attribute__((visibility("hidden"))) int fecgpu_knob_zc_read(void) { return knob(K_ZC_READ); }
extern "C" __attribute__((visibility("hidden"))) int fecgpu_knob_window_sc(void) { return knob(K_WINDOW_SC); }
extern "C" __attribute__((visibility("hidden"))) int fecgpu_knob_host_alloc(void) { return knob(K_HOST_ALLOC); }
extern "C" __attribute__((visibility("hidden"))) void fecgpu_knob_yield(int *slice_kb, int *depth, int *gate_us,
                                                                        int *streams, int *always, int *window_ms) {
  *slice_kb = knob(K_YIELD_SLICE_KB);
  *window_ms = knob(K_YIELD_WINDOW_MS);
  *depth = knob(K_YIELD_DEPTH);
  *gate_us = knob(K_YIELD_GATE_US);
  *streams = knob(K_YIELD_STREAMS);
  *always = knob(K_YIELD_ALWAYS);
}

// CU masks of the block-service reservation (knob svc_reserve_cus = n): worker = 1 gives the last n CUs,
// worker = 0 every other CU.  Returns the mask's words (0: no reservation; the caller makes a plain stream).
extern "C" __attribute__((visibility("hidden"))) int fecgpu_svc_cu_mask(int device, int worker, uint32_t *mask,
                                                                        int max_words) {
  // n > 0: the last n CU indices; n < 0: every (-n)-th CU index counted from the last (-8: the indices
  // c % 8 == 7, one XCD's CUs where the queue's CU numbering interleaves the eight XCDs)
  const int n = knob(K_SVC_RESERVE_CUS), zc = knob(K_ZC_CUS);
  int cus = 0;
  if ((n == 0 && (zc == 0 || worker)) ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus <= (n > 0 ? n : -n) || (cus + 31) / 32 > max_words)
    return 0;
  const int words = (cus + 31) / 32;
  for (int w = 0; w < words; w++) mask[w] = 0;
  if (!worker && zc > 0 && zc < cus) {  // zc_cus: the host-path streams on zc CUs, every (cus / zc)-th index
    const int step = cus / zc;
    for (int c = 0, m = 0; c < cus && m < zc; c += step, m++) mask[c >> 5] |= 1u << (c & 31);
    return words;
  }
  if (n == 0) return 0;
  for (int c = 0; c < cus; c++) {
    const bool reserved = n > 0 ? c >= cus - n : (c % -n) == (-n - 1);
    if (reserved == (worker != 0)) mask[c >> 5] |= 1u << (c & 31);
  }
  return words;
}

static int set_err(int code, const char *fmt, const char *what) {
  snprintf(g_err, sizeof g_err, fmt, what);
  return code;
}

#define HIPCHK(call)                                                                 \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess) return set_err(FECGPU_ERR_HIP, "HIP: %s", hipGetErrorString(e_)); \
  } while (0)

// =============================================================================================
// Workspace layout of the decode plan (bytes per block).
// =============================================================================================
constexpr size_t kWsLdsMax = 4096;  // bytes of workspace records a recover group stages in LDS

struct WsLayout {
  uint32_t em;      // e_max = min(k, r)
  uint32_t off_unk, off_sel, off_slot, off_nz, off_D, off_dep, stride;
};

__host__ __device__ static inline uint32_t pad16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ static inline WsLayout ws_layout(uint32_t k, uint32_t r) {
  WsLayout w;
  w.em = k < r ? k : r;
  uint32_t o = 16;  // header: status, e
  w.off_unk = o;  o += pad16(w.em);
  w.off_sel = o;  o += pad16(w.em);
  w.off_slot = o; o += pad16(k);
  w.off_nz = o;   o += pad16(w.em);
  w.off_D = o;    o += pad16(w.em * k);
  w.off_dep = o;  o += pad16(w.em * w.em);
  w.stride = o;
  return w;
}

__device__ __forceinline__ uint32_t block_fbn(uint64_t b, uint32_t fbn_base, const uint32_t *fbn) {
  return fbn ? fbn[b] : (uint32_t)((fbn_base + b) & 0xffffffu);
}

// TinyMT32 seed of the repair in slot i of block b.  The reference seeds every equation with the
// repair's own FPID (get_coefs(..., rs->repair_fec_payload_id.source_fpid.raw, ...),
// rlc_fec_scheme_gf256.c:200): callers that hold received FPIDs pass them as seeds[b * r + i]
// (the sliding-window framework's repairs carry block number 0 in a block numbered by its window
// start, window_framework_sender.h:239-243 / window_framework_receiver.h:60-86).  Without seeds
// the FPID is the block framework's (fbn_b << 8) | i.
__device__ __forceinline__ uint32_t repair_seed(const uint32_t *seeds, uint64_t b, int r, uint32_t f, uint32_t i) {
  return seeds ? seeds[b * (uint64_t)r + i] : rlc_seed(f, i);
}

// Phase stamps (diagnostic builds only, -DFEC_STAMP; tools/phase_probe.py): workgroup 0's thread 0
// records s_memrealtime (100 MHz) at the marked points of a kernel, in issue order, so a one-block
// launch can be split into its phases.  The shipped library compiles them out.
#ifdef FEC_STAMP
__device__ uint64_t g_fec_stamps[16];
#define FEC_STAMP_AT(i)                                                          \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_fec_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FEC_STAMP_AT(i) do { } while (0)
#endif

static uint32_t grid_for(uint64_t units);
// The data-pass kernels run one group per workgroup (no grid-stride loop); a batch of more groups
// than one grid holds (grid_for's cap) is launched in slices, q0 = the slice's first group.
// The group a workgroup codes.  The dispatcher deals workgroups round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, workgroup dispatch); with `interleave` bit 1 the order is swizzled so each XCD's
// workgroups take one contiguous run of groups -- with interleaved groups, one contiguous run of blocks
// per XCD at a time -- instead of every eighth (bijective for any grid size:
// cdna_hip_programming.md, XCD swizzle).  Bit 0 (interleaved groups) is read by the kernels themselves.
__device__ __forceinline__ uint64_t grp_index(int ilv) {
  const uint32_t orig = blockIdx.x, nwg = gridDim.x;
  if (!(ilv & 2) || nwg <= 8) return orig;
  const uint32_t q = nwg / 8, r = nwg % 8, x = orig % 8;
  return (uint64_t)((x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8);
}

#define FEC_LAUNCH_GROUPS(KERNEL, GROUPS, BLOCK, LDS, STREAM, ...)                                  \
  for (uint64_t q0_ = 0; q0_ < (GROUPS); q0_ += grid_for(GROUPS)) {                               \
    const uint64_t n_ = (GROUPS) - q0_ < grid_for(GROUPS) ? (GROUPS) - q0_ : grid_for(GROUPS);   \
    hipLaunchKernelGGL(KERNEL, dim3((uint32_t)n_), dim3(BLOCK), LDS, STREAM, __VA_ARGS__, q0_);   \
  }

// =============================================================================================
// RLC decode: plan (coefficients only), recover (data), finalize (zero propagation)
// =============================================================================================
// GF(2^8)/0x11D log/exp tables (exp doubled so exp[log a + log b] needs no reduction).
struct alignas(16) GfLogExp { uint8_t exp[512]; uint8_t log[256]; };

constexpr GfLogExp make_logexp() {
  GfLogExp t{};
  uint32_t x = 1;
  for (int i = 0; i < 255; i++) {
    t.exp[i] = (uint8_t)x;
    t.exp[i + 255] = (uint8_t)x;
    t.log[x] = (uint8_t)i;
    x = ((x << 1) ^ ((x & 0x80u) ? 0x11du : 0u)) & 0xffu;
  }
  t.exp[510] = t.exp[0];
  t.exp[511] = t.exp[1];
  t.log[0] = 0;
  return t;
}

__constant__ GfLogExp kLogExp = make_logexp();

// Wave-per-block plan (systems too large for a lane): one wave replays fec_recover's coefficient
// work for one block with the lanes spread over matrix entries.  Elimination step i updates every
// row below the pivot at once (rows are independent within a step: no re-pivoting), and back
// substitution is column-oriented: once x_i is known it is folded into every row above.  GF
// arithmetic is exact, so the solution equals the reference's row-by-row recurrence.
// LDS: log/exp | A[em][empad] | V[em][kpad] | X[em][kpad] (coefficient rows before the solve)
//      | unk, sel, perm int[128] | terms[128] | flag.
struct PlanLds {
  uint8_t *exp, *log, *A, *V, *X, *terms;
  int *unk, *sel, *perm, *flag;
};

__host__ __device__ static inline size_t plan_lds_bytes(uint32_t k, uint32_t r) {
  const WsLayout L = ws_layout(k, r);
  const size_t kpad = pad16(k), empad = pad16(L.em);
  return 768 + pad16((uint32_t)(L.em * kpad * 2 + L.em * empad)) + 4 * (128 * 3) + 128 + 16;
}

__device__ __forceinline__ PlanLds plan_carve(uint8_t *lds, int em, int kpad, int empad) {
  PlanLds p;
  p.exp = lds;
  p.log = lds + 512;
  p.A = lds + 768;
  p.V = p.A + em * empad;
  p.X = p.V + em * kpad;
  int *ints = reinterpret_cast<int *>(lds + 768 + pad16((uint32_t)(em * kpad * 2 + em * empad)));
  p.unk = ints;
  p.sel = ints + 128;
  p.perm = ints + 256;
  p.terms = reinterpret_cast<uint8_t *>(ints + 384);
  p.flag = reinterpret_cast<int *>(p.terms + 128);
  return p;
}

__device__ __forceinline__ bool bit128(uint64_t m0, uint64_t m1, int j) {
  return j < 64 ? ((m0 >> j) & 1) : ((m1 >> (j - 64)) & 1);
}
__device__ __forceinline__ int rank128(uint64_t m0, uint64_t m1, int j) {  // set bits below j
  return j < 64 ? __popcll(m0 & ((1ull << j) - 1)) : __popcll(m0) + __popcll(m1 & ((1ull << (j - 64)) - 1));
}
__device__ __forceinline__ void clip128(uint64_t &m0, uint64_t &m1, int n) {
  if (n < 64) { m0 &= (1ull << n) - 1; m1 = 0; }
  else if (n < 128) m1 &= (1ull << (n - 64)) - 1;
}

// Barrier of the wave plans: the workgroup's (one-wave plan kernels, k_rlc_decode_small) or, when one
// wave of a larger workgroup plans while the others stage rows (WG = false), the wave's own: its LDS
// operations complete in order, so waiting for them orders every lane's later reads after the writes.
template <bool WG>
__device__ __forceinline__ void plan_sync() {
  if constexpr (WG) __syncthreads();
  else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// One block's plan by one wave (row-parallel elimination).  `lds` holds the log/exp tables at 0
// (plan_load_tables) and room for plan_lds_bytes(k, r).  Every lane of the wave must call it.
// (48 lanes, one 16-B load each: one memory round trip, which a one-block decode waits for)
__device__ __forceinline__ void plan_load_tables(uint8_t *lds) {
  static_assert(sizeof(GfLogExp) == 48 * 16, "log/exp tables: 48 x 16 B");
  if (threadIdx.x < 48)
    reinterpret_cast<uint4 *>(lds)[threadIdx.x] = reinterpret_cast<const uint4 *>(&kLogExp)[threadIdx.x];
}

// Common start of the wave plans: the block's unknowns (unk[u] = u-th missing source), its equations
// (sel[e] = e-th present repair, :194-212) and their TinyMT32 coefficient rows X[e][0..k) in LDS.
// Returns n, the number of unknowns, or 0 after writing the "nothing to do" record (:140-144).
template <bool WG>
__device__ __forceinline__ int plan_wave_setup(uint64_t b, int k, int r, uint32_t fbn_base, const uint32_t *fbn,
                                               const uint32_t *seeds, const uint64_t *sp, const uint64_t *rp,
                                               uint8_t *h, const PlanLds &P, int kpad, uint64_t &m0,
                                               uint64_t &m1) {
  const int lane = threadIdx.x;
  uint64_t s0 = sp[2 * b], s1 = sp[2 * b + 1], q0 = rp[2 * b], q1 = rp[2 * b + 1];
  clip128(s0, s1, k);
  clip128(q0, q1, r);
  const int cur_ss = __popcll(s0) + __popcll(s1);
  const int cur_rs = __popcll(q0) + __popcll(q1);
  if (cur_ss + cur_rs == 255) FEC_STAMP_AT(15);  // (never true: orders stamp 1 after the mask loads)
  FEC_STAMP_AT(1);
  plan_sync<WG>();
  // rlc_fec_scheme_gf256.c:140-144
  if (r == 0 || cur_ss == k || cur_ss + cur_rs < k) {
    if (lane == 0) { h[0] = FECGPU_BLOCK_NOTHING; h[1] = 0; }
    return 0;
  }
  const int n = k - cur_ss;  // unknowns == equations (n_eq = min(n_unk, cur_rs) = n_unk)
  m0 = ~s0;
  m1 = ~s1;
  clip128(m0, m1, k);
  for (int j = lane; j < k; j += 64)
    if (bit128(m0, m1, j)) P.unk[rank128(m0, m1, j)] = j;
  for (int i = lane; i < r; i += 64)
    if (bit128(q0, q1, i)) {
      const int e = rank128(q0, q1, i);
      if (e < n) P.sel[e] = i;
    }
  plan_sync<WG>();
  const uint32_t f = block_fbn(b, fbn_base, fbn);
  for (int e = lane; e < n; e += 64) {  // TinyMT32 row of repair sel[e] (get_coefs :117-125)
    Tmt t;
    tmt_init(t, repair_seed(seeds, b, r, f, (uint32_t)P.sel[e]));
    for (int j = 0; j < k; j++) P.X[e * kpad + j] = tmt_coef(t);
  }
  plan_sync<WG>();
  FEC_STAMP_AT(2);
  return n;
}

// Record fields every wave plan writes the same way: unknowns, equations, slot map, status.
__device__ __forceinline__ void plan_wave_finish(uint8_t *h, const WsLayout &L, const PlanLds &P, int k, int n,
                                                 uint64_t m0, uint64_t m1) {
  const int lane = threadIdx.x;
  for (int u = lane; u < n; u += 64) {
    h[L.off_nz + u] = 0;
    h[L.off_unk + u] = (uint8_t)P.unk[u];
    h[L.off_sel + u] = (uint8_t)P.sel[u];
  }
  // slot map: input j = source j if present, else the repair selected for its unknown
  for (int j = lane; j < k; j += 64)
    h[L.off_slot + j] = bit128(m0, m1, j) ? (uint8_t)(0x80 | P.sel[rank128(m0, m1, j)]) : (uint8_t)j;
  if (lane == 0) { h[0] = FECGPU_BLOCK_RECOVERED; h[1] = (uint8_t)n; }
}

template <bool WG = true>
__device__ void plan_wave_block(uint64_t b, int k, int r, uint32_t fbn_base, const uint32_t *fbn,
                                const uint32_t *seeds, const uint64_t *sp, const uint64_t *rp, uint8_t *ws,
                                uint8_t *lds) {
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x;
  const int em = (int)L.em;
  const int kpad = (int)pad16((uint32_t)k);
  const int empad = (int)pad16((uint32_t)em);
  const PlanLds P = plan_carve(lds, em, kpad, empad);
  uint8_t *A = P.A, *V = P.V, *X = P.X, *EXP = P.exp, *LOG = P.log, *terms = P.terms;
  int *unk = P.unk, *perm = P.perm;
  // x * y with y != 0 given as log y
  auto mul_l = [&](uint32_t x, uint32_t ly) -> uint32_t { return x ? EXP[LOG[x] + ly] : 0u; };
  {
    uint8_t *h = ws + b * (uint64_t)L.stride;
    uint64_t m0 = 0, m1 = 0;
    const int n = plan_wave_setup<WG>(b, k, r, fbn_base, fbn, seeds, sp, rp, h, P, kpad, m0, m1);
    if (!n) return;
    // A[e][u] = row_e[unk[u]];  V[e][j] = present j ? row_e[j] : (j == unk[e])
    for (int x = lane; x < n * n; x += 64) {
      const int e = x / n, u = x - e * n;
      A[e * empad + u] = X[e * kpad + unk[u]];
    }
    for (int x = lane; x < n * k; x += 64) {
      const int e = x / k, j = x - e * k;
      V[e * kpad + j] = bit128(m0, m1, j) ? (uint8_t)(unk[e] == j) : X[e * kpad + j];
    }
    plan_sync<WG>();
    // sort_system (:28-40): position i takes the first row with the largest A[.][i].  The scan
    // over rows j >= i is a wave max-reduction of (value << 16 | 0xffff - j), so the largest value
    // wins and, among equal values, the smallest j -- the reference's strict '<' scan.
    for (int i = lane; i < n; i += 64) perm[i] = i;
    plan_sync<WG>();
    for (int i = 0; i < n; i++) {
      uint32_t key = 0;
      for (int j = i + lane; j < n; j += 64) {
        const uint32_t kj = ((uint32_t)A[perm[j] * empad + i] << 16) | (0xffffu - (uint32_t)j);
        key = kj > key ? kj : key;
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)key, off, 64);
        key = o > key ? o : key;
      }
      const int mx = (int)(0xffffu - (key & 0xffffu));
      plan_sync<WG>();  // every lane has read perm[] before it changes
      if (lane == 0) { const int t = perm[i]; perm[i] = perm[mx]; perm[mx] = t; }
      plan_sync<WG>();
    }
    FEC_STAMP_AT(8);
    // forward elimination without re-pivoting (:54-70): row_pk -= (A[pk][i] / A[pi][i]) row_pi for all
    // kk > i at once; inv(0) = 0 makes every term 0 (the block is then flagged below).  A lane owns a
    // column (of A from i on, then of V) and walks the rows below: the pivot row's entry and its log
    // stay in registers, each row's term log is a broadcast LDS read, and the row updates are
    // independent (no division, no dependent chain across rows).
    for (int i = 0; i < n - 1; i++) {
      const int pi = perm[i];
      const uint32_t piv = A[pi * empad + i];
      const int below = n - 1 - i;
      const uint32_t lpiv = LOG[piv];
      for (int x = lane; x < below; x += 64) {  // log of the term, 255 = zero term
        const uint32_t a = A[perm[i + 1 + x] * empad + i];
        const int d = (int)LOG[a] - (int)lpiv;
        terms[x] = (piv && a) ? (uint8_t)(d < 0 ? d + 255 : d) : (uint8_t)255;
      }
      plan_sync<WG>();
      const int wa = n - i, w = wa + k;  // columns i..n-1 of A, then all of V
      for (int c = lane; c < w; c += 64) {
        const bool ina = c < wa;
        const uint32_t pv = ina ? A[pi * empad + i + c] : V[pi * kpad + c - wa];
        if (!pv) continue;
        const uint32_t lp = LOG[pv];
        uint8_t *col = ina ? A + i + c : V + (c - wa);
        const int rs = ina ? empad : kpad;
        for (int rr = 0; rr < below; rr++) {
          const uint32_t t = terms[rr];
          if (t == 255u) continue;
          col[perm[i + 1 + rr] * rs] ^= EXP[lp + t];
        }
      }
      plan_sync<WG>();
    }
    FEC_STAMP_AT(9);
    // the reference crashes iff some diagonal entry is zero (candidate walks to -1, :74-77)
    const bool zd = lane < n && A[perm[lane] * empad + lane] == 0;
    bool ub = __any(zd);
    for (int i = 64 + lane; i < n; i += 64) ub |= A[perm[i] * empad + i] == 0;
    if (__any(ub)) {
      if (lane == 0) { h[0] = FECGPU_BLOCK_REF_UB; h[1] = 0; }
      return;
    }
    // back substitution (:71-114), column-oriented: x_i = V[pi] / A[pi][i], then V[pm] -= A[pm][i] x_i.
    // A lane owns column j of V and X throughout, so the steps need no barrier.
    for (int i = n - 1; i >= 0; i--) {
      const int pi = perm[i];
      const uint32_t li = 255u - LOG[A[pi * empad + i]];
      for (int j = lane; j < k; j += 64) {
        const uint32_t xv = mul_l(V[pi * kpad + j], li);
        X[i * kpad + j] = (uint8_t)xv;
        if (!xv) continue;
        const uint32_t lx = LOG[xv];
        for (int m = 0; m < i; m++) {
          const int pm = perm[m];
          const uint32_t a = A[pm * empad + i];
          if (a) V[pm * kpad + j] ^= EXP[LOG[a] + lx];
        }
      }
    }
    FEC_STAMP_AT(10);
    plan_sync<WG>();
    for (int x = lane; x < n * n; x += 64) {
      const int i = x / n, u = x - i * n;
      h[L.off_dep + i * em + u] = (u > i) && A[perm[i] * empad + u] != 0;
    }
    for (int x = lane; x < n * k; x += 64) {
      const int i = x / k, j = x - i * k;
      h[L.off_D + i * k + j] = X[i * kpad + j];
    }
    plan_wave_finish(h, L, P, k, n, m0, m1);
  }
}

// Register wave plan (n <= EM unknowns, n + k <= 64 C columns; used with EM <= 8, C = 1): the same elimination as
// plan_wave_block with the system in VGPRs.  Lane c owns column c (A column c for c < n, V column
// c - n after it; a second column at c + 64 when C = 2) as EM row registers; rows are swapped in
// place by the sort, so row i is perm[i] of the LDS plan.  Every row index is a compile-time
// constant of the unrolled loops and the per-row scalars (pivot terms, A[m][i]) come from the
// owning lane through readlane, so the only LDS traffic is the log/exp lookups, which are
// independent across rows.  Same record bytes (test_plan_kernels_agree).
template <int EM, int C, bool WG = true>
__device__ void plan_wreg_block(uint64_t b, int k, int r, uint32_t fbn_base, const uint32_t *fbn,
                                const uint32_t *seeds, const uint64_t *sp, const uint64_t *rp, uint8_t *ws,
                                uint8_t *lds) {
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x;
  const int kpad = (int)pad16((uint32_t)k);
  const PlanLds P = plan_carve(lds, (int)L.em, kpad, (int)pad16(L.em));
  const uint8_t *EXP = P.exp, *LOG = P.log, *X = P.X;
  uint8_t *h = ws + b * (uint64_t)L.stride;
  uint64_t m0 = 0, m1 = 0;
  const int n = plan_wave_setup<WG>(b, k, r, fbn_base, fbn, seeds, sp, rp, h, P, kpad, m0, m1);
  if (!n) return;
  uint32_t col[C][EM];
  bool isv[C], live[C];
  int jv[C];
#pragma unroll
  for (int q = 0; q < C; q++) {
    const int c = lane + 64 * q;
    isv[q] = c >= n;
    live[q] = c < n + k;
    const int j = isv[q] ? c - n : P.unk[c < n ? c : 0];
    jv[q] = j;
    const bool present = live[q] && isv[q] && bit128(~m0, ~m1, j);
#pragma unroll
    for (int e = 0; e < EM; e++) {
      uint32_t v = 0;
      if (e < n && live[q]) v = (isv[q] && !present) ? (uint32_t)(P.unk[e] == j) : X[e * kpad + j];
      col[q][e] = v;
    }
  }
  // sort_system (:28-40): position i takes the first row j >= i with the largest A[j][i]; lane i
  // holds column i, so it finds the row and every lane swaps rows i and mx in its registers
#pragma unroll
  for (int i = 0; i < EM; i++) {
    if (i >= n) break;
    uint32_t key = 0;
#pragma unroll
    for (int j = 0; j < EM; j++)
      if (j >= i && j < n) {
        const uint32_t kj = (col[0][j] << 8) | (uint32_t)(255 - j);
        key = kj > key ? kj : key;
      }
    const int mx = 255 - (int)(__builtin_amdgcn_readlane(key, i) & 0xffu);
    if (mx != i) {
#pragma unroll
      for (int q = 0; q < C; q++) {
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < EM; j++)
          if (j > i) vm = j == mx ? col[q][j] : vm;
#pragma unroll
        for (int j = 0; j < EM; j++)
          if (j > i) col[q][j] = j == mx ? col[q][i] : col[q][j];
        col[q][i] = vm;
      }
    }
  }
  // forward elimination without re-pivoting (:54-70): rows below i -= (A[rr][i] / A[i][i]) row i,
  // on A columns >= i and all of V; a zero pivot makes every term zero
#pragma unroll
  for (int i = 0; i < EM - 1; i++) {
    if (i >= n - 1) break;
    const uint32_t lpiv = LOG[col[0][i]];
    const bool pz = col[0][i] == 0;
    uint32_t tl[EM];
#pragma unroll
    for (int rr = 0; rr < EM; rr++) {
      if (rr <= i) continue;
      const uint32_t a = col[0][rr];
      const int d = (int)LOG[a] - (int)lpiv;
      const uint32_t t = (pz || !a) ? 255u : (uint32_t)(d < 0 ? d + 255 : d);
      tl[rr] = __builtin_amdgcn_readlane(t, i);
    }
#pragma unroll
    for (int q = 0; q < C; q++) {
      const uint32_t pv = col[q][i];
      const bool act = live[q] && (isv[q] || lane >= i) && pv != 0;
      const uint32_t lp = LOG[pv];
#pragma unroll
      for (int rr = 0; rr < EM; rr++)
        if (rr > i && rr < n && tl[rr] != 255u && act) col[q][rr] ^= EXP[lp + tl[rr]];
    }
  }
  // the reference crashes iff some diagonal entry is zero (candidate walks to -1, :74-77)
  bool ub = false;
#pragma unroll
  for (int i = 0; i < EM; i++)
    if (i < n) ub |= __builtin_amdgcn_readlane(col[0][i], i) == 0;
  if (ub) {
    if (lane == 0) { h[0] = FECGPU_BLOCK_REF_UB; h[1] = 0; }
    return;
  }
  // dependency flags of the upper-triangular system: A lane u writes column u
  if (lane < n) {
#pragma unroll
    for (int i = 0; i < EM; i++)
      if (i < n) h[L.off_dep + i * L.em + lane] = (lane > i) && col[0][i] != 0;
  }
  // back substitution (:71-114): x_i = V[i] / A[i][i], then V[m] -= A[m][i] x_i for m < i
#pragma unroll
  for (int i = EM - 1; i >= 0; i--) {
    if (i >= n) continue;
    const uint32_t li = 255u - LOG[__builtin_amdgcn_readlane(col[0][i], i)];
    uint32_t la[EM];
#pragma unroll
    for (int m = 0; m < EM; m++) {
      if (m >= i) continue;
      const uint32_t a = __builtin_amdgcn_readlane(col[0][m], i);
      la[m] = a ? (uint32_t)LOG[a] : 255u;
    }
#pragma unroll
    for (int q = 0; q < C; q++) {
      if (!(isv[q] && live[q])) continue;
      const uint32_t xv = col[q][i] ? (uint32_t)EXP[LOG[col[q][i]] + li] : 0u;
      col[q][i] = xv;
      const uint32_t lx = LOG[xv];
#pragma unroll
      for (int m = 0; m < EM; m++)
        if (m < i && la[m] != 255u && xv) col[q][m] ^= EXP[la[m] + lx];
    }
  }
#pragma unroll
  for (int q = 0; q < C; q++)
    if (isv[q] && live[q]) {
#pragma unroll
      for (int i = 0; i < EM; i++)
        if (i < n) h[L.off_D + i * k + jv[q]] = (uint8_t)col[q][i];
    }
  plan_wave_finish(h, L, P, k, n, m0, m1);
}

// Wave plan for one block: the register plan when the system fits (em <= 8, k + em <= 64) and wreg
// is set, else the LDS plan.  Two columns per lane (k + em <= 128) measured slower than the LDS plan
// (k64 e16 180 vs 83 us); 16 rows leave part of the system in scratch (the unrolled elimination
// exceeds the compiler's full-unroll budget), so em <= 8.
__device__ __forceinline__ bool plan_wreg_fits(int k, int r) {
  const int em = k < r ? k : r;
  return em <= 8 && k + em <= 64;
}
template <bool WG = true>
__device__ __forceinline__ void plan_wave_any(int wreg, uint64_t b, int k, int r, uint32_t fbn_base,
                                              const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                              const uint64_t *rp, uint8_t *ws, uint8_t *lds) {
  const int em = k < r ? k : r;
  if (wreg && plan_wreg_fits(k, r)) {
    if (em <= 4) plan_wreg_block<4, 1, WG>(b, k, r, fbn_base, fbn, seeds, sp, rp, ws, lds);
    else plan_wreg_block<8, 1, WG>(b, k, r, fbn_base, fbn, seeds, sp, rp, ws, lds);
    return;
  }
  plan_wave_block<WG>(b, k, r, fbn_base, fbn, seeds, sp, rp, ws, lds);
}

// The register wave plan as its own kernel (k_rlc_plan keeps the LDS plan's smaller register
// footprint for the batches where occupancy counts).
template <int EM>
__global__ __launch_bounds__(64) void k_rlc_plan_wreg(uint64_t nblocks, int k, int r, uint32_t fbn_base,
                                                      const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                                      const uint64_t *rp, uint8_t *ws) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  plan_load_tables(lds);
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    plan_wreg_block<EM, 1>(b, k, r, fbn_base, fbn, seeds, sp, rp, ws, lds);
}

__global__ __launch_bounds__(64) void k_rlc_plan(uint64_t nblocks, int k, int r, uint32_t fbn_base,
                                                 const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                                 const uint64_t *rp, uint8_t *ws) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  plan_load_tables(lds);
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) plan_wave_block(b, k, r, fbn_base, fbn, seeds, sp, rp, ws, lds);
}

// ---------------------------------------------------------------------------------------------
// Lane-per-block plan (small systems): one lane replays fec_recover's coefficient work for one
// block.  GF(2^8) products through log/exp tables in LDS; each lane's working set (A: em x em,
// V: em x k, lists) lives in LDS byte-interleaved across the wave (element e of lane l at
// e * 64 + l), so a wave-uniform step touches 64 consecutive bytes.
// ---------------------------------------------------------------------------------------------

__host__ __device__ static inline uint32_t lane_arena_bytes(uint32_t k, uint32_t r) {
  const uint32_t em = k < r ? k : r;
  return em * em + em * k + 3 * em;
}

// Output records are assembled in LDS (row per lane, padded to an odd dword count so byte
// writes from the 64 lanes spread over the banks) and leave as coalesced dword stores: the wave's
// 64 workspace records are contiguous in HBM.
__host__ __device__ static inline uint32_t plan_out_row(uint32_t stride) { return stride + 4; }

// Records staged in LDS (rows of odw dwords, padded against bank conflicts) leave as coalesced
// dwords of rows of rdw.  Lane positions advance by 64 dwords per step without a division.
__device__ __forceinline__ void copy_records(uint32_t *dst, const uint32_t *src, uint32_t nrows, uint32_t rdw,
                                             uint32_t odw, int lane) {
  const uint32_t drow = 64u / rdw, dcol = 64u - drow * rdw;  // dcol < rdw
  uint32_t row = (uint32_t)lane / rdw, col = (uint32_t)lane - row * rdw;
  for (uint32_t x = lane; x < nrows * rdw; x += 64) {
    dst[x] = src[row * odw + col];
    row += drow;
    col += dcol;
    if (col >= rdw) { col -= rdw; row++; }
  }
}

__host__ __device__ static inline size_t plan_lane_lds(uint32_t k, uint32_t r) {
  return 768 + 64 * (size_t)lane_arena_bytes(k, r) + 64 * (size_t)plan_out_row(ws_layout(k, r).stride);
}

__global__ __launch_bounds__(64) void k_rlc_plan_lane(uint64_t nblocks, int k, int r, uint32_t fbn_base,
                                                      const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                                      const uint64_t *rp, uint8_t *ws) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x;
  const int em = (int)L.em;
  uint8_t *EXP = lds, *LOG = lds + 512;
  plan_load_tables(lds);
  __syncthreads();
  uint8_t *my = lds + 768 + lane;
  const uint32_t orow = plan_out_row(L.stride);
  uint8_t *obase = lds + 768 + 64 * (size_t)lane_arena_bytes((uint32_t)k, (uint32_t)r);
  uint8_t *h = obase + (size_t)lane * orow;  // this lane's workspace record (LDS copy)
  const int oA = 0, oV = em * em, oP = oV + em * k, oU = oP + em, oS = oU + em;
#define AR(e) my[(e) * 64]
  for (uint64_t base = (uint64_t)blockIdx.x * 64; base < nblocks; base += (uint64_t)gridDim.x * 64) {
    const uint64_t b = base + lane;
    if (b < nblocks) do {
      uint64_t s0 = sp[2 * b], s1 = sp[2 * b + 1], q0 = rp[2 * b], q1 = rp[2 * b + 1];
      clip128(s0, s1, k);
      clip128(q0, q1, r);
      const int cur_ss = __popcll(s0) + __popcll(s1);
      const int cur_rs = __popcll(q0) + __popcll(q1);
      if (r == 0 || cur_ss == k || cur_ss + cur_rs < k) {  // rlc_fec_scheme_gf256.c:140-144
        h[0] = FECGPU_BLOCK_NOTHING;
        h[1] = 0;
        break;
      }
      const int n = k - cur_ss;
      uint64_t m0 = ~s0, m1 = ~s1;
      clip128(m0, m1, k);
      {
        int u = 0;
        for (int j = 0; j < k; j++)
          if (bit128(m0, m1, j)) AR(oU + u++) = (uint8_t)j;
        int e = 0;
        for (int i = 0; i < r && e < n; i++)
          if (bit128(q0, q1, i)) AR(oS + e++) = (uint8_t)i;
      }
      const uint32_t f = block_fbn(b, fbn_base, fbn);
      for (int e = 0; e < n; e++) {  // system rows, :194-212
        Tmt t;
        tmt_init(t, repair_seed(seeds, b, r, f, AR(oS + e)));
        int u = 0;
        for (int j = 0; j < k; j++) {
          uint8_t c = tmt_coef(t);
          if (bit128(m0, m1, j)) {
            AR(oA + e * em + u) = c;
            AR(oV + e * k + j) = (uint8_t)(u == e);
            u++;
          } else {
            AR(oV + e * k + j) = c;
          }
        }
        AR(oP + e) = (uint8_t)e;
      }
      for (int i = 0; i < n; i++) {  // sort_system :28-40
        int mx = i;
        for (int j = i + 1; j < n; j++)
          if (AR(oA + AR(oP + mx) * em + i) < AR(oA + AR(oP + j) * em + i)) mx = j;
        uint8_t t = AR(oP + i); AR(oP + i) = AR(oP + mx); AR(oP + mx) = t;
      }
      for (int i = 0; i < n - 1; i++) {  // elimination :54-70
        const int pi = AR(oP + i);
        const uint32_t piv = AR(oA + pi * em + i);
        if (!piv) continue;  // inv(0) = 0: every term is 0, nothing changes
        const uint32_t lip = 255u - LOG[piv];
        for (int kk = i + 1; kk < n; kk++) {
          const int pk = AR(oP + kk);
          const uint32_t a = AR(oA + pk * em + i);
          if (!a) continue;
          const uint32_t lt = LOG[EXP[LOG[a] + lip]];
          for (int u = 0; u < n; u++) {
            uint32_t x = AR(oA + pi * em + u);
            if (x) AR(oA + pk * em + u) ^= EXP[lt + LOG[x]];
          }
          for (int j = 0; j < k; j++) {
            uint32_t x = AR(oV + pi * k + j);
            if (x) AR(oV + pk * k + j) ^= EXP[lt + LOG[x]];
          }
        }
      }
      bool ub = false;  // candidate walks to -1 iff a diagonal entry is zero (:74-77)
      for (int i = 0; i < n; i++) ub |= AR(oA + AR(oP + i) * em + i) == 0;
      if (ub) {
        h[0] = FECGPU_BLOCK_REF_UB;
        h[1] = 0;
        break;
      }
      for (int i = n - 1; i >= 0; i--) {  // back substitution :71-114; X_i stored over V[P[i]]
        const int pi = AR(oP + i);
        const uint32_t li = 255u - LOG[AR(oA + pi * em + i)];
        for (int j = 0; j < k; j++) {
          uint32_t v = AR(oV + pi * k + j);
          for (int u = i + 1; u < n; u++) {
            uint32_t a = AR(oA + pi * em + u);
            uint32_t x = AR(oV + AR(oP + u) * k + j);
            if (a && x) v ^= EXP[LOG[a] + LOG[x]];
          }
          AR(oV + pi * k + j) = v ? EXP[LOG[v] + li] : 0;
        }
        for (int u = 0; u < n; u++) h[L.off_dep + i * em + u] = (u > i) && AR(oA + pi * em + u) != 0;
      }
      for (int i = 0; i < n; i++) {
        const int pi = AR(oP + i);
        for (int j = 0; j < k; j++) h[L.off_D + i * k + j] = AR(oV + pi * k + j);
        h[L.off_nz + i] = 0;
        h[L.off_unk + i] = AR(oU + i);
        h[L.off_sel + i] = AR(oS + i);
      }
      {
        int u = 0;
        for (int j = 0; j < k; j++)
          h[L.off_slot + j] = bit128(m0, m1, j) ? (uint8_t)(0x80 | AR(oS + u++)) : (uint8_t)j;
      }
      h[0] = FECGPU_BLOCK_RECOVERED;
      h[1] = (uint8_t)n;
      } while (0);
    __syncthreads();
    const uint32_t nrows = nblocks - base < 64 ? (uint32_t)(nblocks - base) : 64u;
    copy_records(reinterpret_cast<uint32_t *>(ws + base * (uint64_t)L.stride),
                 reinterpret_cast<const uint32_t *>(obase), nrows, L.stride / 4, orow / 4, lane);
    __syncthreads();
  }
#undef AR
}

// ---------------------------------------------------------------------------------------------
// Register-resident lane-per-block plan for small systems (k <= 4 * KD, e_max <= EM; configs 2-4).
// The same replay as k_rlc_plan_lane, with the lane's system held in VGPRs instead of an LDS
// arena: A rows as packed bytes (u64), V rows as KD dwords.  sort_system's row permutation is
// applied physically (predicated swaps), so the rows leave in P order and need no indirection.
// Row operations multiply a packed row by the lane's scalar with the v_perm product tables of
// fec_device.h (4 bytes per v_perm triple); scalar inverses and products use the log/exp tables
// in LDS.  GF arithmetic is exact, so every byte equals the reference's (rlc_fec_scheme_gf256.c
// :28-115, 178-236), and a zero diagonal after elimination is the reference's crash (:74-77).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t gf_mulc(uint32_t x, const PermTab &t) {
  return gf_mac(0u, perm_selectors(x), t.t01, t.t2);
}

template <int EM>
__device__ __forceinline__ uint64_t gf_mulc_row(uint64_t x, const PermTab &t) {
  if constexpr (EM <= 4) return (uint64_t)gf_mulc((uint32_t)x, t);
  else return (uint64_t)gf_mulc((uint32_t)x, t) | ((uint64_t)gf_mulc((uint32_t)(x >> 32), t) << 32);
}

__device__ __forceinline__ uint32_t col8(uint64_t row, int i) { return (uint32_t)(row >> (8 * i)) & 0xffu; }

// One block's register plan (the lane that calls it holds the whole system); the record goes to h
// in the workspace layout.  EXP / LOG: the log/exp tables (LDS).
template <int KD, int EM>
__device__ __forceinline__ void plan_reg_block(uint64_t b, int k, int r, uint32_t fbn_base, const uint32_t *fbn,
                                               const uint32_t *seeds, const uint64_t *sp, const uint64_t *rp,
                                               uint8_t *h, const uint8_t *EXP, const uint8_t *LOG) {
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  const int em = (int)L.em;
  const uint64_t kmask = k < 64 ? (1ull << k) - 1 : ~0ull;
  const uint64_t s0 = sp[2 * b] & kmask;  // k <= 32: the high word never matters
  uint64_t q0 = rp[2 * b], q1 = rp[2 * b + 1];
  clip128(q0, q1, r);
  const int cur_ss = __popcll(s0);
  const int cur_rs = __popcll(q0) + __popcll(q1);
  if (r == 0 || cur_ss == k || cur_ss + cur_rs < k) {  // rlc_fec_scheme_gf256.c:140-144
    h[0] = FECGPU_BLOCK_NOTHING;
    h[1] = 0;
    return;
  }
  const int n = k - cur_ss;  // <= em <= EM
  const uint64_t miss = ~s0 & kmask;
  uint64_t U = 0, S = 0;  // unknown source ids / selected repair ids, one byte each
  {
    int u = 0;
    for (int j = 0; j < k; j++)
      if ((miss >> j) & 1) U |= (uint64_t)j << (8 * u++);
    int e = 0;
    for (int i = 0; i < r && e < n; i++)
      if (bit128(q0, q1, i)) S |= (uint64_t)i << (8 * e++);
  }
  uint64_t A[EM];
  uint32_t V[EM][KD];
#pragma unroll
  for (int e = 0; e < EM; e++) {
    A[e] = 0;
#pragma unroll
    for (int d = 0; d < KD; d++) V[e][d] = 0;
  }
  const uint32_t f = block_fbn(b, fbn_base, fbn);
#pragma unroll
  for (int e = 0; e < EM; e++) {  // system rows, :194-212
    if (e < n) {
      Tmt t;
      tmt_init(t, repair_seed(seeds, b, r, f, col8(S, e)));
      int u = 0;
#pragma unroll
      for (int j = 0; j < 4 * KD; j++) {
        if (j < k) {
          const uint32_t c = tmt_coef(t);
          const bool ms = (miss >> j) & 1;
          V[e][j >> 2] |= (ms ? (uint32_t)(u == e) : c) << (8 * (j & 3));
          if (ms) A[e] |= (uint64_t)c << (8 * u++);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < EM; i++) {  // sort_system :28-40 (first maximum wins; rows swapped in place)
    if (i < n) {
      int mx = i;
      uint32_t best = col8(A[i], i);
#pragma unroll
      for (int j = i + 1; j < EM; j++)
        if (j < n && best < col8(A[j], i)) { best = col8(A[j], i); mx = j; }
#pragma unroll
      for (int j = i + 1; j < EM; j++) {
        if (j == mx) {
          const uint64_t ta = A[i]; A[i] = A[j]; A[j] = ta;
#pragma unroll
          for (int d = 0; d < KD; d++) { const uint32_t tv = V[i][d]; V[i][d] = V[j][d]; V[j][d] = tv; }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < EM - 1; i++) {  // elimination without re-pivoting :54-70
    const uint32_t piv = col8(A[i], i);
    if (i < n - 1 && piv) {
      const uint32_t lip = 255u - LOG[piv];
#pragma unroll
      for (int kk = i + 1; kk < EM; kk++) {
        const uint32_t a = col8(A[kk], i);
        if (kk < n && a) {
          const PermTab T = perm_table(EXP[LOG[a] + lip]);  // a / piv
          A[kk] ^= gf_mulc_row<EM>(A[i], T);
#pragma unroll
          for (int d = 0; d < KD; d++)
            if (4 * d < k) V[kk][d] ^= gf_mulc(V[i][d], T);
        }
      }
    }
  }
  bool ub = false;  // candidate walks to -1 iff a diagonal entry is zero (:74-77)
#pragma unroll
  for (int i = 0; i < EM; i++) ub |= i < n && col8(A[i], i) == 0;
  if (ub) {
    h[0] = FECGPU_BLOCK_REF_UB;
    h[1] = 0;
    return;
  }
#pragma unroll
  for (int i = EM - 1; i >= 0; i--) {  // back substitution :71-114; X_i replaces row i
    if (i < n) {
#pragma unroll
      for (int u = i + 1; u < EM; u++) {
        const uint32_t a = col8(A[i], u);
        if (u < n && a) {
          const PermTab T = perm_table(a);
#pragma unroll
          for (int d = 0; d < KD; d++)
            if (4 * d < k) V[i][d] ^= gf_mulc(V[u][d], T);
        }
      }
      const PermTab T = perm_table(EXP[255u - LOG[col8(A[i], i)]]);  // 1 / diagonal
#pragma unroll
      for (int d = 0; d < KD; d++)
        if (4 * d < k) V[i][d] = gf_mulc(V[i][d], T);
    }
  }
#pragma unroll
  for (int i = 0; i < EM; i++) {
    if (i < n) {
      uint8_t *D = h + L.off_D + i * k;
      if ((k & 3) == 0) {  // D + 4d is 4-byte aligned: the packed V row as dwords
#pragma unroll
        for (int d = 0; d < KD; d++)
          if (4 * d < k) reinterpret_cast<uint32_t *>(D)[d] = V[i][d];
      } else {
#pragma unroll
        for (int j = 0; j < 4 * KD; j++)
          if (j < k) D[j] = (uint8_t)(V[i][j >> 2] >> (8 * (j & 3)));
      }
      for (int u = 0; u < n; u++) h[L.off_dep + i * em + u] = (u > i) && col8(A[i], u) != 0;
      h[L.off_nz + i] = 0;
      h[L.off_unk + i] = (uint8_t)col8(U, i);
      h[L.off_sel + i] = (uint8_t)col8(S, i);
    }
  }
  {
    int u = 0;
    for (int j = 0; j < k; j++)
      h[L.off_slot + j] = ((miss >> j) & 1) ? (uint8_t)(0x80 | col8(S, u++)) : (uint8_t)j;
  }
  h[0] = FECGPU_BLOCK_RECOVERED;
  h[1] = (uint8_t)n;
}

template <int KD, int EM>
__global__ __launch_bounds__(64) void k_rlc_plan_reg(uint64_t nblocks, int k, int r, uint32_t fbn_base,
                                                     const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                                     const uint64_t *rp, uint8_t *ws) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x;
  const uint8_t *EXP = lds, *LOG = lds + 512;
  plan_load_tables(lds);
  __syncthreads();
  const uint32_t orow = plan_out_row(L.stride);
  uint8_t *h = lds + 768 + (size_t)lane * orow;  // this lane's workspace record (LDS copy)
  for (uint64_t base = (uint64_t)blockIdx.x * 64; base < nblocks; base += (uint64_t)gridDim.x * 64) {
    const uint64_t b = base + lane;
    if (b < nblocks) plan_reg_block<KD, EM>(b, k, r, fbn_base, fbn, seeds, sp, rp, h, EXP, LOG);
    __syncthreads();
    const uint32_t nrows = nblocks - base < 64 ? (uint32_t)(nblocks - base) : 64u;
    copy_records(reinterpret_cast<uint32_t *>(ws + base * (uint64_t)L.stride),
                 reinterpret_cast<const uint32_t *>(lds + 768), nrows, L.stride / 4, orow / 4, lane);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Tiled register plan for systems too large for one lane (configs[4]: k = 64, e = 16): LPB = EM/4
// lanes per block.  Lane q of a block holds columns 4q..4q+3 of A (one dword per row) and V's
// columns [q * 4 KDL, (q + 1) * 4 KDL); an A entry another lane needs (pivots, factors, sort keys)
// comes by ds_bpermute from the lane that owns its column.  The TinyMT32 rows are generated
// cooperatively (lane q: rows q, q + LPB, ...) into LDS.  Row operations and record layout as
// k_rlc_plan_reg; records leave as coalesced dwords.  (rlc_fec_scheme_gf256.c:28-115, 134-236)
// ---------------------------------------------------------------------------------------------
template <int KDL, int EM>
__global__ __launch_bounds__(64) void k_rlc_plan_tile(uint64_t nblocks, int k, int r, uint32_t fbn_base,
                                                      const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                                      const uint64_t *rp, uint8_t *ws) {
  constexpr int LPB = EM / 4;    // lanes per block: one A dword (4 columns) each
  constexpr int BPW = 64 / LPB;  // blocks per wave
  constexpr int CW = 4 * KDL;    // V columns per lane
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x, g = lane / LPB, q = lane % LPB, lane0 = g * LPB;
  const int em = (int)L.em;
  const int kpad = (int)pad16((uint32_t)k);
  const uint8_t *EXP = lds, *LOG = lds + 512;
  uint8_t *CO = lds + 768;                                   // [BPW][EM][kpad] coefficient rows
  const uint32_t orow = plan_out_row(L.stride);
  uint8_t *OUTR = CO + (size_t)BPW * EM * kpad;             // [BPW][orow] records
  plan_load_tables(lds);
  uint8_t *h = OUTR + (size_t)g * orow;
  const uint8_t *crow = CO + (size_t)g * EM * kpad;
  const int c0 = q * CW;
  const uint64_t kmask = k < 64 ? (1ull << k) - 1 : ~0ull;
  auto byte_at = [](uint64_t lo, uint64_t hi, int i) -> uint32_t {
    return (uint32_t)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 0xffu);
  };
  for (uint64_t base = (uint64_t)blockIdx.x * BPW; base < nblocks; base += (uint64_t)gridDim.x * BPW) {
    const uint64_t b = base + g;
    int state = 0, n = 0;  // 0: nothing to do, 1: solve
    uint64_t miss = 0, U0 = 0, U1 = 0, S0 = 0, S1 = 0;
    uint32_t f = 0;
    if (b < nblocks) {
      const uint64_t s0 = sp[2 * b] & kmask;  // k <= 64
      uint64_t q0 = rp[2 * b], q1 = rp[2 * b + 1];
      clip128(q0, q1, r);
      const int cur_ss = __popcll(s0), cur_rs = __popcll(q0) + __popcll(q1);
      if (r == 0 || cur_ss == k || cur_ss + cur_rs < k) {  // rlc_fec_scheme_gf256.c:140-144
        if (q == 0) { h[0] = FECGPU_BLOCK_NOTHING; h[1] = 0; }
      } else {
        state = 1;
        n = k - cur_ss;
        miss = ~s0 & kmask;
        int u = 0;
        for (int j = 0; j < k; j++)
          if ((miss >> j) & 1) {
            if (u < 8) U0 |= (uint64_t)j << (8 * u); else U1 |= (uint64_t)j << (8 * (u - 8));
            u++;
          }
        int e = 0;
        for (int i = 0; i < r && e < n; i++)
          if (bit128(q0, q1, i)) {
            if (e < 8) S0 |= (uint64_t)i << (8 * e); else S1 |= (uint64_t)i << (8 * (e - 8));
            e++;
          }
        f = block_fbn(b, fbn_base, fbn);
      }
    }
    // TinyMT32 rows of the selected repairs (:194-212), lane q: rows q, q + LPB, ...
    for (int e = q; e < EM; e += LPB) {
      if (state && e < n) {
        Tmt t;
        tmt_init(t, repair_seed(seeds, b, r, f, byte_at(S0, S1, e)));
        uint8_t *row = CO + ((size_t)g * EM + e) * kpad;
        for (int j = 0; j < k; j++) row[j] = tmt_coef(t);
      }
    }
    __syncthreads();
    uint32_t A[EM], V[EM][KDL];  // A[e]: columns 4q..4q+3 of row e
#pragma unroll
    for (int e = 0; e < EM; e++) {
      uint32_t x = 0;
#pragma unroll
      for (int bb = 0; bb < 4; bb++) {
        const int u = 4 * q + bb;
        if (state && e < n && u < n) x |= (uint32_t)crow[e * kpad + byte_at(U0, U1, u)] << (8 * bb);
      }
      A[e] = x;
#pragma unroll
      for (int d = 0; d < KDL; d++) {
        const int c = c0 + 4 * d;
        uint32_t y = 0;
        if (state && e < n && c < k) {
          y = *reinterpret_cast<const uint32_t *>(crow + e * kpad + c);  // coefficients of present sources
#pragma unroll
          for (int bb = 0; bb < 4; bb++) {
            const int cc = c + bb;
            if (cc >= k) y &= ~(0xffu << (8 * bb));
            else if ((miss >> cc) & 1) {  // unknown column: identity row of its unknown
              const uint32_t one = (uint32_t)(__popcll(miss & ((1ull << cc) - 1)) == e);
              y = (y & ~(0xffu << (8 * bb))) | (one << (8 * bb));
            }
          }
        }
        V[e][d] = y;
      }
    }
    // A[e][i] from the lane owning column i (every lane of the block runs the same code path)
    auto colA = [&](int e, int i) -> uint32_t {
      return ((uint32_t)__shfl((int)A[e], lane0 + (i >> 2), 64) >> (8 * (i & 3))) & 0xffu;
    };
#pragma unroll
    for (int i = 0; i < EM; i++) {  // sort_system :28-40 (first maximum wins; rows swapped in place)
      int mx = i;
      uint32_t best = colA(i, i);
#pragma unroll
      for (int j = i + 1; j < EM; j++) {
        const uint32_t v = colA(j, i);
        if (j < n && best < v) { best = v; mx = j; }
      }
      if (i < n) {
#pragma unroll
        for (int j = i + 1; j < EM; j++) {
          if (j == mx) {
            const uint32_t t = A[i]; A[i] = A[j]; A[j] = t;
#pragma unroll
            for (int d = 0; d < KDL; d++) { const uint32_t t2 = V[i][d]; V[i][d] = V[j][d]; V[j][d] = t2; }
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < EM - 1; i++) {  // elimination without re-pivoting :54-70
      const uint32_t piv = colA(i, i);
      const uint32_t lip = 255u - LOG[piv];
#pragma unroll
      for (int kk = i + 1; kk < EM; kk++) {
        const uint32_t a = colA(kk, i);
        if (i < n - 1 && piv && kk < n && a) {
          const PermTab T = perm_table(EXP[LOG[a] + lip]);  // a / piv
          A[kk] ^= gf_mulc(A[i], T);
#pragma unroll
          for (int d = 0; d < KDL; d++) V[kk][d] ^= gf_mulc(V[i][d], T);
        }
      }
    }
    bool ub = false;  // candidate walks to -1 iff a diagonal entry is zero (:74-77)
#pragma unroll
    for (int i = 0; i < EM; i++) ub |= i < n && colA(i, i) == 0;
    if (state && ub) {
      if (q == 0) { h[0] = FECGPU_BLOCK_REF_UB; h[1] = 0; }
      state = 0;
    }
#pragma unroll
    for (int i = EM - 1; i >= 0; i--) {  // back substitution :71-114; X_i replaces row i
#pragma unroll
      for (int u = i + 1; u < EM; u++) {
        const uint32_t a = colA(i, u);
        if (state && i < n && u < n && a) {
          const PermTab T = perm_table(a);
#pragma unroll
          for (int d = 0; d < KDL; d++) V[i][d] ^= gf_mulc(V[u][d], T);
        }
      }
      const uint32_t dg = colA(i, i);
      if (state && i < n) {
        const PermTab T = perm_table(EXP[255u - LOG[dg]]);  // 1 / diagonal
#pragma unroll
        for (int d = 0; d < KDL; d++) V[i][d] = gf_mulc(V[i][d], T);
      }
    }
    if (state) {
#pragma unroll
      for (int i = 0; i < EM; i++) {
        if (i < n) {
          uint8_t *D = h + L.off_D + i * k;
#pragma unroll
          for (int d = 0; d < KDL; d++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++)
              if (c0 + 4 * d + bb < k) D[c0 + 4 * d + bb] = (uint8_t)(V[i][d] >> (8 * bb));
#pragma unroll
          for (int bb = 0; bb < 4; bb++) {  // dependency flags of the columns this lane owns
            const int u = 4 * q + bb;
            if (u < n) h[L.off_dep + i * em + u] = (u > i) && ((A[i] >> (8 * bb)) & 0xffu) != 0;
          }
          if (q == 0) {
            h[L.off_nz + i] = 0;
            h[L.off_unk + i] = (uint8_t)byte_at(U0, U1, i);
            h[L.off_sel + i] = (uint8_t)byte_at(S0, S1, i);
          }
        }
      }
      if (q == 0) {
        int u = 0;
        for (int j = 0; j < k; j++)
          h[L.off_slot + j] = ((miss >> j) & 1) ? (uint8_t)(0x80 | byte_at(S0, S1, u++)) : (uint8_t)j;
        h[0] = FECGPU_BLOCK_RECOVERED;
        h[1] = (uint8_t)n;
      }
    }
    __syncthreads();
    const uint32_t nrows = nblocks - base < BPW ? (uint32_t)(nblocks - base) : (uint32_t)BPW;
    copy_records(reinterpret_cast<uint32_t *>(ws + base * (uint64_t)L.stride),
                 reinterpret_cast<const uint32_t *>(OUTR), nrows, L.stride / 4, orow / 4, lane);
    __syncthreads();
  }
}

// per-block decode record in LDS (layout shared with gen_bitslice.py): 16 output addresses |
// ws non-zero-flag address @128 | rt @136 | non-zero flags @144 (written by the asm body)
constexpr int kDecRec = 160, kDecRecNzPtr = 16, kDecRecRt = 34, kDecRecNz = 144;

// The reference's zero/undetermined rule (rlc_fec_scheme_gf256.c:98-101, 218-236) for one block,
// given its non-zero flags: unknown u is inserted iff it is non-zero and every unknown its row
// still references after elimination is itself determined.  Returns the recovered source masks.
__device__ __forceinline__ void rlc_finalize_block(const uint8_t *h, const WsLayout &L, const uint8_t *nzf,
                                                   uint64_t &m0, uint64_t &m1) {
  m0 = m1 = 0;
  const int n = h[1];
  uint64_t det0 = 0, det1 = 0;  // determined unknowns, indexed by u
  for (int u = n - 1; u >= 0; u--) {
    bool ok = nzf[u] != 0;
    for (int v = u + 1; v < n && ok; v++)
      if (h[L.off_dep + u * L.em + v]) ok = v < 64 ? ((det0 >> v) & 1) : ((det1 >> (v - 64)) & 1);
    if (ok) {
      if (u < 64) det0 |= 1ull << u; else det1 |= 1ull << (u - 64);
      const int j = h[L.off_unk + u];
      if (j < 64) m0 |= 1ull << j; else m1 |= 1ull << (j - 64);
    }
  }
}

__global__ void k_rlc_finalize(uint64_t nblocks, int k, int r, const uint8_t *ws, uint8_t *status,
                               uint64_t *recovered) {
  const WsLayout L = ws_layout((uint32_t)k, (uint32_t)r);
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nblocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t *h = ws + b * (uint64_t)L.stride;
    uint64_t m0 = 0, m1 = 0;
    const int st = h[0];
    if (st == FECGPU_BLOCK_RECOVERED) rlc_finalize_block(h, L, h + L.off_nz, m0, m1);
    status[b] = (uint8_t)st;
    recovered[2 * b] = m0;
    recovered[2 * b + 1] = m1;
  }
}

// =============================================================================================
// Bitsliced data path (default): one wave per (block, column chunk of <= 2 KiB); each lane owns
// 32 bytes of the chunk as NP = 32 / VEC pieces (piece p of the chunk at byte VEC * p; lane l
// holds pieces l, l + A, ..., A = active lanes).  The multiply-accumulate runs in the generated
// inline-assembly bodies of bitslice_gen.h; this wrapper stages coefficients and addresses in LDS.
// =============================================================================================
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

struct BsCfg { int vec, nchunks, chunk_bytes; };

// Lane geometry for one chunk of cb bytes: pieces of VEC bytes; when cb is not a multiple of
// VEC the last piece is pulled back to end at cb, overlapping its neighbour.  Overlapping lanes
// compute and store identical bytes (the map is bytewise), so the result is unchanged.
template <int VEC>
struct BsLanes {
  static constexpr int NP = 32 / VEC;
  uint32_t off[NP];
  uint64_t vm[NP];
  int active;
  __device__ __forceinline__ BsLanes(int lane, int cb) {
    const int npieces = (cb + VEC - 1) / VEC;
    active = (npieces + NP - 1) / NP;
#pragma unroll
    for (int q = 0; q < NP; q++) {
      const int piece = lane + active * q;
      const bool ok = lane < active && piece < npieces;
      const int o = piece * VEC < cb - VEC ? piece * VEC : cb - VEC;
      off[q] = ok ? (uint32_t)o : 0u;
      vm[q] = __ballot(ok);
    }
  }
};

#define BS_CALL_ENC(RT)                                                                             \
  do {                                                                                              \
    if constexpr (VEC == 16)                                                                        \
      bs_enc_r##RT##_v16(sp, rpp, L, rslo, rshi, sdl, ll, nsrc, k, rt, ca, ln.off[0], ln.off[1], ln.vm[0], \
                         ln.vm[1]);                                                                \
    else if constexpr (VEC == 8)                                                                    \
      bs_enc_r##RT##_v8(sp, rpp, L, rslo, rshi, sdl, ll, nsrc, k, rt, ca, ln.off[0], ln.off[1], ln.off[2], \
                        ln.off[3],                                                                  \
                        ln.vm[0], ln.vm[1], ln.vm[2], ln.vm[3]);                                    \
    else                                                                                            \
      bs_enc_r##RT##_v4(sp, rpp, L, rslo, rshi, sdl, ll, nsrc, k, rt, ca, ln.off[0], ln.off[1], ln.off[2], \
                        ln.off[3],                                                                  \
                        ln.off[4], ln.off[5], ln.off[6], ln.off[7], ln.vm[0], ln.vm[1], ln.vm[2],   \
                        ln.vm[3], ln.vm[4], ln.vm[5], ln.vm[6], ln.vm[7]);                          \
  } while (0)

#define BS_CALL_DEC(RT)                                                                             \
  do {                                                                                              \
    if constexpr (VEC == 16)                                                                        \
      bs_dec_r##RT##_v16(ia, oa, nsrc, k, ca, ln.off[0], ln.off[1], ln.vm[0], ln.vm[1]);            \
    else if constexpr (VEC == 8)                                                                    \
      bs_dec_r##RT##_v8(ia, oa, nsrc, k, ca, ln.off[0], ln.off[1], ln.off[2], ln.off[3], ln.vm[0],  \
                        ln.vm[1], ln.vm[2], ln.vm[3]);                                              \
    else                                                                                            \
      bs_dec_r##RT##_v4(ia, oa, nsrc, k, ca, ln.off[0], ln.off[1], ln.off[2], ln.off[3], ln.off[4], \
                        ln.off[5], ln.off[6], ln.off[7], ln.vm[0], ln.vm[1], ln.vm[2], ln.vm[3],    \
                        ln.vm[4], ln.vm[5], ln.vm[6], ln.vm[7]);                                    \
  } while (0)

template <int RT, int VEC>
__device__ __forceinline__ void bs_enc_call(uint64_t sp, uint64_t rpp, uint32_t L, uint64_t rstep, uint64_t sdelta,
                                            uint32_t nsrc, uint32_t k, uint32_t rt, uint32_t ca,
                                            const BsLanes<VEC> &ln) {
  const uint32_t rslo = (uint32_t)rstep, rshi = (uint32_t)(rstep >> 32);
  const uint64_t sdl = sdelta + L, ll = L;  // source pointer steps: after a block's k-th row / otherwise
  if constexpr (RT == 1) BS_CALL_ENC(1);
  else if constexpr (RT == 2) BS_CALL_ENC(2);
  else if constexpr (RT == 4) BS_CALL_ENC(4);
  else if constexpr (RT == 8) BS_CALL_ENC(8);
  else BS_CALL_ENC(16);
}

template <int RT, int VEC>
__device__ __forceinline__ void bs_dec_call(uint32_t ia, uint32_t oa, uint32_t nsrc, uint32_t k, uint32_t ca,
                                            const BsLanes<VEC> &ln) {
  if constexpr (RT == 1) BS_CALL_DEC(1);
  else if constexpr (RT == 2) BS_CALL_DEC(2);
  else if constexpr (RT == 4) BS_CALL_DEC(4);
  else if constexpr (RT == 8) BS_CALL_DEC(8);
  else BS_CALL_DEC(16);
}

// Blocks per group: at most 64 / RT (one coefficient lane per (block, repair)), bounded by the LDS
// budget.  Defaults measured in-process (profiles/r01_ab_group.log, three boxes; r02_ab_group*.log):
// - encode tiles of 4 repairs: groups of 2 blocks (round 2, four boxes: k16 r4 -3.0..-4.1 % against
//   4; round 1 had 4 against 16: -2.6..-3.1 %);
// - decode tiles of 4: groups of 8 (k16 e4 -0.8..-1 %);
// - symbols wider than one column chunk (L > 2 KiB): one block per group (k64 r16 L9000 encode
//   -2.3 %, decode -8.3 %: the chunk passes then revisit one block's rows);
// - everything else: 64 / RT.
// Knob "group" (FECGPU_GROUP=N) replaces the defaults with a plain cap (A/B experiments).
// - batches of fewer than min_groups (default 1024, one wave per SIMD) groups: halved until there
//   are that many groups or one block per group.  A group is streamed by one wave, so a batch of 8
//   k32 r8 blocks took 137 us in one group against 22 us for one block
//   (profiles/r02_small_kernel_probe.log).
static inline int bs_group(int RT, int k, int per_j_bytes, int per_block_bytes, bool enc, int nchunks,
                           uint64_t nb) {
  int g = 64 / RT;
  if (const int cap = knob(K_GROUP)) {
    while (g > 1 && g > cap) g >>= 1;
  } else if (nchunks > 1) {
    g = 1;
  } else if (RT == 4) {
    g = enc ? 2 : 8;
  }
  while (g > 1 && g * (k * per_j_bytes + per_block_bytes) > 32768) g >>= 1;
  if (const uint64_t ming = (uint64_t)knob(K_MIN_GROUPS))
    while (g > 1 && (nb + g - 1) / g < ming) g >>= 1;
  return g;
}


// W waves per workgroup can split the repairs of one group of blocks: wave w owns repairs
// r0 + w*RT .. +RT, streaming the same source rows close together in time (L2 serves the
// repeats).  Default W = 1 (see pick_enc_tile); W > 1 is kept for FECGPU_ENC_TILE experiments.
#ifndef FEC_V1_ENC8_WAVES
#define FEC_V1_ENC8_WAVES 1  // set by bitslice_gen.h when 8-repair encode tiles use the compact register map
#endif
#ifndef FEC_V1_ENC4_WAVES
#define FEC_V1_ENC4_WAVES 1  // likewise for 4-repair tiles
#endif
template <int RT, int VEC>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(RT == 8 ? FEC_V1_ENC8_WAVES : RT == 4 ? FEC_V1_ENC4_WAVES : 1)))
void k_rlc_encode_bs(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep,
                                                       uint64_t nblocks, int k, int r, int L, int nchunks,
                                                       int chunk_bytes, uint32_t fbn_base, const uint32_t *fbn,
                                                       int r0, int G, uint64_t sbs, uint32_t fbn_step, int ilv,
                                                       int bw, uint64_t q0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_all[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform for the asm's SGPRs
  constexpr int CSB = FEC_BS_COEF_ROW_BYTES(RT);  // per source: RT (>= 4) u16 case offsets
  uint8_t *lds = lds_all + (size_t)wave * G * k * CSB;
  // bw > 1: the workgroup's waves code bw adjacent groups (knob enc_block_waves); else its waves split the
  // group's repairs (W waves, each RT of them)
  const int r0w = r0 + (bw > 1 ? 0 : wave * RT);
  const int rt = r - r0w < RT ? r - r0w : RT;  // <= 0: this wave has no repairs (waits at barriers)
  // Group q holds G blocks.  Interleaved (ilv): blocks q, q + NG, q + 2 NG, ... so the waves resident
  // at one time stream neighbouring blocks (dense HBM pages); otherwise blocks qG .. qG + G - 1.
  const uint64_t NG = (nblocks + G - 1) / G;
  const uint64_t bstep = (ilv & 1) ? NG : 1;
  {  // one group per wave: no grid-stride loop invariants live across the asm body
    const uint64_t q = bw > 1 ? (q0 + grp_index(ilv)) * bw + wave : q0 + grp_index(ilv);
    const bool live = q < NG;  // a wave past the end still meets its workgroup's barriers
    if (bw == 1 && !live) return;
    const uint64_t b0 = (ilv & 1) ? q : q * G;
    const uint64_t left = !live ? 0 : (ilv & 1) ? (nblocks - q + NG - 1) / NG : nblocks - b0;
    const int ng = left < (uint64_t)G ? (int)left : G;
    __syncthreads();
    FEC_STAMP_AT(5);
    if (live && lane < G * RT) {  // TinyMT32 rows: lane -> (block g of the group, repair r0w + lane % RT)
      const int g = lane / RT, i = lane % RT;
      const uint64_t b = b0 + g * bstep;
      uint16_t *row0 = reinterpret_cast<uint16_t *>(lds + (size_t)g * k * CSB);
      uint16_t *row = row0 + FEC_BS_FIELD_SLOT(RT, i);  // field i of source j
      if (g < ng && i < rt) {
#ifdef FEC_PROBE_CONSTCOEF  // timing probe only (wrong repairs): no TinyMT32 in the group setup
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = FEC_BS_FIELD((uint32_t)(0x53 + j + i) & 0xffu, i);
#else
        Tmt t;
        const uint32_t f = fbn ? fbn[b] : (uint32_t)((fbn_base + b * fbn_step) & 0xffffffu);
        tmt_init(t, rlc_seed(f, (uint32_t)(r0w + i)));
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = FEC_BS_FIELD(tmt_coef(t), i);
#endif
      } else {
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = 0;  // ends the chain: repair i is not live
      }
      if constexpr (RT < 4) {  // the unused fields of a 4-field row end the chain as well
        if (i == 0)
          for (int j = 0; j < k; j++)
            for (int x = RT; x < 4; x++) row0[j * (CSB / 2) + FEC_BS_FIELD_SLOT(RT, x)] = 0;
      }
    }
    __syncthreads();
    FEC_STAMP_AT(6);
    if (rt <= 0 || !live) return;
    for (int ch = 0; ch < nchunks; ch++) {
      const int c0 = ch * chunk_bytes;
      const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
      BsLanes<VEC> ln(lane, cb);
      const uint64_t sp = (uint64_t)(uintptr_t)(src + b0 * sbs + c0);  // G == 1 unless sbs == k * L
      const uint64_t rpp = (uint64_t)(uintptr_t)(rep + (b0 * (uint64_t)r + r0w) * (uint64_t)L + c0);
      const uint64_t rstep = bstep * (uint64_t)r * L;                 // repair rows of the next block
      const uint64_t sdelta = bstep * sbs - (uint64_t)k * L;          // source rows: after the k-th row
      if (lane < ln.active)
        bs_enc_call<RT, VEC>(sp, rpp, (uint32_t)L, rstep, sdelta, (uint32_t)(ng * k), (uint32_t)k, (uint32_t)rt,
                             lds_addr(lds), ln);
    }
#ifdef FEC_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    FEC_STAMP_AT(7);
  }
}

// Setup reads the workspace for all of a group's blocks at once (lanes spread over (block, input)
// pairs), so each group pays one HBM round trip before its data pass, not one per block.
// status != nullptr: single pass (e <= RT for every block, r0 == 0) -- the zero/undetermined
// rule runs here from LDS (non-zero flags from the asm body, dependency masks and unknown ids
// staged during setup) and status[]/recovered[] are written for every block of the group.
// Otherwise the flags are OR-ed into the workspace for k_rlc_finalize.
template <int RT>
struct RecoverLds {
  static constexpr int CSB = FEC_BS_COEF_ROW_BYTES(RT);
  uint8_t *coef;     // [G][k][CSB] u16 case offsets (u fastest), as the asm's chains read them
  uint64_t *intab;   // [G][k] input symbol addresses
  uint8_t *rec;      // [G] x kDecRec records read by the asm body
  uint8_t *gid;      // [64] compacted slot -> block in group
  uint8_t *ecnt;     // [64] unknowns of the block in this pass
  uint8_t *hst, *he; // [64] status and unknown count of block g (read back after the data pass, so they
                     // need no registers across it)
  uint8_t *unk;      // [G][16] unknown -> source index (fused finalize)
  uint32_t *depm;    // [G][16] unknowns row u still references after elimination (fused finalize)
  __host__ __device__ static size_t bytes(int G, int k) {
    return (size_t)G * ((size_t)k * (CSB + 8) + kDecRec + 16 + 64) + 256;
  }
  __device__ RecoverLds(uint8_t *l, int G, int k) {
    coef = l;
    intab = reinterpret_cast<uint64_t *>(l + (size_t)G * k * CSB);
    rec = l + (size_t)G * k * (CSB + 8);
    depm = reinterpret_cast<uint32_t *>(rec + (size_t)G * kDecRec);
    unk = reinterpret_cast<uint8_t *>(depm + G * 16);
    gid = unk + G * 16;
    ecnt = gid + 64;
    hst = ecnt + 64;
    he = hst + 64;
  }
};

// Row of dst that receives the recovered source j (unknown number `unk` of block b): src's layout
// ([block][k] rows, dst_rows == 0) or packed ([block][dst_rows] rows, unknowns in ascending source
// order; fecgpu_rlc_decode_apply_packed).  Packed rows of a block are contiguous, so no written row
// leaves a 128-B line half written next to bytes the pass does not own.
__device__ __forceinline__ uint64_t rec_row(uint64_t b, int k, int j, int dst_rows, int unk) {
  return dst_rows ? b * (uint64_t)dst_rows + (uint64_t)unk : b * (uint64_t)k + (uint64_t)j;
}

// One group of the recover data pass (group q of NG, blocks b0, b0 + bstep, ...); every lane of the
// wave calls it.  dst_rows < 0: row tables (fecgpu_rlc_decode_rows) -- src and rep are the [block][k]
// source-row and [block][r] repair-row device-address tables, and a missing source's entry is the row
// its recovered bytes go to.  k_rlc_recover_bs runs it over a grid-stride loop; k_rlc_decode_small after the
// wave plan of the group's block.
template <int RT, int VEC>
__device__ void recover_bs_group(uint64_t q, uint64_t NG, uint64_t bstep, uint8_t *__restrict__ src,
                                 const uint8_t *__restrict__ rep, uint64_t nblocks, int k, int r, int L, int nchunks,
                                 int chunk_bytes, uint8_t *ws, int r0, int G, uint8_t *status, uint64_t *recovered,
                                 int ilv, uint8_t *dst, uint8_t *lds, uint8_t *wsl = nullptr, int dst_rows = 0) {
  const WsLayout WL = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x;
  RecoverLds<RT> S(lds, G, k);
  {
    const uint64_t b0 = (ilv & 1) ? q : q * G;
    const uint64_t left = (ilv & 1) ? (nblocks - q + NG - 1) / NG : nblocks - b0;
    const int ng = left < (uint64_t)G ? (int)left : G;
    // wsl: the group's workspace records are copied into LDS first, 16 B per lane-piece, so the setup
    // below costs one memory round trip per group instead of a chain of dependent ones (header ->
    // coefficient rows / slots -> unknowns and dependencies)
    if (wsl) {
      const int per = (int)(WL.stride >> 4), np = ng * per;
#pragma unroll 1
      for (int x = lane; x < np; x += 64) {
        const int g = x / per, o = x - g * per;
        reinterpret_cast<uint4 *>(wsl)[x] =
            reinterpret_cast<const uint4 *>(ws + (b0 + g * bstep) * (uint64_t)WL.stride)[o];
      }
      __syncthreads();
    }
    // record of block g of the group (LDS copy or workspace)
    auto recg = [&](int g) -> const uint8_t * {
      return wsl ? wsl + (size_t)g * WL.stride : ws + (b0 + g * bstep) * (uint64_t)WL.stride;
    };
    bool act = false;
    int st = FECGPU_BLOCK_NOTHING, e = 0;
    if (lane < ng) {
#ifdef FEC_PROBE_NOWS  // timing probe only (wrong bytes): the group setup reads no workspace
      st = FECGPU_BLOCK_RECOVERED;
      e = RT < r ? RT : r;
#else
      const uint8_t *h = recg(lane);
      st = h[0];
      e = h[1];
#endif
      act = st == FECGPU_BLOCK_RECOVERED && e > r0;
    }
    const uint64_t am = __ballot(act);
    const int nact = __popcll(am);
    __syncthreads();
    if (status && lane < ng) {
      S.hst[lane] = (uint8_t)st;
      S.he[lane] = (uint8_t)e;
    }
    if (act) {
      const int t = __popcll(am & ((1ull << lane) - 1));
      S.gid[t] = (uint8_t)lane;
      S.ecnt[t] = (uint8_t)(e - r0 < RT ? e - r0 : RT);
    }
    __syncthreads();
    // coefficient rows and input addresses, one (block, input j) pair per lane
    for (int x = lane; x < nact * k; x += 64) {
      const int t = x / k, j = x - t * k;
      const uint64_t b = b0 + S.gid[t] * bstep;
      const int rt = S.ecnt[t];
      const uint8_t *h = recg(S.gid[t]);
      constexpr int NF = RecoverLds<RT>::CSB / 2;  // fields per source (>= 4)
      uint16_t *row = reinterpret_cast<uint16_t *>(S.coef + (size_t)x * RecoverLds<RT>::CSB);
#ifdef FEC_PROBE_NOWS
      (void)h;
#pragma unroll
      for (int u = 0; u < NF; u++)
        row[FEC_BS_FIELD_SLOT(RT, u)] = (u < rt) ? FEC_BS_FIELD((uint32_t)(0x53 + j + u) & 0xffu, u) : (uint16_t)0;
      const uint32_t sl = j < k - rt ? (uint32_t)(j + rt) : (uint32_t)(0x80 | (j - (k - rt)));
#else
#ifdef FEC_PROBE_NOFIELD  // timing probe only (wrong bytes): the records are read, the D bytes are not
#pragma unroll
      for (int u = 0; u < NF; u++)
        row[FEC_BS_FIELD_SLOT(RT, u)] = (u < rt) ? FEC_BS_FIELD((uint32_t)(0x53 + j + u) & 0xffu, u) : (uint16_t)0;
#else
#pragma unroll
      for (int u = 0; u < NF; u++)  // case offset of D[u][j]; 0 past the live unknowns ends the chain
        row[FEC_BS_FIELD_SLOT(RT, u)] = (u < rt) ? FEC_BS_FIELD(h[WL.off_D + (r0 + u) * k + j], u) : (uint16_t)0;
#endif
      const uint32_t sl = h[WL.off_slot + j];
#endif
      if (dst_rows < 0) {  // row tables: src / rep hold the rows' device addresses ([block][k] / [block][r])
        S.intab[x] = (sl & 0x80) ? reinterpret_cast<const uint64_t *>(rep)[b * (uint64_t)r + (sl & 0x7f)]
                                 : reinterpret_cast<const uint64_t *>(src)[b * (uint64_t)k + sl];
      } else {
        const uint8_t *p = (sl & 0x80) ? rep + (b * (uint64_t)r + (sl & 0x7f)) * (uint64_t)L
                                       : src + (b * (uint64_t)k + sl) * (uint64_t)L;
        S.intab[x] = (uint64_t)(uintptr_t)p;
      }
    }
    // records: output addresses, rt, flags; for the fused finalize the dependency masks
    for (int x = lane; x < nact * 16; x += 64) {
      const int t = x >> 4, u = x & 15;
      const uint64_t b = b0 + S.gid[t] * bstep;
      const int rt = S.ecnt[t];
      const uint8_t *h = recg(S.gid[t]);
      uint8_t *rc = S.rec + (size_t)t * kDecRec;
      rc[kDecRecNz + u] = 0;
      if (u < rt) {
#ifdef FEC_PROBE_NOWS
        const int j = u;
#else
        const int j = h[WL.off_unk + r0 + u];
#endif
        reinterpret_cast<uint64_t *>(rc)[u] =
            dst_rows < 0 ? reinterpret_cast<const uint64_t *>(src)[b * (uint64_t)k + j]  // the missing source's row
                         : (uint64_t)(uintptr_t)(dst + rec_row(b, k, j, dst_rows, r0 + u) * (uint64_t)L);
        if (status) {
          uint32_t m = 0;
#ifndef FEC_PROBE_NOWS
          for (int v = u + 1; v < rt; v++) m |= (uint32_t)(h[WL.off_dep + u * WL.em + v] != 0) << v;
#endif
          S.unk[x] = (uint8_t)j;
          S.depm[x] = m;
        }
      }
      if (u == 0) {
        reinterpret_cast<uint64_t *>(rc)[kDecRecNzPtr] =
            (uint64_t)(uintptr_t)(ws + b * (uint64_t)WL.stride + WL.off_nz + r0);
        reinterpret_cast<uint32_t *>(rc)[kDecRecRt] = (uint32_t)rt;
      }
    }
    __syncthreads();
    if (nact) {
      for (int ch = 0; ch < nchunks; ch++) {
        const int c0 = ch * chunk_bytes;
        const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
        BsLanes<VEC> ln(lane, cb);
#pragma unroll
        for (int q = 0; q < BsLanes<VEC>::NP; q++) ln.off[q] += (uint32_t)c0;  // chunk offset
        // nsrc and k go to SGPRs: readfirstlane states their uniformity (a plan inlined into a
        // one-lane branch before this call can leave the compiler unsure of it)
        if (lane < ln.active)
          bs_dec_call<RT, VEC>(lds_addr(S.intab), lds_addr(S.rec),
                               (uint32_t)__builtin_amdgcn_readfirstlane(nact * k),
                               (uint32_t)__builtin_amdgcn_readfirstlane(k), lds_addr(S.coef), ln);
      }
    }
    __syncthreads();
    if (status) {
      const int st2 = lane < ng ? S.hst[lane] : FECGPU_BLOCK_NOTHING;
      const int e2 = lane < ng ? S.he[lane] : 0;
      const bool act2 = st2 == FECGPU_BLOCK_RECOVERED && e2 > r0;
      const uint64_t am2 = __ballot(act2);
      if (lane < ng) {
        const uint64_t b = b0 + lane * bstep;
        uint64_t m0 = 0, m1 = 0;
        if (act2) {  // rlc_fec_scheme_gf256.c:98-101, 218-236 (see rlc_finalize_block)
          const int t = __popcll(am2 & ((1ull << lane) - 1));
          const uint8_t *nzf = S.rec + (size_t)t * kDecRec + kDecRecNz;
          uint32_t det = 0;
          for (int u = e2 - 1; u >= 0; u--) {
            if (nzf[u] && (S.depm[t * 16 + u] & ~det) == 0) {
              det |= 1u << u;
              const int j = S.unk[t * 16 + u];
              if (j < 64) m0 |= 1ull << j; else m1 |= 1ull << (j - 64);
            }
          }
        }
        status[b] = (uint8_t)st2;
        recovered[2 * b] = m0;
        recovered[2 * b + 1] = m1;
      }
    } else {
      for (int x = lane; x < nact * 16; x += 64) {
        const uint8_t *rc = S.rec + (size_t)(x >> 4) * kDecRec;
        if (rc[kDecRecNz + (x & 15)])
          reinterpret_cast<uint8_t *>(reinterpret_cast<const uint64_t *>(rc)[kDecRecNzPtr])[x & 15] = 1;
      }
    }
  }
}

#ifndef FEC_V1_DEC4_WAVES
#define FEC_V1_DEC4_WAVES 1  // set by bitslice_gen.h when 4-unknown decode tiles use the compact register map
#endif
template <int RT, int VEC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT == 4 ? FEC_V1_DEC4_WAVES : 1)))
void k_rlc_recover_bs(uint8_t *__restrict__ src, const uint8_t *__restrict__ rep,
                                                       uint64_t nblocks, int k, int r, int L, int nchunks,
                                                       int chunk_bytes, uint8_t *ws, int r0, int G,
                                                       uint8_t *status, uint64_t *recovered, int ilv,
                                                       uint8_t *dst, uint32_t wsl_off, int dst_rows, uint64_t q0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint64_t NG = (nblocks + G - 1) / G;  // groups; interleaved as in k_rlc_encode_bs
  const uint64_t bstep = (ilv & 1) ? NG : 1;
  // one group per workgroup (the launcher splits batches of more groups than one grid holds): no
  // grid-stride loop whose invariants the compiler would keep live across the asm body (they cost
  // the wave-per-SIMD budget, 168 VGPRs for 3 waves)
  const uint64_t q = q0 + grp_index(ilv);
  if (q < NG)
    recover_bs_group<RT, VEC>(q, NG, bstep, src, rep, nblocks, k, r, L, nchunks, chunk_bytes, ws, r0, G, status,
                              recovered, ilv, dst, lds, wsl_off ? lds + wsl_off : nullptr, dst_rows);
}

// Encode with the rows given by address (fecgpu_rlc_encode_rows): the batching adapter hands the
// kernel the symbols where they lie -- the FEC plugin's registered memory arena -- instead of copying
// them into a packed batch.  src_rows[b * k + j] / rep_rows[b * r + i]: device addresses of source row
// j / repair row i of block b.  Same data body as the recover pass (input addresses and output records
// staged in LDS per group), with the coefficients from TinyMT32 as in k_rlc_encode_bs.
template <int RT, int VEC>
__global__ __launch_bounds__(64) void k_rlc_encode_rows(const uint64_t *__restrict__ src_rows,
                                                        const uint64_t *__restrict__ rep_rows, uint64_t nblocks, int k,
                                                        int r, int L, int nchunks, int chunk_bytes, uint32_t fbn_base,
                                                        const uint32_t *fbn, int r0, int G) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  RecoverLds<RT> S(lds, G, k);
  constexpr int CSB = RecoverLds<RT>::CSB;
  const int lane = threadIdx.x;
  const int rt = r - r0 < RT ? r - r0 : RT;
  const uint64_t NG = (nblocks + G - 1) / G;
  for (uint64_t q = blockIdx.x; q < NG; q += gridDim.x) {
    const uint64_t b0 = q * G;
    const int ng = nblocks - b0 < (uint64_t)G ? (int)(nblocks - b0) : G;
    __syncthreads();
    if (lane < ng * RT) {  // TinyMT32 rows (get_coefs, rlc_fec_scheme_generate_gf256.c:9-17): lane -> (block g, repair)
      const int g = lane / RT, i = lane % RT;
      uint16_t *row0 = reinterpret_cast<uint16_t *>(S.coef + (size_t)g * k * CSB);
      uint16_t *row = row0 + FEC_BS_FIELD_SLOT(RT, i);
      if (i < rt) {
        Tmt t;
        tmt_init(t, rlc_seed(block_fbn(b0 + g, fbn_base, fbn), (uint32_t)(r0 + i)));
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = FEC_BS_FIELD(tmt_coef(t), i);
      } else {
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = 0;  // ends the chain: repair i is not live
      }
      if constexpr (RT < 4) {
        if (i == 0)
          for (int j = 0; j < k; j++)
            for (int x = RT; x < 4; x++) row0[j * (CSB / 2) + FEC_BS_FIELD_SLOT(RT, x)] = 0;
      }
    }
    for (int x = lane; x < ng * k; x += 64) S.intab[x] = src_rows[b0 * k + x];
    for (int x = lane; x < ng * 16; x += 64) {
      const int t = x >> 4, u = x & 15;
      uint8_t *rc = S.rec + (size_t)t * kDecRec;
      rc[kDecRecNz + u] = 0;
      if (u < rt) reinterpret_cast<uint64_t *>(rc)[u] = rep_rows[(b0 + t) * r + r0 + u];
      if (u == 0) reinterpret_cast<uint32_t *>(rc)[kDecRecRt] = (uint32_t)rt;
    }
    __syncthreads();
    for (int ch = 0; ch < nchunks; ch++) {
      const int c0 = ch * chunk_bytes;
      const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
      BsLanes<VEC> ln(lane, cb);
#pragma unroll
      for (int x = 0; x < BsLanes<VEC>::NP; x++) ln.off[x] += (uint32_t)c0;
      if (lane < ln.active)
        bs_dec_call<RT, VEC>(lds_addr(S.intab), lds_addr(S.rec), (uint32_t)__builtin_amdgcn_readfirstlane(ng * k),
                             (uint32_t)__builtin_amdgcn_readfirstlane(k), lds_addr(S.coef), ln);
    }
  }
}

// Decode of a few blocks in ONE launch (the synchronous hooks decode one block per call): each
// workgroup plans its block with the wave plan, then runs the single-pass data pass on it.  The
// plan's record stays in LDS (past both phases' scratch, at rec_off): both phases address a record
// as ws + b * stride, so they get a base that puts block b's record there, and no global round trip
// or fence sits between the plan and the data pass.
template <int RT, int VEC>
__global__ __launch_bounds__(64) void k_rlc_decode_small(uint8_t *__restrict__ src, const uint8_t *__restrict__ rep,
                                                         uint64_t nblocks, int k, int r, int L, int nchunks,
                                                         int chunk_bytes, uint32_t fbn_base, const uint32_t *fbn,
                                                         const uint32_t *seeds, const uint64_t *sp,
                                                         const uint64_t *rp, uint32_t rec_off, uint8_t *status,
                                                         uint64_t *recovered, uint8_t *dst, int wreg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint64_t stride = ws_layout((uint32_t)k, (uint32_t)r).stride;
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    uint8_t *wsx = reinterpret_cast<uint8_t *>(reinterpret_cast<uintptr_t>(lds + rec_off) - b * stride);
    __syncthreads();
    FEC_STAMP_AT(0);
    plan_load_tables(lds);
    plan_wave_any(wreg, b, k, r, fbn_base, fbn, seeds, sp, rp, wsx, lds);
    __syncthreads();
    FEC_STAMP_AT(3);
    recover_bs_group<RT, VEC>(b, nblocks, 1, src, rep, nblocks, k, r, L, nchunks, chunk_bytes, wsx, 0, 1, status,
                              recovered, 0, dst, lds);
#ifdef FEC_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    FEC_STAMP_AT(4);
  }
}

// =============================================================================================
// A few blocks with their rows staged in LDS (the synchronous hooks run one block per call).
// One workgroup of 8 waves per block.  A one-block launch is latency-bound: the bitsliced bodies
// stream a block's rows through ONE wave, a dependent chain of k steps, and from page-locked host
// memory every prefetch window is a PCIe round trip.  Here waves 1-7 fetch all of the block's rows
// into LDS at once (one round trip) while wave 0 computes the coefficients -- TinyMT32 rows (encode)
// or the whole wave plan (decode) -- and then every thread multiply-accumulates one 4-byte word of the
// outputs with the packed v_perm GF multiply (fec_device.h gf_mac), its coefficient tables built once
// per (output, input) pair in LDS.
// =============================================================================================
constexpr int kLdsThreads = 512;
constexpr uint64_t kSmallLdsMaxBlocks = 64;  // batches up to this many blocks (knob small_lds)

// rows [row0, row0 + nrows) of `base` (row stride L bytes) into LDS rows of Lp bytes, by threads
// [t0, kLdsThreads); 16-B pieces when L and the base are 16-B aligned, else dwords
__device__ __forceinline__ void stage_rows_lds(uint8_t *lrows, const uint8_t *base, int nrows, int L, int Lp, int t0) {
  const int tid = (int)threadIdx.x - t0, nt = kLdsThreads - t0;
  if (tid < 0) return;
  if ((L & 15) == 0 && ((uintptr_t)base & 15) == 0) {
    const int pr = L >> 4, tot = nrows * pr;
    for (int x = tid; x < tot; x += nt) {
      const int row = x / pr, c = x - row * pr;
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      *reinterpret_cast<v4u *>(lrows + row * Lp + 16 * c) =
          __builtin_nontemporal_load(reinterpret_cast<const v4u *>(base + (size_t)row * L + 16 * c));
    }
  } else {
    const int pr = L >> 2, tot = nrows * pr;
    for (int x = tid; x < tot; x += nt) {
      const int row = x / pr, c = x - row * pr;
      *reinterpret_cast<uint32_t *>(lrows + row * Lp + 4 * c) =
          __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(base + (size_t)row * L + 4 * c));
    }
  }
}

// packed-multiply tables of a tile of OT outputs x k inputs, input-major ([j][o]: the OT tables an
// input step needs are contiguous, so they load as a few back-to-back broadcast LDS reads); outputs
// past the tile's live ones get the zero coefficient's (all-zero) tables, so the loops need no guards
struct LdsTabs {
  uint4 *t01;
  uint32_t *t2;
};

template <int OT>
__device__ __forceinline__ void build_tabs(LdsTabs T, const uint8_t *coef, int cstride, int o0, int no, int k) {
  for (int x = threadIdx.x; x < OT * k; x += kLdsThreads) {
    const int j = x / OT, o = x - j * OT;
    const PermTab t = perm_table(o < no ? coef[(o0 + o) * cstride + j] : 0u);
    T.t01[x] = t.t01;
    T.t2[x] = t.t2;
  }
}

// out[o][w] = sum_j coef(o, j) * row_j[w] for the tile's outputs o < no, words w of this thread (row j
// at rows + j * rstride dwords); store(o, w, value)
template <int OT, typename Store>
__device__ __forceinline__ void lds_mac_words(const LdsTabs &T, int no, int k, int Lw, const uint32_t *rows,
                                              int rstride, Store store) {
  for (int w = threadIdx.x; w < Lw; w += kLdsThreads) {
    uint32_t acc[OT];
#pragma unroll
    for (int o = 0; o < OT; o++) acc[o] = 0;
#pragma unroll 2
    for (int j = 0; j < k; j++) {
      const Sel sl = perm_selectors(rows[j * rstride + w]);
      const uint4 *t01 = T.t01 + j * OT;
      const uint32_t *t2 = T.t2 + j * OT;
#pragma unroll
      for (int o = 0; o < OT; o++) acc[o] = gf_mac(acc[o], sl, t01[o], t2[o]);
    }
#pragma unroll
    for (int o = 0; o < OT; o++)
      if (o < no) store(o, w, acc[o]);
  }
}

struct EncLdsLayout {
  uint32_t coef, t01, t2, rows, bytes;
  __host__ __device__ EncLdsLayout(int k, int r, int L, int OT) {
    coef = 0;
    t01 = pad16((uint32_t)(r * pad16((uint32_t)k)));
    t2 = t01 + 16u * OT * k;
    rows = pad16(t2 + 4u * OT * k);
    bytes = rows + (uint32_t)k * pad16((uint32_t)L);
  }
};

// One block's encode with its rows staged in LDS, by all kLdsThreads threads (src_b / rep_b: the
// block's k source rows and r repair rows, L bytes each).
template <int RT>
__device__ __forceinline__ void encode_block_lds(uint8_t *lds, const uint8_t *src_b, uint8_t *rep_b, int k, int r,
                                                 int L, uint32_t f) {
  const EncLdsLayout Y(k, r, L, RT);
  const int kpad = (int)pad16((uint32_t)k), Lp = (int)pad16((uint32_t)L), Lw = L >> 2;
  uint8_t *C = lds + Y.coef;
  const LdsTabs T{reinterpret_cast<uint4 *>(lds + Y.t01), reinterpret_cast<uint32_t *>(lds + Y.t2)};
  const uint32_t *rows = reinterpret_cast<const uint32_t *>(lds + Y.rows);
  __syncthreads();
  FEC_STAMP_AT(5);
  if (threadIdx.x < 64) {  // wave 0: the TinyMT32 rows of repairs i (get_coefs, rlc_fec_scheme_generate_gf256.c:9-17)
    for (int i = (int)threadIdx.x; i < r; i += 64) {
      Tmt t;
      tmt_init(t, rlc_seed(f, (uint32_t)i));
      for (int j = 0; j < k; j++) C[i * kpad + j] = tmt_coef(t);
    }
  } else {
    stage_rows_lds(lds + Y.rows, src_b, k, L, Lp, 64);
  }
  uint32_t *rb = reinterpret_cast<uint32_t *>(rep_b);
  for (int i0 = 0; i0 < r; i0 += RT) {  // tiles of RT repairs
    const int no = r - i0 < RT ? r - i0 : RT;
    __syncthreads();
    if (i0 == 0) FEC_STAMP_AT(6);
    build_tabs<RT>(T, C, kpad, i0, no, k);
    __syncthreads();
    lds_mac_words<RT>(T, no, k, Lw, rows, Lp >> 2, [&](int i, int w, uint32_t v) {
      __builtin_nontemporal_store(v, rb + (size_t)(i0 + i) * Lw + w);
    });
  }
#ifdef FEC_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  FEC_STAMP_AT(7);
}

template <int RT>
__global__ __launch_bounds__(kLdsThreads) void k_rlc_encode_lds(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep,
                                                                uint64_t nblocks, int k, int r, int L, uint32_t fbn_base,
                                                                const uint32_t *fbn) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    encode_block_lds<RT>(lds, src + b * (uint64_t)k * L, rep + b * (uint64_t)r * L, k, r, L,
                         block_fbn(b, fbn_base, fbn));
}

struct DecLdsLayout {
  uint32_t rec, nz, t01, t2, rows, bytes;
  __host__ __device__ DecLdsLayout(int k, int r, int L, int OT) {
    const WsLayout W = ws_layout((uint32_t)k, (uint32_t)r);
    rec = pad16((uint32_t)plan_lds_bytes((uint32_t)k, (uint32_t)r));
    nz = rec + W.stride;
    t01 = nz + 16;
    t2 = t01 + 16u * OT * k;
    rows = pad16(t2 + 4u * OT * k);
    bytes = rows + (uint32_t)(k + r) * pad16((uint32_t)L);
  }
};

// One block's decode (block b of the mask / seed / status arrays; src_b, rep_b, dst_b: its rows) with
// its rows staged in LDS, by all kLdsThreads threads; e <= EM unknowns (one pass), the zero /
// undetermined rule at the end (thread 0).
template <int EM>
__device__ __forceinline__ void decode_block_lds(uint8_t *lds, uint64_t b, const uint8_t *src_b, const uint8_t *rep_b,
                                                 uint8_t *dst_b, int k, int r, int L, uint32_t fbn_base,
                                                 const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                                 const uint64_t *rp, uint8_t *status, uint64_t *recovered, int wreg) {
  const DecLdsLayout Y(k, r, L, EM);
  const WsLayout WL = ws_layout((uint32_t)k, (uint32_t)r);
  const int Lp = (int)pad16((uint32_t)L), Lw = L >> 2;
  uint8_t *h = lds + Y.rec;
  uint32_t *nzword = reinterpret_cast<uint32_t *>(lds + Y.nz);
  const LdsTabs T{reinterpret_cast<uint4 *>(lds + Y.t01), reinterpret_cast<uint32_t *>(lds + Y.t2)};
  uint32_t *rows = reinterpret_cast<uint32_t *>(lds + Y.rows);
  __syncthreads();
  if (threadIdx.x < 64) {  // wave 0: the plan (its record lands in LDS: a base that puts block b's there)
    FEC_STAMP_AT(0);
    plan_load_tables(lds);
    plan_wave_any<false>(wreg, b, k, r, fbn_base, fbn, seeds, sp, rp, h - b * (uint64_t)WL.stride, lds);
    if (threadIdx.x == 0) *nzword = 0;
  } else {  // waves 1-7: all k source and r repair rows of the block (absent ones are never read)
    stage_rows_lds(lds + Y.rows, src_b, k, L, Lp, 64);
    stage_rows_lds(lds + Y.rows + k * Lp, rep_b, r, L, Lp, 64);
  }
  __syncthreads();
  FEC_STAMP_AT(3);
  const int st = h[0], n = h[1];
  if (st == FECGPU_BLOCK_RECOVERED) {
    // input j is source j, or for a missing source the repair its slot names: copy those repair rows
    // over the missing sources' rows, so input j is LDS row j
    const int Lq = Lp >> 2;
    for (int x = threadIdx.x; x < n * Lq; x += kLdsThreads) {
      const int u = x / Lq, c = x - u * Lq, j = h[WL.off_unk + u];
      rows[j * Lq + c] = rows[(k + (h[WL.off_slot + j] & 0x7f)) * Lq + c];
    }
    build_tabs<EM>(T, h + WL.off_D, k, 0, n, k);
    __syncthreads();
    uint32_t *db = reinterpret_cast<uint32_t *>(dst_b);
    uint32_t nzm = 0;
    lds_mac_words<EM>(T, n, k, Lw, rows, Lq, [&](int u, int w, uint32_t v) {
      __builtin_nontemporal_store(v, db + (size_t)h[WL.off_unk + u] * Lw + w);
      nzm |= (uint32_t)(v != 0) << u;
    });
    if (nzm) atomicOr(nzword, nzm);
  }
  __syncthreads();
  FEC_STAMP_AT(4);
  if (threadIdx.x == 0) {  // rlc_fec_scheme_gf256.c:98-101, 218-236 (rlc_finalize_block)
    uint64_t m0 = 0, m1 = 0;
    if (st == FECGPU_BLOCK_RECOVERED) {
      uint8_t nzf[16];
      for (int u = 0; u < 16; u++) nzf[u] = (uint8_t)((*nzword >> u) & 1u);
      rlc_finalize_block(h, WL, nzf, m0, m1);
    }
    status[b] = (uint8_t)st;
    recovered[2 * b] = m0;
    recovered[2 * b + 1] = m1;
  }
}

template <int EM>
__global__ __launch_bounds__(kLdsThreads) void k_rlc_decode_lds(const uint8_t *__restrict__ src,
                                                                const uint8_t *__restrict__ rep, uint64_t nblocks, int k,
                                                                int r, int L, uint32_t fbn_base, const uint32_t *fbn,
                                                                const uint32_t *seeds, const uint64_t *sp,
                                                                const uint64_t *rp, uint8_t *status, uint64_t *recovered,
                                                                uint8_t *dst, int wreg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x)
    decode_block_lds<EM>(lds, b, src + b * (uint64_t)k * L, rep + b * (uint64_t)r * L, dst + b * (uint64_t)k * L, k, r,
                         L, fbn_base, fbn, seeds, sp, rp, status, recovered, wreg);
}

// ---------------------------------------------------------------------------------------------
// Resident block service (fecgpu_block_svc_*, the synchronous hooks): one workgroup of kLdsThreads
// threads stays resident and polls a page-locked mailbox, so a one-block call costs a mailbox
// round trip over PCIe instead of a kernel launch and its completion signal.  Requests are the
// LDS-staged single-block encode / decode above on page-locked buffers.  The kernel always ends:
// on the quit flag, after `idle_ticks` without a request, or after `life_ticks` in all
// (s_memrealtime, 100 MHz); the host relaunches it for the next request.
// ---------------------------------------------------------------------------------------------
// The mailbox: the request (everything a block needs beside its rows, so the worker fetches it with
// one parallel load: wave 0's lanes read 16 B each) then the device-written words.
constexpr int kSvcMaxR = 128;
// Request numbers: the host posts n by storing it into req.seq (release); the worker claims a pending
// request by compare-and-swap n -> n | kSvcClaimed before it reads the request, and the host withdraws
// one by compare-and-swap n -> n - 1 (the last number served).  Exactly one of the two succeeds, so a
// withdrawn request is never served and a claimed one is always finished.
constexpr uint64_t kSvcClaimed = 1ull << 63;
struct alignas(64) BlockSvcReq {
  uint64_t seq;                     // request number, written last by the host (release); | kSvcClaimed
  uint32_t op, k, r, L, fbn, wreg;  // op 1 = RLC encode, 2 = RLC decode with per-repair seeds
  uint64_t src, rep, dst;           // device addresses of the block's rows (page-locked host memory)
  uint64_t sp[2], rp[2];            // presence masks (decode)
  uint32_t seeds[kSvcMaxR];         // the repairs' FPID seeds (decode)
};
static_assert(sizeof(BlockSvcReq) % 16 == 0 && sizeof(BlockSvcReq) / 16 <= 64, "one 16-B load per lane of a wave");
struct alignas(64) BlockSvcMailbox {
  BlockSvcReq req;
  uint64_t done;                    // device: last request number finished (release)
  uint64_t recovered[2];            // device: decode outputs
  uint32_t status, pad0;
  uint64_t quit;                    // host: 1 = end the worker
  uint64_t launches;                // device: worker generations started (diagnostics)
  uint64_t stamp[4];                // device: claim, request in LDS, rows coded, before done (s_memrealtime)
};

__device__ __forceinline__ uint64_t sys_load(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kLdsThreads) void k_block_svc(BlockSvcMailbox *mb, uint64_t idle_ticks,
                                                           uint64_t life_ticks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ BlockSvcReq R;
  __shared__ int go;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  uint64_t t_last = t_start, done = 0;
  if (threadIdx.x == 0) {
    done = sys_load(&mb->done);
    __hip_atomic_fetch_add(&mb->launches, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (;;) {
    if (threadIdx.x == 0) {
      int g = 0;
      for (;;) {
        uint64_t s = sys_load(&mb->req.seq);
        // a posted, unclaimed request: claim it (the host may withdraw it at the same moment; one wins)
        if (!(s & kSvcClaimed) && s != done &&
            __hip_atomic_compare_exchange_strong(&mb->req.seq, &s, s | kSvcClaimed, __ATOMIC_ACQ_REL,
                                                 __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) {
          done = s;  // the number this pass serves
          g = 1;
          __hip_atomic_store(&mb->stamp[0], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (sys_load(&mb->quit) || now - t_last > idle_ticks || now - t_start > life_ticks) {
          g = -1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      go = g;
    }
    __syncthreads();
    if (go < 0) break;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // no stale cached copy of the last request or its rows
    if (threadIdx.x < sizeof(BlockSvcReq) / 16) {  // the whole request in one round trip (after the acquire)
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      reinterpret_cast<v4u *>(&R)[threadIdx.x] =
          __builtin_nontemporal_load(reinterpret_cast<const v4u *>(&mb->req) + threadIdx.x);
    }
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(&mb->stamp[1], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int k = (int)R.k, r = (int)R.r, L = (int)R.L;
    const uint32_t em = (uint32_t)(k < r ? k : r);
    if (R.op == 1) {
      uint8_t *src = (uint8_t *)R.src, *rep = (uint8_t *)R.rep;
      if (r <= 4) encode_block_lds<4>(lds, src, rep, k, r, L, R.fbn);
      else if (r <= 8) encode_block_lds<8>(lds, src, rep, k, r, L, R.fbn);
      else encode_block_lds<16>(lds, src, rep, k, r, L, R.fbn);
    } else {
      const uint8_t *src = (const uint8_t *)R.src, *rep = (const uint8_t *)R.rep;
      uint8_t *dst = (uint8_t *)R.dst;
      uint8_t *st = reinterpret_cast<uint8_t *>(&mb->status);
      uint64_t *rec = mb->recovered;
      // masks and seeds from the LDS copy of the request
      if (em <= 4) decode_block_lds<4>(lds, 0, src, rep, dst, k, r, L, 0, nullptr, R.seeds, R.sp, R.rp, st, rec, R.wreg);
      else if (em <= 8) decode_block_lds<8>(lds, 0, src, rep, dst, k, r, L, 0, nullptr, R.seeds, R.sp, R.rp, st, rec, R.wreg);
      else decode_block_lds<16>(lds, 0, src, rep, dst, k, r, L, 0, nullptr, R.seeds, R.sp, R.rp, st, rec, R.wreg);
    }
    if (threadIdx.x == 0)
      __hip_atomic_store(&mb->stamp[2], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every wave's outputs reach host memory first
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(&mb->stamp[3], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->done, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      t_last = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// 16-B pieces whenever a symbol holds one (a symbol length that is not a multiple of 16 gets an
// overlapping last piece, see BsLanes); chunks of <= 2 KiB, every chunk but the last a multiple
// of the piece size.  L is a multiple of 4 (checked at the ABI).
static BsCfg pick_bs_cfg(int L) {
  BsCfg c;
  c.vec = (L >= 16) ? 16 : (L % 8 == 0) ? 8 : 4;
  c.nchunks = (L + 2047) / 2048;
  int cb = (L + c.nchunks - 1) / c.nchunks;
  cb = (cb + c.vec - 1) / c.vec * c.vec;
  c.chunk_bytes = cb;
  return c;
}

// sbs: bytes from one block's first source to the next block's (k * L for packed blocks; a
// sliding window's step * L, where consecutive blocks overlap).  The asm streams a group's
// sources as one run of contiguous rows, so overlapping blocks go one per group.
// Interleaved groups (default): a group's blocks are NG apart, so the resident waves stream
// neighbouring blocks.  FECGPU_INTERLEAVE=0 restores contiguous groups (A/B experiments).
static int interleave_groups() { return knob(K_INTERLEAVE); }

template <int RT, int VEC>
static void launch_encode_bs(const uint8_t *src, uint8_t *rep, uint64_t nb, int k, int r, int L, const BsCfg &c,
                             uint32_t fbn_base, const uint32_t *fbn, int r0, int W, uint64_t sbs, uint32_t fbn_step,
                             hipStream_t s) {
  const int G = sbs == (uint64_t)k * L ? bs_group(RT, k, FEC_BS_COEF_ROW_BYTES(RT), 0, true, c.nchunks, nb) : 1;
  const uint64_t groups = (nb + G - 1) / G;
  // knob enc_block_waves: bw waves per workgroup on adjacent groups (only with whole blocks, one wave's repairs)
  int bw = W == 1 && sbs == (uint64_t)k * L ? knob(K_ENC_BW) : 1;
  if ((uint64_t)bw > groups) bw = 1;
  const int wpw = bw > 1 ? bw : W;  // waves per workgroup
  const size_t lds = (size_t)wpw * G * k * FEC_BS_COEF_ROW_BYTES(RT);
  FEC_LAUNCH_GROUPS((k_rlc_encode_bs<RT, VEC>), (groups + bw - 1) / bw, 64 * wpw, lds, s, src, rep, nb, k, r, L,
                    c.nchunks, c.chunk_bytes, fbn_base, fbn, r0, G, sbs, fbn_step, interleave_groups(), bw)
}

template <int RT, int VEC>
static void launch_recover_bs(uint8_t *src, const uint8_t *rep, uint64_t nb, int k, int r, int L, const BsCfg &c,
                              uint8_t *ws, int r0, uint8_t *status, uint64_t *recovered, hipStream_t s,
                              uint8_t *dst, int dst_rows) {
  const int G = bs_group(RT, k, FEC_BS_COEF_ROW_BYTES(RT) + 8, kDecRec + 80, false, c.nchunks, nb);
  size_t lds = RecoverLds<RT>::bytes(G, k);
  // the group's workspace records staged in LDS by one round trip (knob ws_lds) when they are small
  const size_t wsb = (size_t)G * ws_layout((uint32_t)k, (uint32_t)r).stride;
  uint32_t wsl_off = 0;
  if (knob(K_WS_LDS) && wsb <= kWsLdsMax && ((uintptr_t)ws & 15) == 0) {
    wsl_off = (uint32_t)((lds + 15) & ~(size_t)15);
    lds = wsl_off + wsb;
  }
  const uint64_t groups = (nb + G - 1) / G;
  // knob dec_waves = n: at most n waves per SIMD (the workgroup's LDS sized so 4 n fit a CU's 160 KiB)
  if (const int dw = knob(K_DEC_WAVES)) {
    const size_t cap = (size_t)160 * 1024 / (4 * (size_t)dw) & ~(size_t)15;
    if (lds < cap) lds = cap;
  }
  FEC_LAUNCH_GROUPS((k_rlc_recover_bs<RT, VEC>), groups, 64, lds, s, src, rep, nb, k, r, L, c.nchunks,
                    c.chunk_bytes, ws, r0, G, status, recovered, interleave_groups(), dst, wsl_off, dst_rows)
}

template <int RT, int VEC>
static void launch_encode_rows(const uint64_t *src_rows, const uint64_t *rep_rows, uint64_t nb, int k, int r, int L,
                               const BsCfg &c, uint32_t fbn_base, const uint32_t *fbn, int r0, hipStream_t s) {
  const int G = bs_group(RT, k, FEC_BS_COEF_ROW_BYTES(RT) + 8, kDecRec + 80, false, c.nchunks, nb);
  hipLaunchKernelGGL((k_rlc_encode_rows<RT, VEC>), dim3(grid_for((nb + G - 1) / G)), dim3(64), RecoverLds<RT>::bytes(G, k),
                     s, src_rows, rep_rows, nb, k, r, L, c.nchunks, c.chunk_bytes, fbn_base, fbn, r0, G);
}

// ---------------------------------------------------------------------------------------------
// Shared-coefficient encode (window blocks).  The window framework numbers every block it encodes
// 0 (malloc_fec_block(cnx, 0), window_framework_sender.h:218), so every window's coefficient rows
// are seeded by the repair index alone (rlc_fec_scheme_generate_gf256.c:9-17, 57-61) and are the
// same for all windows.  The windows x bytes space is therefore flattened and cut into 2 KiB
// chunks, one per wave step: lane l owns the 16-B pieces at chunk offsets 16 l and 1024 + 16 l,
// which may lie in two different windows (their sources sit step * L apart, their repairs r * L
// apart, hence separate load and store offsets).  One case per coefficient then covers all 64
// lanes, where a block-at-a-time wave covers ceil(L / 32) of them (38 at L = 1200).
// ---------------------------------------------------------------------------------------------
#define BS_CALL_ENCSC(RT)                                                                          \
  bs_encsc_r##RT##_v16(sp, rpp, (uint32_t)L, 0u, 0u, (uint64_t)L, (uint64_t)L, (uint32_t)k, (uint32_t)k,  \
                       (uint32_t)rt, lds_addr(lds), off[0], off[1], so[0], so[1], vm[0], vm[1])
// With a start table (wrow != nullptr) window w instead begins at row wrow[w] of `sym` -- the
// batching adapter's de-duplicated symbol streams, several connections' runs in one buffer -- and
// the pieces' load offsets are taken from `sym` itself (the host keeps the buffer below 2 GiB).
template <int RT>
__global__ __launch_bounds__(64) void k_rlc_encode_sc(const uint8_t *__restrict__ sym, uint8_t *__restrict__ rep,
                                                      uint64_t nwin, int k, int r, int L, uint64_t step_bytes,
                                                      int r0, const uint32_t *__restrict__ wrow) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int CSB = FEC_BS_COEF_ROW_BYTES(RT);
  const int lane = threadIdx.x;
  const int rt = r - r0 < RT ? r - r0 : RT;
  if (lane < RT) {  // coefficient rows of repairs r0 .. r0 + rt - 1, seed (0 << 8) | i
    uint16_t *row0 = reinterpret_cast<uint16_t *>(lds);
    uint16_t *row = row0 + FEC_BS_FIELD_SLOT(RT, lane);
    if (lane < rt) {
      Tmt t;
      tmt_init(t, rlc_seed(0u, (uint32_t)(r0 + lane)));
      for (int j = 0; j < k; j++) row[j * (CSB / 2)] = FEC_BS_FIELD(tmt_coef(t), lane);
    } else {
      for (int j = 0; j < k; j++) row[j * (CSB / 2)] = 0;
    }
    if constexpr (RT < 4) {
      if (lane == 0)
        for (int j = 0; j < k; j++)
          for (int x = RT; x < 4; x++) row0[j * (CSB / 2) + FEC_BS_FIELD_SLOT(RT, x)] = 0;
    }
  }
  __syncthreads();
  const uint64_t F = nwin * (uint64_t)L;
  const uint64_t nch = (F + 2047) / 2048;
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t F0 = c * 2048, w0 = F0 / (uint64_t)L;
    uint32_t off[2], so[2];
    uint64_t vm[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint64_t p = F0 + 16u * (uint32_t)(lane + 64 * q);
      const bool ok = p < F;
      const uint64_t w = p / (uint64_t)L;
      const uint32_t t = (uint32_t)(p - w * (uint64_t)L);
      if (wrow)
        off[q] = ok ? wrow[w] * (uint32_t)L + t : 0u;
      else
        off[q] = ok ? (uint32_t)((w - w0) * step_bytes + t) : 0u;  // a piece past the end reads row 0
      so[q] = ok ? (uint32_t)((w - w0) * (uint64_t)r * (uint64_t)L + t) : 0u;
      vm[q] = __ballot(ok);
    }
    const uint64_t sp = (uint64_t)(uintptr_t)(wrow ? sym : sym + w0 * step_bytes);
    const uint64_t rpp = (uint64_t)(uintptr_t)(rep + (w0 * (uint64_t)r + (uint64_t)r0) * (uint64_t)L);
    if constexpr (RT == 1) BS_CALL_ENCSC(1);
    else if constexpr (RT == 2) BS_CALL_ENCSC(2);
    else if constexpr (RT == 4) BS_CALL_ENCSC(4);
    else BS_CALL_ENCSC(8);
  }
}

// The shared-coefficient path runs for overlapping windows (step < k): there a source row serves
// k / step windows, which neighbouring chunks code close together in time, and the 2 KiB cases
// pay off (2^21 windows of k30 r4 step 10: 14.25 -> 11.62 ms; k32 r8 step 8: 18.75 -> 13.87 ms;
// k30 r4 step 1: 14.17 -> 8.21 ms).  Windows that do not overlap are independent blocks, and the
// block kernel's interleaved groups stream them better (k32 r8 step 32: 18.96 vs 20.37 ms;
// profiles/r02_ab_window_sc.log).  It takes 16-B pieces (L % 16 == 0, 16-B aligned rows) and
// offsets that fit 32 bits; returns false (the block-at-a-time path then runs) otherwise.
static bool launch_encode_sc(const uint8_t *sym, uint8_t *rep, uint64_t nwin, int k, int r, int L,
                             uint64_t step_bytes, hipStream_t s, const uint32_t *wrow = nullptr,
                             uint64_t nrows = 0) {
  if (!knob(K_WINDOW_SC) || L % 16 || ((uintptr_t)sym | (uintptr_t)rep) % 16) return false;
  if (wrow) {  // start table: absolute 32-bit load offsets
    if ((nrows + (uint64_t)k) * (uint64_t)L >= (1ull << 31)) return false;
    if ((2048u / (uint32_t)L + 2u) * (uint64_t)r * L + (uint64_t)L >= (1ull << 31)) return false;
  } else {
    if (step_bytes >= (uint64_t)k * (uint64_t)L && knob(K_WINDOW_SC) != 2) return false;  // 2: force (tests)
    const uint64_t span = (2048u / (uint32_t)L + 2u) * (step_bytes > (uint64_t)r * L ? step_bytes : (uint64_t)r * L);
    if (span + (uint64_t)L >= (1ull << 31)) return false;
  }
  const uint64_t nch = (nwin * (uint64_t)L + 2047) / 2048;
  for (int r0 = 0; r0 < r; r0 += 8) {
    const int rt = r - r0 < 8 ? r - r0 : 8;
    const size_t lds = (size_t)k * FEC_BS_COEF_ROW_BYTES(8);
    if (rt >= 5)
      hipLaunchKernelGGL((k_rlc_encode_sc<8>), dim3(grid_for(nch)), dim3(64), lds, s, sym, rep, nwin, k, r, L,
                         step_bytes, r0, wrow);
    else if (rt >= 3)
      hipLaunchKernelGGL((k_rlc_encode_sc<4>), dim3(grid_for(nch)), dim3(64), lds, s, sym, rep, nwin, k, r, L,
                         step_bytes, r0, wrow);
    else if (rt == 2)
      hipLaunchKernelGGL((k_rlc_encode_sc<2>), dim3(grid_for(nch)), dim3(64), lds, s, sym, rep, nwin, k, r, L,
                         step_bytes, r0, wrow);
    else
      hipLaunchKernelGGL((k_rlc_encode_sc<1>), dim3(grid_for(nch)), dim3(64), lds, s, sym, rep, nwin, k, r, L,
                         step_bytes, r0, wrow);
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// LDS-ring data path (bs2_* bodies, gen_bitslice.py body2): the sources of a group stream into a
// per-wave LDS ring by LDS-DMA, D-1 rows ahead (up to 1 KiB per wave-instruction, linear in memory
// and in LDS); each step reads its 32 B per lane from the ring into the plane registers.  The rows
// cost no VGPRs, so occupancy is set by the accumulators (RT <= 8: 4 waves per SIMD) and the ring
// depth only by LDS.  16-B pieces only (symbol_size >= 16); blocks of at least D sources.
// ---------------------------------------------------------------------------------------------
#define FEC_BS2_D(MODE, RT) FEC_BS2_D_##MODE##_RT##RT

// ring depths (sources in flight + 1) of the shipped ring bodies: 16-repair / 16-unknown tiles.  A build
// whose generator also emitted 4-unknown ring bodies (FEC_GEN2_TILES=4,16) can run the 4-unknown
// recover tiles on the ring as well (knob ring = 4; A/B experiments)
template <int RT> struct Bs2Depth;
template <> struct Bs2Depth<16> { static constexpr int enc = FEC_BS2_D(ENC, 16), dec = FEC_BS2_D(DEC, 16); };
#ifdef FEC_BS2_D_DEC_RT4
#define FEC_BS2_HAS_RT4 1
template <> struct Bs2Depth<4> { static constexpr int enc = FEC_BS2_D(ENC, 4), dec = FEC_BS2_D(DEC, 4); };
#else
#define FEC_BS2_HAS_RT4 0
#endif
// 8-repair ring encode bodies (FEC_GEN2_TILES=8,16 builds; knob ring = 8; A/B experiments)
#ifdef FEC_BS2_D_ENC_RT8
#define FEC_BS2_HAS_RT8 1
template <> struct Bs2Depth<8> { static constexpr int enc = FEC_BS2_D(ENC, 8), dec = FEC_BS2_D(DEC, 8); };
#else
#define FEC_BS2_HAS_RT8 0
#endif
using Bs2Depth16 = Bs2Depth<16>;

// Lane geometry of one chunk of cb bytes (cb >= 16) as 16-B pieces, the last pulled back to end at cb.
// DMA: instruction 1 moves pieces 0..63 (lane = piece), instruction 2 pieces 64.. (lane = piece - 64);
// piece t lands at ring slot + 16 t.  Compute: lane l (< A = ceil(pieces / 2)) owns pieces l and l + A.
// c0 is added to the global offsets (decode: the table holds row starts; encode passes 0 and offsets
// its base pointers instead).
struct Bs2Lanes {
  uint32_t g1, g2, rd1, rd2, off0, off1;
  uint64_t vmlo, vmhi, vm0, vm1;
  int npieces;
  __device__ __forceinline__ Bs2Lanes(int lane, int cb, uint32_t c0, uint32_t ring) {
    npieces = (cb + 15) / 16;
    const int A = (npieces + 1) / 2;
    auto gofs = [&](int t) { return (uint32_t)(t * 16 < cb - 16 ? t * 16 : cb - 16); };
    const bool d1 = lane < npieces, d2 = lane + 64 < npieces;
    g1 = c0 + (d1 ? gofs(lane) : 0u);
    g2 = c0 + (d2 ? gofs(lane + 64) : 0u);
    vmlo = __ballot(d1);
    vmhi = __ballot(d2);
    const int p1 = lane + A;
    const bool ok0 = lane < A, ok1 = lane < A && p1 < npieces;
    rd1 = ring + (ok0 ? 16u * (uint32_t)lane : 0u);  // LDS addresses in slot 0 (steps add the slot)
    rd2 = ring + (ok1 ? 16u * (uint32_t)p1 : 0u);
    off0 = ok0 ? c0 + gofs(lane) : 0u;
    off1 = ok1 ? c0 + gofs(p1) : 0u;
    vm0 = __ballot(ok0);
    vm1 = __ballot(ok1);
  }
};

static inline uint32_t bs2_slot_bytes(int) { return FEC_BS2_SLOT; }  // the bodies address slots by immediates

// The lane id recomputed on the spot (v_mbcnt), opaque to the compiler: the RT = 16 ring bodies
// leave it v0-v7, and their own lane arguments take six of those, so a lane-derived value the
// compiler keeps live across a body (a hoisted 16 * (lane + 64), a block's header bytes) is spilled
// to scratch and reloaded per item.  Deriving the lane values afresh per item / after the loop keeps
// nothing per lane live across the asm.
__device__ __forceinline__ int lane_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

#define BS2_LANE_ARGS ln.g1, ln.g2, ln.vmlo, ln.vmhi, ln.rd1, ln.rd2, ln.off0, ln.off1, ln.vm0, ln.vm1
#define BS2_CALL_ENC(RT, ND) \
  bs2_enc_r##RT##_d##ND(sp, rpp, (uint32_t)L, rslo, rshi, sdl, ll, (uint32_t)rt, nsrc, (uint32_t)k, ca, ring, \
                        BS2_LANE_ARGS)
#define BS2_CALL_DEC(RT, ND) \
  bs2_dec_r##RT##_d##ND(ia, oa, nsrc, (uint32_t)k, ca, ring, BS2_LANE_ARGS)

template <int RT>
__device__ __forceinline__ void bs2_enc_call(bool two, uint64_t sp, uint64_t rpp, int L, uint32_t rslo, uint32_t rshi,
                                             uint64_t sdl, uint64_t ll, int rt, uint32_t nsrc, int k, uint32_t ca,
                                             uint32_t ring, const Bs2Lanes &ln) {
#if FEC_BS2_HAS_RT8
  if constexpr (RT == 8) {
    if (two) BS2_CALL_ENC(8, 2); else BS2_CALL_ENC(8, 1);
    return;
  }
#endif
  if (two) BS2_CALL_ENC(16, 2); else BS2_CALL_ENC(16, 1);
}

template <int RT>
__device__ __forceinline__ void bs2_dec_call(bool two, uint32_t ia, uint32_t oa, uint32_t nsrc, int k, uint32_t ca,
                                             uint32_t ring, const Bs2Lanes &ln) {
#if FEC_BS2_HAS_RT4
  if constexpr (RT == 4) {
    if (two) BS2_CALL_DEC(4, 2); else BS2_CALL_DEC(4, 1);
    return;
  }
#endif
  if (two) BS2_CALL_DEC(16, 2); else BS2_CALL_DEC(16, 1);
}

// W waves per workgroup split a group's repairs (wave w: repairs r0 + w RT ..), each with its own
// coefficient rows and ring; they read the same source rows close together in time (L2 serves the
// repeats).  W = 1 unless a tile knob asks for more.
// CW (chunk waves): symbols wider than one column chunk (L > 2 KiB, e.g. configs[4]'s 9000 B).  A
// workgroup of kCwWaves waves codes a group of G blocks as the list of its (block, chunk) items --
// wave w takes items w, w + kCwWaves, ... -- so each round codes kCwWaves consecutive chunks at once,
// sharing the group's coefficient rows (one TinyMT32 pass) and each wave streaming its own ring.
// Neighbouring chunks of a row advance together, so the 128-B lines they share (chunk and row
// boundaries are not line-aligned) are fetched once and hit in L2 for the other wave, instead of
// being re-fetched by the next chunk pass of one wave tens of microseconds later.  Four waves per
// workgroup: the waves of a workgroup are spread evenly over the CU's four SIMDs, so a 5-wave
// workgroup holds two slots on every SIMD and halved the resident waves (+68 % time at k64 r16
// L9000, profiles/r03_ab_chunk_waves_5wave_wg.log).
constexpr int kCwWaves = 4;

template <int RT, bool CW>
#ifndef FEC_BS2_RT16_WAVES
#define FEC_BS2_RT16_WAVES 3
#endif
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(RT == 16 && FEC_BS2_BASE <= 8 ? FEC_BS2_RT16_WAVES
                                                                    : RT == 8 ? 4 : 1)))
void k_rlc_encode_bs2(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep,
                                                        uint64_t nblocks, int k, int r, int L, int nchunks,
                                                        int chunk_bytes, uint32_t fbn_base, const uint32_t *fbn,
                                                        int r0, int G, uint64_t sbs, uint32_t fbn_step, int ilv,
                                                        uint32_t slotb, uint64_t q0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_all[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int CSB = FEC_BS_COEF_ROW_BYTES(RT);
  constexpr int D = Bs2Depth<RT>::enc;
  const uint32_t coef_bytes = pad16((uint32_t)(G * k * CSB));
  // CW: one set of coefficient rows for the group, then a ring per wave; otherwise rows + ring per wave
  uint8_t *lds = CW ? lds_all : lds_all + (size_t)wave * (coef_bytes + D * slotb);
  const uint32_t ring = CW ? lds_addr(lds_all) + coef_bytes + (uint32_t)wave * D * slotb : lds_addr(lds) + coef_bytes;
  if constexpr (!CW) r0 += wave * RT;
  const int rt = r - r0 < RT ? r - r0 : RT;  // <= 0: this wave has no repairs (waits at barriers)
  const uint64_t NG = (nblocks + G - 1) / G;
  const uint64_t bstep = (ilv & 1) ? NG : 1;
  {  // one group per workgroup: no grid-stride loop invariants live across the asm body
    const uint64_t q = q0 + grp_index(ilv);
    if (q >= NG) return;
    const uint64_t b0 = (ilv & 1) ? q : q * G;
    const uint64_t left = (ilv & 1) ? (nblocks - q + NG - 1) / NG : nblocks - b0;
    const int ng = left < (uint64_t)G ? (int)left : G;
    __syncthreads();
    if ((CW ? (int)threadIdx.x : lane) < G * RT) {  // TinyMT32 rows: lane -> (block g, repair r0 + lane % RT)
      // (CW: wave 0's lanes only, G * RT <= 64)
      const int g = lane / RT, i = lane % RT;
      const uint64_t b = b0 + g * bstep;
      uint16_t *row0 = reinterpret_cast<uint16_t *>(lds + (size_t)g * k * CSB);
      uint16_t *row = row0 + FEC_BS_FIELD_SLOT(RT, i);
      if (g < ng && i < rt) {
        Tmt t;
        const uint32_t f = fbn ? fbn[b] : (uint32_t)((fbn_base + b * fbn_step) & 0xffffffu);
        tmt_init(t, rlc_seed(f, (uint32_t)(r0 + i)));
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = FEC_BS_FIELD(tmt_coef(t), i);
      } else {
        for (int j = 0; j < k; j++) row[j * (CSB / 2)] = 0;
      }
      if constexpr (RT < 4) {
        if (i == 0)
          for (int j = 0; j < k; j++)
            for (int x = RT; x < 4; x++) row0[j * (CSB / 2) + FEC_BS_FIELD_SLOT(RT, x)] = 0;
      }
    }
    __syncthreads();
    if (rt <= 0) return;
    if constexpr (CW) {  // items (block g, chunk ch), one block's k rows per body call
      for (int it = wave; it < ng * nchunks; it += kCwWaves) {
        const int g = it / nchunks, ch = it - g * nchunks;
        const int c0 = ch * chunk_bytes;
        const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
        const Bs2Lanes ln(lane_fresh(), cb, 0u, ring);
        const uint64_t b = b0 + g * bstep;
        const uint64_t sp = (uint64_t)(uintptr_t)(src + b * sbs + c0);
        const uint64_t rpp = (uint64_t)(uintptr_t)(rep + (b * (uint64_t)r + r0) * (uint64_t)L + c0);
        bs2_enc_call<RT>(ln.npieces > 64, sp, rpp, L, 0u, 0u, (uint64_t)L, (uint64_t)L, rt, (uint32_t)k, k,
                     lds_addr(lds + (size_t)g * k * CSB), ring, ln);
      }
    } else {
      for (int ch = 0; ch < nchunks; ch++) {
        const int c0 = ch * chunk_bytes;
        const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
        const Bs2Lanes ln(lane_fresh(), cb, 0u, ring);
        const uint64_t sp = (uint64_t)(uintptr_t)(src + b0 * sbs + c0);
        const uint64_t rpp = (uint64_t)(uintptr_t)(rep + (b0 * (uint64_t)r + r0) * (uint64_t)L + c0);
        const uint64_t rstep = bstep * (uint64_t)r * L;
        const uint64_t sdelta = bstep * sbs - (uint64_t)k * L;
        const uint32_t rslo = (uint32_t)rstep, rshi = (uint32_t)(rstep >> 32);
        const uint64_t sdl = sdelta + L, ll = (uint64_t)L;
        bs2_enc_call<RT>(ln.npieces > 64, sp, rpp, L, rslo, rshi, sdl, ll, rt, (uint32_t)(ng * k), k, lds_addr(lds), ring,
                     ln);
      }
    }
  }
}

// CW: as in k_rlc_encode_bs2, kCwWaves waves code the group's (block, chunk) items; the setup is
// spread over every thread of the workgroup and wave 0 writes the statuses once all items are done.
template <int RT, bool CW>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(RT == 16 ? 3 : RT >= 4 ? 4 : 1)))
void k_rlc_recover_bs2(uint8_t *__restrict__ src, const uint8_t *__restrict__ rep,
                                                        uint64_t nblocks, int k, int r, int L, int nchunks,
                                                        int chunk_bytes, uint8_t *ws, int r0, int G,
                                                        uint8_t *status, uint64_t *recovered, int ilv,
                                                        uint8_t *dst, uint32_t slotb, int dst_rows, uint64_t q0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const WsLayout WL = ws_layout((uint32_t)k, (uint32_t)r);
  const int lane = threadIdx.x & 63;
  const int wave = CW ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  const int tid = CW ? (int)threadIdx.x : lane, nthr = CW ? (int)blockDim.x : 64;
  RecoverLds<RT> S(lds, G, k);
  const uint32_t ring = lds_addr(lds) + (uint32_t)pad16((uint32_t)RecoverLds<RT>::bytes(G, k)) +
                        (uint32_t)wave * Bs2Depth<RT>::dec * slotb;
  const uint64_t NG = (nblocks + G - 1) / G;
  const uint64_t bstep = (ilv & 1) ? NG : 1;
  {  // one group per workgroup: no grid-stride loop invariants live across the asm body
    const uint64_t q = q0 + grp_index(ilv);
    if (q >= NG) return;
    const uint64_t b0 = (ilv & 1) ? q : q * G;
    const uint64_t left = (ilv & 1) ? (nblocks - q + NG - 1) / NG : nblocks - b0;
    const int ng = left < (uint64_t)G ? (int)left : G;
    bool act = false;
    int st = FECGPU_BLOCK_NOTHING, e = 0;
    if (lane < ng) {  // every wave reads the group's headers (the same values)
      const uint8_t *h = ws + (b0 + lane * bstep) * (uint64_t)WL.stride;
      st = h[0];
      e = h[1];
      act = st == FECGPU_BLOCK_RECOVERED && e > r0;
    }
    const uint64_t am = __ballot(act);
    const int nact = __popcll(am);
    __syncthreads();
    if (act && wave == 0) {
      const int t = __popcll(am & ((1ull << lane) - 1));
      S.gid[t] = (uint8_t)lane;
      S.ecnt[t] = (uint8_t)(e - r0 < RT ? e - r0 : RT);
    }
    __syncthreads();
    for (int x = tid; x < nact * k; x += nthr) {
      const int t = x / k, j = x - t * k;
      const uint64_t b = b0 + S.gid[t] * bstep;
      const int rt = S.ecnt[t];
      const uint8_t *h = ws + b * (uint64_t)WL.stride;
      constexpr int NF = RecoverLds<RT>::CSB / 2;
      uint16_t *row = reinterpret_cast<uint16_t *>(S.coef + (size_t)x * RecoverLds<RT>::CSB);
#pragma unroll
      for (int u = 0; u < NF; u++)
        row[FEC_BS_FIELD_SLOT(RT, u)] = (u < rt) ? FEC_BS_FIELD(h[WL.off_D + (r0 + u) * k + j], u) : (uint16_t)0;
      const uint32_t sl = h[WL.off_slot + j];
      const uint8_t *p = (sl & 0x80) ? rep + (b * (uint64_t)r + (sl & 0x7f)) * (uint64_t)L
                                     : src + (b * (uint64_t)k + sl) * (uint64_t)L;
      S.intab[x] = (uint64_t)(uintptr_t)p;
    }
    for (int x = tid; x < nact * 16; x += nthr) {
      const int t = x >> 4, u = x & 15;
      const uint64_t b = b0 + S.gid[t] * bstep;
      const int rt = S.ecnt[t];
      const uint8_t *h = ws + b * (uint64_t)WL.stride;
      uint8_t *rc = S.rec + (size_t)t * kDecRec;
      rc[kDecRecNz + u] = 0;
      if (u < rt) {
#ifdef FEC_PROBE_NOWS
        const int j = u;
#else
        const int j = h[WL.off_unk + r0 + u];
#endif
        reinterpret_cast<uint64_t *>(rc)[u] = (uint64_t)(uintptr_t)(dst + rec_row(b, k, j, dst_rows, r0 + u) * (uint64_t)L);
        if (status) {
          uint32_t m = 0;
#ifndef FEC_PROBE_NOWS
          for (int v = u + 1; v < rt; v++) m |= (uint32_t)(h[WL.off_dep + u * WL.em + v] != 0) << v;
#endif
          S.unk[x] = (uint8_t)j;
          S.depm[x] = m;
        }
      }
      if (u == 0) {
        reinterpret_cast<uint64_t *>(rc)[kDecRecNzPtr] = (uint64_t)(uintptr_t)(h + WL.off_nz + r0);
        reinterpret_cast<uint32_t *>(rc)[kDecRecRt] = (uint32_t)rt;
      }
    }
    __syncthreads();
    if constexpr (CW) {  // items (active block t, chunk ch); the chunks' non-zero flags OR together
      for (int it = wave; it < nact * nchunks; it += kCwWaves) {
        const int t = it / nchunks, ch = it - t * nchunks;
        const int c0 = ch * chunk_bytes;
        const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
        const Bs2Lanes ln(lane_fresh(), cb, (uint32_t)c0, ring);
        bs2_dec_call<RT>(ln.npieces > 64, lds_addr(S.intab + (size_t)t * k), lds_addr(S.rec + (size_t)t * kDecRec),
                     (uint32_t)k, k, lds_addr(S.coef + (size_t)t * k * RecoverLds<RT>::CSB), ring, ln);
      }
    } else if (nact) {
      for (int ch = 0; ch < nchunks; ch++) {
        const int c0 = ch * chunk_bytes;
        const int cb = L - c0 < chunk_bytes ? L - c0 : chunk_bytes;
        const Bs2Lanes ln(lane_fresh(), cb, (uint32_t)c0, ring);
        bs2_dec_call<RT>(ln.npieces > 64, lds_addr(S.intab), lds_addr(S.rec), (uint32_t)(nact * k), k,
                         lds_addr(S.coef), ring, ln);
      }
    }
    __syncthreads();
    if (wave != 0) return;
    if (status) {
      const int ln0 = lane_fresh();  // the header bytes read again rather than kept across the bodies
      if (ln0 < ng) {
        const uint64_t b = b0 + ln0 * bstep;
        const uint8_t *h = ws + b * (uint64_t)WL.stride;
        const int st = h[0], e = h[1];
        uint64_t m0 = 0, m1 = 0;
        if (st == FECGPU_BLOCK_RECOVERED && e > r0) {  // rlc_fec_scheme_gf256.c:98-101, 218-236 (see rlc_finalize_block)
          const int t = __popcll(am & ((1ull << ln0) - 1));
          const uint8_t *nzf = S.rec + (size_t)t * kDecRec + kDecRecNz;
          uint32_t det = 0;
          for (int u = e - 1; u >= 0; u--) {
            if (nzf[u] && (S.depm[t * 16 + u] & ~det) == 0) {
              det |= 1u << u;
              const int j = S.unk[t * 16 + u];
              if (j < 64) m0 |= 1ull << j; else m1 |= 1ull << (j - 64);
            }
          }
        }
        status[b] = (uint8_t)st;
        recovered[2 * b] = m0;
        recovered[2 * b + 1] = m1;
      }
    } else {
      for (int x = lane_fresh(); x < nact * 16; x += 64) {
        const uint8_t *rc = S.rec + (size_t)(x >> 4) * kDecRec;
        if (rc[kDecRecNz + (x & 15)])
          reinterpret_cast<uint8_t *>(reinterpret_cast<const uint64_t *>(rc)[kDecRecNzPtr])[x & 15] = 1;
      }
    }
  }
}

// Groups for the ring path: as bs_group, then halved until the workgroup's LDS (coefficient rows or
// decode staging + the ring) leaves room for `waves` waves per CU (160 KiB of LDS per CU).
static inline int bs2_group(int RT, int k, int per_j, int per_block, bool enc, int nchunks, size_t ring_bytes,
                            int waves, uint64_t nb) {
  int g = bs_group(RT, k, per_j, per_block, enc, nchunks, nb);
  const size_t budget = (size_t)160 * 1024 / (size_t)waves;
  while (g > 1 && (size_t)g * (k * per_j + per_block) + 256 + ring_bytes > budget) g >>= 1;
  return g;
}

// Target waves per CU for the ring kernels (VGPR-limited occupancy of the bodies: RT <= 4: 5,
// RT = 8: 4, RT = 16: 2 waves per SIMD).
// resident waves per CU the LDS budget is sized for (RT = 16 reaches 3 per SIMD only with the
// two-temporary register map of a FEC_GEN2_BASE=8 build)
#ifndef FEC_BS2_RT4_WAVES_PER_CU
#define FEC_BS2_RT4_WAVES_PER_CU 16
#endif
static inline int bs2_waves_per_cu(int RT) {
  return RT <= 4 ? FEC_BS2_RT4_WAVES_PER_CU : RT == 8 ? 16 : FEC_BS2_BASE <= 8 ? 4 * FEC_BS2_RT16_WAVES : 8;
}

// Chunk waves (knob chunk_waves, default on): symbols wider than one column chunk are coded by
// workgroups of kCwWaves waves over groups of up to 64 / RT blocks (k_rlc_encode_bs2 /
// k_rlc_recover_bs2 CW), the group halved until the workgroup's LDS fits 64 KiB.
static int cw_group(int RT, int k, int per_j, int per_block, size_t ring_bytes, uint64_t nb) {
  if (!knob(K_CHUNK_WAVES)) return 0;
  int g = 64 / RT;
  while (g > 1 && (uint64_t)g > nb) g >>= 1;
  while (g >= 1 && (size_t)g * (k * per_j + per_block) + 256 + kCwWaves * ring_bytes > 65536) g >>= 1;
  return g;
}

template <int RT>
static void launch_encode_bs2(const uint8_t *src, uint8_t *rep, uint64_t nb, int k, int r, int L, const BsCfg &c,
                              uint32_t fbn_base, const uint32_t *fbn, int r0, int W, uint64_t sbs, uint32_t fbn_step,
                              hipStream_t s) {
  const uint32_t slotb = bs2_slot_bytes(c.chunk_bytes);
  const size_t ring_bytes = (size_t)Bs2Depth<RT>::enc * slotb;
  const int CSB = FEC_BS_COEF_ROW_BYTES(RT);
  if (int G = (W == 1 && c.nchunks > 1) ? cw_group(RT, k, CSB, 0, ring_bytes, nb) : 0) {
    if (sbs != (uint64_t)k * L) G = 1;  // overlapping blocks (windows): one per group
    const size_t lds = pad16((uint32_t)(G * k * CSB)) + kCwWaves * ring_bytes;
    FEC_LAUNCH_GROUPS((k_rlc_encode_bs2<RT, true>), (nb + G - 1) / G, 64 * kCwWaves, lds, s, src, rep, nb, k, r, L,
                      c.nchunks, c.chunk_bytes, fbn_base, fbn, r0, G, sbs, fbn_step, interleave_groups(), slotb)
    return;
  }
  const int G = sbs == (uint64_t)k * L
                    ? bs2_group(RT, k, CSB, 0, true, c.nchunks, ring_bytes, bs2_waves_per_cu(RT), nb)
                    : 1;
  const size_t coef = pad16((uint32_t)(G * k * CSB));
  FEC_LAUNCH_GROUPS((k_rlc_encode_bs2<RT, false>), (nb + G - 1) / G, 64 * W, (size_t)W * (coef + ring_bytes), s,
                    src, rep, nb, k, r, L, c.nchunks, c.chunk_bytes, fbn_base, fbn, r0, G, sbs, fbn_step,
                    interleave_groups(), slotb)
}

template <int RT>
static void launch_recover_bs2(uint8_t *src, const uint8_t *rep, uint64_t nb, int k, int r, int L, const BsCfg &c,
                               uint8_t *ws, int r0, uint8_t *status, uint64_t *recovered, hipStream_t s,
                               uint8_t *dst, int dst_rows) {
  const uint32_t slotb = bs2_slot_bytes(c.chunk_bytes);
  const size_t ring_bytes = (size_t)Bs2Depth<RT>::dec * slotb;
  const int per_j = FEC_BS_COEF_ROW_BYTES(RT) + 8, per_block = kDecRec + 80;
  if (const int G = c.nchunks > 1 ? cw_group(RT, k, per_j, per_block, ring_bytes, nb) : 0) {
    const size_t lds = pad16((uint32_t)RecoverLds<RT>::bytes(G, k)) + kCwWaves * ring_bytes;
    FEC_LAUNCH_GROUPS((k_rlc_recover_bs2<RT, true>), (nb + G - 1) / G, 64 * kCwWaves, lds, s, src, rep, nb, k, r, L,
                      c.nchunks, c.chunk_bytes, ws, r0, G, status, recovered, interleave_groups(), dst, slotb, dst_rows)
    return;
  }
  const int G = bs2_group(RT, k, per_j, per_block, false, c.nchunks, ring_bytes, bs2_waves_per_cu(RT), nb);
  const size_t stage = pad16((uint32_t)RecoverLds<RT>::bytes(G, k));
  FEC_LAUNCH_GROUPS((k_rlc_recover_bs2<RT, false>), (nb + G - 1) / G, 64, stage + ring_bytes, s, src, rep, nb, k, r,
                    L, c.nchunks, c.chunk_bytes, ws, r0, G, status, recovered, interleave_groups(), dst, slotb, dst_rows)
}

// The ring path applies to 16-repair / 16-unknown tiles of 16-B pieces (symbol_size >= 16) and blocks
// of at least D sources (one epilogue in any wait window, see gen_bitslice.py body2); knob ring = 0
// keeps those tiles on the register-prefetch body (A/B).
static bool use_ring(int rt, uint32_t k, const BsCfg &cfg, bool enc) {
  if (knob(K_RING) == 0 || cfg.vec != 16) return false;
  if (rt == 16) return (int)k >= (enc ? Bs2Depth16::enc : Bs2Depth16::dec);
#if FEC_BS2_HAS_RT8
  if (rt == 8 && enc && knob(K_RING) == 8) return (int)k >= Bs2Depth<8>::enc;
#endif
#if FEC_BS2_HAS_RT4
  if (rt == 4 && !enc && knob(K_RING) == 4) return (int)k >= Bs2Depth<4>::dec;
#endif
  return false;
}

#if FEC_BS2_HAS_RT4
#define FEC_BS2_DISPATCH_DEC(FN, ...) \
  if (rt == 4) FN<4>(__VA_ARGS__); else FN<16>(__VA_ARGS__);
#else
#define FEC_BS2_DISPATCH_DEC(FN, ...) FN<16>(__VA_ARGS__);
#endif
#if FEC_BS2_HAS_RT8
#define FEC_BS2_DISPATCH(FN, ...) \
  if (rt == 8) FN<8>(__VA_ARGS__); else FN<16>(__VA_ARGS__);
#else
#define FEC_BS2_DISPATCH(FN, ...) FN<16>(__VA_ARGS__);
#endif

#define FEC_BS_DISPATCH(FN, ...)                                                   \
  switch (rt * 100 + cfg.vec) {                                                    \
    case 116: FN<1, 16>(__VA_ARGS__); break;  case 108: FN<1, 8>(__VA_ARGS__); break;   \
    case 104: FN<1, 4>(__VA_ARGS__); break;   case 216: FN<2, 16>(__VA_ARGS__); break;  \
    case 208: FN<2, 8>(__VA_ARGS__); break;   case 204: FN<2, 4>(__VA_ARGS__); break;   \
    case 416: FN<4, 16>(__VA_ARGS__); break;  case 408: FN<4, 8>(__VA_ARGS__); break;   \
    case 404: FN<4, 4>(__VA_ARGS__); break;   case 816: FN<8, 16>(__VA_ARGS__); break;  \
    case 808: FN<8, 8>(__VA_ARGS__); break;   case 804: FN<8, 4>(__VA_ARGS__); break;   \
    case 1616: FN<16, 16>(__VA_ARGS__); break; case 1608: FN<16, 8>(__VA_ARGS__); break; \
    default: FN<16, 4>(__VA_ARGS__); break;                                        \
  }

// The case tails build jump targets from the table's upper address bits and a 16-bit offset, so
// the table must sit on a 64 KiB boundary at run time (the code object asks for it: .p2align 16).
// Checked once per device, on a private stream, before the first bitsliced launch; a misplaced
// table fails the call instead of jumping into the wrong code.
static std::atomic<int> g_tab_state[64];  // 0 unknown, 1 checked, -1 misaligned
static int bs_table_check() {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return set_err(FECGPU_ERR_NO_DEVICE, "%s", "device index out of range");
  int st = g_tab_state[dev].load();
  if (st == 0) {
    uint64_t *d = nullptr, h[2] = {0, 0};
    hipStream_t ps;
    HIPCHK(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&d, sizeof h));
    hipLaunchKernelGGL(fec_bs_case_table_addr, dim3(1), dim3(64), 0, ps, d);
    HIPCHK(hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, ps));
    HIPCHK(hipStreamSynchronize(ps));
    HIPCHK(hipFree(d));
    HIPCHK(hipStreamDestroy(ps));
    st = (h[0] != 0 && (h[0] & 0xFFFF) == 0 && h[1] != 0 && (h[1] & 0xFFFF) == 0) ? 1 : -1;
    g_tab_state[dev].store(st);
  }
  if (st < 0) return set_err(FECGPU_ERR_HIP, "%s", "GF(256) case table is not 64 KiB-aligned in device memory");
  return FECGPU_OK;
}

// =============================================================================================
// XOR scheme
// =============================================================================================
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ V vxor(V a, V b) { return a ^ b; }

// One thread per 16-B (or 4-B) column piece of a block.  KC > 0: k fixed at compile time, so
// the k row loads are issued back to back; I: 32-bit index arithmetic when nblocks * Lv < 2^32
// (a 64-bit division per piece is most of the non-memory work otherwise).
template <typename V, int KC, typename I>
__global__ __launch_bounds__(256) void k_xor_encode(const V *__restrict__ src, V *__restrict__ rep,
                                                    uint64_t nblocks, int k_rt, int Lv_rt) {
  const int k = KC ? KC : k_rt;
  const I Lv = (I)Lv_rt, total = (I)(nblocks * (uint64_t)Lv_rt);
  for (I t = (I)blockIdx.x * (I)blockDim.x + (I)threadIdx.x; t < total; t += (I)gridDim.x * (I)blockDim.x) {
    const I b = t / Lv, c = t - b * Lv;
    const V *p = src + (uint64_t)b * (uint64_t)k * (uint64_t)Lv + c;
    V a = __builtin_nontemporal_load(p);
#pragma unroll
    for (int j = 1; j < (KC ? KC : 1); j++) a = vxor(a, __builtin_nontemporal_load(p + (uint64_t)j * Lv));
    if (!KC)
      for (int j = 1; j < k; j++) a = vxor(a, __builtin_nontemporal_load(p + (uint64_t)j * Lv));
    __builtin_nontemporal_store(a, rep + (uint64_t)b * Lv + c);
  }
}

// xor_fec_scheme.c:41-74.  status: RECOVERED when exactly the preconditions hold and the
// repair is present; REF_UB when they hold with the repair absent (NULL dereference).
template <typename V, int KC, typename I>
__global__ __launch_bounds__(256) void k_xor_decode(V *__restrict__ src, const V *__restrict__ rep,
                                                    uint64_t nblocks, int k_rt, int Lv_rt,
                                                    const uint64_t *sp, const uint64_t *rp,
                                                    uint8_t *status, uint64_t *recovered, V *__restrict__ dst) {
  const int k = KC ? KC : k_rt;
  const I Lv = (I)Lv_rt, total = (I)(nblocks * (uint64_t)Lv_rt);
  for (I t = (I)blockIdx.x * (I)blockDim.x + (I)threadIdx.x; t < total; t += (I)gridDim.x * (I)blockDim.x) {
    const I b = t / Lv, c = t - b * Lv;
    uint64_t s0 = sp[2 * (uint64_t)b], s1 = sp[2 * (uint64_t)b + 1];
    if (k < 64) { s0 &= (1ull << k) - 1; s1 = 0; } else if (k < 128) s1 &= (1ull << ((k - 64) & 63)) - 1;
    const int cur_ss = __popcll(s0) + __popcll(s1);
    const int cur_rs = (int)(rp[2 * (uint64_t)b] & 1);
    int st = FECGPU_BLOCK_NOTHING, miss = -1;
    if (cur_ss + cur_rs == k) {
      if (!cur_rs) st = FECGPU_BLOCK_REF_UB;
      else {
        st = FECGPU_BLOCK_RECOVERED;
        uint64_t m0 = ~s0, m1 = ~s1;
        if (k < 64) { m0 &= (1ull << k) - 1; m1 = 0; } else if (k < 128) m1 &= (1ull << ((k - 64) & 63)) - 1;
        miss = m1 ? 127 - __clzll(m1) : 63 - __clzll(m0);  // LAST missing index (:54-58)
      }
    }
    if (st == FECGPU_BLOCK_RECOVERED) {  // streaming rows: non-temporal like the encode
      const V *p = src + (uint64_t)b * (uint64_t)k * Lv + c;
      V a = __builtin_nontemporal_load(rep + (uint64_t)b * Lv + c);
      if (KC) {  // exactly one source is missing: the k - 1 present rows, loads back to back
#pragma unroll
        for (int jj = 0; jj < (KC ? KC - 1 : 1); jj++)
          a = vxor(a, __builtin_nontemporal_load(p + (uint64_t)(jj + (jj >= miss)) * Lv));
      } else {
        for (int j = 0; j < k; j++)
          if (j != miss) a = vxor(a, __builtin_nontemporal_load(p + (uint64_t)j * Lv));
      }
      // dst: one row per block (the recovered symbol in a row of its own, as fec_recover allocates it
      // anew, :54-58); else in place, at the missing source's slot
      __builtin_nontemporal_store(a, dst ? dst + (uint64_t)b * Lv + c : src + ((uint64_t)b * k + miss) * Lv + c);
    }
    if (c == 0) {
      status[b] = (uint8_t)st;
      recovered[2 * (uint64_t)b] = (st == FECGPU_BLOCK_RECOVERED && miss < 64) ? 1ull << miss : 0;
      recovered[2 * (uint64_t)b + 1] = (st == FECGPU_BLOCK_RECOVERED && miss >= 64) ? 1ull << (miss - 64) : 0;
    }
  }
}

// k = 2..8 and 16 get a compile-time row count; other k take the runtime loop.
struct XorEnc {
  template <typename V, int KC, typename I, typename... A>
  static void go(uint32_t grid, hipStream_t s, A... a) {
    hipLaunchKernelGGL((k_xor_encode<V, KC, I>), dim3(grid), dim3(256), 0, s, a...);
  }
};
struct XorDec {
  template <typename V, int KC, typename I, typename... A>
  static void go(uint32_t grid, hipStream_t s, A... a) {
    hipLaunchKernelGGL((k_xor_decode<V, KC, I>), dim3(grid), dim3(256), 0, s, a...);
  }
};
template <typename V, typename OP, typename I, typename... A>
static void xor_dispatch_k(uint32_t k, uint32_t grid, hipStream_t s, A... a) {
  switch (k) {
    case 2: OP::template go<V, 2, I>(grid, s, a...); break;
    case 3: OP::template go<V, 3, I>(grid, s, a...); break;
    case 4: OP::template go<V, 4, I>(grid, s, a...); break;
    case 5: OP::template go<V, 5, I>(grid, s, a...); break;
    case 6: OP::template go<V, 6, I>(grid, s, a...); break;
    case 8: OP::template go<V, 8, I>(grid, s, a...); break;
    case 16: OP::template go<V, 16, I>(grid, s, a...); break;
    default: OP::template go<V, 0, I>(grid, s, a...); break;
  }
}
// 32-bit element indices: a batch with more index positions than that runs as several launches
// (xor_sub_batch), so one instantiation per (vector width, k) serves every size.
static uint64_t xor_sub_batch(uint64_t nblocks, int Lv, uint32_t grid) {
  const uint64_t lim = ((1ull << 32) - 1 - (uint64_t)grid * 256) / (uint64_t)Lv;
  return nblocks < lim ? nblocks : lim;
}

// FEC frames for batched repair symbols (the block framework's get_repair_payload_from_queue +
// write_fec_frame, block_framework_sender.h:100-133, protoops/write_fec_frame.c): frame (b, i) =
// 0x2a | BE16(len << 1 | fin=1) | offset=1 | BE64((fbn_b << 8) | i) | nss | nrs | repair bytes.
// One thread per output dword; the payload sits 14 bytes into the frame, so each output dword
// is assembled from two aligned source dwords with v_alignbyte.  Bytes past 14 + len are zeroed.
__device__ __forceinline__ uint32_t frame_header_byte(int o, uint32_t len, uint64_t raw, uint32_t nss, uint32_t nrs) {
  const uint32_t v16 = (len << 1) | 1u;
  switch (o) {
    case 0: return 0x2a;
    case 1: return (v16 >> 8) & 0xff;
    case 2: return v16 & 0xff;
    case 3: return 1;
    case 12: return nss;
    case 13: return nrs;
    default: return (uint32_t)(raw >> (8 * (11 - o))) & 0xff;  // o = 4..11, big-endian
  }
}

__global__ void k_write_repair_frames(const uint32_t *__restrict__ rep, uint64_t nframes, uint32_t r, uint32_t Lw,
                                      uint32_t len, uint32_t fbn_base, const uint32_t *fbn, uint32_t nss,
                                      uint32_t nrs, uint32_t *__restrict__ frames, uint32_t fw) {
  const uint64_t total = nframes * fw;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t f = t / fw;
    const uint32_t w = (uint32_t)(t - f * fw);
    const uint64_t b = f / r;
    const uint32_t i = (uint32_t)(f - b * r);
    const uint32_t *row = rep + f * (uint64_t)Lw;
    uint32_t out;
    if (w >= 4) {  // bytes 4w .. 4w+3 = payload bytes 4w-14 .. 4w-11 = row dwords (w-4) [2..3], (w-3) [0..1]
      const uint32_t lo = (w - 4) < Lw ? row[w - 4] : 0u, hi = (w - 3) < Lw ? row[w - 3] : 0u;
      out = __builtin_amdgcn_alignbyte(hi, lo, 2);
    } else {
      const uint32_t fb = fbn ? fbn[b] : (uint32_t)((fbn_base + b) & 0xffffffu);
      const uint64_t raw = ((uint64_t)fb << 8) | i;
      out = 0;
      for (int q = 0; q < 4; q++) {
        const int o = 4 * (int)w + q;
        const uint32_t byte = o < 14 ? frame_header_byte(o, len, raw, nss, nrs)
                                     : (row[0] >> (8 * (o - 14))) & 0xff;  // o = 14, 15: payload 0, 1
        out |= byte << (8 * q);
      }
    }
    // zero the bytes past the frame's end (14 + len) within the slot
    const int valid = (int)(14 + len) - 4 * (int)w;
    if (valid <= 0) out = 0;
    else if (valid < 4) out &= (1u << (8 * valid)) - 1u;
    frames[f * fw + w] = out;
  }
}

// Fast path (16-B aligned rows and slots): a thread per 16-B output chunk over all frames, so the
// frame slots are written as one contiguous run (a wave per frame left 52 of its 128 lane slots
// idle on 1216-B slots).  Chunk c of a frame holds payload bytes 16c-14 .. 16c+1 = source dwords
// 4c-4 .. 4c shifted by 2 bytes; chunk 0 is the header.  I: 32-bit chunk indices when they fit.
template <typename I>
__global__ __launch_bounds__(256) void k_write_repair_frames16(const uint32_t *__restrict__ rep, uint64_t nframes,
                                                               uint32_t r, uint32_t Lw, uint32_t len,
                                                               uint32_t fbn_base, const uint32_t *fbn, uint32_t nss,
                                                               uint32_t nrs, uint32_t *__restrict__ frames,
                                                               uint32_t fw) {
  const I nchunks = (I)(fw / 4), total = (I)(nframes * (fw / 4));
  u32x4 *out = reinterpret_cast<u32x4 *>(frames);
  for (I t = (I)blockIdx.x * (I)blockDim.x + (I)threadIdx.x; t < total; t += (I)gridDim.x * (I)blockDim.x) {
    const I f = t / nchunks;
    const uint32_t c = (uint32_t)(t - f * nchunks);
    const uint32_t *row = rep + (uint64_t)f * Lw;
    u32x4 o;
    if (c == 0) {
      const uint64_t b = (uint64_t)f / r;
      const uint32_t i = (uint32_t)((uint64_t)f - b * r);
      const uint32_t fb = fbn ? fbn[b] : (uint32_t)((fbn_base + b) & 0xffffffu);
      const uint64_t raw = ((uint64_t)fb << 8) | i;
      uint32_t wv[4];
      for (int w = 0; w < 4; w++) {
        uint32_t v = 0;
        for (int q = 0; q < 4; q++) {
          const int ob = 4 * w + q;
          const uint32_t byte = ob < 14 ? frame_header_byte(ob, len, raw, nss, nrs) : (row[0] >> (8 * (ob - 14))) & 0xff;
          v |= byte << (8 * q);
        }
        wv[w] = v;
      }
      o = u32x4{wv[0], wv[1], wv[2], wv[3]};
    } else {
      const uint32_t d0 = 4 * (c - 1);
      const u32x4 a = d0 + 3 < Lw ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(row + d0))
                                  : u32x4{0, 0, 0, 0};
      const uint32_t e = d0 + 4 < Lw ? row[d0 + 4] : 0u;
      o = u32x4{__builtin_amdgcn_alignbyte(a.y, a.x, 2), __builtin_amdgcn_alignbyte(a.z, a.y, 2),
                __builtin_amdgcn_alignbyte(a.w, a.z, 2), __builtin_amdgcn_alignbyte(e, a.w, 2)};
    }
    const int valid = (int)(14 + len) - 16 * (int)c;  // zero the slot past the frame's end
    if (valid < 16) {
      uint32_t m[4];
      for (int w = 0; w < 4; w++) {
        const int vb = valid - 4 * w;
        m[w] = vb <= 0 ? 0u : vb >= 4 ? 0xffffffffu : (1u << (8 * vb)) - 1u;
      }
      o = u32x4{o.x & m[0], o.y & m[1], o.z & m[2], o.w & m[3]};
    }
    __builtin_nontemporal_store(o, out + t);
  }
}

__global__ void k_synth_fill(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t offset) {
  // one 8-byte word of the stream per thread; unaligned head/tail handled bytewise
  const uint64_t first = offset >> 3, last = (offset + nbytes + 7) >> 3;
  for (uint64_t w = first + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < last;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (w + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    const uint64_t o0 = w << 3;
    if (o0 >= offset && o0 + 8 <= offset + nbytes && ((o0 - offset) & 7) == 0 &&
        (((uintptr_t)(dst + (o0 - offset))) & 7) == 0) {
      *reinterpret_cast<uint64_t *>(dst + (o0 - offset)) = z;
    } else {
      for (int i = 0; i < 8; i++) {
        uint64_t o = o0 + i;
        if (o >= offset && o < offset + nbytes) dst[o - offset] = (uint8_t)(z >> (8 * i));
      }
    }
  }
}

// =============================================================================================
// Launch configuration
// =============================================================================================
static int pick_rt(uint32_t r) { return r >= 16 ? 16 : r >= 8 ? 8 : r >= 4 ? 4 : r >= 2 ? 2 : 1; }

static uint32_t grid_for(uint64_t units) {
  const uint64_t cap = 1u << 22;
  return (uint32_t)(units < cap ? (units ? units : 1) : cap);
}

static int check_common(const void *a, const void *b, uint64_t nblocks, uint32_t k, uint32_t r,
                        uint32_t L) {
  if (nblocks == 0) return FECGPU_OK;
  if (!a || !b) return set_err(FECGPU_ERR_INVALID, "%s", "NULL symbol buffer");
  if (k < 1 || k > FECGPU_MAX_K) return set_err(FECGPU_ERR_INVALID, "%s", "k out of range [1,128]");
  if (r > FECGPU_MAX_R) return set_err(FECGPU_ERR_INVALID, "%s", "r out of range [0,128]");
  if (L == 0 || (L & 3) || L > 65532) return set_err(FECGPU_ERR_INVALID, "%s", "symbol_size must be a positive multiple of 4 (<= 65532)");
  if (((uintptr_t)a & 3) || ((uintptr_t)b & 3)) return set_err(FECGPU_ERR_INVALID, "%s", "buffers must be 4-byte aligned");
  return FECGPU_OK;
}

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

const char *fecgpu_version(void) { return FECGPU_VERSION; }
const char *fecgpu_last_error(void) { return g_err; }

int fecgpu_init(int device) {
  std::call_once(g_knob_once, knobs_default);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device)
    return set_err(FECGPU_ERR_NO_DEVICE, "%s", "no HIP device");
  hipDeviceProp_t p;
  HIPCHK(hipGetDeviceProperties(&p, device));
  if (strncmp(p.gcnArchName, "gfx950", 6) != 0)
    return set_err(FECGPU_ERR_NO_DEVICE, "device is %s, engine is built for gfx950", p.gcnArchName);
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  if (cur != device) HIPCHK(hipSetDevice(device));
  const int rc = bs_table_check();
  if (cur != device) HIPCHK(hipSetDevice(cur));
  return rc;
}

// The values each knob accepts: a tile of 3 repairs would
// dispatch a 16-repair body while stepping r0 by 3, a negative group cap would become a huge
// unsigned one.
static bool knob_value_ok(int id, int v) {
  switch (id) {
    case K_PLAN: return v >= PLAN_AUTO && v <= PLAN_WREG;
    case K_ENC_RT: return v == 0 || v == 1 || v == 2 || v == 4 || v == 8 || v == 16;
    case K_ENC_W: return v >= 0 && v <= 4;
    case K_ENC_BW: return v == 1 || v == 2 || v == 4;
    case K_RING: return v == 0 || v == 2 || (v == 4 && FEC_BS2_HAS_RT4) || (v == 8 && FEC_BS2_HAS_RT8);
    case K_WINDOW_SC: return v >= 0 && v <= 2;
    case K_GROUP: case K_MIN_GROUPS: return v >= 0;
    case K_DEC_WAVES: return v >= 0 && v <= 8;
    case K_YIELD_SLICE_KB: return v >= 0 && v <= (1 << 20);
    case K_YIELD_DEPTH: return v >= 1 && v <= 16;
    case K_YIELD_GATE_US: return v >= 0 && v <= 10000;
    case K_YIELD_STREAMS: return v >= 1 && v <= 4;
    case K_YIELD_WINDOW_MS: return v >= 0 && v <= 600000;
    case K_SVC_RESERVE_CUS: return v >= -64 && v <= 128;
    case K_HOST_ALLOC: return v >= 0 && v <= 2;
    case K_ZC_CUS: return v >= 0 && v <= 256;
    case K_INTERLEAVE: return v >= 0 && v <= 3;
    default: return v == 0 || v == 1;  // on / off knobs
  }
}

int fecgpu_set_knob(const char *name, int value) {
  std::call_once(g_knob_once, knobs_default);
  for (int i = 0; i < K_N; i++)
    if (name && !strcmp(name, kKnobName[i])) {
      if (!knob_value_ok(i, value)) return set_err(FECGPU_ERR_INVALID, "value out of range for knob %s", name);
      g_knob[i].store(value, std::memory_order_relaxed);
      return FECGPU_OK;
    }
  return set_err(FECGPU_ERR_INVALID, "unknown knob %s", name ? name : "(null)");
}

int fecgpu_get_knob(const char *name, int *value) {
  std::call_once(g_knob_once, knobs_default);
  for (int i = 0; i < K_N; i++)
    if (name && value && !strcmp(name, kKnobName[i])) {
      *value = g_knob[i].load(std::memory_order_relaxed);
      return FECGPU_OK;
    }
  return set_err(FECGPU_ERR_INVALID, "unknown knob %s", name ? name : "(null)");
}

#ifdef FEC_STAMP
int fecgpu_debug_stamps(uint64_t out[16]) {  // diagnostic builds: the phase stamps of the last launch
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fec_stamps), 16 * sizeof(uint64_t)));
  return FECGPU_OK;
}
#endif

void fecgpu_host_registry_stats(uint64_t *hits, uint64_t *misses);  // host_path.hip (library-internal)
void fecgpu_host_yield_stats(uint64_t *slices, uint64_t *waits);      // host_path.hip (library-internal)

void fecgpu_get_stats(fecgpu_stats_t *out) {
  out->encode_calls = g_stats[0].load();
  out->encode_blocks = g_stats[1].load();
  out->decode_calls = g_stats[2].load();
  out->decode_blocks = g_stats[3].load();
  fecgpu_host_registry_stats(&out->pinned_registry_hits, &out->pinned_registry_misses);
  fecgpu_host_yield_stats(&out->yield_slices, &out->yield_waits);
}

// Encode tiling: repairs per wave (RT) and waves per workgroup sharing the source stream.
// Knobs enc_tile_rt / enc_tile_waves (FECGPU_ENC_TILE="RT,W") override (A/B experiments).
struct EncTile { int rt, waves; };
static EncTile pick_enc_tile(uint32_t r) {
  if (const int a = knob(K_ENC_RT)) {  // knobs enc_tile_rt / enc_tile_waves (FECGPU_ENC_TILE="RT,W")
    const int b = knob(K_ENC_W);
    return {a, b >= 1 && b <= 4 ? b : 1};
  }
  // measured (profiles/r01_tile_ab.log): splitting repairs over waves repeats the transpose and
  // table work per wave and loses more VALU than the occupancy gains (k32r8 4x2: +34 %,
  // k64r16 8x2: +10 %), so one wave carries up to 16 repairs
  return {pick_rt(r), 1};
}

int fecgpu_rlc_encode(const void *src, void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                      uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn, void *stream) {
  int rc = check_common(src, rep, nblocks, k, r, symbol_size);
  if (rc || nblocks == 0 || r == 0) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (nblocks <= kSmallLdsMaxBlocks && knob(K_SMALL_LDS) && !knob(K_ENC_RT)) {
    const EncLdsLayout Y((int)k, (int)r, (int)symbol_size, r <= 4 ? 4 : r <= 8 ? 8 : 16);
    if (Y.bytes <= 65536) {
      const uint32_t grid = (uint32_t)nblocks;
      if (r <= 4)
        hipLaunchKernelGGL(k_rlc_encode_lds<4>, dim3(grid), dim3(kLdsThreads), Y.bytes, s, (const uint8_t *)src,
                           (uint8_t *)rep, nblocks, (int)k, (int)r, (int)symbol_size, fbn_base, fbn);
      else if (r <= 8)
        hipLaunchKernelGGL(k_rlc_encode_lds<8>, dim3(grid), dim3(kLdsThreads), Y.bytes, s, (const uint8_t *)src,
                           (uint8_t *)rep, nblocks, (int)k, (int)r, (int)symbol_size, fbn_base, fbn);
      else
        hipLaunchKernelGGL(k_rlc_encode_lds<16>, dim3(grid), dim3(kLdsThreads), Y.bytes, s, (const uint8_t *)src,
                           (uint8_t *)rep, nblocks, (int)k, (int)r, (int)symbol_size, fbn_base, fbn);
      HIPCHK(hipGetLastError());
      g_stats[0]++;
      g_stats[1] += nblocks;
      return FECGPU_OK;
    }
  }
  if (int rc2 = bs_table_check()) return rc2;
  const BsCfg cfg = pick_bs_cfg((int)symbol_size);
  const EncTile et = pick_enc_tile(r);
  const int rt = et.rt;
  if (use_ring(rt, k, cfg, true)) {
    for (int r0 = 0; r0 < (int)r; r0 += rt * et.waves) {
      FEC_BS2_DISPATCH(launch_encode_bs2, (const uint8_t *)src, (uint8_t *)rep, nblocks, (int)k, (int)r,
                       (int)symbol_size, cfg, fbn_base, fbn, r0, et.waves, (uint64_t)k * symbol_size, 1u, s)
    }
  } else {
    for (int r0 = 0; r0 < (int)r; r0 += et.rt * et.waves) {
      FEC_BS_DISPATCH(launch_encode_bs, (const uint8_t *)src, (uint8_t *)rep, nblocks, (int)k, (int)r,
                      (int)symbol_size, cfg, fbn_base, fbn, r0, et.waves, (uint64_t)k * symbol_size, 1u, s)
    }
  }
  HIPCHK(hipGetLastError());
  g_stats[0]++;
  g_stats[1] += nblocks;
  return FECGPU_OK;
}

int fecgpu_rlc_encode_rows(const uint64_t *src_rows, const uint64_t *rep_rows, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn, void *stream) {
  int rc = check_common(src_rows, rep_rows, nblocks, k, r, symbol_size);
  if (rc || nblocks == 0 || r == 0) return rc;
  if (int rc2 = bs_table_check()) return rc2;
  hipStream_t s = (hipStream_t)stream;
  const BsCfg cfg = pick_bs_cfg((int)symbol_size);
  const int rt = pick_rt(r);
  for (int r0 = 0; r0 < (int)r; r0 += rt) {
    FEC_BS_DISPATCH(launch_encode_rows, src_rows, rep_rows, nblocks, (int)k, (int)r, (int)symbol_size, cfg, fbn_base,
                    fbn, r0, s)
  }
  HIPCHK(hipGetLastError());
  g_stats[0]++;
  g_stats[1] += nblocks;
  return FECGPU_OK;
}

int fecgpu_rlc_window_encode(const void *symbols, uint64_t nwindows, uint32_t step, uint32_t k, uint32_t r,
                             uint32_t symbol_size, void *rep, void *stream) {
  int rc = check_common(symbols, rep, nwindows, k, r, symbol_size);
  if (rc || nwindows == 0 || r == 0) return rc;
  if (step == 0) return set_err(FECGPU_ERR_INVALID, "%s", "window step must be >= 1");
  if (int rc2 = bs_table_check()) return rc2;
  const BsCfg cfg = pick_bs_cfg((int)symbol_size);
  const int rt = pick_rt(r);
  if (!launch_encode_sc((const uint8_t *)symbols, (uint8_t *)rep, nwindows, (int)k, (int)r, (int)symbol_size,
                        (uint64_t)step * symbol_size, (hipStream_t)stream)) {
    for (int r0 = 0; r0 < (int)r; r0 += rt) {
      FEC_BS_DISPATCH(launch_encode_bs, (const uint8_t *)symbols, (uint8_t *)rep, nwindows, (int)k, (int)r,
                      (int)symbol_size, cfg, 0u, nullptr, r0, 1, (uint64_t)step * symbol_size, 0u,
                      (hipStream_t)stream)
    }
  }
  HIPCHK(hipGetLastError());
  g_stats[0]++;
  g_stats[1] += nwindows;
  return FECGPU_OK;
}

int fecgpu_rlc_window_encode_table(const void *symbols, uint64_t nrows, const uint32_t *wrow, uint64_t nwindows,
                                   uint32_t k, uint32_t r, uint32_t symbol_size, void *rep, void *stream) {
  int rc = check_common(symbols, rep, nwindows, k, r, symbol_size);
  if (rc || nwindows == 0 || r == 0) return rc;
  if (!wrow || nrows < k) return set_err(FECGPU_ERR_INVALID, "%s", "window start table missing or stream shorter than k");
  if (symbol_size % 16 || ((uintptr_t)symbols | (uintptr_t)rep) % 16)
    return set_err(FECGPU_ERR_INVALID, "%s", "window table encode needs 16-B rows (symbol_size %% 16 == 0, aligned)");
  if (int rc2 = bs_table_check()) return rc2;
  if (!launch_encode_sc((const uint8_t *)symbols, (uint8_t *)rep, nwindows, (int)k, (int)r, (int)symbol_size, 0,
                        (hipStream_t)stream, wrow, nrows))
    return set_err(FECGPU_ERR_INVALID, "%s", "window table encode: stream of 2 GiB or more, or window_sc knob 0");
  HIPCHK(hipGetLastError());
  g_stats[0]++;
  g_stats[1] += nwindows;
  return FECGPU_OK;
}

int fecgpu_xor_encode(const void *src, void *rep, uint64_t nblocks, uint32_t k, uint32_t symbol_size,
                      void *stream) {
  int rc = check_common(src, rep, nblocks, k, 1, symbol_size);
  if (rc || nblocks == 0) return rc;
  hipStream_t s = (hipStream_t)stream;
  const bool v4 = (symbol_size % 16) == 0 && ((uintptr_t)src % 16) == 0 && ((uintptr_t)rep % 16) == 0;
  const int Lv = (int)(v4 ? symbol_size / 16 : symbol_size / 4);
  const uint32_t gmax = 1u << 20;
  for (uint64_t b0 = 0, n; b0 < nblocks; b0 += n) {
    n = xor_sub_batch(nblocks - b0, Lv, gmax);
    const uint64_t total = n * (uint64_t)Lv;
    const uint32_t grid = (uint32_t)((total + 255) / 256 < gmax ? (total + 255) / 256 : gmax);
    const uint64_t so = b0 * k * (uint64_t)Lv, ro = b0 * (uint64_t)Lv;  // in vectors
    if (v4)
      xor_dispatch_k<u32x4, XorEnc, uint32_t>(k, grid, s, (const u32x4 *)src + so, (u32x4 *)rep + ro, n, (int)k, Lv);
    else
      xor_dispatch_k<uint32_t, XorEnc, uint32_t>(k, grid, s, (const uint32_t *)src + so, (uint32_t *)rep + ro, n,
                                                 (int)k, Lv);
  }
  HIPCHK(hipGetLastError());
  g_stats[0]++;
  g_stats[1] += nblocks;
  return FECGPU_OK;
}

size_t fecgpu_rlc_decode_workspace(uint64_t nblocks, uint32_t k, uint32_t r) {
  return (size_t)nblocks * ws_layout(k, r).stride;
}

static int decode_args(const void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r, uint32_t L,
                       const void *a, const void *b, const void *c, const void *d, void *ws, size_t wsb) {
  int rc = check_common(src, rep, nblocks, k, r, L);
  if (rc) return rc;
  if (nblocks && (!a || !b || !c || !d || !ws)) return set_err(FECGPU_ERR_INVALID, "%s", "NULL mask/status/workspace");
  if (nblocks && wsb < fecgpu_rlc_decode_workspace(nblocks, k, r))
    return set_err(FECGPU_ERR_NOMEM, "%s", "decode workspace too small");
  return FECGPU_OK;
}

// Up to this many blocks a wave per block plans fastest: the lane-parallel plans (reg / tile / lane)
// take one lane's dependent chain whatever the batch, e.g. k32 e8 70 us against the register wave
// plan's 17-26 us at 65-4096 blocks; they win from ~8192 blocks on
// (profiles/r02_plan_crossover_wreg.log).
constexpr uint64_t kPlanWaveMaxBlocks = 4096;

static int decode_plan_impl(uint64_t nblocks, uint32_t k, uint32_t r, uint32_t fbn_base, const uint32_t *fbn,
                            const uint32_t *seeds, const uint64_t *src_present, const uint64_t *rep_present,
                            void *workspace, size_t workspace_bytes, void *stream) {
  static const uint32_t dummy = 0;
  int rc = decode_args(&dummy, &dummy, nblocks, k, r, 4, src_present, rep_present, &dummy, &dummy, workspace,
                       workspace_bytes);
  if (rc || nblocks == 0) return rc;
  hipStream_t s = (hipStream_t)stream;
  uint8_t *ws = (uint8_t *)workspace;
  const size_t lane_lds = plan_lane_lds(k, r);
  // knob "plan" (FECGPU_PLAN=reg|tile|lane|wave) overrides the size rule (A/B experiments; the tests
  // compare the plan kernels on the same inputs through fecgpu_set_knob)
  int force = knob(K_PLAN);
  // the wave kernel takes the register plan wherever it fits unless the LDS wave plan is forced
  const int wreg = force != PLAN_WAVE;
  if (force == PLAN_WREG) force = PLAN_WAVE;
  const uint32_t em = ws_layout(k, r).em;
  // up to kPlanWaveMaxBlocks blocks (the synchronous hooks run one): every block gets its own wave
  // and the wave plan's row-parallel elimination, instead of a lane's serial replay -- one-block
  // recover hook 47 -> 40 us (profiles/r02_hook_plan.log)
  if (force == 0 && nblocks <= kPlanWaveMaxBlocks && plan_lds_bytes(k, r) <= 65536) force = PLAN_WAVE;
  if ((force == 0 || force == 3) && k <= 32 && em <= 8) {
    const size_t reg_lds = 768 + 64 * (size_t)plan_out_row(ws_layout(k, r).stride);
    const uint64_t groups = (nblocks + 63) / 64;
#define FEC_PLAN_REG(KD, EM)                                                                         \
  hipLaunchKernelGGL((k_rlc_plan_reg<KD, EM>), dim3(grid_for(groups)), dim3(64), reg_lds, s, nblocks, \
                     (int)k, (int)r, fbn_base, fbn, seeds, src_present, rep_present, ws)
    if (k <= 16 && em <= 4) FEC_PLAN_REG(4, 4);
    else if (k <= 16) FEC_PLAN_REG(4, 8);
    else if (em <= 4) FEC_PLAN_REG(8, 4);
    else FEC_PLAN_REG(8, 8);
#undef FEC_PLAN_REG
    HIPCHK(hipGetLastError());
    return FECGPU_OK;
  }
  if ((force == 0 || force == 4) && k <= 64 && em <= 16) {  // FECGPU_PLAN=tile
    constexpr int BPW = 16, EM = 16;  // k_rlc_plan_tile<4, 16>: 4 lanes per block
    const size_t tile_lds = 768 + (size_t)BPW * EM * pad16(k) + (size_t)BPW * plan_out_row(ws_layout(k, r).stride);
    if (tile_lds > 65536) {
      static bool raised = false;
      if (!raised) {
        HIPCHK(hipFuncSetAttribute((const void *)k_rlc_plan_tile<4, 16>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        raised = true;
      }
    }
    const uint64_t groups = (nblocks + BPW - 1) / BPW;
    hipLaunchKernelGGL((k_rlc_plan_tile<4, 16>), dim3(grid_for(groups)), dim3(64), tile_lds, s, nblocks,
                       (int)k, (int)r, fbn_base, fbn, seeds, src_present, rep_present, ws);
    HIPCHK(hipGetLastError());
    return FECGPU_OK;
  }
  if (force != 1 && (lane_lds <= 64 * 1024 || force == 2) && lane_lds <= 160 * 1024) {
    if (lane_lds > 65536) {
      static bool raised = false;
      if (!raised) {
        HIPCHK(hipFuncSetAttribute((const void *)k_rlc_plan_lane, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024));
        raised = true;
      }
    }
    const uint64_t groups = (nblocks + 63) / 64;
    hipLaunchKernelGGL(k_rlc_plan_lane, dim3(grid_for(groups)), dim3(64), lane_lds, s, nblocks, (int)k,
                       (int)r, fbn_base, fbn, seeds, src_present, rep_present, ws);
  } else {
    const size_t plan_lds = plan_lds_bytes(k, r);
    if (plan_lds > 65536) {
      static bool raised = false;
      if (!raised) {
        HIPCHK(hipFuncSetAttribute((const void *)k_rlc_plan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)plan_lds));
        raised = true;
      }
    }
    if (wreg && em <= 8 && k + em <= 64) {
#define FEC_PLAN_WREG(EM)                                                                                  \
  hipLaunchKernelGGL((k_rlc_plan_wreg<EM>), dim3(grid_for(nblocks)), dim3(64), plan_lds, s, nblocks, (int)k, \
                     (int)r, fbn_base, fbn, seeds, src_present, rep_present, ws)
      if (em <= 4) FEC_PLAN_WREG(4);
      else FEC_PLAN_WREG(8);
#undef FEC_PLAN_WREG
    } else {
      hipLaunchKernelGGL(k_rlc_plan, dim3(grid_for(nblocks)), dim3(64), plan_lds, s, nblocks, (int)k, (int)r,
                         fbn_base, fbn, seeds, src_present, rep_present, ws);
    }
  }
  HIPCHK(hipGetLastError());
  return FECGPU_OK;
}

int fecgpu_rlc_decode_plan(uint64_t nblocks, uint32_t k, uint32_t r, uint32_t fbn_base, const uint32_t *fbn,
                           const uint64_t *src_present, const uint64_t *rep_present, void *workspace,
                           size_t workspace_bytes, void *stream) {
  return decode_plan_impl(nblocks, k, r, fbn_base, fbn, nullptr, src_present, rep_present, workspace,
                          workspace_bytes, stream);
}

int fecgpu_rlc_decode_plan_seeded(uint64_t nblocks, uint32_t k, uint32_t r, const uint32_t *rep_seed,
                                  const uint64_t *src_present, const uint64_t *rep_present, void *workspace,
                                  size_t workspace_bytes, void *stream) {
  if (nblocks && r && !rep_seed) return set_err(FECGPU_ERR_INVALID, "%s", "NULL rep_seed");
  return decode_plan_impl(nblocks, k, r, 0, nullptr, rep_seed, src_present, rep_present, workspace,
                          workspace_bytes, stream);
}

static int launch_finalize(uint64_t nblocks, uint32_t k, uint32_t r, uint8_t *status, uint64_t *recovered,
                           const uint8_t *ws, hipStream_t s) {
  const uint32_t fgrid = (uint32_t)((nblocks + 255) / 256 < 65536 ? (nblocks + 255) / 256 : 65536);
  hipLaunchKernelGGL(k_rlc_finalize, dim3(fgrid), dim3(256), 0, s, nblocks, (int)k, (int)r, ws, status, recovered);
  HIPCHK(hipGetLastError());
  return FECGPU_OK;
}

// The data pass of decode; recovered symbols go to dst (same [block][k][L] layout as src; dst == src
// is the in-place form).  Inputs are only ever read from src/rep, outputs only written to dst.
static int decode_apply_impl(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k,
                             uint32_t r, uint32_t symbol_size, uint8_t *status, uint64_t *recovered,
                             void *workspace, size_t workspace_bytes, hipStream_t s, int dst_rows = 0) {
  static const uint64_t dummy = 0;
  int rc = decode_args(src, rep, nblocks, k, r, symbol_size, &dummy, &dummy, status, recovered, workspace,
                       workspace_bytes);
  if (rc || nblocks == 0) return rc;
  if (!dst) return set_err(FECGPU_ERR_INVALID, "%s", "NULL output buffer");
  if ((uintptr_t)dst % 4) return set_err(FECGPU_ERR_INVALID, "%s", "output buffer must be 4-byte aligned");
  g_stats[2]++;  // decode calls / blocks are counted at the data pass (fecgpu_rlc_decode and the staged API)
  g_stats[3] += nblocks;
  uint8_t *ws = (uint8_t *)workspace;
  const WsLayout L = ws_layout(k, r);
  // decode passes: the smallest tile covering e_max (one pass, finalize fused) up to 16 unknowns
  const int rt = L.em <= 1 ? 1 : L.em <= 2 ? 2 : L.em <= 4 ? 4 : L.em <= 8 ? 8 : 16;
  if (r == 0) return launch_finalize(nblocks, k, r, status, recovered, ws, s);
  if (int rc2 = bs_table_check()) return rc2;
  const BsCfg cfg = pick_bs_cfg((int)symbol_size);
  const bool fused = (int)L.em <= rt;  // one pass covers every unknown of every block
  const bool ring = use_ring(rt, k, cfg, false);
  for (int r0 = 0; r0 < (int)L.em; r0 += rt) {
    if (ring) {
      FEC_BS2_DISPATCH_DEC(launch_recover_bs2, (uint8_t *)src, (const uint8_t *)rep, nblocks, (int)k, (int)r,
                       (int)symbol_size, cfg, ws, r0, fused ? status : nullptr, fused ? recovered : nullptr, s,
                       (uint8_t *)dst, dst_rows)
    } else {
      FEC_BS_DISPATCH(launch_recover_bs, (uint8_t *)src, (const uint8_t *)rep, nblocks, (int)k, (int)r,
                      (int)symbol_size, cfg, ws, r0, fused ? status : nullptr, fused ? recovered : nullptr, s,
                      (uint8_t *)dst, dst_rows)
    }
  }
  HIPCHK(hipGetLastError());
  return fused ? FECGPU_OK : launch_finalize(nblocks, k, r, status, recovered, ws, s);
}

int fecgpu_rlc_decode_apply(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                            uint32_t symbol_size, uint8_t *status, uint64_t *recovered, void *workspace,
                            size_t workspace_bytes, void *stream) {
  return decode_apply_impl(src, rep, src, nblocks, k, r, symbol_size, status, recovered, workspace,
                           workspace_bytes, (hipStream_t)stream);
}

int fecgpu_rlc_decode_apply_to(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k,
                               uint32_t r, uint32_t symbol_size, uint8_t *status, uint64_t *recovered,
                               void *workspace, size_t workspace_bytes, void *stream) {
  return decode_apply_impl(src, rep, dst, nblocks, k, r, symbol_size, status, recovered, workspace,
                           workspace_bytes, (hipStream_t)stream);
}

int fecgpu_rlc_decode_apply_packed(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k,
                                   uint32_t r, uint32_t symbol_size, uint8_t *status, uint64_t *recovered,
                                   void *workspace, size_t workspace_bytes, void *stream) {
  const uint32_t em = k < r ? k : r;
  return decode_apply_impl(src, rep, dst, nblocks, k, r, symbol_size, status, recovered, workspace,
                           workspace_bytes, (hipStream_t)stream, em ? (int)em : 1);
}

int fecgpu_rlc_decode_rows(const uint64_t *src_rows, const uint64_t *rep_rows, uint64_t nblocks, uint32_t k,
                           uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed, const uint64_t *src_present,
                           const uint64_t *rep_present, uint8_t *status, uint64_t *recovered, void *workspace,
                           size_t workspace_bytes, void *stream) {
  int rc = decode_args(src_rows, rep_rows, nblocks, k, r, symbol_size, src_present, rep_present, status, recovered,
                       workspace, workspace_bytes);
  if (rc || nblocks == 0) return rc;
  if (r && !rep_seed) return set_err(FECGPU_ERR_INVALID, "%s", "NULL rep_seed");
  hipStream_t s = (hipStream_t)stream;
  if ((rc = decode_plan_impl(nblocks, k, r, 0, nullptr, rep_seed, src_present, rep_present, workspace,
                             workspace_bytes, s)))
    return rc;
  g_stats[2]++;
  g_stats[3] += nblocks;
  uint8_t *ws = (uint8_t *)workspace;
  const WsLayout WL = ws_layout(k, r);
  if (r == 0) return launch_finalize(nblocks, k, r, status, recovered, ws, s);
  if (int rc2 = bs_table_check()) return rc2;
  const int rt = WL.em <= 1 ? 1 : WL.em <= 2 ? 2 : WL.em <= 4 ? 4 : WL.em <= 8 ? 8 : 16;
  const BsCfg cfg = pick_bs_cfg((int)symbol_size);
  const bool fused = (int)WL.em <= rt;
  // the register-prefetch recover pass for every tile size (the LDS-ring pass computes its row
  // addresses from packed buffers); dst_rows = -1 selects the row tables
  for (int r0 = 0; r0 < (int)WL.em; r0 += rt) {
    FEC_BS_DISPATCH(launch_recover_bs, (uint8_t *)src_rows, (const uint8_t *)rep_rows, nblocks, (int)k, (int)r,
                    (int)symbol_size, cfg, ws, r0, fused ? status : nullptr, fused ? recovered : nullptr, s,
                    (uint8_t *)nullptr, -1)
  }
  HIPCHK(hipGetLastError());
  return fused ? FECGPU_OK : launch_finalize(nblocks, k, r, status, recovered, ws, s);
}

extern "C++" {
template <int RT, int VEC>
static void launch_decode_small(uint8_t *src, const uint8_t *rep, uint64_t nb, int k, int r, int L, const BsCfg &c,
                                uint32_t fbn_base, const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp,
                                const uint64_t *rp, uint8_t *ws, uint8_t *status, uint64_t *recovered, uint8_t *dst,
                                hipStream_t s) {
  const size_t pl = plan_lds_bytes((uint32_t)k, (uint32_t)r), rl = RecoverLds<RT>::bytes(1, k);
  const uint32_t rec_off = pad16((uint32_t)(pl > rl ? pl : rl));  // the plan record, past both phases' scratch
  (void)ws;  // the record never leaves the workgroup
  const size_t lds = rec_off + pad16(ws_layout((uint32_t)k, (uint32_t)r).stride);
  hipLaunchKernelGGL((k_rlc_decode_small<RT, VEC>), dim3((uint32_t)nb), dim3(64), lds, s, src, rep, nb, k, r,
                     L, c.nchunks, c.chunk_bytes, fbn_base, fbn, seeds, sp, rp, rec_off, status, recovered, dst,
                     knob(K_PLAN) != PLAN_WAVE);
}
}  // extern "C++"

// Below this many blocks a decode is one launch (k_rlc_decode_small): plan and data pass per
// workgroup.  One-block recover hook p50 46 us (lane plan + data pass, two launches) -> 40 (wave
// plan, two launches) -> 37 (one launch) (profiles/r02_hook_plan.log, r02_hook_small.log; the
// first line of the latter is this path, the second the forced lane-register plan).
constexpr uint64_t kDecodeSmallMaxBlocks = 64;

// Plan + apply; recovered rows to dst (dst == src: in place).  seeds != nullptr: per-repair seeds.
static int decode_impl(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k, uint32_t r,
                       uint32_t L, uint32_t fbn_base, const uint32_t *fbn, const uint32_t *seeds,
                       const uint64_t *sp, const uint64_t *rp, uint8_t *status, uint64_t *recovered, void *ws,
                       size_t wsb, hipStream_t s) {
  int rc = decode_args(src, rep, nblocks, k, r, L, sp, rp, status, recovered, ws, wsb);
  if (rc || nblocks == 0) return rc;
  if (!dst) return set_err(FECGPU_ERR_INVALID, "%s", "NULL output buffer");
  if ((uintptr_t)dst % 4) return set_err(FECGPU_ERR_INVALID, "%s", "output buffer must be 4-byte aligned");
  const WsLayout WL = ws_layout(k, r);
  // a few blocks with their rows in LDS: one launch, the plan beside the row fetch
  if (nblocks <= kSmallLdsMaxBlocks && r > 0 && WL.em <= 16 && knob(K_PLAN) == 0 && knob(K_SMALL_LDS)) {
    const DecLdsLayout Y((int)k, (int)r, (int)L, WL.em <= 4 ? 4 : WL.em <= 8 ? 8 : 16);
    if (Y.bytes <= 65536) {
      g_stats[2]++;
      g_stats[3] += nblocks;
      const int wreg = knob(K_PLAN) != PLAN_WAVE;
#define FEC_DEC_LDS(EM)                                                                                          \
  hipLaunchKernelGGL(k_rlc_decode_lds<EM>, dim3((uint32_t)nblocks), dim3(kLdsThreads), Y.bytes, s, (const uint8_t *)src, \
                     (const uint8_t *)rep, nblocks, (int)k, (int)r, (int)L, fbn_base, fbn, seeds, sp, rp, status,      \
                     recovered, (uint8_t *)dst, wreg)
      if (WL.em <= 4) FEC_DEC_LDS(4);
      else if (WL.em <= 8) FEC_DEC_LDS(8);
      else FEC_DEC_LDS(16);
#undef FEC_DEC_LDS
      HIPCHK(hipGetLastError());
      return FECGPU_OK;
    }
  }
  // the one-launch path: a few blocks, one data pass (e <= 16), the default kernels (no knob forces a
  // plan kernel or another data path)
  if (nblocks <= kDecodeSmallMaxBlocks && r > 0 && WL.em <= 16 && knob(K_PLAN) == 0 &&
      plan_lds_bytes(k, r) <= 65536) {
    const BsCfg cfg = pick_bs_cfg((int)L);
    const int rt = WL.em <= 1 ? 1 : WL.em <= 2 ? 2 : WL.em <= 4 ? 4 : WL.em <= 8 ? 8 : 16;
    if (!use_ring(rt, k, cfg, false)) {
      if (int rc2 = bs_table_check()) return rc2;
      g_stats[2]++;
      g_stats[3] += nblocks;
      FEC_BS_DISPATCH(launch_decode_small, (uint8_t *)src, (const uint8_t *)rep, nblocks, (int)k, (int)r, (int)L,
                      cfg, fbn_base, fbn, seeds, sp, rp, (uint8_t *)ws, status, recovered, (uint8_t *)dst, s)
      HIPCHK(hipGetLastError());
      return FECGPU_OK;
    }
  }
  rc = decode_plan_impl(nblocks, k, r, fbn_base, fbn, seeds, sp, rp, ws, wsb, s);
  if (rc) return rc;
  return decode_apply_impl(src, rep, dst, nblocks, k, r, L, status, recovered, ws, wsb, s);
}

int fecgpu_rlc_decode(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                      uint32_t symbol_size, uint32_t fbn_base, const uint32_t *fbn,
                      const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                      uint64_t *recovered, void *workspace, size_t workspace_bytes, void *stream) {
  return decode_impl(src, rep, src, nblocks, k, r, symbol_size, fbn_base, fbn, nullptr, src_present, rep_present,
                     status, recovered, workspace, workspace_bytes, (hipStream_t)stream);
}

int fecgpu_rlc_decode_seeded(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t r,
                             uint32_t symbol_size, const uint32_t *rep_seed, const uint64_t *src_present,
                             const uint64_t *rep_present, uint8_t *status, uint64_t *recovered, void *workspace,
                             size_t workspace_bytes, void *stream) {
  if (nblocks && r && !rep_seed) return set_err(FECGPU_ERR_INVALID, "%s", "NULL rep_seed");
  return decode_impl(src, rep, src, nblocks, k, r, symbol_size, 0, nullptr, rep_seed, src_present, rep_present,
                     status, recovered, workspace, workspace_bytes, (hipStream_t)stream);
}

// host_path.hip: decode with the recovered rows to dst (library-internal)
extern "C" __attribute__((visibility("hidden"))) int fecgpu_rlc_decode_to_internal(
    const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k, uint32_t r, uint32_t L,
    uint32_t fbn_base, const uint32_t *fbn, const uint32_t *seeds, const uint64_t *sp, const uint64_t *rp,
    uint8_t *status, uint64_t *recovered, void *ws, size_t wsb, void *stream) {
  return decode_impl(src, rep, dst, nblocks, k, r, L, fbn_base, fbn, seeds, sp, rp, status, recovered, ws, wsb,
                     (hipStream_t)stream);
}

static int xor_decode_impl(void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k, uint32_t symbol_size,
                           const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                           uint64_t *recovered, void *stream) {
  int rc = check_common(src, rep, nblocks, k, 1, symbol_size);
  if (rc || nblocks == 0) return rc;
  if (!src_present || !rep_present || !status || !recovered)
    return set_err(FECGPU_ERR_INVALID, "%s", "NULL mask/status");
  hipStream_t s = (hipStream_t)stream;
  const bool v4 = (symbol_size % 16) == 0 && ((uintptr_t)src % 16) == 0 && ((uintptr_t)rep % 16) == 0 &&
                  ((uintptr_t)dst % 16) == 0;
  const int Lv = (int)(v4 ? symbol_size / 16 : symbol_size / 4);
  const uint32_t gmax = 1u << 20;
  for (uint64_t b0 = 0, n; b0 < nblocks; b0 += n) {
    n = xor_sub_batch(nblocks - b0, Lv, gmax);
    const uint64_t total = n * (uint64_t)Lv;
    const uint32_t grid = (uint32_t)((total + 255) / 256 < gmax ? (total + 255) / 256 : gmax);
    const uint64_t so = b0 * k * (uint64_t)Lv, ro = b0 * (uint64_t)Lv;  // in vectors
    if (v4)
      xor_dispatch_k<u32x4, XorDec, uint32_t>(k, grid, s, (u32x4 *)src + so, (const u32x4 *)rep + ro, n, (int)k, Lv,
                                              src_present + 2 * b0, rep_present + 2 * b0, status + b0,
                                              recovered + 2 * b0, dst ? (u32x4 *)dst + ro : (u32x4 *)nullptr);
    else
      xor_dispatch_k<uint32_t, XorDec, uint32_t>(k, grid, s, (uint32_t *)src + so, (const uint32_t *)rep + ro, n,
                                                 (int)k, Lv, src_present + 2 * b0, rep_present + 2 * b0, status + b0,
                                                 recovered + 2 * b0, dst ? (uint32_t *)dst + ro : (uint32_t *)nullptr);
  }
  HIPCHK(hipGetLastError());
  g_stats[2]++;
  g_stats[3] += nblocks;
  return FECGPU_OK;
}

int fecgpu_xor_decode(void *src, const void *rep, uint64_t nblocks, uint32_t k, uint32_t symbol_size,
                      const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                      uint64_t *recovered, void *stream) {
  return xor_decode_impl(src, rep, nullptr, nblocks, k, symbol_size, src_present, rep_present, status, recovered,
                         stream);
}

int fecgpu_xor_decode_to(const void *src, const void *rep, void *dst, uint64_t nblocks, uint32_t k,
                         uint32_t symbol_size, const uint64_t *src_present, const uint64_t *rep_present,
                         uint8_t *status, uint64_t *recovered, void *stream) {
  if (!dst) return set_err(FECGPU_ERR_INVALID, "%s", "NULL dst");
  return xor_decode_impl(const_cast<void *>(src), rep, dst, nblocks, k, symbol_size, src_present, rep_present,
                         status, recovered, stream);
}

int fecgpu_write_repair_frames(const void *rep, uint64_t nblocks, uint32_t r, uint32_t symbol_size,
                               uint16_t data_length, uint32_t fbn_base, const uint32_t *fbn, uint8_t nss, uint8_t nrs,
                               void *frames, uint32_t frame_stride, void *stream) {
  if (!rep || !frames) return set_err(FECGPU_ERR_INVALID, "%s", "NULL buffer");
  if (symbol_size % 4 || frame_stride % 4) return set_err(FECGPU_ERR_INVALID, "%s", "sizes must be multiples of 4");
  if (data_length > symbol_size || data_length > 0x7fff || frame_stride < 14u + data_length)
    return set_err(FECGPU_ERR_INVALID, "%s", "data_length exceeds the symbol, 15 bits or the frame slot");
  if (!nblocks || !r) return FECGPU_OK;
  const uint64_t nf = nblocks * r, total = nf * (frame_stride / 4);
  if (symbol_size % 16 == 0 && frame_stride % 16 == 0 && ((uintptr_t)rep | (uintptr_t)frames) % 16 == 0) {
    const uint64_t chunks = nf * (frame_stride / 16), wg = (chunks + 255) / 256;
    const uint32_t grid = (uint32_t)(wg < (1u << 20) ? wg : (1u << 20));
    if (chunks < (1ull << 32) - (uint64_t)grid * 256)
      hipLaunchKernelGGL(k_write_repair_frames16<uint32_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                         (const uint32_t *)rep, nf, r, symbol_size / 4, (uint32_t)data_length, fbn_base, fbn,
                         (uint32_t)nss, (uint32_t)nrs, (uint32_t *)frames, frame_stride / 4);
    else
      hipLaunchKernelGGL(k_write_repair_frames16<uint64_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                         (const uint32_t *)rep, nf, r, symbol_size / 4, (uint32_t)data_length, fbn_base, fbn,
                         (uint32_t)nss, (uint32_t)nrs, (uint32_t *)frames, frame_stride / 4);
  } else {
    const uint32_t grid = (uint32_t)((total + 255) / 256 < (1u << 20) ? (total + 255) / 256 : (1u << 20));
    hipLaunchKernelGGL(k_write_repair_frames, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint32_t *)rep,
                       nf, r, symbol_size / 4, (uint32_t)data_length, fbn_base, fbn, (uint32_t)nss, (uint32_t)nrs,
                       (uint32_t *)frames, frame_stride / 4);
  }
  HIPCHK(hipGetLastError());
  return FECGPU_OK;
}

// ---- resident block service (k_block_svc) ----
struct fecgpu_block_svc {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;          // recorded after each worker launch: complete once it has ended
  BlockSvcMailbox *mb = nullptr;    // page-locked, coherent
  BlockSvcMailbox *mb_dev = nullptr;
  uint64_t seq = 0;
  bool launched = false;
  uint64_t deadline_us = 2000;      // a request not served by then is withdrawn (svc_withdraw)
  uint64_t backoff_until = 0;       // after a withdrawal the calls take the launch path until then (us)
  uint64_t misses = 0;              // requests withdrawn at the deadline
  uint64_t t_launch_us = 0;         // the running worker's launch, host clock
  uint64_t t_done_us = 0;           // the last request it finished, host clock
  uint64_t t_post_us = 0, t_seen_us = 0;  // the last served request: posted / seen done (diagnostics)
  std::mutex mu;
};

static uint64_t svc_now_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

// Hook requests in flight (posted, not yet returned) across every service of the process, and the
// time of the last one: the zero-copy bulk paths (host_path.hip, Pacer) slice their launches while
// hooks are in use and start no slice while one is pending.
static std::atomic<int> g_svc_pending{0};
static std::atomic<uint64_t> g_svc_last_us{0};
extern "C" __attribute__((visibility("hidden"))) int fecgpu_svc_hooks_pending(void) { return g_svc_pending.load(); }
extern "C" __attribute__((visibility("hidden"))) uint64_t fecgpu_svc_last_request_us(void) {
  return g_svc_last_us.load(std::memory_order_relaxed);
}
// after a withdrawn request the hooks use the launch path for this long: a worker that was not
// scheduled within the deadline is most likely queued behind a long kernel, and so would the next be
constexpr uint64_t kSvcBackoffUs = 50000;

// worker lifetime: ends after 20 ms without a request (the next call relaunches it) and after 50 ms
// in all (s_memrealtime: 100 MHz).  The worker runs on a stream of the greatest priority, which the
// runtime maps to a hardware queue of its own unless the process creates other such streams; should
// it share one, kernels queued behind the resident worker wait at most its lifetime (sustained hook
// traffic then pays one relaunch per 50 ms).
constexpr uint64_t kSvcIdleTicks = 2000000, kSvcLifeTicks = 5000000;
constexpr uint32_t kSvcLds = 60 * 1024;  // dynamic LDS of the worker (the mailbox copy is static)

fecgpu_block_svc_t *fecgpu_block_svc_create(int device) {
  if (fecgpu_init(device) != FECGPU_OK) return nullptr;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(device) != hipSuccess) return nullptr;
  auto *v = new fecgpu_block_svc;
  v->device = device;
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
  uint32_t cu_mask[16];
  const int mw = fecgpu_svc_cu_mask(device, 1, cu_mask, 16);
  bool ok = (mw ? hipExtStreamCreateWithCUMask(&v->stream, (uint32_t)mw, cu_mask)
                : hipStreamCreateWithPriority(&v->stream, hipStreamNonBlocking, prio_greatest)) == hipSuccess &&
            hipEventCreateWithFlags(&v->ev, hipEventDisableTiming) == hipSuccess &&
            // fine-grained (coherent) explicitly: the host's compare-and-swap on req.seq (svc_unpost) and
            // the worker's system-scope claim must be atomic against each other over PCIe
            hipHostMalloc((void **)&v->mb, sizeof(BlockSvcMailbox), hipHostMallocMapped | hipHostMallocCoherent) ==
                hipSuccess;
  if (ok) {
    memset(v->mb, 0, sizeof(BlockSvcMailbox));
    ok = hipHostGetDevicePointer((void **)&v->mb_dev, v->mb, 0) == hipSuccess &&
         hipFuncSetAttribute((const void *)k_block_svc, hipFuncAttributeMaxDynamicSharedMemorySize, kSvcLds) ==
             hipSuccess;
  }
  (void)hipSetDevice(cur);
  if (!ok) {
    (void)hipGetLastError();
    fecgpu_block_svc_destroy(v);
    return nullptr;
  }
  return v;
}

void fecgpu_block_svc_destroy(fecgpu_block_svc_t *v) {
  if (!v) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(v->device);
  if (v->mb) __atomic_store_n(&v->mb->quit, 1ull, __ATOMIC_RELEASE);
  if (v->launched) (void)hipEventSynchronize(v->ev);  // the worker sees quit within a poll
  if (v->ev) (void)hipEventDestroy(v->ev);
  if (v->stream) (void)hipStreamDestroy(v->stream);
  if (v->mb) (void)hipHostFree(v->mb);
  (void)hipSetDevice(cur);
  delete v;
}

// (re)launch the worker unless one is running.  A worker that finished a request within the last 5 ms
// and was launched less than 30 ms ago is running for sure (it ends after 20 ms idle, 50 ms in all):
// then no runtime call is made, one fewer per hook beside a bulk job's own launches and event waits in
// the same runtime (a worker that faults is still caught by the poll loop's periodic query).
static int svc_ensure(fecgpu_block_svc_t *v) {
  if (v->launched) {
    const uint64_t now = svc_now_us();
    if (now - v->t_done_us < 5000 && now - v->t_launch_us < 30000) return FECGPU_OK;
    if (hipEventQuery(v->ev) == hipErrorNotReady) return FECGPU_OK;
  }
  (void)hipGetLastError();
  __atomic_store_n(&v->mb->quit, 0ull, __ATOMIC_RELEASE);
  hipLaunchKernelGGL(k_block_svc, dim3(1), dim3(kLdsThreads), kSvcLds, v->stream, v->mb_dev, kSvcIdleTicks,
                     kSvcLifeTicks);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(v->ev, v->stream));
  v->launched = true;
  v->t_launch_us = svc_now_us();
  v->t_done_us = 0;
  return FECGPU_OK;
}

// Takes back request `seq` unless a worker has claimed it: compare-and-swap seq -> seq - 1 (the last
// number served), against the worker's claim seq -> seq | kSvcClaimed.  Returns true when the request
// is withdrawn (no worker can serve it later, when its rows are the caller's again); false when a
// worker claimed it first and is serving it.
static bool svc_unpost(fecgpu_block_svc_t *v, uint64_t seq) {
  uint64_t expect = seq;
  if (__atomic_compare_exchange_n(&v->mb->req.seq, &expect, seq - 1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
    v->seq = seq - 1;
    return true;
  }
  return false;
}

// A claimed request is being served: wait for it, as long as its worker lives (a worker that ended or
// faulted without finishing it reports an error).
static int svc_wait_claimed(fecgpu_block_svc_t *v, uint64_t seq) {
  for (uint64_t spin = 1;; spin++) {
    if (__atomic_load_n(&v->mb->done, __ATOMIC_ACQUIRE) == seq) return FECGPU_OK;
    __builtin_ia32_pause();
    if ((spin & 1023) == 0) {
      const hipError_t q = hipEventQuery(v->ev);
      if (q == hipErrorNotReady) continue;
      if (__atomic_load_n(&v->mb->done, __ATOMIC_ACQUIRE) == seq) return FECGPU_OK;
      return set_err(FECGPU_ERR_HIP, "block service: worker ended without finishing a claimed request (%s)",
                     hipGetErrorString(q));
    }
  }
}

// Takes request `seq` back on an error path; a request a worker has claimed is waited for instead.
static int svc_abandon(fecgpu_block_svc_t *v, uint64_t seq, int rc) {
  if (svc_unpost(v, seq)) return rc;
  const int w = svc_wait_claimed(v, seq);
  return w ? w : rc;
}

// The deadline passed with request `seq` unserved.  If no worker has claimed it, it is withdrawn on
// the spot -- no wait for the worker, which may be queued behind a long kernel: it starts when the
// GPU lets it, finds nothing pending and serves later requests or ends on its idle limit -- and the
// call returns FECGPU_ERR_INVALID, so the caller runs the block through the launch path, as for a
// block the service does not take; the next calls skip the service for a while and the withdrawal is
// counted.  If a worker claimed it in the meantime it is running now and is waited for (OK).
static int svc_withdraw(fecgpu_block_svc_t *v, uint64_t seq) {
  if (!svc_unpost(v, seq)) return svc_wait_claimed(v, seq);
  v->misses++;
  v->backoff_until = svc_now_us() + kSvcBackoffUs;
  return set_err(FECGPU_ERR_INVALID, "%s", "block service: deadline passed, request withdrawn");
}

// Posts the request already written into the mailbox and waits for its completion, at most
// v->deadline_us before it is withdrawn (svc_withdraw).  The request number is posted only once a
// worker is running or launched, and taken back on every error return.
static int svc_run_posted(fecgpu_block_svc_t *v, uint64_t t0);
static int svc_run(fecgpu_block_svc_t *v) {
  const uint64_t t0 = svc_now_us();
  if (t0 < v->backoff_until) return FECGPU_ERR_INVALID;  // a recent withdrawal: the launch path for now
  g_svc_last_us.store(t0, std::memory_order_relaxed);
  g_svc_pending.fetch_add(1);
  const int rc = svc_run_posted(v, t0);
  g_svc_pending.fetch_sub(1);
  if (rc == FECGPU_OK) v->t_done_us = svc_now_us();
  return rc;
}
static int svc_run_posted(fecgpu_block_svc_t *v, uint64_t t0) {
  if (int rc = svc_ensure(v)) return rc;
  const uint64_t seq = v->seq + 1;
  v->seq = seq;
  __atomic_store_n(&v->mb->req.seq, seq, __ATOMIC_RELEASE);
  const uint64_t t_post = svc_now_us();
  for (uint64_t spin = 1;; spin++) {
    if (__atomic_load_n(&v->mb->done, __ATOMIC_ACQUIRE) == seq) {
      v->t_post_us = t_post;
      v->t_seen_us = svc_now_us();
      return FECGPU_OK;
    }
    __builtin_ia32_pause();
    if ((spin & 255) == 0 && svc_now_us() - t0 > v->deadline_us) return svc_withdraw(v, seq);
    if ((spin & 1023) == 0) {
      const hipError_t q = hipEventQuery(v->ev);
      if (q == hipErrorNotReady) continue;
      if (q != hipSuccess)
        return svc_abandon(v, seq, set_err(FECGPU_ERR_HIP, "block service: %s", hipGetErrorString(q)));
      // the worker ended (idle limit reached as the request was posted): the next one serves it
      if (__atomic_load_n(&v->mb->done, __ATOMIC_ACQUIRE) == seq) return FECGPU_OK;
      if (int rc = svc_ensure(v)) return svc_abandon(v, seq, rc);
    }
  }
}

int fecgpu_host_device_address(const void *p, size_t bytes, uint64_t *dev);  // host_path.hip

static bool svc_addr(const void *p, size_t n, uint64_t *d) { return fecgpu_host_device_address(p, n, d) == FECGPU_OK; }

int fecgpu_block_svc_rlc_encode(fecgpu_block_svc_t *v, const void *src, void *rep, uint32_t k, uint32_t r,
                                uint32_t symbol_size, uint32_t fbn) {
  if (!v || !knob(K_BLOCK_SVC)) return FECGPU_ERR_INVALID;
  if (int rc = check_common(src, rep, 1, k, r, symbol_size)) return rc;
  if (!r) return FECGPU_OK;
  const int OT = r <= 4 ? 4 : r <= 8 ? 8 : 16;
  if (EncLdsLayout((int)k, (int)r, (int)symbol_size, OT).bytes > kSvcLds)
    return set_err(FECGPU_ERR_INVALID, "%s", "block service: block too large for its LDS");
  uint64_t ds, dr;
  if (!svc_addr(src, (size_t)k * symbol_size, &ds) || !svc_addr(rep, (size_t)r * symbol_size, &dr))
    return set_err(FECGPU_ERR_INVALID, "%s", "block service: buffers must be page-locked");
  std::lock_guard<std::mutex> g(v->mu);
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  if (cur != v->device) HIPCHK(hipSetDevice(v->device));
  BlockSvcReq *m = &v->mb->req;
  m->op = 1; m->k = k; m->r = r; m->L = symbol_size; m->fbn = fbn & 0xffffffu;
  m->src = ds; m->rep = dr;
  const int rc = svc_run(v);
  if (cur != v->device) (void)hipSetDevice(cur);
  if (!rc) {
    g_stats[0]++;
    g_stats[1]++;
  }
  return rc;
}

int fecgpu_block_svc_rlc_decode_seeded(fecgpu_block_svc_t *v, const void *src, const void *rep, void *dst, uint32_t k,
                                       uint32_t r, uint32_t symbol_size, const uint32_t *rep_seed,
                                       const uint64_t *src_present, const uint64_t *rep_present, uint8_t *status,
                                       uint64_t *recovered) {
  if (!v || !knob(K_BLOCK_SVC)) return FECGPU_ERR_INVALID;
  if (int rc = check_common(src, rep, 1, k, r, symbol_size)) return rc;
  if (!dst || !rep_seed || !src_present || !rep_present || !status || !recovered || r == 0)
    return set_err(FECGPU_ERR_INVALID, "%s", "block service: NULL argument or r == 0");
  const uint32_t em = k < r ? k : r;
  if (em > 16 || r > (uint32_t)kSvcMaxR || knob(K_PLAN) != 0 ||
      DecLdsLayout((int)k, (int)r, (int)symbol_size, em <= 4 ? 4 : em <= 8 ? 8 : 16).bytes > kSvcLds)
    return set_err(FECGPU_ERR_INVALID, "%s", "block service: block too large for its LDS");
  uint64_t a[3];
  if (!svc_addr(src, (size_t)k * symbol_size, &a[0]) || !svc_addr(rep, (size_t)r * symbol_size, &a[1]) ||
      !svc_addr(dst, (size_t)k * symbol_size, &a[2]))
    return set_err(FECGPU_ERR_INVALID, "%s", "block service: symbol rows must be page-locked");
  std::lock_guard<std::mutex> g(v->mu);
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  if (cur != v->device) HIPCHK(hipSetDevice(v->device));
  BlockSvcReq *m = &v->mb->req;
  m->op = 2; m->k = k; m->r = r; m->L = symbol_size; m->fbn = 0; m->wreg = knob(K_PLAN) != PLAN_WAVE;
  m->src = a[0]; m->rep = a[1]; m->dst = a[2];
  m->sp[0] = src_present[0]; m->sp[1] = src_present[1];
  m->rp[0] = rep_present[0]; m->rp[1] = rep_present[1];
  memcpy(m->seeds, rep_seed, (size_t)r * 4);
  const int rc = svc_run(v);
  if (cur != v->device) (void)hipSetDevice(cur);
  if (!rc) {
    *status = (uint8_t)v->mb->status;
    recovered[0] = v->mb->recovered[0];
    recovered[1] = v->mb->recovered[1];
    g_stats[2]++;
    g_stats[3]++;
  }
  return rc;
}

uint64_t fecgpu_block_svc_launches(const fecgpu_block_svc_t *v) {
  return v && v->mb ? __atomic_load_n(&v->mb->launches, __ATOMIC_ACQUIRE) : 0;
}

int fecgpu_block_svc_set_deadline(fecgpu_block_svc_t *v, uint64_t deadline_us) {
  if (!v) return FECGPU_ERR_INVALID;
  std::lock_guard<std::mutex> g(v->mu);
  v->deadline_us = deadline_us;
  v->backoff_until = 0;
  return FECGPU_OK;
}

int fecgpu_block_svc_last_stamps(fecgpu_block_svc_t *v, uint64_t out[6]) {
  if (!v || !out || !v->mb) return FECGPU_ERR_INVALID;
  std::lock_guard<std::mutex> g(v->mu);
  for (int i = 0; i < 4; i++) out[i] = __atomic_load_n(&v->mb->stamp[i], __ATOMIC_ACQUIRE);
  out[4] = v->t_post_us;
  out[5] = v->t_seen_us;
  return FECGPU_OK;
}

uint64_t fecgpu_block_svc_deadline_misses(fecgpu_block_svc_t *v) {
  if (!v) return 0;
  std::lock_guard<std::mutex> g(v->mu);
  return v->misses;
}

int fecgpu_block_svc_worker_running(fecgpu_block_svc_t *v) {
  if (!v) return FECGPU_ERR_INVALID;
  std::lock_guard<std::mutex> g(v->mu);
  if (!v->launched) return 0;
  const hipError_t q = hipEventQuery(v->ev);
  if (q == hipErrorNotReady) return 1;
  return q == hipSuccess ? 0 : set_err(FECGPU_ERR_HIP, "block service: worker ended with %s", hipGetErrorString(q));
}

int fecgpu_synth_fill(void *dst, uint64_t nbytes, uint64_t seed, uint64_t offset, void *stream) {
  if (!dst) return set_err(FECGPU_ERR_INVALID, "%s", "NULL dst");
  if (!nbytes) return FECGPU_OK;
  const uint64_t words = ((offset + nbytes + 7) >> 3) - (offset >> 3) + 1;
  const uint32_t grid = (uint32_t)((words + 255) / 256 < (1u << 20) ? (words + 255) / 256 : (1u << 20));
  hipLaunchKernelGGL(k_synth_fill, dim3(grid), dim3(256), 0, (hipStream_t)stream, (uint8_t *)dst, nbytes,
                     seed, offset);
  HIPCHK(hipGetLastError());
  return FECGPU_OK;
}

}  // extern "C"
