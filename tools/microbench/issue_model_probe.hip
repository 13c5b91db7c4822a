// Issue-model probe for the bitsliced data path's dispatch: how fast can W waves per SIMD issue
// (a) straight-line independent VALU, (b) VALU with a few independent SALU ops mixed in,
// (c) 8-VALU "cases" chained by s_setpc_b64 (the case-table dispatch), (d) the same with the
// 3-SALU chain tail.  Reports wave64 VALU instructions per SIMD per cycle (at the measured clock)
// and per-case cycles.  build: hipcc --offload-arch=gfx950 -O3 issue_model_probe.hip -o issue_model_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

#define X8 "v_xor_b32 v40, v41, v40\n v_xor_b32 v42, v41, v42\n v_xor_b32 v43, v41, v43\n v_xor_b32 v44, v41, v44\n" \
           "v_xor_b32 v45, v41, v45\n v_xor_b32 v46, v41, v46\n v_xor_b32 v47, v41, v47\n v_xor_b32 v48, v41, v48\n"
#define S3 "s_add_u32 s40, s40, 8\n s_lshr_b64 s[42:43], s[42:43], 16\n s_pack_ll_b32_b16 s44, s42, s45\n"

// the straight-line modes need the SALU text pasted in at compile time
#define STRAIGHT(NAME, TAIL)                                                                          \
  __global__ __launch_bounds__(64) void NAME(unsigned *out, int trips) {                              \
    unsigned r;                                                                                        \
    asm volatile(                                                                                      \
        "v_mov_b32 v40, 1\n v_mov_b32 v41, 3\n v_mov_b32 v42, 5\n v_mov_b32 v43, 7\n v_mov_b32 v44, 9\n" \
        "v_mov_b32 v45, 11\n v_mov_b32 v46, 13\n v_mov_b32 v47, 15\n v_mov_b32 v48, 17\n"             \
        "s_mov_b32 s46, %1\n s_mov_b64 s[42:43], -1\n s_mov_b32 s45, 0\n"                              \
        ".Lloop%=:\n" X8 TAIL X8 TAIL X8 TAIL X8 TAIL                                                  \
        "s_sub_u32 s46, s46, 1\n s_cbranch_scc0 .Lloop%=\n"                                            \
        "v_xor_b32 %0, v40, v48\n"                                                                     \
        : "=v"(r) : "s"(trips)                                                                          \
        : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "s40", "s41", "s42", "s43",   \
          "s44", "s45", "s46", "scc");                                                                  \
    out[blockIdx.x] = r;                                                                               \
  }
STRAIGHT(k_straight, "")
STRAIGHT(k_straight_salu, S3)

// chained units: unit A ends with a jump to unit B and B back to A (through the loop counter)
#define CHAINED(NAME, TAIL)                                                                           \
  __global__ __launch_bounds__(64) void NAME(unsigned *out, int trips) {                              \
    unsigned r;                                                                                        \
    asm volatile(                                                                                      \
        "v_mov_b32 v40, 1\n v_mov_b32 v41, 3\n v_mov_b32 v42, 5\n v_mov_b32 v43, 7\n v_mov_b32 v44, 9\n" \
        "v_mov_b32 v45, 11\n v_mov_b32 v46, 13\n v_mov_b32 v47, 15\n v_mov_b32 v48, 17\n"             \
        "s_mov_b32 s46, %1\n s_mov_b64 s[42:43], -1\n s_mov_b32 s45, 0\n"                              \
        "s_getpc_b64 s[50:51]\n.Lpa%=:\n s_add_u32 s50, s50, .LA%= - .Lpa%=\n s_addc_u32 s51, s51, 0\n"   \
        "s_getpc_b64 s[52:53]\n.Lpb%=:\n s_add_u32 s52, s52, .LB%= - .Lpb%=\n s_addc_u32 s53, s53, 0\n"   \
        "s_getpc_b64 s[54:55]\n.Lpc%=:\n s_add_u32 s54, s54, .LC%= - .Lpc%=\n s_addc_u32 s55, s55, 0\n"   \
        "s_getpc_b64 s[56:57]\n.Lpd%=:\n s_add_u32 s56, s56, .LD%= - .Lpd%=\n s_addc_u32 s57, s57, 0\n"   \
        "s_setpc_b64 s[50:51]\n"                                                                       \
        ".p2align 6\n.LA%=:\n" X8 TAIL "s_setpc_b64 s[52:53]\n"                                         \
        ".p2align 6\n.LB%=:\n" X8 TAIL "s_setpc_b64 s[54:55]\n"                                         \
        ".p2align 6\n.LC%=:\n" X8 TAIL "s_setpc_b64 s[56:57]\n"                                         \
        ".p2align 6\n.LD%=:\n" X8 TAIL                                                                  \
        "s_sub_u32 s46, s46, 1\n s_cbranch_scc1 .Lend%=\n s_setpc_b64 s[50:51]\n"                      \
        ".Lend%=:\n v_xor_b32 %0, v40, v48\n"                                                          \
        : "=v"(r) : "s"(trips)                                                                          \
        : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "s40", "s41", "s42", "s43",   \
          "s44", "s45", "s46", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "scc");          \
    out[blockIdx.x] = r;                                                                               \
  }
CHAINED(k_chain, "")
CHAINED(k_chain_salu, S3)

__global__ void k_clock(unsigned long long *t) {
  // wall-clock (constant 100 MHz) vs shader clock over a busy loop: the shader clock rate
  unsigned long long c0 = clock64(), w0 = wall_clock64();
  unsigned x = threadIdx.x;
  for (int i = 0; i < (1 << 22); i++) x = x * 1664525u + 1013904223u;
  unsigned long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { t[0] = c1 - c0; t[1] = w1 - w0; t[2] = x; }
}

typedef void (*KFn)(unsigned *, int);

static double run(KFn fn, int waves_per_simd, int trips, unsigned *o) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = 1024 * waves_per_simd;
  float ms, best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(64), 0, 0, o, trips);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep) best = std::min(best, ms);
  }
  return best;
}

int main() {
  unsigned *o;
  CK(hipMalloc(&o, 1 << 20));
  unsigned long long *t;
  CK(hipMalloc(&t, 64));
  hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, t);
  unsigned long long h[3];
  CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
  int wall_khz = 0;
  CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  const double ghz = (double)h[0] / ((double)h[1] / (wall_khz * 1e3)) / 1e9;
  printf("shader clock (1 busy wave): %.3f GHz\n", ghz);
  const int trips = 20000;
  struct { const char *name; KFn fn; int valu_per_trip, salu_per_trip; } ks[] = {
      {"straight 8V", k_straight, 32, 2}, {"straight 8V+3S", k_straight_salu, 32, 14},
      {"chain 8V+jump", k_chain, 32, 6}, {"chain 8V+3S+jump", k_chain_salu, 32, 18}};
  for (auto &kk : ks) {
    for (int w : {1, 2, 3, 4, 6, 8}) {
      const double ms = run(kk.fn, w, trips, o);
      const double units = 4.0 * trips;                 // units per wave
      const double cyc = ms * 1e-3 * ghz * 1e9;         // at the one-wave clock (approximate)
      printf("%-18s W=%d: %8.3f ms  VALU/SIMD/cycle %.3f  cycles per unit per wave %.1f\n", kk.name, w, ms,
             w * units * 8 / cyc, cyc / units);
    }
  }
  return 0;
}
