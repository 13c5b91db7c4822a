// Block-pattern probe: the RLC encode's memory pattern (per block: k = 16 source rows of 1200 B
// read, r = 4 repair rows written; one wave accumulates one block at a time, 38 lanes x 2 x 16 B
// per row) with trivial XOR compute, under different block -> wave assignments and occupancy.
// Separates the pattern's own HBM ceiling from the bitsliced arithmetic's cost.
// Build: hipcc --offload-arch=gfx950 -O3 block_pattern_probe.hip -o block_pattern_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef PK
#define PK 16
#define PR 4
#define PL 1200
#endif
constexpr int K = PK, R = PR, L = PL;  // -DPK=32 -DPR=8 for configs[3]'s rows

// wave per group of G blocks; ilv: group q = blocks q, q + NG, ...; else qG .. qG + G - 1
// WIDE: lane l holds 16-B pieces l and l + 64 (64 + 11 lanes per 1200-B row) instead of l and l + 38
template <int G, bool ILV, bool NTS, bool WIDE = false, bool NTL = false>
__global__ __launch_bounds__(64) void enc_pattern(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep,
                                                  uint64_t nblocks) {
  const int lane = threadIdx.x;
  constexpr int A = WIDE ? 64 : (L / 16 + 1) / 2;  // lanes of the first piece row
  if (lane >= A) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok1 = lane + A < L / 16;
  const uint64_t NG = (nblocks + G - 1) / G;
  for (uint64_t q = blockIdx.x; q < NG; q += gridDim.x) {
    for (int g = 0; g < G; g++) {
      const uint64_t b = ILV ? q + g * NG : q * G + g;
      if (b >= nblocks) break;
      const uint8_t *sb = src + b * K * L;
      u32x4 x0 = 0, x1 = 0;
      for (int j0 = 0; j0 < K; j0 += 8) {  // 8 rows in flight at a time (the asm keeps P = 4..8)
        u32x4 a0[8], a1[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const u32x4 *p0 = (const u32x4 *)(sb + (j0 + j) * L + o0), *p1 = (const u32x4 *)(sb + (j0 + j) * L + o1);
          a0[j] = j0 + j < K ? (NTL ? __builtin_nontemporal_load(p0) : *p0) : (u32x4)0;
          a1[j] = (ok1 && j0 + j < K) ? (NTL ? __builtin_nontemporal_load(p1) : *p1) : (u32x4)0;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) { x0 ^= a0[j]; x1 ^= a1[j]; }
      }
      uint8_t *rb = rep + b * R * L;
#pragma unroll
      for (int i = 0; i < R; i++) {
        u32x4 v0 = x0 + (uint32_t)i, v1 = x1 + (uint32_t)i;
        if (NTS) {
          __builtin_nontemporal_store(v0, (u32x4 *)(rb + i * L + o0));
          if (ok1) __builtin_nontemporal_store(v1, (u32x4 *)(rb + i * L + o1));
        } else {
          *(u32x4 *)(rb + i * L + o0) = v0;
          if (ok1) *(u32x4 *)(rb + i * L + o1) = v1;
        }
      }
    }
  }
}

// persistent: grid = W resident waves; round m, step g: wave w takes block m G W + g W + w, so the
// resident waves sweep one dense window of W blocks at a time
template <int G>
__global__ __launch_bounds__(64) void enc_pattern_persist(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep,
                                                          uint64_t nblocks) {
  const int lane = threadIdx.x;
  if (lane >= 38) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + 38);
  const bool ok1 = lane + 38 < 75;
  const uint64_t W = gridDim.x;
  for (uint64_t base = 0; base < nblocks; base += G * W) {
    for (int g = 0; g < G; g++) {
      const uint64_t b = base + g * W + blockIdx.x;
      if (b >= nblocks) break;
      const uint8_t *sb = src + b * K * L;
      u32x4 x0 = 0, x1 = 0;
      for (int j0 = 0; j0 < K; j0 += 8) {
        u32x4 a0[8], a1[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          a0[j] = j0 + j < K ? *(const u32x4 *)(sb + (j0 + j) * L + o0) : (u32x4)0;
          a1[j] = (ok1 && j0 + j < K) ? *(const u32x4 *)(sb + (j0 + j) * L + o1) : (u32x4)0;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) { x0 ^= a0[j]; x1 ^= a1[j]; }
      }
      uint8_t *rb = rep + b * R * L;
#pragma unroll
      for (int i = 0; i < R; i++) {
        __builtin_nontemporal_store(x0 + (uint32_t)i, (u32x4 *)(rb + i * L + o0));
        if (ok1) __builtin_nontemporal_store(x1 + (uint32_t)i, (u32x4 *)(rb + i * L + o1));
      }
    }
  }
}

// LIN: the same bytes, but each wave-instruction reads 1 KiB of the block's contiguous k x L
// source region in order (lane l, instruction m: bytes 1024 m + 16 l), and writes the r x L repair
// region the same way: every access is a run of whole 128-B lines except at region ends.  (A real
// kernel would need an LDS transpose to get column-aligned symbols back; this measures whether the
// denser shape is worth one.)
template <int G, bool ILV, bool NTL = true>
__global__ __launch_bounds__(64) void enc_pattern_lin(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep,
                                                      uint64_t nblocks) {
  const int lane = threadIdx.x;
  constexpr int NP = K * L / 16, NI = (NP + 63) / 64;  // 16-B pieces, instructions per block
  constexpr int RP = R * L / 16, RI = (RP + 63) / 64;
  const uint64_t NG = (nblocks + G - 1) / G;
  for (uint64_t q = blockIdx.x; q < NG; q += gridDim.x) {
    for (int g = 0; g < G; g++) {
      const uint64_t b = ILV ? q + g * NG : q * G + g;
      if (b >= nblocks) break;
      const uint8_t *sb = src + b * K * L;
      u32x4 x = 0;
      for (int m0 = 0; m0 < NI; m0 += 8) {
        u32x4 a[8];
#pragma unroll
        for (int m = 0; m < 8; m++) {
          const int pc = (m0 + m) * 64 + lane;
          const u32x4 *pp = (const u32x4 *)(sb + 16 * pc);
          a[m] = (m0 + m < NI && pc < NP) ? (NTL ? __builtin_nontemporal_load(pp) : *pp) : (u32x4)0;
        }
#pragma unroll
        for (int m = 0; m < 8; m++) x ^= a[m];
      }
      uint8_t *rb = rep + b * R * L;
#pragma unroll
      for (int m = 0; m < RI; m++) {
        const int pc = m * 64 + lane;
        if (pc < RP) __builtin_nontemporal_store(x + (uint32_t)m, (u32x4 *)(rb + 16 * pc));
      }
    }
  }
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint64_t nb = (uint64_t)(1 << 20) * 16 / K;  // ~20 GB of sources
  uint8_t *src, *rep;
  CK(hipMalloc(&src, nb * K * L)); CK(hipMalloc(&rep, nb * R * L));
  CK(hipMemset(src, 3, nb * K * L)); CK(hipMemset(rep, 0, nb * R * L));
  const double bytes = (double)nb * (K + R) * L;
  auto run = [&](const char *name, size_t lds, auto kern, uint64_t groups) {
    float best = 1e9;
    for (int it = 0; it < 5; it++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3((uint32_t)groups), dim3(64), lds, 0, src, rep, nb);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (it) best = std::min(best, ms);
    }
    printf("%-48s %8.3f ms  %7.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  // LDS caps residency: 13 KiB per workgroup -> 12 waves per CU (3 per SIMD, the asm kernels'
  // occupancy); 0 -> as many as the VGPRs allow
  for (size_t lds : {(size_t)0, (size_t)13 << 10}) {
    char nm[96];
#define RUNP(G, ILV, NTS)                                                                        \
    snprintf(nm, sizeof nm, "G%-2d %s nts%d %s", G, ILV ? "interleaved" : "contiguous", NTS,      \
             lds ? "3 waves/SIMD" : "max occupancy");                                            \
    run(nm, lds, enc_pattern<G, ILV, NTS>, (nb + G - 1) / G);
    RUNP(1, false, true)
    RUNP(4, false, true)
    RUNP(8, true, true)
    RUNP(16, false, true)
    RUNP(4, true, true)
    RUNP(16, true, true)
    RUNP(16, true, false)
    snprintf(nm, sizeof nm, "G16 interleaved WIDE lanes %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern<16, true, true, true>, (nb + 15) / 16);
    snprintf(nm, sizeof nm, "G1 contiguous WIDE lanes %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern<1, false, true, true>, nb);
    snprintf(nm, sizeof nm, "G1 contiguous LIN %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern_lin<1, false>, nb);
    snprintf(nm, sizeof nm, "G4 interleaved LIN %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern_lin<4, true>, (nb + 3) / 4);
    snprintf(nm, sizeof nm, "G16 interleaved LIN %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern_lin<16, true>, (nb + 15) / 16);
    snprintf(nm, sizeof nm, "G16 interleaved LIN ld-default %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern_lin<16, true, false>, (nb + 15) / 16);
    snprintf(nm, sizeof nm, "G16 interleaved nt loads %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern<16, true, true, false, true>, (nb + 15) / 16);
    snprintf(nm, sizeof nm, "G1 contiguous nt loads %s", lds ? "3 waves/SIMD" : "max occupancy");
    run(nm, lds, enc_pattern<1, false, true, false, true>, nb);
    if (getenv("LIN_ONLY")) continue;
    if (lds) {
      for (int W : {3072, 2048, 6144}) {
        snprintf(nm, sizeof nm, "G16 persistent W=%d 3 waves/SIMD", W);
        run(nm, lds, enc_pattern_persist<16>, (uint64_t)W);
        snprintf(nm, sizeof nm, "G4 persistent W=%d 3 waves/SIMD", W);
        run(nm, lds, enc_pattern_persist<4>, (uint64_t)W);
      }
    }
  }
  return 0;
}
