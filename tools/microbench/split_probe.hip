// Split probe (round 4): can the FEC block pattern stream faster than one wave per block?
// Trivial XOR compute, the engine's block-major layout src[b][k][L], rep[b][r][L], L = 1200.
//   col G1        one wave per block, 38 lanes x 2 x 16 B per row, 8 rows in flight (the kernels today)
//   split Wn      n waves per block (workgroup), wave w takes rows w, w + n, ...; partial sums meet
//                 in LDS (one ds_write + barrier + n ds_reads per lane and piece), wave w writes
//                 repairs i = w mod n
//   lin Wn        n waves per block, each wave-instruction reads 1 KiB of the block's contiguous
//                 k x L region (whole 128-B lines); outputs written the same way
// (An LDS-DMA variant of lin faulted the GPU twice in round 4 -- an illegal address from the DMA whose
// cause was not found -- and was removed; the LDS-DMA ring bodies of the engine are measured instead.)
// Occupancy is set by the dynamic LDS per workgroup (3 or 4 waves per SIMD, as the kernels run).
// Build: hipcc --offload-arch=gfx950 -O3 -DPK=32 -DPR=8 split_probe.hip -o split_probe_k32
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
#endif
constexpr int K = PK, R = PR, L = 1200;
constexpr int A = (L / 16 + 1) / 2;  // 38 lanes own 2 pieces of 16 B (the last one 1)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}

__global__ __launch_bounds__(64) void col(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep, uint64_t nb) {
  const int lane = threadIdx.x;
  if (lane >= A) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok1 = lane + A < L / 16;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    u32x4 x0 = 0, x1 = 0;
    for (int j0 = 0; j0 < K; j0 += 8) {
      u32x4 a0[8], a1[8];
#pragma unroll
      for (int jj = 0; jj < 8; jj++) {
        const uint8_t *p = src + (b * K + j0 + jj) * (uint64_t)L;
        a0[jj] = ld<true>((const u32x4 *)(p + o0));
        a1[jj] = ok1 ? ld<true>((const u32x4 *)(p + o1)) : (u32x4)0;
      }
#pragma unroll
      for (int jj = 0; jj < 8; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
    }
#pragma unroll
    for (int i = 0; i < R; i++) {
      uint8_t *p = rep + (b * R + i) * (uint64_t)L;
      __builtin_nontemporal_store(x0 + (uint32_t)i, (u32x4 *)(p + o0));
      if (ok1) __builtin_nontemporal_store(x1 + (uint32_t)i, (u32x4 *)(p + o1));
    }
  }
}

// colU / adj Wn: col's one wave per block with U rows in flight; adj packs W such waves in a workgroup
// on adjacent blocks (wave w of workgroup q: block q W + w) -- fewer distinct regions in flight without
// any reduction between the waves.
template <int U, int W>
__global__ __launch_bounds__(64 * W) void adj(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep, uint64_t nb) {
  const int lane = threadIdx.x & 63;
  if (lane >= A) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok1 = lane + A < L / 16;
  const uint64_t b = (uint64_t)blockIdx.x * W + (threadIdx.x >> 6);
  if (b >= nb) return;
  u32x4 x0 = 0, x1 = 0;
  for (int j0 = 0; j0 < K; j0 += U) {
    u32x4 a0[U], a1[U];
#pragma unroll
    for (int jj = 0; jj < U; jj++) {
      const uint8_t *p = src + (b * K + j0 + jj) * (uint64_t)L;
      a0[jj] = ld<true>((const u32x4 *)(p + o0));
      a1[jj] = ok1 ? ld<true>((const u32x4 *)(p + o1)) : (u32x4)0;
    }
#pragma unroll
    for (int jj = 0; jj < U; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
  }
#pragma unroll
  for (int i = 0; i < R; i++) {
    uint8_t *p = rep + (b * R + i) * (uint64_t)L;
    __builtin_nontemporal_store(x0 + (uint32_t)i, (u32x4 *)(p + o0));
    if (ok1) __builtin_nontemporal_store(x1 + (uint32_t)i, (u32x4 *)(p + o1));
  }
}

// dec: the decode apply's pattern -- per block the k - E received sources (E = R erased, at rotating
// slots) and the E repairs, read in slot order, and E recovered rows written packed to dst[b][E][L]
// (the bench's apply); `sorted` reads the received sources first, then the repairs.
template <bool SORTED>
__global__ __launch_bounds__(64) void dec(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep, uint64_t nb) {
  const int lane = threadIdx.x;
  if (lane >= A) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok1 = lane + A < L / 16;
  const uint64_t b = blockIdx.x;
  const int e0 = (int)((b * 7) % K);  // erased sources e0, e0 + K/R, ... (mod K)
  const uint8_t *rp = rep + b * (uint64_t)R * L;  // repairs read from rep; recovered rows written after them
  uint8_t *dst = rep + (nb + b) * (uint64_t)R * L;
  const uint8_t *rows[K];
  int nr = 0, ne = 0;
#pragma unroll
  for (int j = 0; j < K; j++) {
    bool er = false;
#pragma unroll
    for (int u = 0; u < R; u++) er |= j == (e0 + u * (K / R)) % K;
    if (er) {
      if (!SORTED) rows[nr++] = rp + (uint64_t)(ne++) * L;  // the equation that replaces it, in its slot
    } else {
      rows[nr++] = src + (b * K + j) * (uint64_t)L;
    }
  }
  if (SORTED)
    for (int u = 0; u < R; u++) rows[nr++] = rp + (uint64_t)u * L;
  u32x4 x0 = 0, x1 = 0;
  for (int j0 = 0; j0 < K; j0 += 8) {
    u32x4 a0[8], a1[8];
#pragma unroll
    for (int jj = 0; jj < 8; jj++) {
      a0[jj] = ld<true>((const u32x4 *)(rows[j0 + jj] + o0));
      a1[jj] = ok1 ? ld<true>((const u32x4 *)(rows[j0 + jj] + o1)) : (u32x4)0;
    }
#pragma unroll
    for (int jj = 0; jj < 8; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
  }
#pragma unroll
  for (int i = 0; i < R; i++) {
    uint8_t *p = dst + (uint64_t)i * L;
    __builtin_nontemporal_store(x0 + (uint32_t)i, (u32x4 *)(p + o0));
    if (ok1) __builtin_nontemporal_store(x1 + (uint32_t)i, (u32x4 *)(p + o1));
  }
}

template <int W, bool NT>
__global__ __launch_bounds__(64 * W) void split(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep, uint64_t nb) {
  __shared__ u32x4 red[2][W][2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int KW = K / W, U = KW < 8 ? KW : 8;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok0 = lane < A, ok1 = lane + A < L / 16;
  int par = 0;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x, par ^= 1) {
    u32x4 x0 = 0, x1 = 0;
    for (int i0 = 0; i0 < KW; i0 += U) {
      u32x4 a0[U], a1[U];
#pragma unroll
      for (int jj = 0; jj < U; jj++) {
        const int j = w + W * (i0 + jj);
        const uint8_t *p = src + (b * K + j) * (uint64_t)L;
        a0[jj] = ok0 ? ld<NT>((const u32x4 *)(p + o0)) : (u32x4)0;
        a1[jj] = ok1 ? ld<NT>((const u32x4 *)(p + o1)) : (u32x4)0;
      }
#pragma unroll
      for (int jj = 0; jj < U; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
    }
    red[par][w][0][lane] = x0;
    red[par][w][1][lane] = x1;
    __syncthreads();  // one barrier per block: the parity buffers keep block b+1's writes off b's reads
    u32x4 y0 = 0, y1 = 0;
#pragma unroll
    for (int v = 0; v < W; v++) { y0 ^= red[par][v][0][lane]; y1 ^= red[par][v][1][lane]; }
    for (int i = w; i < R; i += W) {
      uint8_t *p = rep + (b * R + i) * (uint64_t)L;
      if (ok0) __builtin_nontemporal_store(y0 + (uint32_t)i, (u32x4 *)(p + o0));
      if (ok1) __builtin_nontemporal_store(y1 + (uint32_t)i, (u32x4 *)(p + o1));
    }
  }
}

// lin: the block's k*L source bytes as NPI = k*L/16 pieces; wave-instruction q covers pieces
// 64 q .. 64 q + 63 (1 KiB), wave w takes q = w, w + W, ...
template <int W>
__global__ __launch_bounds__(64 * W) void lin(const uint8_t *__restrict__ src, uint8_t *__restrict__ rep, uint64_t nb) {
  constexpr int NPI = K * L / 16, NQ = (NPI + 63) / 64, NPO = R * L / 16, NQO = (NPO + 63) / 64;
  constexpr int QW = (NQ + W - 1) / W, U = 8;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const u32x4 *s = (const u32x4 *)(src + b * (uint64_t)K * L);
    u32x4 x = 0;
    for (int q0 = 0; q0 < QW; q0 += U) {
      u32x4 a[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int pc = 64 * (w + W * (q0 + u)) + lane;
        a[u] = (q0 + u < QW && pc < NPI) ? ld<true>(s + pc) : (u32x4)0;
      }
#pragma unroll
      for (int u = 0; u < U; u++) x ^= a[u];
    }
    u32x4 *o = (u32x4 *)(rep + b * (uint64_t)R * L);
    for (int q = w; q < NQO; q += W) {
      const int pc = 64 * q + lane;
      if (pc < NPO) __builtin_nontemporal_store(x + (uint32_t)q, o + pc);
    }
  }
}

int main(int argc, char **argv) {
  const bool adj_only = argc > 1, dec_only = argc > 1 && argv[1][0] == 'd';
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint64_t nb = (uint64_t)(1 << 20) * 16 / K;  // 2^20 blocks at k16, 2^19 at k32 (19.3 GB)
  uint8_t *src, *rep;
  CK(hipMalloc(&src, nb * K * L)); CK(hipMalloc(&rep, 2 * nb * R * L));  // dec: recovered rows after the repairs
  CK(hipMemset(src, 3, nb * K * L)); CK(hipMemset(rep, 5, 2 * nb * R * L));
  const double bytes = (double)nb * (K + R) * L;
  printf("# k%d r%d L%d, %llu blocks, %.2f GB per launch\n", K, R, L, (unsigned long long)nb, bytes / 1e9);
  auto run = [&](const char *name, auto kern, int W, size_t lds_per_wave, size_t stat, int per_wg = 1) {
    // grid: one workgroup per block (the engine's one-group-per-workgroup launch); dynamic LDS tops
    // the kernel's static LDS up to lds_per_wave per wave
    const size_t lds = lds_per_wave * W > stat ? lds_per_wave * W - stat : 0;
    float best = 1e9, sum = 0;
    int n = 0;
    for (int it = 0; it < 5; it++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3((uint32_t)((nb + per_wg - 1) / per_wg)), dim3(64 * W), lds, 0, src, rep, nb);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (it) { best = std::min(best, ms); sum += ms; n++; }
    }
    printf("%-40s %8.3f ms (mean %7.3f)  %7.0f GB/s\n", name, best, sum / n, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  for (int rep_ = 0; rep_ < 3; rep_++) {
    for (size_t per : {(size_t)13 << 10, (size_t)10 << 10}) {  // 3 / 4 waves per SIMD
      const int wps = per == ((size_t)13 << 10) ? 3 : 4;
      char nm[96];
#define RUNK(NAME, KERN, W, STAT)                                \
      snprintf(nm, sizeof nm, "%-22s %d waves/SIMD", NAME, wps); \
      run(nm, KERN, W, per, STAT);
#define RUNA(NAME, KERN, W)                                      \
      snprintf(nm, sizeof nm, "%-22s %d waves/SIMD", NAME, wps); \
      run(nm, KERN, W, per, 0, W);
      RUNK("col G1", col, 1, 0)
      if (dec_only) {
        RUNK("dec slot order", dec<false>, 1, 0)
        RUNK("dec sorted", dec<true>, 1, 0)
        continue;
      }
      if (!adj_only) {
        RUNK("split W2 nt", (split<2, true>), 2, 4096 * 2)
        RUNK("split W4 nt", (split<4, true>), 4, 4096 * 4)
        RUNK("split W4 default", (split<4, false>), 4, 4096 * 4)
        RUNK("split W8 nt", (split<8, true>), 8, 4096 * 8)
        RUNK("lin W1", lin<1>, 1, 0)
        RUNK("lin W4", lin<4>, 4, 0)
        RUNK("lin W8", lin<8>, 8, 0)
      }
      RUNA("adj U8 W1", (adj<8, 1>), 1)
      RUNA("adj U16 W1", (adj<16, 1>), 1)
      RUNA("adj U4 W1", (adj<4, 1>), 1)
      RUNA("adj U8 W2", (adj<8, 2>), 2)
      RUNA("adj U8 W4", (adj<8, 4>), 4)
      RUNA("adj U8 W8", (adj<8, 8>), 8)
      RUNA("adj U16 W4", (adj<16, 4>), 4)
      RUNK("split W4 nt", (split<4, true>), 4, 4096 * 4)
    }
  }
  return 0;
}
