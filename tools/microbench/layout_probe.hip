// Layout probe: the RLC encode / decode-apply memory pattern with trivial XOR compute under two
// device layouts of a batch of FEC blocks:
//   block-major  src[b][j][L], rep[b][i][L]   (each block's rows contiguous; the engine's layout so far)
//   symbol-major src[j][b][L], rep[i][b][L]   (row j of consecutive blocks contiguous)
// One wave per group of G blocks (interleaved: group q = blocks q, q + NG, ...), 38 lanes x 2 x 16 B
// per 1200-B row, P rows in flight, as the bitsliced kernels stream them.  The decode pattern reads
// k - e source rows and e repair rows (erasures at rotating positions) and writes e rows to dst.
// Build: hipcc --offload-arch=gfx950 -O3 layout_probe.hip -o layout_probe
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
constexpr int K = PK, R = PR, L = PL;

struct Lay {
  uint64_t nb;
  bool sm;
  __device__ __forceinline__ uint64_t row(uint64_t b, int j, int rows) const {  // byte offset of row j of block b
    return sm ? ((uint64_t)j * nb + b) * L : (b * rows + j) * (uint64_t)L;
  }
};

// Random-erasure decode (round 3): MODE 1 = the R erased sources of block b are a random R-subset
// (one of 64 fixed masks, picked by a hash of b), read in slot order as the recover pass does;
// MODE 2 = the same, the recovered rows written packed (out[b][i]) instead of at their slots.
// Combined layout (round 6, COMB_ONLY): each block's k sources and r repairs contiguous, blk[b][k + r][L].
// MODE 3 = random erasures read from it in slot order, recovered rows packed to out[b][i]; MODE 4 = the
// same written into the erased slots; MODE 5 = encode: sources read, repairs written to the block's tail.
__constant__ uint32_t kEras[64];
__device__ __forceinline__ int nth_bit(uint32_t m, int n) {
  for (int i = 0; i < n; i++) m &= m - 1;
  return __ffs(m) - 1;
}

template <int G, bool DEC, int MODE = 0>
__global__ __launch_bounds__(64) void pattern(const uint8_t *__restrict__ src, const uint8_t *__restrict__ rep,
                                              uint8_t *__restrict__ out, uint64_t nblocks, int sm) {
  const int lane = threadIdx.x;
  constexpr int A = (L / 16 + 1) / 2;
  if (lane >= A) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok1 = lane + A < L / 16;
  const Lay ly{nblocks, sm != 0};
  const uint64_t NG = (nblocks + G - 1) / G;
  for (uint64_t q = blockIdx.x; q < NG; q += gridDim.x) {
    for (int g = 0; g < G; g++) {
      const uint64_t b = q + g * NG;
      if (b >= nblocks) break;
      const int e0 = (int)(b % (K - R + 1));  // decode: sources e0 .. e0 + R - 1 erased
      u32x4 x0 = 0, x1 = 0;
      for (int j0 = 0; j0 < K; j0 += 8) {
        u32x4 a0[8], a1[8];
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
          const int j = j0 + jj;
          const uint8_t *p = MODE >= 3 ? src + (b * (K + R) + j) * (uint64_t)L : src + ly.row(b, j, K);
          if (MODE >= 3 && MODE <= 4) {
            const uint32_t m = kEras[(b * 0x9E3779B1u >> 7) & 63];
            if ((m >> j) & 1) p = src + (b * (K + R) + K + __popc(m & ((1u << j) - 1))) * (uint64_t)L;
          } else if (MODE == 1 || MODE == 2) {
            const uint32_t m = kEras[(b * 0x9E3779B1u >> 7) & 63];
            if ((m >> j) & 1) p = rep + ly.row(b, __popc(m & ((1u << j) - 1)), R);
          } else if (DEC && j >= e0 && j < e0 + R) {
            p = rep + ly.row(b, j - e0, R);
          }
          a0[jj] = j < K ? __builtin_nontemporal_load((const u32x4 *)(p + o0)) : (u32x4)0;
          a1[jj] = (ok1 && j < K) ? __builtin_nontemporal_load((const u32x4 *)(p + o1)) : (u32x4)0;
        }
#pragma unroll
        for (int jj = 0; jj < 8; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
      }
#pragma unroll
      for (int i = 0; i < R; i++) {
        uint8_t *p = DEC ? out + ly.row(b, e0 + i, K) : out + ly.row(b, i, R);
        if (MODE == 1) p = out + ly.row(b, nth_bit(kEras[(b * 0x9E3779B1u >> 7) & 63], i), K);
        if (MODE == 2 || MODE == 3) p = out + ly.row(b, i, R);
        if (MODE == 4) p = out + (b * (K + R) + nth_bit(kEras[(b * 0x9E3779B1u >> 7) & 63], i)) * (uint64_t)L;
        if (MODE == 5) p = out + (b * (K + R) + K + i) * (uint64_t)L;
        __builtin_nontemporal_store(x0 + (uint32_t)i, (u32x4 *)(p + o0));
        if (ok1) __builtin_nontemporal_store(x1 + (uint32_t)i, (u32x4 *)(p + o1));
      }
    }
  }
}

// Split pattern (round 3): W waves per block (one workgroup per block), wave w XORs the rows
// w, w + W, ... (ILV: the W waves read W adjacent rows at a time) or the contiguous chunk
// [w K/W, (w + 1) K/W); the partials meet in LDS and wave w writes the output rows i = w mod W.  The
// resident waves then work on W times fewer blocks at once (a smaller window of HBM pages).
template <int W, bool ILV>
__global__ __launch_bounds__(64 * W) void split(const uint8_t *__restrict__ src, const uint8_t *__restrict__ rep,
                                                uint8_t *__restrict__ out, uint64_t nblocks, int) {
  __shared__ u32x4 red[W][2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int A = (L / 16 + 1) / 2;
  constexpr int KW = K / W;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + A);
  const bool ok0 = lane < A, ok1 = lane + A < L / 16;
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    u32x4 x0 = 0, x1 = 0;
    for (int i0 = 0; i0 < KW; i0 += 4) {
      u32x4 a0[4], a1[4];
#pragma unroll
      for (int jj = 0; jj < 4; jj++) {
        const int i = i0 + jj;
        const int j = ILV ? w + W * i : w * KW + i;
        const uint8_t *p = src + (b * K + j) * (uint64_t)L;
        a0[jj] = (ok0 && i < KW) ? __builtin_nontemporal_load((const u32x4 *)(p + o0)) : (u32x4)0;
        a1[jj] = (ok1 && i < KW) ? __builtin_nontemporal_load((const u32x4 *)(p + o1)) : (u32x4)0;
      }
#pragma unroll
      for (int jj = 0; jj < 4; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
    }
    red[w][0][lane] = x0;
    red[w][1][lane] = x1;
    __syncthreads();
    u32x4 y0 = 0, y1 = 0;
#pragma unroll
    for (int v = 0; v < W; v++) { y0 ^= red[v][0][lane]; y1 ^= red[v][1][lane]; }
    for (int i = w; i < R; i += W) {
      uint8_t *p = out + (b * R + i) * (uint64_t)L;
      if (ok0) __builtin_nontemporal_store(y0 + (uint32_t)i, (u32x4 *)(p + o0));
      if (ok1) __builtin_nontemporal_store(y1 + (uint32_t)i, (u32x4 *)(p + o1));
    }
    __syncthreads();
  }
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint64_t nb = (uint64_t)(1 << 20) * 16 / K;
  uint8_t *src, *rep, *dst;
  CK(hipMalloc(&src, nb * (K + R) * L)); CK(hipMalloc(&rep, nb * R * L)); CK(hipMalloc(&dst, nb * (K + R) * L));
  CK(hipMemset(src, 3, nb * (K + R) * L)); CK(hipMemset(rep, 5, nb * R * L)); CK(hipMemset(dst, 0, nb * (K + R) * L));
  auto run = [&](const char *name, size_t lds, auto kern, uint64_t groups, int sm, bool dec, uint8_t *outp = nullptr) {
    float best = 1e9;
    for (int it = 0; it < 6; it++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3((uint32_t)groups), dim3(64), lds, 0, src, rep, outp ? outp : dec ? dst : rep, nb, sm);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (it) best = std::min(best, ms);
    }
    const double bytes = (double)nb * (K + R) * L;
    printf("%-58s %8.3f ms  %7.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  auto runw = [&](const char *name, size_t lds, auto kern, int W) {
    float best = 1e9;
    for (int it = 0; it < 6; it++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3((uint32_t)nb), dim3(64 * W), lds, 0, src, rep, rep, nb, 0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (it) best = std::min(best, ms);
    }
    const double bytes = (double)nb * (K + R) * L;
    printf("%-58s %8.3f ms  %7.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  printf("# k%d r%d L%d, %llu blocks\n", K, R, L, (unsigned long long)nb);
  {
    uint32_t em[64];
    srand(7);
    for (int i = 0; i < 64; i++) {
      uint32_t m = 0;
      while (__builtin_popcount(m) < R) m |= 1u << (rand() % K);
      em[i] = m;
    }
    CK(hipMemcpyToSymbol(HIP_SYMBOL(kEras), em, sizeof em));
  }
  if (getenv("COMB_ONLY")) {  // two arrays (src, rep) against one combined block-major array, alternating
    for (int it = 0; it < 3; it++)
      for (size_t lds : {(size_t)13 << 10, (size_t)10 << 10}) {
        const int wps = lds == ((size_t)13 << 10) ? 3 : 4;
        char nm[96];
#define RUNC(G_, M_, D_, NAME_)                                                                     \
        snprintf(nm, sizeof nm, "%s G%-2d %d waves/SIMD", NAME_, G_, wps);                          \
        run(nm, lds, pattern<G_, D_, M_>, (nb + G_ - 1) / G_, 0, true, M_ >= 4 ? src : nullptr);
        RUNC(1, 2, true, "decode two arrays, packed out  ") RUNC(1, 3, true, "decode combined,   packed out  ")
        RUNC(1, 4, true, "decode combined,   in place    ") RUNC(2, 2, true, "decode two arrays, packed out  ")
        RUNC(2, 3, true, "decode combined,   packed out  ")
        snprintf(nm, sizeof nm, "encode two arrays               G1  %d waves/SIMD", wps);
        run(nm, lds, pattern<1, false>, nb, 0, false);
        RUNC(1, 5, false, "encode combined (repairs in tail)")
      }
    return 0;
  }
  if (getenv("DEC_ONLY")) {  // decode patterns: contiguous erased run / random erasures / random + packed output
    for (size_t lds : {(size_t)13 << 10, (size_t)10 << 10}) {
      const int wps = lds == ((size_t)13 << 10) ? 3 : 4;
      char nm[96];
#define RUND(G_, M_)                                                                              \
      snprintf(nm, sizeof nm, "decode G%-2d %s %d waves/SIMD", G_,                                \
               M_ == 0 ? "erased run      " : M_ == 1 ? "random erasures " : "random, packed  ", wps); \
      run(nm, lds, pattern<G_, true, M_>, (nb + G_ - 1) / G_, 0, true);
      RUND(8, 0) RUND(8, 1) RUND(8, 2) RUND(2, 1) RUND(2, 2) RUND(1, 1) RUND(1, 2)
      snprintf(nm, sizeof nm, "encode G2  block-major  %d waves/SIMD", wps);
      run(nm, lds, pattern<2, false>, (nb + 1) / 2, 0, false);
    }
    return 0;
  }
  if (getenv("SPLIT_ONLY")) {  // encode pattern: one wave per block vs W waves per block
    for (int rep = 0; rep < 6; rep++) {  // alternating, so drift hits every variant alike
      const size_t per = rep & 1 ? (size_t)10 << 10 : (size_t)13 << 10;  // LDS per wave: 3 / 4 waves per SIMD
      const int wps = per == ((size_t)13 << 10) ? 3 : 4;
      char nm[96];
      snprintf(nm, sizeof nm, "encode G1  block-major  %d waves/SIMD", wps);
      run(nm, per, pattern<1, false>, nb, 0, false);
      snprintf(nm, sizeof nm, "encode G2  block-major  %d waves/SIMD", wps);
      run(nm, per, pattern<2, false>, (nb + 1) / 2, 0, false);
#define RUNS(W_, I_)                                                                              \
      snprintf(nm, sizeof nm, "encode split W%d %s %d waves/SIMD", W_, I_ ? "rows-ilv  " : "rows-chunk", wps); \
      runw(nm, per * W_ - sizeof(u32x4) * W_ * 128, split<W_, I_>, W_);
      RUNS(2, true) RUNS(2, false) RUNS(4, true) RUNS(4, false)
    }
    return 0;
  }
  for (size_t lds : {(size_t)13 << 10, (size_t)10 << 10}) {  // 3 / 4 waves per SIMD
    for (int dec = 0; dec < 2; dec++)
      for (int sm = 0; sm < 2; sm++) {
        char nm[96];
#define RUNP(G)                                                                                   \
        snprintf(nm, sizeof nm, "%s G%-2d %s %d waves/SIMD", dec ? "decode" : "encode", G,          \
                 sm ? "symbol-major" : "block-major ", lds == (13u << 10) ? 3 : 4);                 \
        run(nm, lds, dec ? pattern<G, true> : pattern<G, false>, (nb + G - 1) / G, sm, dec);
        RUNP(1) RUNP(2) RUNP(4) RUNP(8)
      }
  }
  return 0;
}
