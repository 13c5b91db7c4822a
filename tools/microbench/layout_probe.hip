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

template <int G, bool DEC>
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
          const uint8_t *p = src + ly.row(b, j, K);
          if (DEC && j >= e0 && j < e0 + R) p = rep + ly.row(b, j - e0, R);
          a0[jj] = j < K ? __builtin_nontemporal_load((const u32x4 *)(p + o0)) : (u32x4)0;
          a1[jj] = (ok1 && j < K) ? __builtin_nontemporal_load((const u32x4 *)(p + o1)) : (u32x4)0;
        }
#pragma unroll
        for (int jj = 0; jj < 8; jj++) { x0 ^= a0[jj]; x1 ^= a1[jj]; }
      }
#pragma unroll
      for (int i = 0; i < R; i++) {
        uint8_t *p = DEC ? out + ly.row(b, e0 + i, K) : out + ly.row(b, i, R);
        __builtin_nontemporal_store(x0 + (uint32_t)i, (u32x4 *)(p + o0));
        if (ok1) __builtin_nontemporal_store(x1 + (uint32_t)i, (u32x4 *)(p + o1));
      }
    }
  }
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint64_t nb = (uint64_t)(1 << 20) * 16 / K;
  uint8_t *src, *rep, *dst;
  CK(hipMalloc(&src, nb * K * L)); CK(hipMalloc(&rep, nb * R * L)); CK(hipMalloc(&dst, nb * K * L));
  CK(hipMemset(src, 3, nb * K * L)); CK(hipMemset(rep, 5, nb * R * L)); CK(hipMemset(dst, 0, nb * K * L));
  auto run = [&](const char *name, size_t lds, auto kern, uint64_t groups, int sm, bool dec) {
    float best = 1e9;
    for (int it = 0; it < 6; it++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3((uint32_t)groups), dim3(64), lds, 0, src, rep, dec ? dst : rep, nb, sm);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (it) best = std::min(best, ms);
    }
    const double bytes = (double)nb * (K + R) * L;
    printf("%-58s %8.3f ms  %7.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  printf("# k%d r%d L%d, %llu blocks\n", K, R, L, (unsigned long long)nb);
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
