// Ceiling probe for the RLC data path's memory pattern (k sources in, r repairs out per block,
// 1200-B symbols, [block][symbol][byte] layout) with trivial compute (XOR), to separate the
// memory-pattern limit from the GF arithmetic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// V1: one wave per group of G blocks, 38 lanes x 2 x 16 B per symbol (the bitsliced kernel's mapping)
template <int R, int P, bool NT, int ST = 0>
__global__ __launch_bounds__(64) void v1(const uint8_t *src, uint8_t *rep, int nblocks, int k, int L, int G) {
  const int lane = threadIdx.x;
  const int act = 38;
  if (lane >= act) return;
  const uint32_t o0 = 16 * lane, o1 = 16 * (lane + 38);
  const bool ok1 = lane + 38 < 75;
  for (int g0 = blockIdx.x * G; g0 < nblocks; g0 += gridDim.x * G) {
    int ng = nblocks - g0 < G ? nblocks - g0 : G;
    const uint8_t *s = src + (size_t)g0 * k * L;
    for (int g = 0; g < ng; g++) {
      u32x4 acc[R][2];
      for (int i = 0; i < R; i++) acc[i][0] = acc[i][1] = 0;
      const uint8_t *sb = s + (size_t)g * k * L;
#pragma unroll 4
      for (int j = 0; j < k; j++) {
        const u32x4 *p0 = (const u32x4 *)(sb + (size_t)j * L + o0);
        const u32x4 *p1 = (const u32x4 *)(sb + (size_t)j * L + o1);
        u32x4 a = NT ? __builtin_nontemporal_load(p0) : *p0;
        u32x4 b = ok1 ? (NT ? __builtin_nontemporal_load(p1) : *p1) : (u32x4)0;
#pragma unroll
        for (int i = 0; i < R; i++) { acc[i][0] ^= a; acc[i][1] ^= b; }
      }
      uint8_t *rb = rep + ((size_t)(g0 + g) * R) * L;
      for (int i = 0; i < R; i++) {
        if (ST == 1) {
          __builtin_nontemporal_store(acc[i][0], (u32x4 *)(rb + (size_t)i * L + o0));
          if (ok1) __builtin_nontemporal_store(acc[i][1], (u32x4 *)(rb + (size_t)i * L + o1));
        } else {
          *(u32x4 *)(rb + (size_t)i * L + o0) = acc[i][0];
          if (ok1) *(u32x4 *)(rb + (size_t)i * L + o1) = acc[i][1];
        }
      }
    }
  }
}

// V3: flat streaming, all lanes busy: thread t -> (block, 16-B chunk), 64 lanes contiguous
template <int R>
__global__ __launch_bounds__(256) void v3(const uint8_t *src, uint8_t *rep, int nblocks, int k, int L) {
  const int cpb = L / 16;
  const size_t total = (size_t)nblocks * cpb;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    size_t b = t / cpb, c = t % cpb;
    const u32x4 *p = (const u32x4 *)(src + b * k * L + 16 * c);
    u32x4 a = 0;
    for (int j = 0; j < k; j++) a ^= __builtin_nontemporal_load(p + j * (L / 16));
    for (int i = 0; i < R; i++) __builtin_nontemporal_store(a, (u32x4 *)(rep + (b * R + i) * L + 16 * c));
  }
}

int main() {
  const int L = 1200;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct Cfg { int k, R, nb; } cfgs[] = {{16, 4, 1 << 20}, {32, 8, 1 << 21}};
  for (auto c : cfgs) {
    size_t sb = (size_t)c.nb * c.k * L, rb = (size_t)c.nb * c.R * L;
    uint8_t *src, *rep;
    CK(hipMalloc(&src, sb)); CK(hipMalloc(&rep, rb));
    CK(hipMemset(src, 3, sb));
    double bytes = (double)(sb + rb);
    auto run = [&](const char *name, auto launch) {
      float best = 1e9;
      for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (it) best = std::min(best, ms);
      }
      printf("k=%d r=%d %-28s %8.3f ms  %7.0f GB/s\n", c.k, c.R, name, best, bytes / (best * 1e-3) / 1e9);
    };
    int G = 8;
    int groups = (c.nb + G - 1) / G;
    if (c.R == 4) {
      run("v1 wave/block 38 lanes", [&] { v1<4, 4, false><<<groups, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 nontemporal loads", [&] { v1<4, 4, true><<<groups, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 grid/4", [&] { v1<4, 4, true><<<groups / 4, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 nt stores", [&] { v1<4, 4, false, 1><<<groups, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 G=16", [&] { v1<4, 4, false><<<(c.nb + 15) / 16, 64>>>(src, rep, c.nb, c.k, L, 16); });
      run("v1 G=2", [&] { v1<4, 4, false><<<(c.nb + 1) / 2, 64>>>(src, rep, c.nb, c.k, L, 2); });
      run("v3 flat all lanes", [&] { v3<4><<<8192, 256>>>(src, rep, c.nb, c.k, L); });
    } else {
      run("v1 wave/block 38 lanes", [&] { v1<8, 4, false><<<groups, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 nontemporal loads", [&] { v1<8, 4, true><<<groups, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 nt stores", [&] { v1<8, 4, false, 1><<<groups, 64>>>(src, rep, c.nb, c.k, L, G); });
      run("v1 G=2", [&] { v1<8, 4, false><<<(c.nb + 1) / 2, 64>>>(src, rep, c.nb, c.k, L, 2); });
      run("v3 flat all lanes", [&] { v3<8><<<8192, 256>>>(src, rep, c.nb, c.k, L); });
    }
    CK(hipFree(src)); CK(hipFree(rep));
  }
  return 0;
}
