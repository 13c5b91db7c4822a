// Copy-style probe: does the launch pattern (one-shot vs grid-stride, items per thread, blit
// engine) move the plain-streaming ceiling of hbm_ceiling_probe.hip?  The FEC kernels are judged
// against the best of these.  Build: hipcc --offload-arch=gfx950 -O3 copy_style_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) { if constexpr (NT) return __builtin_nontemporal_load(p); else return *p; }
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) { if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v; }

// one-shot copy: each workgroup of 256 copies U * 256 units (coalesced, U in flight per thread)
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_oneshot(const u32x4 *__restrict__ in, u32x4 *__restrict__ out) {
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = ld<NT>(in + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; u++) st<NT>(out + base + u * 256, v[u]);
}

// one-shot 4:1 mix shaped like encode k=4 r=1: a wave reads 4 consecutive 1-KiB rows, writes 1
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void mix41_oneshot(const u32x4 *__restrict__ in, u32x4 *__restrict__ out) {
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const u32x4 *p = in + w * 256 + lane;
  u32x4 a = ld<NTL>(p) ^ ld<NTL>(p + 64) ^ ld<NTL>(p + 128) ^ ld<NTL>(p + 192);
  st<NTS>(out + w * 64 + lane, a);
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const size_t nb = (size_t)8 << 30;  // 8 GiB each way, far beyond the 256 MiB Infinity Cache
  u32x4 *in, *out;
  CK(hipMalloc(&in, nb)); CK(hipMalloc(&out, nb));
  CK(hipMemset(in, 3, nb)); CK(hipMemset(out, 0, nb));
  const size_t units = nb / 16;
  auto run = [&](const char *name, double bytes, auto launch) {
    float best = 1e9;
    for (int it = 0; it < 5; it++) {
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (it) best = std::min(best, ms);
    }
    printf("%-40s %8.3f ms  %7.0f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  run("hipMemcpyAsync D2D", 2.0 * nb, [&] { CK(hipMemcpyAsync(out, in, nb, hipMemcpyDeviceToDevice, 0)); });
  run("copy one-shot U1", 2.0 * nb, [&] { copy_oneshot<1, false><<<units / 256, 256>>>(in, out); });
  run("copy one-shot U4", 2.0 * nb, [&] { copy_oneshot<4, false><<<units / 1024, 256>>>(in, out); });
  run("copy one-shot U4 nt", 2.0 * nb, [&] { copy_oneshot<4, true><<<units / 1024, 256>>>(in, out); });
  run("copy one-shot U8 nt", 2.0 * nb, [&] { copy_oneshot<8, true><<<units / 2048, 256>>>(in, out); });
  run("copy one-shot U16 nt", 2.0 * nb, [&] { copy_oneshot<16, true><<<units / 4096, 256>>>(in, out); });
  // 4:1 mix: reads nb, writes nb / 4
  run("mix4:1 one-shot", 1.25 * nb, [&] { mix41_oneshot<false, false><<<units / 1024, 256>>>(in, out); });
  run("mix4:1 one-shot nt/nt", 1.25 * nb, [&] { mix41_oneshot<true, true><<<units / 1024, 256>>>(in, out); });
  run("mix4:1 one-shot ld/nt", 1.25 * nb, [&] { mix41_oneshot<false, true><<<units / 1024, 256>>>(in, out); });
  return 0;
}
