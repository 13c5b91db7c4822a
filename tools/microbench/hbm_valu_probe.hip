// Calibration probe for the FEC kernels' two candidate bounds on MI355X:
//   (1) HBM streaming rates: copy / read-only / write-only with 16-B lanes;
//   (2) VALU issue rate of the ops the GF(256) multiply uses (v_perm_b32, v_bitop3_b32).
// Not part of the product; results are quoted in DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__global__ void k_copy(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += st) d[i] = s[i];
}
__global__ void k_read(const uint4* __restrict__ s, unsigned* __restrict__ d, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  unsigned a = 0;
  for (; i < n; i += st) { uint4 v = s[i]; a ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (a == 0x12345678u) d[0] = a;
}
__global__ void k_write(uint4* __restrict__ d, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += st) d[i] = make_uint4(i, i, i, i);
}
// 8 independent chains; per iteration 8 v_perm + 8 v_bitop3 = 16 VALU ops per lane
__global__ void k_valu(unsigned* out, int iters, unsigned t0, unsigned t1) {
  unsigned x[8];
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 2654435761u + j;
  unsigned a = t0 ^ threadIdx.x, b = t1 + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      unsigned p = __builtin_amdgcn_perm(a, b, x[j]);
      x[j] = __builtin_amdgcn_bitop3_b32(x[j], p, a, 0x96);
    }
  }
  unsigned r = 0;
  for (int j = 0; j < 8; ++j) r ^= x[j];
  if (r == 0x9e3779b9u) out[0] = r;
}

int main(int argc, char** argv) {
  size_t bytes = (size_t)4 << 30;
  size_t n = bytes / 16;
  uint4 *a, *b; unsigned* o;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 1, bytes)); CK(hipMemset(b, 2, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (int g : grids) {
    float ms; double best_c = 0, best_r = 0, best_w = 0;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0)); k_copy<<<g, 256>>>(a, b, n); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); best_c = std::max(best_c, 2.0 * bytes / (ms * 1e-3) / 1e9);
      CK(hipEventRecord(e0)); k_read<<<g, 256>>>(a, o, n); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); best_r = std::max(best_r, 1.0 * bytes / (ms * 1e-3) / 1e9);
      CK(hipEventRecord(e0)); k_write<<<g, 256>>>(b, n); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); best_w = std::max(best_w, 1.0 * bytes / (ms * 1e-3) / 1e9);
    }
    printf("grid %6d x256: copy %.0f GB/s (r+w)  read %.0f GB/s  write %.0f GB/s\n", g, best_c, best_r, best_w);
  }
  int iters = 4096;
  int blocks_list[] = {256, 512, 1024, 2048, 4096, 8192};
  for (int blocks : blocks_list) {
    float ms, best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0)); k_valu<<<blocks, 256>>>(o, iters, 0x03020100u, 0x07060504u); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms);
    }
    double ops = (double)blocks * 256 * iters * 16;
    printf("valu blocks %5d (waves/SIMD %.1f): %.1f T lane-ops/s (perm+bitop3)\n", blocks, blocks * 4.0 / 1024, ops / (best * 1e-3) / 1e12);
  }
  return 0;
}
