// tools/microbench/glds_probe.hip -- semantics of global_load_lds_dwordx4 on gfx950 (inline asm):
// where the bytes land in LDS for (a) M0 base, (b) an immediate offset, (c) 8-byte-aligned (not
// 16-byte-aligned) global addresses, (d) exec-masked lanes.  Prints PASS/FAIL lines.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void probe(const uint8_t *g, uint32_t *out, int mode) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[8192];
  const int lane = threadIdx.x;
  for (int i = lane; i < 8192 / 4; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = 0xdeadbeefu;
  __syncthreads();
  const uint32_t ldsbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)lds;
  uint64_t base = (uint64_t)(uintptr_t)g;
  uint32_t voff = 16u * lane;
  uint32_t keep;
  if (mode == 0) {  // plain: M0 = ldsbase + 64, global g + 16 lane
    asm volatile("s_mov_b32 %0, m0\n s_mov_b32 m0, %1\n s_nop 0\n global_load_lds_dwordx4 %2, %3\n s_waitcnt vmcnt(0)\n s_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(ldsbase + 64), "v"(voff), "s"(base) : "memory");
  } else if (mode == 1) {  // immediate offset 1024
    asm volatile("s_mov_b32 %0, m0\n s_mov_b32 m0, %1\n s_nop 0\n global_load_lds_dwordx4 %2, %3 offset:1024\n s_waitcnt vmcnt(0)\n s_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(ldsbase + 64), "v"(voff), "s"(base) : "memory");
  } else if (mode == 2) {  // 8-byte aligned global base (g + 8)
    asm volatile("s_mov_b32 %0, m0\n s_mov_b32 m0, %1\n s_nop 0\n global_load_lds_dwordx4 %2, %3\n s_waitcnt vmcnt(0)\n s_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(ldsbase + 64), "v"(voff), "s"(base + 8) : "memory");
  } else {  // exec mask: lanes >= 11 off
    uint64_t em = (1ull << 11) - 1;
    uint64_t sv;
    asm volatile("s_mov_b32 %0, m0\n s_mov_b32 m0, %2\n s_mov_b64 %1, exec\n s_mov_b64 exec, %5\n s_nop 0\n global_load_lds_dwordx4 %3, %4\n s_mov_b64 exec, %1\n s_waitcnt vmcnt(0)\n s_mov_b32 m0, %0"
                 : "=&s"(keep), "=&s"(sv) : "s"(ldsbase + 64), "v"(voff), "s"(base), "s"(em) : "memory");
  }
  __syncthreads();
  for (int i = lane; i < 8192 / 4; i += 64) out[i] = reinterpret_cast<uint32_t *>(lds)[i];
}

int main() {
  uint8_t *g; uint32_t *o;
  hipMalloc(&g, 8192); hipMalloc(&o, 8192);
  uint8_t h[8192];
  for (int i = 0; i < 8192; i++) h[i] = (uint8_t)(i * 7 + (i >> 8));
  hipMemcpy(g, h, 8192, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 4; mode++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, g, o, mode);
    uint32_t r[2048];
    hipMemcpy(r, o, 8192, hipMemcpyDeviceToHost);
    const uint8_t *rb = (const uint8_t *)r;
    // find where byte 0 of the expected source landed
    int gsh = mode == 1 ? 1024 : mode == 2 ? 8 : 0;
    int nl = mode == 3 ? 11 : 64;
    int found = -1;
    for (int o2 = 0; o2 + 16 * nl <= 8192 && found < 0; o2 += 4) {
      bool ok = true;
      for (int i = 0; i < 16 * nl && ok; i++) ok = rb[o2 + i] == h[gsh + i];
      if (ok) found = o2;
    }
    int beyond = 0;  // bytes written outside [found, found + 16 nl)
    for (int i = 0; i < 8192; i += 4)
      if (r[i / 4] != 0xdeadbeefu && (found < 0 || i < found || i >= found + 16 * nl)) beyond++;
    printf("mode %d: data (global +%d, %d lanes) found at LDS offset %d (expected 64 or 64+1024); stray dwords %d\n",
           mode, gsh, nl, found, beyond);
  }
  return 0;
}
