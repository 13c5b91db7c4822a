// Test infrastructure only (never linked into the product): a kernel that holds every CU's whole LDS
// for a bounded time, so that any other kernel launched meanwhile -- the block service's worker --
// stays queued behind it.  Used by tests/test_block_svc_gpu.py to check that a hook call's wait is
// bounded by its deadline when the worker cannot start.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void k_gpu_hog(uint64_t ticks) {
  extern __shared__ uint32_t lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  if (threadIdx.x == 0) lds[0] = 1;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(20);
}

static hipEvent_t g_done = nullptr;
static hipStream_t g_stream = nullptr;

// Holds every CU (one workgroup with 160 KiB of LDS each) for `ms` milliseconds (capped at 2000) on a
// stream of its own.  Returns 0, or a HIP error code.
extern "C" int gpu_hog_launch(int ms) {
  if (ms < 0) ms = 0;
  if (ms > 2000) ms = 2000;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) return 1;
  const uint32_t lds = 160u * 1024u;
  if (hipFuncSetAttribute((const void *)k_gpu_hog, hipFuncAttributeMaxDynamicSharedMemorySize, lds)) return 2;
  if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking)) return 3;
  if (!g_done && hipEventCreateWithFlags(&g_done, hipEventDisableTiming)) return 4;
  hipLaunchKernelGGL(k_gpu_hog, dim3(cus), dim3(64), lds, g_stream, (uint64_t)ms * 100000u);
  if (hipGetLastError()) return 5;
  if (hipEventRecord(g_done, g_stream)) return 6;
  return 0;
}

// Waits for the last hog to end.
extern "C" int gpu_hog_wait(void) { return g_done ? (int)hipEventSynchronize(g_done) : 0; }
