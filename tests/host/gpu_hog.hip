// Test infrastructure only (never linked into the product): a kernel that holds every CU's whole LDS
// until it is released (or at most a bounded time), so that any other kernel launched meanwhile -- the
// block service's worker -- stays queued behind it.  Used by tests/test_block_svc_gpu.py to check that a
// hook call's wait is bounded by its deadline when the worker cannot start.  The tests wait on states,
// not on sleeps: each workgroup counts itself resident in page-locked memory, and the hog ends when the
// host releases it.
#include <hip/hip_runtime.h>
#include <cstdint>

struct HogFlags {
  uint32_t resident;  // workgroups that have started (each holds one CU's whole LDS)
  uint32_t stop;      // set by the host: every workgroup ends at its next poll
};

__global__ void k_gpu_hog(uint64_t ticks, HogFlags *f) {
  extern __shared__ uint32_t lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  if (threadIdx.x == 0) {
    lds[0] = 1;
    __hip_atomic_fetch_add(&f->resident, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks &&
         !__hip_atomic_load(&f->stop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM))
    __builtin_amdgcn_s_sleep(20);
}

static hipEvent_t g_done = nullptr;
static hipStream_t g_stream = nullptr;
static HogFlags *g_flags = nullptr;  // page-locked, fine-grained
static HogFlags *g_flags_dev = nullptr;
static int g_wgs = 0;

// Holds every CU (one workgroup with 160 KiB of LDS each) until gpu_hog_release() or for at most `ms`
// milliseconds (capped at 5000) on a stream of its own.  Returns 0, or a nonzero setup error.
extern "C" int gpu_hog_launch(int ms) {
  if (ms < 0) ms = 0;
  if (ms > 5000) ms = 5000;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) return 1;
  const uint32_t lds = 160u * 1024u;
  if (hipFuncSetAttribute((const void *)k_gpu_hog, hipFuncAttributeMaxDynamicSharedMemorySize, lds)) return 2;
  if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking)) return 3;
  if (!g_done && hipEventCreateWithFlags(&g_done, hipEventDisableTiming)) return 4;
  if (!g_flags) {
    if (hipHostMalloc((void **)&g_flags, sizeof(HogFlags), hipHostMallocMapped | hipHostMallocCoherent)) return 7;
    if (hipHostGetDevicePointer((void **)&g_flags_dev, g_flags, 0)) return 8;
  }
  if (hipEventSynchronize(g_done)) return 9;  // the previous hog has ended before the flags are reset
  __atomic_store_n(&g_flags->resident, 0u, __ATOMIC_RELEASE);
  __atomic_store_n(&g_flags->stop, 0u, __ATOMIC_RELEASE);
  g_wgs = cus;
  hipLaunchKernelGGL(k_gpu_hog, dim3(cus), dim3(64), lds, g_stream, (uint64_t)ms * 100000u, g_flags_dev);
  if (hipGetLastError()) return 5;
  if (hipEventRecord(g_done, g_stream)) return 6;
  return 0;
}

// Workgroups of the last hog that have started, and how many it has: every CU is held once they match.
extern "C" int gpu_hog_resident(void) { return g_flags ? (int)__atomic_load_n(&g_flags->resident, __ATOMIC_ACQUIRE) : 0; }
extern "C" int gpu_hog_workgroups(void) { return g_wgs; }

// 1 while the last hog is still running.
extern "C" int gpu_hog_running(void) { return g_done && hipEventQuery(g_done) == hipErrorNotReady; }

// Ends the last hog at its next poll and waits for it.
extern "C" int gpu_hog_release(void) {
  if (g_flags) __atomic_store_n(&g_flags->stop, 1u, __ATOMIC_RELEASE);
  return g_done ? (int)hipEventSynchronize(g_done) : 0;
}

// Waits for the last hog to end (its time limit, or a release).
extern "C" int gpu_hog_wait(void) { return g_done ? (int)hipEventSynchronize(g_done) : 0; }
