// Probe (round 6, verdict weak 6): can a resident worker take its request and its input rows from device
// memory the CPU writes through the BAR, instead of polling and reading page-locked host memory -- whose
// reads stall for about a bulk kernel while a zero-copy bulk job saturates the host-read path
// (profiles/r06_svc_phase_probe.log)?
//
// 1. Fine-grained device memory (hipExtMallocWithFlags, hipDeviceMallocFinegrained), made accessible to the
//    CPU agent (hsa_amd_agents_allow_access); the CPU writes a request (19,200 B of rows + a sequence word).
// 2. A one-workgroup worker polls the sequence word in device memory, reads the rows from device memory,
//    folds them into 64 words, writes those and its done word to page-locked host memory.
// 3. A bulk kernel streams page-locked host memory (the zero-copy bulk job's read pattern) meanwhile.
// Host-side latency per request (CPU copy + post -> done seen), idle and under the bulk load, p50 / p99.
// Every kernel ends on its own: the worker after `calls` requests or a time limit, the bulk kernel after a
// fixed number of passes or a stop word.
//   build: hipcc --offload-arch=gfx950 -O2 vram_mailbox_probe.hip -o vram_mailbox_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <immintrin.h>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      exit(1);                                                                                   \
    }                                                                                            \
  } while (0)

constexpr int kRowBytes = 19200;  // k16 x 1200 B

struct Box {          // in fine-grained device memory (written by the CPU)
  uint64_t seq;       // request number, written last
  uint64_t pad[15];
  uint8_t rows[kRowBytes];
};
struct Out {          // in page-locked host memory (written by the worker)
  uint64_t done;
  uint64_t pad[15];
  uint32_t fold[64];
};

__global__ void k_worker(Box *box, Out *out, uint64_t calls, uint64_t life_ticks) {
  __shared__ uint64_t go;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t served = 0;
  while (served < calls) {
    if (threadIdx.x == 0) {
      uint64_t s;
      for (;;) {
        s = __hip_atomic_load(&box->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (s == served + 1) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > life_ticks) { s = 0; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      go = s;
    }
    __syncthreads();
    if (go == 0) return;
    const uint64_t t_seen = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(box->rows);
    for (int i = threadIdx.x; i < kRowBytes / 4; i += blockDim.x)
      acc ^= __hip_atomic_load(&w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // outputs by plain (posted) stores: an atomic on host memory is a round trip like a read
    if (threadIdx.x < 64) out->fold[threadIdx.x] = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    served++;
    if (threadIdx.x == 0) {
      out->pad[1] = t_seen;
      out->pad[2] = __builtin_amdgcn_s_memrealtime();  // rows read and folded, outputs written, fence passed
      __hip_atomic_store(&out->done, served, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
  }
}

// streams `bytes` of page-locked host memory `passes` times (sum into a sink), or until *stop
__global__ void k_bulk(const uint4 *src, size_t n16, int passes, const volatile int *stop, uint32_t *sink) {
  uint32_t acc = 0;
  for (int p = 0; p < passes; p++) {
    if (*stop) break;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
      const uint4 v = src[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

static hsa_status_t find_cpu(hsa_agent_t a, void *d) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *(hsa_agent_t *)d = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

static void run(const char *tag, Box *box, Out *out, int calls, std::vector<uint8_t> &rows) {
  std::vector<double> lat;
  lat.reserve(calls);
  for (int c = 1; c <= calls; c++) {
    rows[0] = (uint8_t)c;
    const auto t0 = std::chrono::steady_clock::now();
    memcpy(box->rows, rows.data(), kRowBytes);  // CPU -> device memory through the BAR (write-combined)
    _mm_sfence();                                // the rows leave the write-combining buffers before the post
    __atomic_store_n(&box->seq, (uint64_t)c + 0, __ATOMIC_RELEASE);
    _mm_sfence();                                // and the post itself now, not when a buffer times out
    while (__atomic_load_n(&out->done, __ATOMIC_ACQUIRE) < (uint64_t)c) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        printf("%s: request %d not served within 2 s\n", tag, c);
        return;
      }
    }
    lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(lat.begin(), lat.end());
  printf("%s: %d requests, p50 %.1f us, p90 %.1f us, p99 %.1f us, max %.1f us\n", tag, calls, lat[lat.size() / 2],
         lat[lat.size() * 9 / 10], lat[lat.size() * 99 / 100], lat.back());
  fflush(stdout);
}

int main(int argc, char **argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 2000;
  const bool host_box = argc > 2 && !strcmp(argv[2], "host");  // the baseline: the mailbox in host memory
  // device memory: fine-grained (cached in L2: a CPU write through the BAR is not seen until the line
  // leaves the L2) or uncached (every access of the worker goes to HBM)
  const unsigned dflags = argc > 2 && !strcmp(argv[2], "vram") ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
  CK(hipSetDevice(0));
  Box *box = nullptr;
  if (host_box) {
    CK(hipHostMalloc((void **)&box, sizeof(Box), hipHostMallocMapped | hipHostMallocCoherent));
    memset(box, 0, sizeof(Box));
    printf("mailbox and rows in page-locked host memory (baseline)\n");
  } else {
    CK(hipExtMallocWithFlags((void **)&box, sizeof(Box), dflags));
    CK(hipMemset(box, 0, sizeof(Box)));
    hsa_agent_t cpu{};
    if (hsa_iterate_agents(find_cpu, &cpu) != HSA_STATUS_INFO_BREAK) { printf("no CPU agent\n"); return 1; }
    const hsa_status_t st = hsa_amd_agents_allow_access(1, &cpu, nullptr, box);
    printf("mailbox and rows in %s device memory; allow_access(CPU): %d\n",
           dflags == hipDeviceMallocUncached ? "uncached" : "fine-grained", (int)st);
    if (st != HSA_STATUS_SUCCESS) return 1;
  }
  CK(hipDeviceSynchronize());
  // a CPU write and read back through the pointer (faults here if the BAR does not map it)
  box->pad[0] = 0xC0FFEE;
  printf("CPU read back %#lx\n", (unsigned long)box->pad[0]);
  Out *out = nullptr;
  CK(hipHostMalloc((void **)&out, sizeof(Out), hipHostMallocMapped | hipHostMallocCoherent));
  memset(out, 0, sizeof(Out));
  std::vector<uint8_t> rows(kRowBytes, 0x5A);
  {  // CPU write speed into device memory
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 200; i++) memcpy(box->rows, rows.data(), kRowBytes);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 200;
    printf("CPU memcpy of %d B into device memory: %.2f us (%.2f GB/s)\n", kRowBytes, us, kRowBytes / us / 1e3);
  }
  hipStream_t sw, sb;
  CK(hipStreamCreateWithFlags(&sw, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  const uint64_t life = 20ull * 100000000ull;  // 20 s at 100 MHz
  hipLaunchKernelGGL(k_worker, dim3(1), dim3(256), 0, sw, box, out, (uint64_t)(2 * calls), life);
  CK(hipGetLastError());
  run("idle (no bulk job)", box, out, calls, rows);
  // the bulk job: 1 GiB of page-locked host memory streamed by the whole chip
  const size_t bulk_bytes = 1ull << 30;
  uint4 *hb = nullptr;
  int *stop = nullptr;
  uint32_t *sink = nullptr;
  CK(hipHostMalloc((void **)&hb, bulk_bytes, hipHostMallocMapped));
  memset(hb, 1, bulk_bytes);
  CK(hipHostMalloc((void **)&stop, 64, hipHostMallocMapped | hipHostMallocCoherent));
  *stop = 0;
  CK(hipMalloc((void **)&sink, 64));
  hipLaunchKernelGGL(k_bulk, dim3(2048), dim3(256), 0, sb, hb, bulk_bytes / 16, 400, (const volatile int *)stop, sink);
  CK(hipGetLastError());
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  // the served count continues from `calls`: shift the numbering
  std::vector<double> lat, cp, wk;
  for (int c = calls + 1; c <= 2 * calls; c++) {
    rows[0] = (uint8_t)c;
    const auto t0 = std::chrono::steady_clock::now();
    memcpy(box->rows, rows.data(), kRowBytes);
    _mm_sfence();
    __atomic_store_n(&box->seq, (uint64_t)c, __ATOMIC_RELEASE);
    _mm_sfence();
    const auto t1 = std::chrono::steady_clock::now();
    bool ok = true;
    while (__atomic_load_n(&out->done, __ATOMIC_ACQUIRE) < (uint64_t)c)
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) { ok = false; break; }
    if (!ok) { printf("loaded: request %d not served within 2 s\n", c); break; }
    lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    cp.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    wk.push_back((double)(__atomic_load_n(&out->pad[2], __ATOMIC_ACQUIRE) - out->pad[1]) / 100.0);
  }
  if (!cp.empty()) {
    std::sort(cp.begin(), cp.end());
    std::sort(wk.begin(), wk.end());
    printf("loaded phases: host copy + post p50 %.1f p99 %.1f us; worker seen -> outputs fenced p50 %.1f p99 %.1f us\n",
           cp[cp.size() / 2], cp[cp.size() * 99 / 100], wk[wk.size() / 2], wk[wk.size() * 99 / 100]);
  }
  const bool bulk_running = hipStreamQuery(sb) == hipErrorNotReady;
  *stop = 1;
  CK(hipStreamSynchronize(sb));
  CK(hipStreamSynchronize(sw));
  if (!lat.empty()) {
    std::sort(lat.begin(), lat.end());
    printf("loaded (bulk job streaming page-locked host memory%s): %zu requests, p50 %.1f us, p90 %.1f us, p99 %.1f "
           "us, max %.1f us\n", bulk_running ? ", still running at the end" : ", ENDED before the requests did",
           lat.size(), lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat[lat.size() * 99 / 100], lat.back());
  }
  return 0;
}
