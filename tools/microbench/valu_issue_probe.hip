// VALU issue-rate probe: which 32-bit integer ops issue at full SIMD-32 rate on gfx950.
// Each kernel runs 16 independent register chains of one instruction (inline asm, so the
// compiler cannot fuse or reorder). Reports lane-ops/s for the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

#define BODY16(INS) \
  asm volatile( \
    INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7) \
    INS(8) INS(9) INS(10) INS(11) INS(12) INS(13) INS(14) INS(15) \
    : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
      "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) \
    : "v"(a), "v"(b));

#define I_XOR(n)    "v_xor_b32 %" #n ", %16, %" #n "\n"
#define I_AND(n)    "v_and_b32 %" #n ", %16, %" #n "\n"
#define I_LSHR(n)   "v_lshrrev_b32 %" #n ", 3, %" #n "\n"
#define I_PERM(n)   "v_perm_b32 %" #n ", %16, %17, %" #n "\n"
#define I_BITOP3(n) "v_bitop3_b32 %" #n ", %16, %17, %" #n " bitop3:0x96\n"
#define I_BFI(n)    "v_bfi_b32 %" #n ", %16, %17, %" #n "\n"
#define I_FMA(n)    "v_fma_f32 %" #n ", %16, %17, %" #n "\n"
#define I_XOR_E64(n) "v_xor_b32_e64 %" #n ", %16, %" #n "\n"

template <int OP>
__global__ void k(unsigned* out, int iters) {
  unsigned x[16];
  for (int j = 0; j < 16; ++j) x[j] = threadIdx.x * 2654435761u + j;
  unsigned a = 0x03020100u ^ blockIdx.x, b = 0x07060504u;
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) { BODY16(I_XOR) }
    if constexpr (OP == 1) { BODY16(I_AND) }
    if constexpr (OP == 2) { BODY16(I_LSHR) }
    if constexpr (OP == 3) { BODY16(I_PERM) }
    if constexpr (OP == 4) { BODY16(I_BITOP3) }
    if constexpr (OP == 5) { BODY16(I_BFI) }
    if constexpr (OP == 6) { BODY16(I_FMA) }
    if constexpr (OP == 7) { BODY16(I_XOR_E64) }
  }
  unsigned r = 0;
  for (int j = 0; j < 16; ++j) r ^= x[j];
  if (r == 0x9e3779b9u) out[0] = r;
}

// 64-bit shifts (two dwords per op): does v_lshlrev_b64 issue at full rate?  16 chains of 64 bits.
#define BODY16W(INS) \
  asm volatile( \
    INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7) \
    INS(8) INS(9) INS(10) INS(11) INS(12) INS(13) INS(14) INS(15) \
    : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]), \
      "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), "+v"(y[13]), "+v"(y[14]), "+v"(y[15]));
#define I_SHL64(n)  "v_lshlrev_b64 %" #n ", 3, %" #n "\n"
#define I_SHR64(n)  "v_lshrrev_b64 %" #n ", 3, %" #n "\n"
#define I_SHL32P(n) "v_lshlrev_b32 %" #n ", 3, %" #n "\n"

template <int OP>
__global__ void kw(unsigned* out, int iters) {
  unsigned long long y[16];
  for (int j = 0; j < 16; ++j) y[j] = threadIdx.x * 0x9E3779B97F4A7C15ull + j;
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) { BODY16W(I_SHL64) }
    if constexpr (OP == 1) { BODY16W(I_SHR64) }
  }
  unsigned long long r = 0;
  for (int j = 0; j < 16; ++j) r ^= y[j];
  if (r == 0x9e3779b9u) out[0] = (unsigned)r;
}

template <int OP>
void runw(const char* name, unsigned* o) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int iters = 2048, blocks = 8192;
  float ms, best = 1e9;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0)); kw<OP><<<blocks, 256>>>(o, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms);
  }
  double ops = (double)blocks * 256 * iters * 16;
  printf("%-10s blocks %5d: %6.1f T lane-ops/s (64-bit ops; x2 for dwords)\n", name, blocks, ops / (best * 1e-3) / 1e12);
}

template <int OP>
void run(const char* name, unsigned* o) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int iters = 2048;
  int blist[] = {1024, 2048, 8192};
  for (int blocks : blist) {
    float ms, best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0)); k<OP><<<blocks, 256>>>(o, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms);
    }
    double ops = (double)blocks * 256 * iters * 16;
    printf("%-10s blocks %5d: %6.1f T lane-ops/s\n", name, blocks, ops / (best * 1e-3) / 1e12);
  }
}

int main() {
  unsigned* o; CK(hipMalloc(&o, 64));
  run<0>("v_xor", o); run<7>("v_xor_e64", o); run<1>("v_and", o); run<2>("v_lshrrev", o);
  run<3>("v_perm", o); run<4>("v_bitop3", o); run<5>("v_bfi", o); run<6>("v_fma_f32", o);
  runw<0>("v_lshl_b64", o); runw<1>("v_lshr_b64", o);
  return 0;
}
