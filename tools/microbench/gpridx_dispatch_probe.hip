// Mechanism probe for the bitsliced encode kernel (gfx950):
//  (1) s_set_gpr_idx_on(SRC0,DST) offsets VOP3 v_bitop3_b32 and VOP2 v_xor_b32 dst/src0 only;
//  (2) computed call into a code table inside one inline-asm statement: s_swappc_b64 / s_setpc_b64;
//  (3) v_bitop3_b32 truth tables: 0x96 = a^b^c, 0xCA = (a & b) | (~a & c).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void probe(uint32_t *out, const uint32_t *in, uint32_t c0, uint32_t c1, uint32_t mask) {
  int l = threadIdx.x;
  uint32_t a = in[4 * l], b = in[4 * l + 1], c = in[4 * l + 2], d = in[4 * l + 3];
  uint32_t o[16], mux;
  asm volatile(
      "v_mov_b32 v60, %[a]\n v_mov_b32 v61, %[b]\n v_mov_b32 v62, %[c]\n v_mov_b32 v63, %[d]\n"
      "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
      "v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v46, 0\n v_mov_b32 v47, 0\n"
      "v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n"
      "v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n v_mov_b32 v54, 0\n v_mov_b32 v55, 0\n"
      "s_getpc_b64 s[20:21]\n"
      ".Lpc_%=:\n"
      "s_add_u32 s20, s20, .Ltab_%= - .Lpc_%=\n"
      "s_addc_u32 s21, s21, 0\n"
      // call 1: repair 0, case c0
      "s_lshl_b32 s24, %[c0], 6\n"
      "s_add_u32 s26, s20, s24\n s_addc_u32 s27, s21, 0\n"
      "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
      "s_swappc_b64 s[22:23], s[26:27]\n"
      "s_set_gpr_idx_off\n"
      // call 2: repair 1 (offset 8), case c1
      "s_lshl_b32 s24, %[c1], 6\n"
      "s_add_u32 s26, s20, s24\n s_addc_u32 s27, s21, 0\n"
      "s_set_gpr_idx_on 8, gpr_idx(SRC0,DST)\n"
      "s_swappc_b64 s[22:23], s[26:27]\n"
      "s_set_gpr_idx_off\n"
      // call 3: repair 1 again, case 2 (tests accumulation)
      "s_set_gpr_idx_on 8, gpr_idx(SRC0,DST)\n"
      "s_add_u32 s26, s20, 128\n s_addc_u32 s27, s21, 0\n"
      "s_swappc_b64 s[22:23], s[26:27]\n"
      "s_set_gpr_idx_off\n"
      "s_branch .Lend_%=\n"
      ".p2align 6\n"
      ".Ltab_%=:\n"
      // case 0 (64 B): acc[0] ^= T0^T1 ; acc[1] ^= T2 ; return
      "v_bitop3_b32 v40, v40, v60, v61 bitop3:0x96\n"
      "v_xor_b32 v41, v41, v62\n"
      "s_setpc_b64 s[22:23]\n"
      ".p2align 6\n"
      // case 1: acc[2] ^= T3 ; acc[7] ^= T0^T3 ; return
      "v_xor_b32 v42, v42, v63\n"
      "v_bitop3_b32 v47, v47, v60, v63 bitop3:0x96\n"
      "s_setpc_b64 s[22:23]\n"
      ".p2align 6\n"
      // case 2: acc[0] ^= T1^T2 ; return
      "v_bitop3_b32 v40, v40, v61, v62 bitop3:0x96\n"
      "s_setpc_b64 s[22:23]\n"
      ".p2align 6\n"
      ".Lend_%=:\n"
      "v_mov_b32 %[o0], v40\n v_mov_b32 %[o1], v41\n v_mov_b32 %[o2], v42\n v_mov_b32 %[o7], v47\n"
      "v_mov_b32 %[o8], v48\n v_mov_b32 %[o9], v49\n v_mov_b32 %[o10], v50\n v_mov_b32 %[o15], v55\n"
      "v_bitop3_b32 %[mux], %[m], %[a], %[b] bitop3:0xCA\n"
      : [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o7] "=&v"(o[7]), [o8] "=&v"(o[8]),
        [o9] "=&v"(o[9]), [o10] "=&v"(o[10]), [o15] "=&v"(o[15]), [mux] "=&v"(mux)
      : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [c0] "s"(c0), [c1] "s"(c1), [m] "s"(mask)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52",
        "v53", "v54", "v55", "v60", "v61", "v62", "v63", "s20", "s21", "s22", "s23", "s24", "s26",
        "s27", "m0", "scc");
  out[16 * l + 0] = o[0]; out[16 * l + 1] = o[1]; out[16 * l + 2] = o[2]; out[16 * l + 3] = o[7];
  out[16 * l + 4] = o[8]; out[16 * l + 5] = o[9]; out[16 * l + 6] = o[10]; out[16 * l + 7] = o[15];
  out[16 * l + 8] = mux;
}

int main() {
  uint32_t h_in[256], h_out[1024];
  for (int i = 0; i < 256; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ (i << 7);
  uint32_t *d_in, *d_out;
  CK(hipMalloc(&d_in, sizeof h_in)); CK(hipMalloc(&d_out, sizeof h_out));
  CK(hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice));
  CK(hipMemset(d_out, 0, sizeof h_out));
  uint32_t mask = 0x0F0F5533u;
  probe<<<1, 64>>>(d_out, d_in, 0, 1, mask);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; l++) {
    uint32_t a = h_in[4 * l], b = h_in[4 * l + 1], c = h_in[4 * l + 2], d = h_in[4 * l + 3];
    // call1 (acc0, case0): acc0[0]=a^b, acc0[1]=c.  call2 (acc1, case1): acc1[2]=d, acc1[7]=a^d.
    // call3 (acc1, case2): acc1[0]=b^c.
    uint32_t exp[9] = {a ^ b, c, 0, 0, b ^ c, 0, d, a ^ d, (mask & a) | (~mask & b)};
    for (int t = 0; t < 9; t++)
      if (h_out[16 * l + t] != exp[t]) {
        if (bad < 10) printf("lane %d slot %d got %08x exp %08x\n", l, t, h_out[16 * l + t], exp[t]);
        bad++;
      }
  }
  printf(bad ? "PROBE FAIL (%d mismatches)\n" : "PROBE OK: gpr_idx(SRC0,DST) on VOP3+VOP2, swappc table, bitop3 0x96/0xCA\n", bad);
  return bad != 0;
}
