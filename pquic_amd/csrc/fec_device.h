// pquic_amd/csrc/fec_device.h -- device-side building blocks of the FEC engine (gfx950).
//
//   * TinyMT32 coefficient streams, bit-exact with plugins/fec/prng/tinymt32.c:60-161,301-315
//     and get_coefs (rlc_fec_scheme_generate_gf256.c:9-17).
//   * GF(2^8)/0x11D scalar arithmetic (gf256/swif_symbol.c:16-29) for the elimination.
//   * The packed GF multiply-accumulate of the one-block kernels (k_rlc_encode_lds,
//     k_rlc_decode_lds, k_block_svc; the batched data path is bit-sliced, bitslice_gen.h): a
//     byte-wise product by a constant c is split over the bit fields
//     x = x[2:0] | x[5:3] << 3 | x[7:6] << 6, and each field is looked up with one v_perm_b32 in
//     an 8-entry product table held in a pair of 32-bit registers (c*x[2:0], c*(x[5:3] << 3),
//     c*(x[7:6] << 6)); the three partial products are XOR-ed in with v_bitop3_b32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fecdev {

// ---------------------------------------------------------------- TinyMT32 ------------
constexpr uint32_t kMat1 = 0x8f7011eeu, kMat2 = 0xfc78ff1fu, kTmat = 0x3793fdffu;

struct Tmt { uint32_t s0, s1, s2, s3; };

__device__ __forceinline__ void tmt_next(Tmt &t) {
  uint32_t y = t.s3;
  uint32_t x = (t.s0 & 0x7fffffffu) ^ t.s1 ^ t.s2;
  x ^= x << 1;
  y ^= (y >> 1) ^ x;
  t.s0 = t.s1;
  t.s1 = t.s2;
  t.s2 = x ^ (y << 10);
  t.s3 = y;
  uint32_t m = 0u - (y & 1u);
  t.s1 ^= m & kMat1;
  t.s2 ^= m & kMat2;
}

__device__ __forceinline__ uint32_t tmt_temper(const Tmt &t) {
  uint32_t t1 = t.s0 + (t.s2 >> 8);
  uint32_t t0 = t.s3 ^ t1;
  return t0 ^ ((0u - (t1 & 1u)) & kTmat);
}

__device__ __forceinline__ void tmt_init(Tmt &t, uint32_t seed) {
  uint32_t st[4] = {seed, kMat1, kMat2, kTmat};
#pragma unroll
  for (uint32_t i = 1; i < 8; i++) {
    uint32_t p = st[(i - 1) & 3];
    st[i & 3] ^= i + 1812433253u * (p ^ (p >> 30));
  }
  if ((st[0] & 0x7fffffffu) == 0 && st[1] == 0 && st[2] == 0 && st[3] == 0) {
    st[0] = 'T'; st[1] = 'I'; st[2] = 'N'; st[3] = 'Y';
  }
  t.s0 = st[0]; t.s1 = st[1]; t.s2 = st[2]; t.s3 = st[3];
#pragma unroll
  for (int i = 0; i < 8; i++) tmt_next(t);
}

__device__ __forceinline__ uint8_t tmt_coef(Tmt &t) {
  tmt_next(t);
  uint8_t c = (uint8_t)tmt_temper(t);
  return c ? c : 1;
}

__device__ __forceinline__ uint32_t rlc_seed(uint32_t fbn, uint32_t i) {
  return ((fbn & 0xffffffu) << 8) | (i & 0xffu);
}

// ---------------------------------------------------------------- GF(2^8) scalar ------
__device__ __forceinline__ uint32_t gf_xtime(uint32_t a) {  // a < 256
  return (a << 1) ^ ((a >> 7) * 0x11du);  // the carry's 0x100 cancels bit 8 of a << 1
}

__device__ __forceinline__ uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    p ^= (b & 1u) ? a : 0u;
    b >>= 1;
    a = gf_xtime(a);
  }
  return p;
}

// Multiplicative inverse: a^254 (a^(2^8-2)); inv(0) = 0 like the reference's table.
__device__ __forceinline__ uint32_t gf_inv(uint32_t a) {
  uint32_t r = 1, b = a;
#pragma unroll
  for (int i = 0; i < 8; i++) {  // 254 = 0b11111110
    if ((254u >> i) & 1u) r = gf_mul(r, b);
    b = gf_mul(b, b);
  }
  return a ? r : 0u;
}

// ---------------------------------------------------------------- perm tables ---------
// Five dwords per coefficient: {T0lo, T0hi, T1lo, T1hi} and T2.
struct PermTab { uint4 t01; uint32_t t2; };

__device__ __forceinline__ uint32_t bcast8(uint32_t x) {  // byte 0 of x in all four bytes
  return __builtin_amdgcn_perm(0u, x, 0x00000000u);
}

// The 4-entry half tables {0, a, b, a^b} packed in one dword.
__device__ __forceinline__ uint32_t pair_table(uint32_t a, uint32_t b) {
  return (a << 8) | (b << 16) | ((a ^ b) << 24);
}

__device__ __forceinline__ PermTab perm_table(uint32_t c) {
  uint32_t p[8];
  p[0] = c;
#pragma unroll
  for (int i = 1; i < 8; i++) p[i] = gf_xtime(p[i - 1]);  // c * 2^i
  // t01: bytes x = 0..7 of c * x[2:0] (dwords 0-1) and c * (x << 3) (dwords 2-3); the upper
  // half of an 8-entry table is the lower half XOR the product of its top bit
  PermTab t;
  const uint32_t lo0 = pair_table(p[0], p[1]), lo3 = pair_table(p[3], p[4]);
  t.t01 = make_uint4(lo0, lo0 ^ bcast8(p[2]), lo3, lo3 ^ bcast8(p[5]));
  t.t2 = pair_table(p[6], p[7]);  // c * (x << 6), x < 4
  return t;
}

struct Sel { uint32_t s0, s1, s2; };

__device__ __forceinline__ Sel perm_selectors(uint32_t s) {
  Sel r;
  r.s0 = s & 0x07070707u;
  r.s1 = (s >> 3) & 0x07070707u;
  r.s2 = (s >> 6) & 0x03030303u;
  return r;
}

// acc ^= c * s (bytewise), with c's table in registers and s pre-split into selectors.
__device__ __forceinline__ uint32_t gf_mac(uint32_t acc, const Sel &x, const uint4 &t01, uint32_t t2) {
  uint32_t p0 = __builtin_amdgcn_perm(t01.y, t01.x, x.s0);
  uint32_t p1 = __builtin_amdgcn_perm(t01.w, t01.z, x.s1);
  uint32_t p2 = __builtin_amdgcn_perm(t2, t2, x.s2);
  return __builtin_amdgcn_bitop3_b32(acc, p0, p1, 0x96) ^ p2;  // 0x96: 3-input XOR
}

}  // namespace fecdev
