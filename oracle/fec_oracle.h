/*
 * oracle/fec_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A clean-room CPU restatement of the arithmetic on PQUIC's plugins/fec hot path:
 *   GF(2^8)/0x11D tables, TinyMT32 coefficient streams, RLC and XOR encode, and a
 *   reference-faithful RLC / XOR recover (same repair selection, same row sort,
 *   elimination without re-pivoting, same "undetermined" bookkeeping).
 * Every function cites the reference file:line it restates (paths relative to
 * p-quic/pquic, plugins/fec/...).
 *
 * Parity is PINNED: tests/golden/ holds fixtures produced by the reference's own
 * scheme sources compiled natively (oracle/ref/, output in oracle/_ref/), and the
 * CPU test suite checks this restatement against them byte for byte.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product (pquic_amd/, libpquic_fec.so) never links it.
 */
#ifndef PQUIC_FEC_ORACLE_H
#define PQUIC_FEC_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Outcome of a reference recover on one block (fec_recover's observable result). */
#define ORACLE_DEC_RECOVERED   0   /* recovery ran; fec_recover returned 0            */
#define ORACLE_DEC_NOTHING     1   /* a precondition failed; nothing recovered        */
#define ORACLE_DEC_REF_UB      2   /* reference indexes x[-1] / overflows: it crashes  */

/* --- GF(2^8), polynomial 0x11D (gf256/swif_symbol.c:16-29, generated_table_code.c:4-14) --- */
void oracle_gf_tables(uint8_t *mul /* 65536, [a][b] */, uint8_t *inv /* 256 */);
uint8_t oracle_gf_mul(uint8_t a, uint8_t b);

/* --- TinyMT32 coefficients (prng/tinymt32.c:60-161,301-315; get_coefs
 *     rlc_fec_scheme_generate_gf256.c:9-17) --- */
uint32_t oracle_tinymt32_first(uint32_t seed);          /* first generate_uint32 after init */
void oracle_tinymt32_stream(uint32_t seed, int n, uint32_t *out);
void oracle_rlc_coefs(uint32_t seed, int n, uint8_t *coefs);
uint32_t oracle_rlc_seed(uint32_t fbn, uint32_t repair_index);

/* --- Per-block functions with the reference's variable-length symbols. ---
 * src[j] == NULL marks a missing source, rep[i] == NULL a missing repair. */
int oracle_rlc_encode_block(uint32_t fbn, int k, int r,
                            const uint8_t *const *src, const uint16_t *src_len,
                            uint8_t *const *rep /* r buffers >= max len */,
                            uint16_t *rep_len);
int oracle_xor_encode_block(int k, int r,
                            const uint8_t *const *src, const uint16_t *src_len,
                            uint8_t *rep, uint16_t *rep_len);
/* Returns ORACLE_DEC_*.  out[j] receives recovered source j (max_length bytes),
 * recovered[j] is set to 1 for every source the reference would insert. */
int oracle_rlc_decode_block(uint32_t fbn, int k, int r,
                            const uint8_t *const *src, const uint16_t *src_len,
                            const uint8_t *const *rep, const uint16_t *rep_len,
                            const uint32_t *rep_seed /* NULL: oracle_rlc_seed(fbn, i) */,
                            uint8_t *const *out, uint16_t *out_len, uint8_t *recovered);
int oracle_xor_decode_block(int k, int r,
                            const uint8_t *const *src, const uint16_t *src_len,
                            const uint8_t *const *rep, const uint16_t *rep_len,
                            uint8_t *out, uint16_t *out_len, int *recovered_index);

/* --- Batched, fixed-size layout (the same layout the device engine uses) ---
 * src: [nblocks][k][L] bytes, rep: [nblocks][r][L] bytes, L % 4 == 0 not required.
 * fbn of block b = (fbn_base + b) & 0xFFFFFF.  nthreads <= 0 -> one per online core.
 * Presence masks: bit j of src_present[b*2 + (j>>6)], same for repairs.
 * status[b] = ORACLE_DEC_*, recovered[b*2..] = mask of recovered sources.            */
int oracle_rlc_encode_batch(const uint8_t *src, uint8_t *rep, uint64_t nblocks,
                            int k, int r, int L, uint32_t fbn_base, int nthreads);
int oracle_rlc_decode_batch(uint8_t *src, const uint8_t *rep, uint64_t nblocks,
                            int k, int r, int L, uint32_t fbn_base,
                            const uint64_t *src_present, const uint64_t *rep_present,
                            uint8_t *status, uint64_t *recovered, int nthreads);
int oracle_xor_encode_batch(const uint8_t *src, uint8_t *rep, uint64_t nblocks,
                            int k, int L, int nthreads);
int oracle_xor_decode_batch(uint8_t *src, const uint8_t *rep, uint64_t nblocks,
                            int k, int L, const uint64_t *src_present,
                            const uint64_t *rep_present, uint8_t *status,
                            uint64_t *recovered, int nthreads);

/* Synthetic bytes used by tests and bench.py: byte o of the
 * stream is byte (o & 7) of splitmix64(seed + (o >> 3) * golden). */
void oracle_synth_fill(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t offset);
int oracle_cpu_count(void);

#ifdef __cplusplus
}
#endif
#endif
