/*
 * include/pquic_fec_protoops.h -- drop-in protocol operations for PQUIC's plugins/fec
 * scheme hooks, backed by the MI355X engine (include/fecgpu.h).
 *
 * The reference ships three scheme pluglets per FEC scheme, compiled to eBPF and run by
 * uBPF, declared by the manifests plugins/fec/fec_scheme_rlc_gf256.plugin:1-3 and
 * plugins/fec/fec_scheme_xor.plugin:1-3:
 *
 *   protoop id                    reference pluglet (RLC / XOR)                      replaced by
 *   create_fec_schemes            create_rlc_fec_scheme_gf256.c:46-59 / create_xor_fec_scheme.c:4-9
 *                                                                 pquic_fec_{rlc,xor}_create_fec_schemes
 *   fec_generate_repair_symbols   rlc_fec_scheme_generate_gf256.c:24-77 / xor_fec_scheme_generate.c:41-78
 *                                                                 pquic_fec_{rlc,xor}_generate_repair_symbols
 *   fec_recover                   rlc_fec_scheme_gf256.c:134-251 / xor_fec_scheme.c:41-74
 *                                                                 pquic_fec_{rlc,xor}_recover
 *
 * Every function has the reference's protocol_operation signature
 * (picoquic/picoquic_internal.h:582: protoop_arg_t op(picoquic_cnx_t *)), reads its inputs
 * with get_cnx(cnx, AK_CNX_INPUT, i), writes outputs with set_cnx(cnx, AK_CNX_OUTPUT, i, v)
 * and returns the same codes as the pluglet it replaces.  Repair / recovered symbols are
 * allocated with the caller's my_malloc, exactly like malloc_repair_symbol /
 * malloc_source_symbol (plugins/fec/fec.h:201-231), so the framework frees them as before.
 *
 * picoquic's accessors are bound at run time (pquic_fec_bind_host) so that this library
 * does not link against picoquic; see INTEGRATION.md for the registration stub.
 */
#ifndef PQUIC_FEC_PROTOOPS_H
#define PQUIC_FEC_PROTOOPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- picoquic plugin ABI (picoquic/picoquic.h:333, getset.h:11,339-341) ---- */
typedef uint64_t protoop_arg_t;
typedef struct st_picoquic_cnx_t picoquic_cnx_t;
typedef uint16_t access_key_t;
#define PQUIC_AK_CNX_INPUT  0x00
#define PQUIC_AK_CNX_OUTPUT 0x01
#define PQUIC_ERROR_MEMORY  0x405   /* PICOQUIC_ERROR_MEMORY = PICOQUIC_ERROR_CLASS + 5 */
#define PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK 100   /* plugins/fec/fec.h:8 */

/* ---- layout-compatible view of the reference FEC data model (plugins/fec/fec.h:44-130),
 *      x86-64 SysV; sizes pinned by tests/golden/layout.json ---- */
typedef union {
    uint32_t raw;
    struct __attribute__((__packed__)) { uint8_t symbol_number; uint32_t fec_block_number : 24; } f;
} pquic_source_fpid_t;

typedef union {
    uint64_t raw;
    struct __attribute__((__packed__)) {
        pquic_source_fpid_t source_fpid;   /* symbol_number | fec_block_number << 8 */
        uint32_t fec_scheme_specific;
    } f;
} pquic_repair_fpid_t;

typedef struct {
    pquic_repair_fpid_t fpid;            /* repair_fec_payload_id */
    uint16_t data_length : 15;
    uint8_t *data;
} pquic_repair_symbol_t;

typedef struct {
    pquic_source_fpid_t fpid;            /* source_fec_payload_id (fec_block_offset, fbn) */
    uint16_t data_length : 15;
    uint8_t *data;
} pquic_source_symbol_t;

typedef struct __attribute__((__packed__)) {
    uint32_t fec_block_number;
    uint8_t total_source_symbols;
    uint8_t total_repair_symbols;
    uint8_t current_source_symbols;
    uint8_t current_repair_symbols;
    pquic_source_symbol_t *source_symbols[PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK];
    pquic_repair_symbol_t *repair_symbols[PQUIC_FEC_MAX_SYMBOLS_PER_BLOCK];
} pquic_fec_block_t;

/* ---- host accessors (picoquic/getset.h:28,38; picoquic/memory.h:6,8) ---- */
typedef struct {
    protoop_arg_t (*get_cnx)(picoquic_cnx_t *cnx, access_key_t ak, uint16_t param);
    void (*set_cnx)(picoquic_cnx_t *cnx, access_key_t ak, uint16_t param, protoop_arg_t val);
    void *(*my_malloc)(picoquic_cnx_t *cnx, unsigned int size);
    void (*my_free)(picoquic_cnx_t *cnx, void *ptr);
    /* optional: the skip_frame protoop (helper_skip_frame, plugins/helpers.h:234-245); needed
     * only by pquic_fec_packet_payload_to_source_symbol */
    int (*skip_frame)(picoquic_cnx_t *cnx, uint8_t *bytes, size_t bytes_max, size_t *consumed, int *pure_ack);
} pquic_fec_host_api_t;

/* Bind picoquic's accessors; returns 0.  Until bound every protoop returns
 * PQUIC_FEC_ERR_UNBOUND.  `device` selects the HIP device the schemes use. */
int pquic_fec_bind_host(const pquic_fec_host_api_t *api, int device);
#define PQUIC_FEC_ERR_UNBOUND 0x41B     /* PICOQUIC_ERROR_UNEXPECTED_ERROR */

/* Scheme object handed out by create_fec_schemes (outputs 0 and 1, like the reference's
 * rlc_gf256_fec_scheme_t*).  Opaque to the framework. */
typedef struct pquic_fec_scheme pquic_fec_scheme_t;

/* ---- the protocol operations ---- */
protoop_arg_t pquic_fec_rlc_create_fec_schemes(picoquic_cnx_t *cnx);
protoop_arg_t pquic_fec_rlc_generate_repair_symbols(picoquic_cnx_t *cnx);
protoop_arg_t pquic_fec_rlc_recover(picoquic_cnx_t *cnx);
protoop_arg_t pquic_fec_xor_create_fec_schemes(picoquic_cnx_t *cnx);
protoop_arg_t pquic_fec_xor_generate_repair_symbols(picoquic_cnx_t *cnx);
protoop_arg_t pquic_fec_xor_recover(picoquic_cnx_t *cnx);

/* packet_payload_to_source_symbol (protoops/packet_payload_to_source_symbol.c:6-36, manifest
 * fec_core.plugin:20): inputs [0] payload bytes, [1] symbol buffer, [2] payload length,
 * [3] packet number; returns the symbol length, PQUIC_ERROR_MEMORY for a NULL buffer, or
 * PQUIC_FEC_ERR_UNBOUND without a bound skip_frame.  The pluglet's store to
 * bpf_state.current_symbol_length is not reproduced: both callers overwrite or never read it
 * (incoming_encrypted.c:29-33, schedule_frames_on_path.c:47). */
protoop_arg_t pquic_fec_packet_payload_to_source_symbol(picoquic_cnx_t *cnx);

/* Counters of adapter activity (calls, blocks the reference would have crashed on; calls whose request
 * the resident block service withdrew at its deadline, which then took the launch path --
 * fecgpu_block_svc_set_deadline). */
typedef struct {
    uint64_t generate_calls, recover_calls, recovered_symbols, ref_ub_blocks, errors;
    uint64_t svc_deadline_misses;
} pquic_fec_protoop_stats_t;
void pquic_fec_protoop_stats(pquic_fec_protoop_stats_t *out);

/* Layout self-description for tests: {sizeof block, source, repair, offsetof source_symbols,
 * repair_symbols, source data, repair data, sizeof repair fpid}. */
int pquic_fec_layout(uint64_t out[8]);

#ifdef __cplusplus
}
#endif
#endif
