/*
 * pquic_fec_frames.h -- wire codecs of the FEC plugin's frames and source-symbol header
 * (SURVEY §8f rows 2 and 4), host C, plus the device-side FEC-frame writer for batched
 * repair symbols (fecgpu_write_fec_frames in fecgpu.h).
 *
 * Byte formats follow the reference exactly, quirks included, and are pinned by
 * tests/golden/frames.json (generated from the reference's own code):
 *   FEC frame      0x2a | BE16 (data_length << 1 | fin) | offset | BE64 repair FPID raw | nss | nrs
 *                  (fec.h:175-194; fec_frame_header_t is a packed struct whose first 16 bits are
 *                  the fin bit then the 15-bit length, written as one big-endian u16)
 *   SOURCE_FPID    0x29 | BE32 source FPID raw                          (fec_protoops.h:92-100)
 *   RECOVERED      0x2b | n | first packet number as a HOST-ORDER u64 | (range, gap) bytes...
 *                  (protoops/write_simple_recovered_frame.c, parse_simple_recovered_frame.c)
 *   source symbol  0x10 | BE64 packet number | frames        (packet_payload_to_source_symbol.c)
 */
#ifndef PQUIC_FEC_FRAMES_H
#define PQUIC_FEC_FRAMES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQUIC_FEC_MAGIC_NUMBER 0x10   /* fec.h:5 */
#define PQUIC_FEC_SOURCE_FPID_TYPE 0x29
#define PQUIC_FEC_FEC_TYPE 0x2a
#define PQUIC_FEC_RECOVERED_TYPE 0x2b
#define PQUIC_FEC_FRAME_HEADER_BYTES 14  /* type byte + packed fec_frame_header_t (13) */
#define PQUIC_FEC_SOURCE_SYMBOL_HEADER_BYTES 9

typedef struct {
    uint8_t fin;              /* 1 bit */
    uint16_t data_length;     /* 15 bits */
    uint8_t offset;
    uint64_t repair_fpid_raw; /* repair_fpid_t.raw: sn | fbn << 8 | fec_scheme_specific << 32 */
    uint8_t nss, nrs;
} pquic_fec_frame_header_t;

/* write_fec_frame_header (fec.h:184-194): 14 bytes including the type byte.  Returns 14. */
size_t pquic_fec_write_fec_frame_header(const pquic_fec_frame_header_t *h, uint8_t *out);
/* parse_fec_frame_header (fec.h:175-183); `in` points at the type byte (14 bytes readable). */
void pquic_fec_parse_fec_frame_header(const uint8_t *in, pquic_fec_frame_header_t *h);

/* helper_write_source_fpid_frame (fec_protoops.h:92-100): 0 and *consumed = 5, or
 * PQUIC_FEC_FRAME_BUFFER_TOO_SMALL when bytes_max < 5. */
#define PQUIC_FEC_FRAME_BUFFER_TOO_SMALL 0x410  /* PICOQUIC_ERROR_FRAME_BUFFER_TOO_SMALL (picoquic.h:65) */
int pquic_fec_write_sfpid_frame(uint32_t source_fpid_raw, uint8_t *out, size_t bytes_max, size_t *consumed);
/* parse_sfpid_frame (fec.h); `in` points at the type byte. */
uint32_t pquic_fec_parse_sfpid_frame(const uint8_t *in);

/* write_simple_recovered_frame.c: 0 with *consumed bytes written, or -1 with *consumed = 0
 * (no packets, buffer too small, or packet numbers not strictly increasing by at most 255). */
int pquic_fec_write_recovered_frame(const uint64_t *packets, uint8_t n, uint8_t *bytes, const uint8_t *bytes_max,
                                    size_t *consumed);
/* parse_simple_recovered_frame.c: the first byte after the frame, or NULL when malformed;
 * packets[] (room for 255) and *n receive the packet numbers as the reference reconstructs
 * them. */
const uint8_t *pquic_fec_parse_recovered_frame(const uint8_t *bytes, const uint8_t *bytes_max, uint64_t *packets,
                                               uint8_t *n);

/* packet_payload_to_source_symbol.c:16-18: the 9-byte source-symbol prefix. Returns 9. */
size_t pquic_fec_source_symbol_header(uint64_t packet_number, uint8_t *out);

/* The transport's frame skipper (picoquic skip_frame protoop, picoquic_internal.h:1185,
 * run by helper_skip_frame, plugins/helpers.h:234-245): *consumed = length of the frame at
 * bytes.  Its return value is ignored, like the reference does. */
typedef int (*pquic_fec_skip_frame_fn)(void *ctx, const uint8_t *bytes, size_t bytes_max, size_t *consumed,
                                       int *pure_ack);

/* packet_payload_to_source_symbol.c:6-36: builds the source symbol of a packet into buffer
 * (room for 9 + payload_length bytes): the 9-byte prefix, then every frame of the payload
 * except ACK (0x02), PADDING (0x00) and CRYPTO (0x06), frames delimited by `skip`.  Returns
 * the symbol length 9 + copied bytes.  A skipper that consumes 0 bytes ends the walk (the
 * reference would loop forever there). */
uint32_t pquic_fec_payload_to_source_symbol(const uint8_t *payload, uint32_t payload_length, uint64_t packet_number,
                                            uint8_t *buffer, pquic_fec_skip_frame_fn skip, void *ctx);

#ifdef __cplusplus
}
#endif
#endif
