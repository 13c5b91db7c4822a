/*
 * include/pquic_fec_cc.h -- recovered-packet bookkeeping and congestion-control notification of
 * the FEC plugin, host C.
 *
 * Replaces, behaviour for behaviour:
 *   recovered_packets_buffer_t              plugins/fec/fec_protoops.h:12-16 (50-entry ring in bpf_state)
 *   enqueue_recovered_packet_to_buffer      fec_protoops.h:122-129
 *   dequeue_recovered_packet_from_buffer    fec_protoops.h:137-143
 *   enqueue_recovered_packets               fec_protoops.h:145-149
 *   process_recovered_frame                 protoops/process_simple_recovered_frame.c:5-16 (enqueue the
 *                                           packet numbers of a parsed RECOVERED frame)
 *   maybe_notify_recovered_packets_to_cc    fec_protoops.h:151-184, run by the pre-hook of
 *                                           prepare_packet_ready (protoops/maybe_notify_recovered_packets_to_cc.c)
 *
 * The notification walks the transport's retransmit queue, so the transport accessors the
 * reference reaches through get_cnx / get_path / get_pkt_ctx / get_pkt / set_pkt_ctx
 * (picoquic/getset.h) and the helper protoops it runs (plugins/helpers.h:175-206, 274-280,
 * 835-840) are bound as a table of callbacks (pquic_fec_transport_api_t); INTEGRATION.md shows
 * picoquic's.  Pinned by tests/golden/cc_cases.json: event logs of the reference pluglet itself.
 */
#ifndef PQUIC_FEC_CC_H
#define PQUIC_FEC_CC_H

#include <stdint.h>

#include "pquic_fec_protoops.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PQUIC_FEC_MAX_RECOVERED_PACKETS_IN_BUFFER 50  /* fec_protoops.h:7 */
#define PQUIC_CONGESTION_NOTIFICATION_REPEAT 1         /* picoquic_congestion_notification_repeat (picoquic.h:832) */

/* Same layout as the reference's recovered_packets_buffer_t (fec_protoops.h:12-16). */
typedef struct {
    uint32_t start;
    uint32_t size;
    uint64_t packet_numbers[PQUIC_FEC_MAX_RECOVERED_PACKETS_IN_BUFFER];
} pquic_fec_recovered_packets_buffer_t;

/* enqueue_recovered_packet_to_buffer: a full ring drops its oldest entry. */
void pquic_fec_enqueue_recovered_packet(pquic_fec_recovered_packets_buffer_t *b, uint64_t packet_number);
/* enqueue_recovered_packets / process_recovered_frame: n packet numbers in order. */
void pquic_fec_enqueue_recovered_packets(pquic_fec_recovered_packets_buffer_t *b, const uint64_t *packet_numbers,
                                         uint8_t n);
/* dequeue_recovered_packet_from_buffer: the oldest entry, or (uint64_t)-1 when empty. */
uint64_t pquic_fec_dequeue_recovered_packet(pquic_fec_recovered_packets_buffer_t *b);

/* The transport as the reference pluglet sees it.  Packets, paths and packet contexts are opaque. */
typedef struct {
    void *(*path)(picoquic_cnx_t *cnx);                              /* get_cnx(cnx, AK_CNX_PATH, 0) */
    void *(*application_pkt_ctx)(void *path);                        /* get_path(path, AK_PATH_PKT_CTX,
                                                                         picoquic_packet_context_application) */
    void *(*retransmit_oldest)(void *pkt_ctx);                       /* get_pkt_ctx(.., AK_PKTCTX_RETRANSMIT_OLDEST) */
    void *(*next_packet)(void *packet);                              /* get_pkt(.., AK_PKT_NEXT_PACKET) */
    uint64_t (*sequence_number)(void *packet);                       /* get_pkt(.., AK_PKT_SEQUENCE_NUMBER) */
    int (*is_pure_ack)(void *packet);                                /* get_pkt(.., AK_PKT_IS_PURE_ACK) */
    uint64_t (*latest_cc_notification_time)(void *pkt_ctx);          /* get_pkt_ctx(.., AK_PKTCTX_LATEST_
                                                                         RETRANSMIT_CC_NOTIFICATION_TIME) */
    void (*set_latest_cc_notification_time)(void *pkt_ctx, uint64_t t); /* set_pkt_ctx(same key) */
    uint64_t (*smoothed_rtt)(void *path);                            /* get_path(.., AK_PATH_SMOOTHED_RTT, 0) */
    /* protoop retransmit_needed_by_packet (helper_retransmit_needed_by_packet, helpers.h:175-192) */
    int (*retransmit_needed)(picoquic_cnx_t *cnx, void *packet, uint64_t current_time, int *timer_based);
    /* protoop packet_was_lost (helper_packet_was_lost, helpers.h:835-840) */
    void (*packet_was_lost)(picoquic_cnx_t *cnx, void *packet, void *path);
    /* protoop dequeue_retransmit_packet (helper_dequeue_retransmit_packet, helpers.h:274-280) */
    void (*dequeue_retransmit_packet)(picoquic_cnx_t *cnx, void *packet, int should_free);
    /* protoop congestion_algorithm_notify (helper_congestion_algorithm_notify, helpers.h:194-206) */
    void (*congestion_notify)(picoquic_cnx_t *cnx, void *path, int notification, uint64_t rtt_measurement,
                              uint64_t nb_bytes_acknowledged, uint64_t lost_packet_number, uint64_t current_time);
} pquic_fec_transport_api_t;

/* maybe_notify_recovered_packets_to_cc (fec_protoops.h:151-184): walks the retransmit queue from
 * its oldest packet; a queued packet whose number is the oldest recovered one is, if the transport
 * would retransmit it now, declared lost and dequeued (without CC notification of a loss: a
 * "repeat" notification only when the last one is at least one smoothed RTT old and the packet is
 * not a pure ACK), and the recovered number is consumed; recovered numbers older than the queue
 * position are dropped; the walk stops at the first recovered packet not yet due. */
void pquic_fec_maybe_notify_recovered_packets_to_cc(picoquic_cnx_t *cnx, const pquic_fec_transport_api_t *t,
                                                    pquic_fec_recovered_packets_buffer_t *b, uint64_t current_time);

#ifdef __cplusplus
}
#endif
#endif
