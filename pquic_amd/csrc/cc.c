/*
 * pquic_amd/csrc/cc.c -- recovered-packet ring and congestion-control notification of the FEC
 * plugin (include/pquic_fec_cc.h).  Host C; each function restates the reference routine it
 * names, pinned by the reference pluglet's own event logs (tests/golden/cc_cases.json).
 */
#include "pquic_fec_cc.h"

#define NBUF PQUIC_FEC_MAX_RECOVERED_PACKETS_IN_BUFFER

/* fec_protoops.h:122-129 */
void pquic_fec_enqueue_recovered_packet(pquic_fec_recovered_packets_buffer_t *b, uint64_t packet_number) {
    b->packet_numbers[(b->start + b->size) % NBUF] = packet_number;
    if (b->size < NBUF)
        b->size++;
    else
        b->start = (b->start + 1) % NBUF;  /* the oldest entry was just overwritten */
}

/* fec_protoops.h:145-149 */
void pquic_fec_enqueue_recovered_packets(pquic_fec_recovered_packets_buffer_t *b, const uint64_t *packet_numbers,
                                         uint8_t n) {
    for (int i = 0; i < n; i++) pquic_fec_enqueue_recovered_packet(b, packet_numbers[i]);
}

/* fec_protoops.h:137-143 */
uint64_t pquic_fec_dequeue_recovered_packet(pquic_fec_recovered_packets_buffer_t *b) {
    if (b->size == 0) return (uint64_t)-1;
    const uint64_t pn = b->packet_numbers[b->start];
    b->size--;
    b->start = (b->start + 1) % NBUF;
    return pn;
}

/* fec_protoops.h:151-184 */
void pquic_fec_maybe_notify_recovered_packets_to_cc(picoquic_cnx_t *cnx, const pquic_fec_transport_api_t *t,
                                                    pquic_fec_recovered_packets_buffer_t *b, uint64_t current_time) {
    void *path = t->path(cnx);
    void *pkt_ctx = t->application_pkt_ctx(path);
    void *p = t->retransmit_oldest(pkt_ctx);
    while (b->size > 0 && p) {
        void *next = t->next_packet(p);
        const uint64_t pn = t->sequence_number(p);
        const uint64_t first = b->packet_numbers[b->start];
        if (pn == first) {
            int timer_based = 0;
            if (!t->retransmit_needed(cnx, p, current_time, &timer_based))
                break;  /* not considered lost yet, and later packets were sent later (:161-165) */
            const uint64_t notify_at = t->latest_cc_notification_time(pkt_ctx) + t->smoothed_rtt(path);
            const int pure_ack = t->is_pure_ack(p) != 0;
            t->packet_was_lost(cnx, p, path);
            t->dequeue_retransmit_packet(cnx, p, 1);
            if (current_time >= notify_at && !pure_ack) {  /* as the core does (:172) */
                t->set_latest_cc_notification_time(pkt_ctx, current_time);
                t->congestion_notify(cnx, path, PQUIC_CONGESTION_NOTIFICATION_REPEAT, 0, 0, pn, current_time);
            }
            pquic_fec_dequeue_recovered_packet(b);
        } else if (pn > first) {
            pquic_fec_dequeue_recovered_packet(b);  /* already gone from the retransmit queue (:178-180) */
        }
        p = next;
    }
}
