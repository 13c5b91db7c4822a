/*
 * tests/host/integration_stub.c -- TEST INFRASTRUCTURE: the reference-side binding from
 * INTEGRATION.md §2-§4, compiled against picoquic's real headers (survey container only),
 * proving the adapter header is type-compatible with picoquic's plugin ABI.
 */
#include "picoquic.h"
#include "picoquic_internal.h"
#include "getset.h"
#include "memory.h"
#include "uthash.h"
#include "pquic_fec_protoops.h"

static int fec_skip_frame(picoquic_cnx_t *cnx, uint8_t *bytes, size_t bytes_max, size_t *consumed,
                          int *pure_ack) {
    protoop_arg_t outs[PROTOOPARGS_MAX];
    int ret = (int)protoop_prepare_and_run_noparam(cnx, &PROTOOP_NOPARAM_SKIP_FRAME, outs, bytes, bytes_max,
                                                   *consumed, *pure_ack);
    *consumed = (size_t)outs[0];
    *pure_ack = (int)outs[1];
    return ret;
}

void pquic_fec_install(int hip_device) {
    static const pquic_fec_host_api_t api = {get_cnx, set_cnx, my_malloc, my_free, fec_skip_frame};
    pquic_fec_bind_host(&api, hip_device);
}

static protoop_plugin_t *fec_plugin(picoquic_cnx_t *cnx) {
    protoop_plugin_t *p = NULL;
    HASH_FIND_STR(cnx->plugins, "be.michelfra.fecxor", p);
    return p;
}
static void *fec_malloc(picoquic_cnx_t *cnx, unsigned int n) {
    protoop_plugin_t *p = fec_plugin(cnx);
    return p->memory_manager.my_malloc(p, n);
}
static void fec_free(picoquic_cnx_t *cnx, void *ptr) { my_free_in_core(fec_plugin(cnx), ptr); }

void pquic_fec_install_native(picoquic_cnx_t *cnx) {
    static const pquic_fec_host_api_t api = {get_cnx, set_cnx, fec_malloc, fec_free};
    pquic_fec_bind_host(&api, 0);
    static protoop_id_t pid_create = {.id = "create_fec_schemes"};
    static protoop_id_t pid_gen = {.id = "fec_generate_repair_symbols"};
    static protoop_id_t pid_rec = {.id = "fec_recover"};
    register_noparam_protoop(cnx, &pid_create, pquic_fec_rlc_create_fec_schemes);
    register_noparam_protoop(cnx, &pid_gen, pquic_fec_rlc_generate_repair_symbols);
    register_noparam_protoop(cnx, &pid_rec, pquic_fec_rlc_recover);
    static protoop_id_t pid_capture = {.id = "packet_payload_to_source_symbol"};
    register_noparam_protoop(cnx, &pid_capture, pquic_fec_packet_payload_to_source_symbol);
}
