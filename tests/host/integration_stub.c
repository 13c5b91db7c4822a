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
#include <stdio.h>
#include <string.h>

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

/* The FEC plugin composition the host inserted: its name is the first line of the manifest it loaded
 * (plugins/fec/fec.plugin:1 "be.michelfra.fecxor"; fec_rlc_gf256_window.plugin:1, _uniform.plugin:1 and
 * _no_rf.plugin:1 "be.michelfra.fecrlc"; fec_rlc_gf256_window_protect_end_of_stream_only_inflight.plugin:1
 * "be.michelfra.fecrlcgf256").  Plugins are hashed by that name (picoquic/plugin.c:836).  With no name
 * given, the connection's plugin whose name starts with "be.michelfra.fec" is taken. */
static char g_fec_plugin_name[PROTOOPPLUGINNAME_MAX];

static protoop_plugin_t *fec_plugin(picoquic_cnx_t *cnx) {
    protoop_plugin_t *p = NULL, *tmp;
    if (g_fec_plugin_name[0]) {
        HASH_FIND_STR(cnx->plugins, g_fec_plugin_name, p);
        return p;
    }
    HASH_ITER(hh, cnx->plugins, p, tmp) {
        if (strncmp(p->name, "be.michelfra.fec", 16) == 0) return p;
    }
    return NULL;
}
/* NULL when the connection has no FEC plugin: the protoop then returns PICOQUIC_ERROR_MEMORY */
static void *fec_malloc(picoquic_cnx_t *cnx, unsigned int n) {
    protoop_plugin_t *p = fec_plugin(cnx);
    return p ? p->memory_manager.my_malloc(p, n) : NULL;
}
static void fec_free(picoquic_cnx_t *cnx, void *ptr) {
    protoop_plugin_t *p = fec_plugin(cnx);
    if (p && ptr) my_free_in_core(p, ptr);
}

void pquic_fec_install_native(picoquic_cnx_t *cnx, const char *fec_plugin_name) {
    snprintf(g_fec_plugin_name, sizeof g_fec_plugin_name, "%s", fec_plugin_name ? fec_plugin_name : "");
    static const pquic_fec_host_api_t api = {get_cnx, set_cnx, fec_malloc, fec_free, NULL};
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
