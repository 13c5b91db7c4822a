/*
 * tests/host/integration_driver.c -- TEST INFRASTRUCTURE (survey container only: it needs picoquic's
 * headers from the reference tree).  Drives INTEGRATION.md §4's native registration (Option B,
 * integration_stub.c, included here so its static allocator shims are reachable) on connections built
 * from picoquic's own structures: for every shipped FEC composition name, a connection holding that
 * plugin next to a decoy plugin, each with a private arena standing in for memory[PLUGIN_MEMORY].  The
 * registered create_fec_schemes must allocate its scheme inside the FEC plugin's arena; on a
 * connection without a FEC plugin it must return PICOQUIC_ERROR_MEMORY.  Exit status 0 = all pass.
 *
 * Only what picoquic would supply beside the plugin structures is defined here: the connection
 * accessors get_cnx / set_cnx (outputs only), register_noparam_protoop (records the operation),
 * my_malloc / my_free / my_free_in_core (the plugin's arena is a bump allocator over its memory[]),
 * and an inert plugin_run_protoop_internal behind the stub's skip_frame (never called).
 */
#include "integration_stub.c"
#include <stdlib.h>

static protoop_arg_t g_out[PROTOOPARGS_MAX];
protoop_arg_t get_cnx(picoquic_cnx_t *cnx, access_key_t ak, uint16_t param) {
    (void)cnx; (void)ak; (void)param;
    return 0;
}
void set_cnx(picoquic_cnx_t *cnx, access_key_t ak, uint16_t param, protoop_arg_t val) {
    (void)cnx;
    if (ak == AK_CNX_OUTPUT && param < PROTOOPARGS_MAX) g_out[param] = val;
}
void *my_malloc(picoquic_cnx_t *cnx, unsigned int size) { (void)cnx; return malloc(size); }
void my_free(picoquic_cnx_t *cnx, void *ptr) { (void)cnx; free(ptr); }

static long g_arena_live;
static void *arena_malloc(protoop_plugin_t *p, unsigned int size) {
    size_t *used = (size_t *)p->memory_manager.ctx;
    size = (size + 15u) & ~15u;
    if (*used + size > PLUGIN_MEMORY) return NULL;
    void *r = p->memory + *used;
    *used += size;
    g_arena_live++;
    return r;
}
void my_free_in_core(protoop_plugin_t *p, void *ptr) {
    if ((uint8_t *)ptr < (uint8_t *)p->memory || (uint8_t *)ptr >= (uint8_t *)p->memory + PLUGIN_MEMORY) abort();
    g_arena_live--;
}

static protocol_operation g_create;
int register_noparam_protoop(picoquic_cnx_t *cnx, protoop_id_t *pid, protocol_operation op) {
    (void)cnx;
    if (strcmp(pid->id, "create_fec_schemes") == 0) g_create = op;
    return 0;
}
protoop_id_t PROTOOP_NOPARAM_SKIP_FRAME = {.id = "skip_frame"};
protoop_arg_t plugin_run_protoop_internal(picoquic_cnx_t *cnx, const protoop_params_t *pp) {
    (void)cnx; (void)pp;
    return 0;  /* skip_frame is only bound by Option A's installer, never called here */
}

static protoop_plugin_t *mk_plugin(const char *name, size_t *used) {
    protoop_plugin_t *p = calloc(1, sizeof *p);
    if (!p) abort();
    snprintf(p->name, sizeof p->name, "%s", name);
    p->memory_manager.my_malloc = arena_malloc;
    p->memory_manager.ctx = used;
    return p;
}

/* one connection with plugins {decoy, fec_name (if any)}; returns 0 when the scheme lands in the FEC
 * plugin's arena (or, without one, when the operation reports PICOQUIC_ERROR_MEMORY) */
static int run_case(const char *fec_name, const char *configured) {
    picoquic_cnx_t *cnx = calloc(1, sizeof *cnx);
    size_t used_decoy = 0, used_fec = 0;
    protoop_plugin_t *decoy = mk_plugin("be.michelfra.multipath", &used_decoy), *fec = NULL;
    HASH_ADD_STR(cnx->plugins, name, decoy);
    if (fec_name) {
        fec = mk_plugin(fec_name, &used_fec);
        HASH_ADD_STR(cnx->plugins, name, fec);
    }
    g_create = NULL;
    memset(g_out, 0, sizeof g_out);
    pquic_fec_install_native(cnx, configured);
    int bad = 0;
    protoop_arg_t ret = g_create ? g_create(cnx) : (protoop_arg_t)-1;
    if (fec_name) {
        uint8_t *s = (uint8_t *)(uintptr_t)g_out[0];
        bad = ret != 0 || !s || s < (uint8_t *)fec->memory || s >= (uint8_t *)fec->memory + PLUGIN_MEMORY ||
              g_out[1] != g_out[0] || used_decoy != 0 || used_fec == 0;
        if (!bad) fec_free(cnx, s);
    } else {
        bad = ret != PICOQUIC_ERROR_MEMORY || used_decoy != 0;
    }
    printf("%-28s configured=%-24s ret=0x%llx fec_arena=%zu decoy_arena=%zu %s\n", fec_name ? fec_name : "(none)",
           configured ? configured : "(prefix)", (unsigned long long)ret, used_fec, used_decoy, bad ? "FAIL" : "ok");
    HASH_CLEAR(hh, cnx->plugins);
    free(decoy);
    free(fec);
    free(cnx);
    return bad;
}

int main(void) {
    /* the first line of each shipped FEC composition manifest */
    static const char *names[] = {"be.michelfra.fecxor", "be.michelfra.fecrlc", "be.michelfra.fecrlcgf256"};
    int bad = 0;
    for (int i = 0; i < 3; i++) {
        bad |= run_case(names[i], names[i]);  /* the name the host inserted, passed at install */
        bad |= run_case(names[i], NULL);      /* no name: found by its prefix */
    }
    bad |= run_case(NULL, NULL);
    bad |= run_case(NULL, "be.michelfra.fecrlc");
    bad |= g_arena_live != 0;
    printf("%s (arena allocations still live: %ld)\n", bad ? "FAILED" : "all ok", g_arena_live);
    return bad;
}
