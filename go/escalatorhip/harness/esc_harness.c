/*
 * esc_harness.c — plain-C stand-in for the cgo shim (go/escalatorhip/escalatorhip.go).
 *
 * There is no Go toolchain in this image, so the shim cannot be compiled here.  This
 * harness makes the same ABI calls in the same order as the shim's methods, with the
 * same object structs the shim fills from *v1.Pod / *v1.Node, so the call sequence a Go
 * host would run is exercised end to end:
 *
 *   NewContext          esc_ctx_create
 *   NewContextMulti     esc_ctx_create_multi (argv[2] = number of shards: the device of
 *                       the input listed that many times, the peer exchange on one GPU)
 *   (*Context).Load     esc_packer_create, esc_packer_add_pods, esc_packer_add_nodes,
 *                       esc_packer_set_tracker (dry-mode groups), esc_packer_view,
 *                       esc_load_pods, esc_load_nodes, esc_packer_destroy
 *   (*Context).Calibrate esc_k1_calibrate (once, after the first state)
 *   (*Context).SetSelections esc_set_order_in_step, esc_set_selections (slack 1)
 *   (*Context).RunOnce  esc_set_state, esc_step, esc_sync, esc_results, esc_selections
 *   (*Context).Order    esc_sort_nodes, esc_group_order (taintOldestN / untaintNewestN)
 *   CalculatePodsRequestsTotal / CalculateNodesCapacityTotal
 *                       esc_pods_requests_total, esc_nodes_capacity_total
 *   calcPercentUsage / calcScaleUpDelta
 *                       esc_calc_percent_usage, esc_calc_scale_up_delta
 *
 * Input (argv[1]): whitespace-separated tokens written by tests/harness_io.py.  Strings
 * are "s" + percent-encoded bytes (so "s" alone is the empty string).  Output (stdout):
 * one record per line, parsed by the same module.  Without a gfx950 device the shim's
 * device calls return ESC_E_NODEV; the harness prints "nodev <call>" and exits 0 after
 * the host-side calls (packer, scalar math) have run.
 */
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "escalator_hip.h"

/* ------------------------------------------------------------ token reader */
typedef struct { char* buf; size_t pos, len; } rd_t;

static void die(const char* what) {
    fprintf(stderr, "esc_harness: %s\n", what);
    exit(2);
}

static char* tok(rd_t* r) {
    while (r->pos < r->len && (r->buf[r->pos] == ' ' || r->buf[r->pos] == '\n' || r->buf[r->pos] == '\t')) r->pos++;
    if (r->pos >= r->len) die("unexpected end of input");
    char* t = r->buf + r->pos;
    while (r->pos < r->len && r->buf[r->pos] != ' ' && r->buf[r->pos] != '\n' && r->buf[r->pos] != '\t') r->pos++;
    if (r->pos < r->len) r->buf[r->pos++] = 0;
    return t;
}

static int64_t num(rd_t* r) {
    char* t = tok(r);
    char* end;
    errno = 0;
    long long v = strtoll(t, &end, 10);
    if (*end || errno) die("bad integer");
    return (int64_t)v;
}

static void expect(rd_t* r, const char* word) {
    if (strcmp(tok(r), word)) die(word);
}

static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    die("bad escape");
    return 0;
}

/* Decodes in place: the token's own bytes hold the shorter result. */
static const char* str(rd_t* r) {
    char* t = tok(r);
    if (t[0] != 's') die("string token must start with 's'");
    char* o = t;
    for (const char* p = t + 1; *p; p++) {
        if (*p == '%') {
            if (!p[1] || !p[2]) die("bad escape");
            *o++ = (char)(hexv(p[1]) * 16 + hexv(p[2]));
            p += 2;
        } else {
            *o++ = *p;
        }
    }
    *o = 0;
    return t;
}

static void* cal(size_t n, size_t sz) {
    void* p = calloc(n ? n : 1, sz);
    if (!p) die("out of memory");
    return p;
}

/* Arrays handed to the library: NULL when empty, as the cgo shim's ptr() passes them (the
 * ABI takes NULL with a zero count for every array). */
static void* arr(size_t n, size_t sz) { return n ? cal(n, sz) : NULL; }

static esc_request req(rd_t* r) {
    esc_request q;
    q.cpu_m = num(r);
    q.mem_b = num(r);
    q.has_cpu = (int32_t)num(r);
    q.has_mem = (int32_t)num(r);
    return q;
}

/* ------------------------------------------------------------ objects */
static void read_pod(rd_t* r, esc_pod_obj* o) {
    memset(o, 0, sizeof(*o));
    o->n_owner_kinds = (int32_t)num(r);
    const char** kinds = arr((size_t)o->n_owner_kinds, sizeof(char*));
    for (int i = 0; i < o->n_owner_kinds; i++) kinds[i] = str(r);
    o->owner_kinds = kinds;
    o->has_config_source = (int32_t)num(r);
    o->config_source = str(r);
    o->n_node_selector = (int32_t)num(r);
    esc_kv* sel = arr((size_t)o->n_node_selector, sizeof(esc_kv));
    for (int i = 0; i < o->n_node_selector; i++) { sel[i].key = str(r); sel[i].value = str(r); }
    o->node_selector = sel;
    o->has_affinity = (int32_t)num(r);
    o->has_node_affinity = (int32_t)num(r);
    o->has_pod_affinity = (int32_t)num(r);
    o->has_pod_anti_affinity = (int32_t)num(r);
    o->has_required = (int32_t)num(r);
    o->n_exprs = (int32_t)num(r);
    esc_selector_expr* ex = arr((size_t)o->n_exprs, sizeof(esc_selector_expr));
    for (int i = 0; i < o->n_exprs; i++) {
        ex[i].key = str(r);
        ex[i].op = str(r);
        ex[i].n_values = (int32_t)num(r);
        const char** vals = arr((size_t)ex[i].n_values, sizeof(char*));
        for (int v = 0; v < ex[i].n_values; v++) vals[v] = str(r);
        ex[i].values = vals;
        ex[i].term = (int32_t)num(r);
    }
    o->exprs = ex;
    o->n_containers = (int32_t)num(r);
    esc_request* cs = arr((size_t)o->n_containers, sizeof(esc_request));
    for (int i = 0; i < o->n_containers; i++) cs[i] = req(r);
    o->containers = cs;
    o->n_init_containers = (int32_t)num(r);
    esc_request* ic = arr((size_t)o->n_init_containers, sizeof(esc_request));
    for (int i = 0; i < o->n_init_containers; i++) ic[i] = req(r);
    o->init_containers = ic;
    o->has_overhead = (int32_t)num(r);
    o->overhead = req(r);
}

static void read_node(rd_t* r, esc_node_obj* o) {
    memset(o, 0, sizeof(*o));
    o->name = str(r);
    o->n_labels = (int32_t)num(r);
    esc_kv* lb = arr((size_t)o->n_labels, sizeof(esc_kv));
    for (int i = 0; i < o->n_labels; i++) { lb[i].key = str(r); lb[i].value = str(r); }
    o->labels = lb;
    o->unschedulable = (int32_t)num(r);
    o->n_taints = (int32_t)num(r);
    const char** tk = arr((size_t)o->n_taints, sizeof(char*));
    for (int i = 0; i < o->n_taints; i++) tk[i] = str(r);
    o->taint_keys = tk;
    o->allocatable = req(r);
    o->created_unix_ns = num(r);
}

/* ------------------------------------------------------------ the shim's sequence */
static int device_call(const char* name, int32_t rc) {
    if (rc == ESC_E_NODEV) {
        printf("nodev %s\n", name);
        return 1;
    }
    if (rc != ESC_OK) {
        fprintf(stderr, "esc_harness: %s: %s (%d)\n", name, esc_strerror(rc), rc);
        exit(1);
    }
    return 0;
}

static void host_call(const char* name, int32_t rc) {
    if (rc != ESC_OK) {
        fprintf(stderr, "esc_harness: %s: %s (%d)\n", name, esc_strerror(rc), rc);
        exit(1);
    }
}

static uint64_t bits(double d) {
    uint64_t u;
    memcpy(&u, &d, sizeof u);
    return u;
}

int main(int argc, char** argv) {
    if (argc != 2 && argc != 3) die("usage: esc_harness <input> [shards]");
    const int32_t shards = argc == 3 ? (int32_t)atoi(argv[2]) : 0;
    if (argc == 3 && (shards < 1 || shards > 16)) die("shards must be 1..16");
    FILE* f = fopen(argv[1], "rb");
    if (!f) die("cannot open input");
    rd_t r = {0};
    fseek(f, 0, SEEK_END);
    r.len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    r.buf = cal(r.len + 1, 1);
    if (fread(r.buf, 1, r.len, f) != r.len) die("short read");
    fclose(f);

    expect(&r, "ESCH1");
    expect(&r, "device");
    int32_t device = (int32_t)num(&r);
    expect(&r, "groups");
    int32_t G = (int32_t)num(&r);
    esc_group_spec* groups = cal((size_t)G, sizeof(esc_group_spec));
    for (int g = 0; g < G; g++) {
        groups[g].name = str(&r);
        groups[g].label_key = str(&r);
        groups[g].label_value = str(&r);
        groups[g].min_nodes = (int32_t)num(&r);
        groups[g].max_nodes = (int32_t)num(&r);
        groups[g].taint_upper_pct = (int32_t)num(&r);
        groups[g].taint_lower_pct = (int32_t)num(&r);
        groups[g].scale_up_pct = (int32_t)num(&r);
        groups[g].slow_removal_rate = (int32_t)num(&r);
        groups[g].fast_removal_rate = (int32_t)num(&r);
        groups[g].dry_mode = (int32_t)num(&r);
    }
    expect(&r, "states");
    esc_group_state* states = cal((size_t)G, sizeof(esc_group_state));
    for (int g = 0; g < G; g++) {
        states[g].locked = (int32_t)num(&r);
        states[g].requested_nodes = (int32_t)num(&r);
        states[g].cached_cpu_m = num(&r);
        states[g].cached_mem_b = num(&r);
    }
    expect(&r, "pods");
    int64_t P = num(&r);
    esc_pod_obj* pods = arr((size_t)P, sizeof(esc_pod_obj));
    for (int64_t i = 0; i < P; i++) read_pod(&r, &pods[i]);
    expect(&r, "nodes");
    int64_t N = num(&r);
    esc_node_obj* nodes = arr((size_t)N, sizeof(esc_node_obj));
    for (int64_t i = 0; i < N; i++) read_node(&r, &nodes[i]);
    expect(&r, "trackers");
    int32_t T = (int32_t)num(&r);
    int32_t* trk_group = cal((size_t)T, sizeof(int32_t));
    int64_t* trk_n = cal((size_t)T, sizeof(int64_t));
    const char*** trk_names = cal((size_t)T, sizeof(char**));
    for (int t = 0; t < T; t++) {
        trk_group[t] = (int32_t)num(&r);
        trk_n[t] = num(&r);
        trk_names[t] = arr((size_t)trk_n[t], sizeof(char*));
        for (int64_t i = 0; i < trk_n[t]; i++) trk_names[t][i] = str(&r);
    }
    expect(&r, "end");

    if (esc_abi_version() != ESC_ABI_VERSION) die("ABI version mismatch");
    printf("abi %d\n", esc_abi_version());

    /* NewContext / NewContextMulti */
    esc_ctx* ctx = NULL;
    int32_t rc;
    if (shards) {
        int32_t devs[16];
        for (int i = 0; i < shards; i++) devs[i] = device;
        rc = esc_ctx_create_multi(groups, G, devs, shards, &ctx);
        if (device_call("esc_ctx_create_multi", rc)) return 0;
    } else {
        rc = esc_ctx_create(groups, G, device, 0, 1, &ctx);
        if (device_call("esc_ctx_create", rc)) return 0;
    }

    /* scalar math (calcPercentUsage / calcScaleUpDelta): host-only, runs without a device */
    {
        double cpu = 0, mem = 0;
        int32_t st = esc_calc_percent_usage(20000, 40000, 20000, 80000, 10, &cpu, &mem);
        printf("pct %d %016" PRIx64 " %016" PRIx64 "\n", st, bits(cpu), bits(mem));
        int64_t d = 0;
        st = esc_calc_scale_up_delta(10, cpu, mem, 20000, 40000, 0, 0, 70, &d);
        printf("delta %d %" PRId64 "\n", st, d);
    }

    /* (*Context).Load */
    esc_packer* pk = NULL;
    host_call("esc_packer_create", esc_packer_create(ctx, &pk));
    host_call("esc_packer_add_pods", esc_packer_add_pods(pk, pods, P));
    host_call("esc_packer_add_nodes", esc_packer_add_nodes(pk, nodes, N));
    for (int t = 0; t < T; t++)
        host_call("esc_packer_set_tracker", esc_packer_set_tracker(pk, trk_group[t], trk_names[t], trk_n[t]));
    esc_pod_soa ps;
    esc_node_soa ns;
    host_call("esc_packer_view", esc_packer_view(pk, &ps, &ns));
    printf("packed %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 "\n", ps.n_pods, ps.n_xc, ps.n_xp,
           ns.n_nodes, ns.n_trk);
    rc = esc_load_pods(ctx, &ps, 0);
    if (device_call("esc_load_pods", rc)) {
        esc_packer_destroy(pk);
        esc_ctx_destroy(ctx);
        return 0;
    }
    device_call("esc_load_nodes", esc_load_nodes(ctx, &ns, 0, ns.n_nodes));
    esc_packer_destroy(pk);      /* inputs are never retained: the snapshot lives in HBM */

    /* (*Context).SetSelections(1, 0): the walks' first nodes come with every decision */
    device_call("esc_set_order_in_step", esc_set_order_in_step(ctx, 1));
    device_call("esc_set_selections", esc_set_selections(ctx, 1, 0));

    /* (*Context).RunOnce */
    device_call("esc_set_state", esc_set_state(ctx, states));
    device_call("esc_k1_calibrate", esc_k1_calibrate(ctx, 2));     /* (*Context).Calibrate */
    device_call("esc_step", esc_step(ctx));
    device_call("esc_sync", esc_sync(ctx));
    esc_group_totals* tot = cal((size_t)G, sizeof(esc_group_totals));
    esc_group_decision* dec = cal((size_t)G, sizeof(esc_group_decision));
    device_call("esc_results", esc_results(ctx, tot, dec));
    for (int g = 0; g < G; g++) {
        const esc_group_totals* t = &tot[g];
        printf("totals %d %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64
               " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 "\n",
               g, t->pod_cpu_m, t->pod_mem_b, t->n_pods, t->node_cpu_m, t->node_mem_b, t->n_nodes, t->n_untainted,
               t->n_tainted, t->n_cordoned, t->first_node, t->first_cpu_m, t->first_mem_b, t->flags);
        const esc_group_decision* d = &dec[g];
        char msg[160] = "";
        if (d->taint_status == ESC_ST_ERR_TAINT_MIN)
            esc_taint_error(t->n_untainted, groups[g].min_nodes, msg, (int32_t)sizeof msg);
        printf("decision %d %016" PRIx64 " %016" PRIx64 " %" PRId64 " %" PRId64 " %" PRId64 " %" PRId64 " %d %d %d\n",
               g, bits(d->cpu_pct), bits(d->mem_pct), d->delta, d->n_to_taint, d->cached_cpu_m, d->cached_mem_b,
               d->status, d->branch, d->taint_status);
        printf("status %d %s|%s\n", g, d->status ? esc_status_string(d->status) : "", msg);
    }
    {   /* RunOnce's esc_selections: one call into the context's persistent buffer, a second
           only when it was short (ESC_E_LIMIT: the sizes are known, the buffer grows) */
        int32_t* which = cal((size_t)G, sizeof(int32_t));
        int64_t* off = cal((size_t)G + 1, sizeof(int64_t));
        int64_t total = 0, cap = 4;                      /* small on purpose: the grow path runs */
        int64_t* sel = cal((size_t)cap, sizeof(int64_t));
        int32_t rc = esc_selections(ctx, which, off, sel, cap, &total);
        if (rc == ESC_E_LIMIT) {
            free(sel);
            cap = total;
            sel = cal((size_t)(cap ? cap : 1), sizeof(int64_t));
            rc = esc_selections(ctx, which, off, sel, cap, &total);
        }
        device_call("esc_selections", rc);
        for (int g = 0; g < G; g++) {
            printf("select %d %d %" PRId64, g, which[g], off[g + 1] - off[g]);
            for (int64_t i = off[g]; i < off[g + 1]; i++) printf(" %" PRId64, sel[i]);
            printf("\n");
        }
    }
    device_call("esc_sort_nodes", esc_sort_nodes(ctx));
    int64_t* idx = cal((size_t)(N ? N : 1), sizeof(int64_t));
    for (int g = 0; g < G; g++) {
        for (int which = 0; which < 2; which++) {
            int64_t n = 0;
            device_call("esc_group_order", esc_group_order(ctx, g, which, idx, N, &n));
            printf("order %d %d %" PRId64, g, which, n);
            for (int64_t i = 0; i < n && i < N; i++) printf(" %" PRId64, idx[i]);
            printf("\n");
        }
    }

    /* CalculatePodsRequestsTotal / CalculateNodesCapacityTotal on the whole lists */
    int64_t mem = 0, cpu = 0;
    rc = esc_pods_requests_total(ctx, pods, P, &mem, &cpu);
    if (rc == ESC_E_LIMIT) printf("list_pods overflow\n");
    else { device_call("esc_pods_requests_total", rc); printf("list_pods %" PRId64 " %" PRId64 "\n", mem, cpu); }
    rc = esc_nodes_capacity_total(ctx, nodes, N, &mem, &cpu);
    if (rc == ESC_E_LIMIT) printf("list_nodes overflow\n");
    else { device_call("esc_nodes_capacity_total", rc); printf("list_nodes %" PRId64 " %" PRId64 "\n", mem, cpu); }

    host_call("esc_ctx_destroy", esc_ctx_destroy(ctx));
    printf("done\n");
    return 0;
}
