/*
 * esc_oracle.c — CPU oracle over the packed snapshot (SoA) format.
 *
 * TEST INFRASTRUCTURE ONLY: linked by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, never by the product.  It restates the reference's semantics
 * independently of the HIP kernels, on the same inputs, at sizes the Python literal
 * oracle (oracle/oracle.py) cannot reach:
 *
 *   orc_totals      single pass: FilteredPodsLister.List + ComputePodResourceRequest +
 *                   CalculatePodsRequestsTotal (pkg/k8s/pod_listers.go:33,
 *                   pkg/k8s/scheduler/types.go:72-89, pkg/k8s/util.go:27-38), and
 *                   FilteredNodesLister.List + filterNodes + CalculateNodesCapacityTotal
 *                   (node_listers.go:33, pkg/controller/controller.go:120-154,
 *                   util.go:41-51), allNodes[0] (controller.go:208-211).  Exact sums in
 *                   __int128 (Quantity.Add's checked int64 add -> overflow flag).
 *   orc_totals_par  orc_totals over n host threads (OpenMP): the optimised all-core
 *                   "B-opt" CPU baseline of BASELINE.md §4.
 *   orc_ref_scan    the same totals computed the way the reference computes them: one
 *                   full scan of every pod per group (controller.go:416 loops groups,
 *                   each List() rescans everything) — the "port" CPU baseline.
 *   orc_decide      scaleNodeGroup's decision arithmetic (controller.go:192-351),
 *                   calcPercentUsage / calcScaleUpDelta (pkg/controller/util.go:13-81),
 *                   scaleDownTaint clamp (scale_down.go:138-158).
 *   orc_try_remove  TryRemoveTaintedNodes (scale_down.go:51-136) for one group, with
 *                   CreateNodeNameToInfoMap / NodePodsRemaining / NodeEmpty
 *                   (node_state.go:10-65) over the pods' node bindings; reference-shaped
 *                   (the group's pods rescanned per call).
 *   orc_order       taintOldestN / untaintNewestN orderings (scale_down.go:171-205,
 *                   scale_up.go:118-163, sort.go:6-39); ties by index (Go's sort.Sort
 *                   is unstable, so its tie order is not reproducible).
 *
 * Parity of this file is pinned through oracle/oracle.py (checked against every
 * transcribed reference test in tests/golden/) by tests/test_pack_parity.py.
 * Group membership: a pod / node carries interned (key, value) pair ids (pair0 + xp,
 * label0 + xl); group g selects pair gpair[g] (the numbering rule of
 * include/escalator_hip.h, restated in oracle/soa.py from the group specs).  A pod is
 * in a non-default group g iff gpair[g] is among its pairs (NewPodAffinityFilterFunc,
 * node_group.go:218-253); a node iff gpair[g] is among its label pairs
 * (NewNodeLabelFilterFunc, node_group.go:278-287).
 * Build: gcc -O2 -ffp-contract=off (oracle/Makefile).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NONE 0xFFFFFFFFu
#define PF_DS 1u
#define PF_STATIC 2u
#define PF_SEL 4u
#define PF_AFF 8u
#define PF_OVH 16u
#define NF_UNSCHED 1u
#define NF_TAINTED 2u
#define NF_TRACKED 4u

typedef __int128 i128;

static uint32_t xreg(uint32_t f) { return (f >> 8) & 0xFF; }
static uint32_t xinit(uint32_t f) { return (f >> 16) & 0xFF; }
static uint32_t xctr(uint32_t f) { return xreg(f) + xinit(f) + ((f & PF_OVH) ? 1 : 0); }
static uint32_t xpair(uint32_t f) { return (f >> 24) & 0x3F; }
static uint32_t xlbl(uint32_t f) { return (f >> 8) & 0xFF; }

/* ComputePodResourceRequest — scheduler/types.go:72-89 (int64 += wraps; init max). */
static void pod_request(uint32_t f, uint32_t cpu0, int64_t mem0, const int64_t* xc_cpu, const int64_t* xc_mem,
                        uint64_t* o, int64_t* cpu, int64_t* mem) {
    uint64_t c = cpu0, m = (uint64_t)mem0;
    for (uint32_t r = 0; r < xreg(f); ++r, ++*o) { c += (uint64_t)xc_cpu[*o]; m += (uint64_t)xc_mem[*o]; }
    for (uint32_t r = 0; r < xinit(f); ++r, ++*o) {
        if ((int64_t)m < xc_mem[*o]) m = (uint64_t)xc_mem[*o];   /* Resource.SetMaxResource :36 */
        if ((int64_t)c < xc_cpu[*o]) c = (uint64_t)xc_cpu[*o];
    }
    if (f & PF_OVH) { c += (uint64_t)xc_cpu[*o]; m += (uint64_t)xc_mem[*o]; ++*o; }
    *cpu = (int64_t)c;
    *mem = (int64_t)m;
}

typedef struct { i128 pcpu, pmem, ncpu, nmem; int64_t npod, nunt, ntaint, ncord, first; } Acc;

static int fits64(i128 v) { return v >= (i128)INT64_MIN && v <= (i128)INT64_MAX; }

static int is_tracked(const int32_t* tn, const int32_t* tg, int64_t n_trk, int64_t node, int32_t g) {
    int64_t lo = 0, hi = n_trk;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (tn[mid] < node || (tn[mid] == node && tg[mid] < g)) lo = mid + 1; else hi = mid;
    }
    return lo < n_trk && tn[lo] == node && tg[lo] == g;
}

/* filterNodes class: 0 untainted, 1 tainted, 2 cordoned (controller.go:125-150). */
static int node_class(uint32_t f, int dry, const int32_t* tn, const int32_t* tg, int64_t n_trk, int64_t i,
                      int32_t g) {
    if (dry) return ((f & NF_TRACKED) && is_tracked(tn, tg, n_trk, i, g)) ? 1 : 0;
    if (f & NF_UNSCHED) return 2;
    return (f & NF_TAINTED) ? 1 : 0;
}

/* pair id -> groups selecting it, ascending (a chain head[q] -> nxt[g]); pods skip the
 * default group (client.go:58-64 gives it NewPodDefaultFilterFunc instead). */
typedef struct { int32_t* head; int32_t* nxt; uint32_t n_gp; } PairIdx;

static int pair_idx(PairIdx* x, const uint32_t* gpair, uint32_t n_gp, int32_t G, int32_t skip) {
    x->head = (int32_t*)malloc(sizeof(int32_t) * (n_gp + 1));
    x->nxt = (int32_t*)malloc(sizeof(int32_t) * ((size_t)G + 1));
    x->n_gp = n_gp;
    if (!x->head || !x->nxt) return -1;
    for (uint32_t q = 0; q < n_gp; ++q) x->head[q] = -1;
    for (int32_t g = G - 1; g >= 0; --g) {
        x->nxt[g] = -1;
        if (g == skip || gpair[g] >= n_gp) continue;
        x->nxt[g] = x->head[gpair[g]];
        x->head[gpair[g]] = g;
    }
    return 0;
}

static void pair_idx_free(PairIdx* x) { free(x->head); free(x->nxt); }

static int32_t first_group(const PairIdx* x, uint32_t q) { return q < x->n_gp ? x->head[q] : -1; }

static void emit_out(const Acc* a, int32_t G, const int64_t* ncpu, const int64_t* nmem, int64_t* out) {
    for (int32_t g = 0; g < G; ++g) {
        int64_t* o = out + (int64_t)g * 13;
        int64_t fl = 0;
        if (!fits64(a[g].pcpu) || !fits64(a[g].pmem)) fl |= 1;
        if (!fits64(a[g].ncpu) || !fits64(a[g].nmem)) fl |= 2;
        o[0] = (int64_t)a[g].pcpu; o[1] = (int64_t)a[g].pmem; o[2] = a[g].npod;
        o[3] = (int64_t)a[g].ncpu; o[4] = (int64_t)a[g].nmem;
        o[5] = a[g].nunt + a[g].ntaint + a[g].ncord; o[6] = a[g].nunt; o[7] = a[g].ntaint; o[8] = a[g].ncord;
        o[9] = a[g].first;
        o[10] = a[g].first >= 0 ? ncpu[a[g].first] : 0;
        o[11] = a[g].first >= 0 ? nmem[a[g].first] : 0;
        o[12] = fl;
    }
}

static void node_pass(Acc* a, int64_t lo, int64_t hi, const uint32_t* nflags, const uint32_t* label0,
                      const int64_t* ncpu, const int64_t* nmem, const uint32_t* xl, const int32_t* tn,
                      const int32_t* tg, int64_t n_trk, const uint8_t* dry, int64_t n_all, const PairIdx* px) {
    uint64_t q = 0;
    for (int64_t i = 0; i < lo && i < n_all; ++i) q += xlbl(nflags[i]);
    for (int64_t i = lo; i < hi; ++i) {
        const uint32_t f = nflags[i];
        const uint32_t nx = xlbl(f);
        for (uint32_t k = 0; k <= nx; ++k) {
            const uint32_t pr = k == 0 ? label0[i] : xl[q++];
            for (int32_t g = first_group(px, pr); g >= 0; g = px->nxt[g]) {
                if (a[g].first < 0) a[g].first = i;        /* allNodes[0] in lister order */
                const int c = node_class(f, dry[g], tn, tg, n_trk, i, g);
                if (c == 0) { a[g].nunt++; a[g].ncpu += ncpu[i]; a[g].nmem += nmem[i]; }
                else if (c == 1) a[g].ntaint++;
                else a[g].ncord++;
            }
        }
    }
}

int orc_totals(int64_t n_pods, const uint32_t* flags, const uint32_t* cpu0, const int64_t* mem0,
               const uint32_t* pair0, const int64_t* xc_cpu, const int64_t* xc_mem, const uint32_t* xp,
               int64_t n_nodes, const uint32_t* nflags, const uint32_t* label0, const int64_t* ncpu,
               const int64_t* nmem, const uint32_t* xl, const int32_t* tn, const int32_t* tg, int64_t n_trk,
               int64_t node_lo, int64_t node_hi, int32_t G, int32_t default_group, const uint32_t* gpair,
               uint32_t n_gp, const uint8_t* dry, int64_t* out) {
    Acc* a = (Acc*)calloc((size_t)G, sizeof(Acc));
    PairIdx pp, np;
    if (!a || pair_idx(&pp, gpair, n_gp, G, default_group) || pair_idx(&np, gpair, n_gp, G, -1)) return -1;
    for (int32_t g = 0; g < G; ++g) a[g].first = -1;
    uint64_t oc = 0, op = 0;
    for (int64_t p = 0; p < n_pods; ++p) {
        const uint32_t f = flags[p];
        if (f & PF_DS) { oc += xctr(f); op += xpair(f); continue; }   /* node_group.go:221,259 */
        int64_t cpu, mem;
        pod_request(f, cpu0[p], mem0[p], xc_cpu, xc_mem, &oc, &cpu, &mem);
        /* default filter: !static && no nodeSelector && affinity blocks nothing (node_group.go:263-273) */
        if (default_group >= 0 && !(f & (PF_STATIC | PF_SEL | PF_AFF))) {
            a[default_group].pcpu += cpu; a[default_group].pmem += mem; a[default_group].npod++;
        }
        const uint32_t nx = xpair(f);
        for (uint32_t k = 0; k <= nx; ++k) {
            const uint32_t pr = k == 0 ? pair0[p] : xp[op++];
            for (int32_t g = first_group(&pp, pr); g >= 0; g = pp.nxt[g]) {
                a[g].pcpu += cpu; a[g].pmem += mem; a[g].npod++;
            }
        }
    }
    node_pass(a, node_lo, node_hi, nflags, label0, ncpu, nmem, xl, tn, tg, n_trk, dry, n_nodes, &np);
    emit_out(a, G, ncpu, nmem, out);
    pair_idx_free(&pp);
    pair_idx_free(&np);
    free(a);
    return 0;
}

/* The "B-opt" CPU baseline: orc_totals' single
 * pass split over n_threads host threads (OpenMP), each with private per-group
 * accumulators merged at the end.  Pod ranges start at record offsets found by a parallel
 * count + prefix of the per-pod record counts.  Same outputs as orc_totals. */
int orc_totals_par(int64_t n_pods, const uint32_t* flags, const uint32_t* cpu0, const int64_t* mem0,
                   const uint32_t* pair0, const int64_t* xc_cpu, const int64_t* xc_mem, const uint32_t* xp,
                   int64_t n_nodes, const uint32_t* nflags, const uint32_t* label0, const int64_t* ncpu,
                   const int64_t* nmem, const uint32_t* xl, const int32_t* tn, const int32_t* tg, int64_t n_trk,
                   int64_t node_lo, int64_t node_hi, int32_t G, int32_t default_group, const uint32_t* gpair,
                   uint32_t n_gp, const uint8_t* dry, int32_t n_threads, int64_t* out) {
    if (n_threads < 1) n_threads = 1;
    const int T = n_threads;
    Acc* acc = (Acc*)calloc((size_t)G * (size_t)T, sizeof(Acc));
    uint64_t* oc0 = (uint64_t*)calloc((size_t)T + 1, sizeof(uint64_t));
    uint64_t* op0 = (uint64_t*)calloc((size_t)T + 1, sizeof(uint64_t));
    PairIdx pp, np;
    if (!acc || !oc0 || !op0 || pair_idx(&pp, gpair, n_gp, G, default_group) || pair_idx(&np, gpair, n_gp, G, -1))
        return -1;
    for (int64_t k = 0; k < (int64_t)G * T; ++k) acc[k].first = -1;
    int rc = 0;
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        const int64_t lo = n_pods * t / T, hi = n_pods * (t + 1) / T;
        uint64_t c = 0, q = 0;
        for (int64_t p = lo; p < hi; ++p) { c += xctr(flags[p]); q += xpair(flags[p]); }
        oc0[t + 1] = c;
        op0[t + 1] = q;
#pragma omp barrier
#pragma omp single
        for (int k = 0; k < T; ++k) { oc0[k + 1] += oc0[k]; op0[k + 1] += op0[k]; }
        Acc* a = acc + (size_t)G * t;
        uint64_t oc = oc0[t], op = op0[t];
        for (int64_t p = lo; p < hi; ++p) {
            const uint32_t f = flags[p];
            if (f & PF_DS) { oc += xctr(f); op += xpair(f); continue; }
            int64_t cpu, mem;
            pod_request(f, cpu0[p], mem0[p], xc_cpu, xc_mem, &oc, &cpu, &mem);
            if (default_group >= 0 && !(f & (PF_STATIC | PF_SEL | PF_AFF))) {
                a[default_group].pcpu += cpu; a[default_group].pmem += mem; a[default_group].npod++;
            }
            const uint32_t nx = xpair(f);
            for (uint32_t k = 0; k <= nx; ++k) {
                const uint32_t pr = k == 0 ? pair0[p] : xp[op++];
                for (int32_t g = first_group(&pp, pr); g >= 0; g = pp.nxt[g]) {
                    a[g].pcpu += cpu; a[g].pmem += mem; a[g].npod++;
                }
            }
        }
        /* nodes: contiguous thread ranges, so the lowest thread with a member holds allNodes[0] */
        const int64_t span = node_hi - node_lo;
        node_pass(a, node_lo + span * t / T, node_lo + span * (t + 1) / T, nflags, label0, ncpu, nmem, xl, tn, tg,
                  n_trk, dry, n_nodes, &np);
#pragma omp barrier
        /* merge: thread t owns groups [G*t/T, G*(t+1)/T) */
        for (int32_t g = (int32_t)((int64_t)G * t / T); g < (int32_t)((int64_t)G * (t + 1) / T); ++g) {
            Acc s = acc[g];
            for (int k = 1; k < T; ++k) {
                const Acc* b = &acc[(size_t)G * k + g];
                s.pcpu += b->pcpu; s.pmem += b->pmem; s.ncpu += b->ncpu; s.nmem += b->nmem;
                s.npod += b->npod; s.nunt += b->nunt; s.ntaint += b->ntaint; s.ncord += b->ncord;
                if (s.first < 0) s.first = b->first;
            }
            acc[g] = s;
        }
    }
    emit_out(acc, G, ncpu, nmem, out);
    pair_idx_free(&pp);
    pair_idx_free(&np);
    free(acc);
    free(oc0);
    free(op0);
    return rc;
}

/* Reference-shaped: every group rescans every pod and re-evaluates its filter and the
 * pod's request (controller.go:416 -> scaleNodeGroup -> Pods.List() -> filterFunc per pod
 * -> CalculatePodsRequestsTotal).  Groups [g_lo, g_hi) only, so a bounded sample can be
 * timed. */
int orc_ref_scan(int64_t n_pods, const uint32_t* flags, const uint32_t* cpu0, const int64_t* mem0,
                 const uint32_t* pair0, const int64_t* xc_cpu, const int64_t* xc_mem, const uint32_t* xp,
                 int64_t n_nodes, const uint32_t* nflags, const uint32_t* label0, const int64_t* ncpu,
                 const int64_t* nmem, const uint32_t* xl, const int32_t* tn, const int32_t* tg, int64_t n_trk,
                 int32_t G, int32_t default_group, const uint32_t* gpair, const uint8_t* dry, int32_t g_lo,
                 int32_t g_hi, int64_t* out) {
    Acc* a = (Acc*)calloc((size_t)G, sizeof(Acc));
    if (!a) return -1;
    for (int32_t g = 0; g < G; ++g) a[g].first = -1;
    for (int32_t g = g_lo; g < g_hi; ++g) {
        uint64_t oc = 0, op = 0;
        for (int64_t p = 0; p < n_pods; ++p) {
            const uint32_t f = flags[p];
            const uint64_t oc0 = oc;
            oc += xctr(f);
            int member = 0;
            if (!(f & PF_DS)) {
                if (g == default_group) {
                    member = !(f & (PF_STATIC | PF_SEL | PF_AFF));
                } else {
                    const uint32_t nx = xpair(f);          /* NodeSelector[K]==V || In(K,V) */
                    for (uint32_t k = 0; k <= nx && !member; ++k) {
                        uint32_t h = k == 0 ? pair0[p] : xp[op + k - 1];
                        member = (h == gpair[g]);
                    }
                }
            }
            op += xpair(f);
            if (!member) continue;
            int64_t cpu, mem;
            uint64_t o = oc0;
            pod_request(f, cpu0[p], mem0[p], xc_cpu, xc_mem, &o, &cpu, &mem);
            a[g].pcpu += cpu; a[g].pmem += mem; a[g].npod++;
        }
        /* nodes: every group rescans all nodes too (node_listers.go:33) */
        uint64_t q = 0;
        for (int64_t i = 0; i < n_nodes; ++i) {
            const uint32_t f = nflags[i];
            int member = 0;
            for (uint32_t k = 0; k <= xlbl(f); ++k) {              /* Labels[K] == V */
                uint32_t h = k == 0 ? label0[i] : xl[q + k - 1];
                member |= (h == gpair[g]);
            }
            q += xlbl(f);
            if (!member) continue;
            if (a[g].first < 0) a[g].first = i;
            const int c = node_class(f, dry[g], tn, tg, n_trk, i, g);
            if (c == 0) { a[g].nunt++; a[g].ncpu += ncpu[i]; a[g].nmem += nmem[i]; }
            else if (c == 1) a[g].ntaint++;
            else a[g].ncord++;
        }
    }
    emit_out(a, G, ncpu, nmem, out);
    free(a);
    return 0;
}

/* ------------------------------------------------------------ decision math */
static const double MAXF = 1.7976931348623157e308;

static int64_t milli_mem(int64_t b) { return (int64_t)((uint64_t)b * 1000u); }   /* Quantity.MilliValue */

static double go_max(double x, double y) {                                   /* math.Max */
    if (isinf(x) && x > 0) return x;
    if (isinf(y) && y > 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? y : x;
    return x > y ? x : y;
}

static int64_t go_int(double x) {                                            /* int(float64) on amd64 */
    if (isnan(x) || !(x < 9223372036854775808.0) || !(x >= -9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

/* calcPercentUsage — util.go:58-81.  Returns 0 or 3 (divide by zero). */
int orc_percent(int64_t cpu_req, int64_t mem_req, int64_t cpu_cap, int64_t mem_cap, int64_t n_unt, double* cpu,
                double* mem) {
    int64_t a = cpu_req, b = milli_mem(mem_req), c = cpu_cap, d = milli_mem(mem_cap);
    if (a == 0 && b == 0 && c == 0 && d == 0 && n_unt == 0) { *cpu = 0; *mem = 0; return 0; }
    if (c == 0 || d == 0) {
        if (n_unt == 0) { *cpu = MAXF; *mem = MAXF; return 0; }
        *cpu = 0; *mem = 0; return 3;
    }
    *cpu = (double)a / (double)c * 100;
    *mem = (double)b / (double)d * 100;
    return 0;
}

/* calcScaleUpDelta — util.go:13-46.  Returns 0 or 4 (negative delta). */
int orc_scale_up(int64_t n_unt, double cpu, double mem, int64_t cpu_req, int64_t mem_req, int64_t ccpu, int64_t cmem,
                 int32_t thr, int64_t* delta) {
    double nc = (double)n_unt, t = (double)thr, a, b;
    if (cpu == MAXF || mem == MAXF) {
        if (ccpu == 0 || cmem == 0) { *delta = 1; return 0; }
        a = ceil((double)cpu_req / (double)ccpu / t * 100);
        b = ceil((double)milli_mem(mem_req) / (double)milli_mem(cmem) / t * 100);
    } else {
        a = ceil(nc * ((cpu - t) / t));
        b = ceil(nc * ((mem - t) / t));
    }
    *delta = go_int(go_max(a, b));
    return *delta < 0 ? 4 : 0;
}

/* params[g]: min,max,upper,lower,up,slow,fast,dry,locked,requested,cached_cpu,cached_mem
 * totals[g]: emit_out layout.  dec_f[g]: cpu,mem.  dec_i[g]: delta,n_to_taint,cached_cpu,
 * cached_mem,status,branch,taint_status (branch codes as ESC_BR_*). */
void orc_decide(int32_t G, const int64_t* params, const int64_t* totals, double* dec_f, int64_t* dec_i) {
    for (int32_t g = 0; g < G; ++g) {
        const int64_t* p = params + (int64_t)g * 12;
        const int64_t* t = totals + (int64_t)g * 13;
        double* df = dec_f + (int64_t)g * 2;
        int64_t* di = dec_i + (int64_t)g * 7;
        const int64_t n_pods = t[2], n_nodes = t[5], n_unt = t[6];
        int64_t delta = 0, ntt = 0, status = 0, branch = 8, tst = 0;
        double cpu = 0, mem = 0;
        int64_t ccpu = n_nodes > 0 ? t[10] : p[10];                    /* controller.go:208 */
        int64_t cmem = n_nodes > 0 ? t[11] : p[11];
        if (n_nodes == 0 && n_pods == 0) branch = 0;                     /* :233 */
        else if (n_nodes < p[0]) { branch = 1; status = 1; }             /* :238 */
        else if (n_nodes > p[1]) { branch = 1; status = 2; }             /* :247 */
        else if (t[12]) { branch = 1; status = 5; }
        else if (n_unt < p[0]) { branch = 2; delta = p[0] - n_unt; }     /* :281 */
        else {
            int st = orc_percent(t[0], t[1], t[3], t[4], n_unt, &cpu, &mem);
            if (st) { branch = 3; status = st; }
            else if (p[8]) { branch = 4; delta = p[9]; }                 /* :317 */
            else {
                double mx = go_max(cpu, mem);
                if (mx < (double)p[3]) { branch = 5; delta = -p[6]; }
                else if (mx < (double)p[2]) { branch = 6; delta = -p[5]; }
                else if (mx > (double)p[4]) {
                    branch = 7;
                    status = orc_scale_up(n_unt, cpu, mem, t[0], t[1], ccpu, cmem, (int32_t)p[4], &delta);
                }
                if (status == 0 && delta < 0) {                          /* scale_down.go:143-158 */
                    ntt = -delta;
                    if (n_unt - ntt < p[0]) {
                        ntt = n_unt - p[0];
                        if (ntt < 0) { tst = 6; ntt = 0; }
                    }
                }
            }
        }
        df[0] = cpu; df[1] = mem;
        di[0] = delta; di[1] = ntt; di[2] = ccpu; di[3] = cmem; di[4] = status; di[5] = branch; di[6] = tst;
    }
}

/* --------------------------------------------------------------- ordering */
typedef struct { int64_t key; int64_t idx; } KI;

static int cmp_ki(const void* a, const void* b) {
    const KI* x = (const KI*)a;
    const KI* y = (const KI*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* which 0: untainted oldest-first; 1: tainted newest-first.  Returns the member count;
 * writes up to cap indices. */
int64_t orc_order(int64_t n_nodes, const uint32_t* nflags, const uint32_t* label0, const int64_t* created,
                  const uint32_t* xl, const int32_t* tn, const int32_t* tg, int64_t n_trk, int64_t lo, int64_t hi,
                  const uint8_t* dry, const uint32_t* gpair, int32_t group, int32_t which, int64_t* out,
                  int64_t cap) {
    KI* v = (KI*)malloc(sizeof(KI) * (size_t)(hi - lo + 1));
    int64_t m = 0;
    uint64_t q = 0;
    for (int64_t i = 0; i < lo && i < n_nodes; ++i) q += xlbl(nflags[i]);
    for (int64_t i = lo; i < hi; ++i) {
        const uint32_t f = nflags[i];
        int member = 0;
        for (uint32_t k = 0; k <= xlbl(f); ++k) {
            uint32_t h = k == 0 ? label0[i] : xl[q + k - 1];
            member |= (h == gpair[group]);
        }
        q += xlbl(f);
        if (!member) continue;
        const int c = node_class(f, dry[group], tn, tg, n_trk, i, group);
        if (c != which) continue;
        v[m].key = which == 0 ? created[i] : -created[i];
        v[m].idx = i;
        ++m;
    }
    qsort(v, (size_t)m, sizeof(KI), cmp_ki);
    for (int64_t i = 0; i < m && i < cap; ++i) out[i] = v[i].idx;
    free(v);
    return m;
}

/* (*Controller).TryRemoveTaintedNodes — scale_down.go:51-136, one group.  The group's
 * NodeInfoMap (controller.go:259 -> CreateNodeNameToInfoMap, node_state.go:10-39) is
 * restated as occ[node] = the group's non-daemonset pods bound to the node
 * (NodePodsRemaining, node_state.go:48-65; pods bound to no / an unknown node are dropped,
 * node_state.go:31-36).  Then its tainted nodes (filterNodes, controller.go:125-150) in
 * snapshot order: safeFromDeletion (:39-46), GetToBeRemovedTime (taint.go:91-103;
 * taint_s INT64_MIN = none), now.Sub(taintedTime) (saturating, as time.Time.Sub) against
 * the soft / hard grace (:71-99), deletions only when not in dry mode.
 * res = {n_candidates, n_delete, pods_remaining}; out = deleted node indices.  */
int64_t orc_try_remove(int64_t n_pods, const uint32_t* flags, const uint32_t* pair0, const uint32_t* xp,
                       const uint32_t* pod_node, int64_t n_nodes, const uint32_t* nflags, const uint32_t* label0,
                       const uint32_t* xl, const int32_t* tn, const int32_t* tg, int64_t n_trk,
                       const int64_t* taint_s, const uint8_t* no_delete, const uint8_t* dry,
                       const uint32_t* gpair, int32_t default_group, int32_t group, int64_t now_ns, int64_t soft_ns,
                       int64_t hard_ns, int64_t* res, int64_t* out, int64_t cap) {
    int64_t* occ = (int64_t*)calloc((size_t)n_nodes + 1, sizeof(int64_t));
    if (!occ) return -1;
    const uint32_t q = gpair[group];
    uint64_t op = 0;
    for (int64_t p = 0; p < n_pods; ++p) {
        const uint32_t f = flags[p], nx = xpair(f);
        int in = 0;
        if (group == default_group) {
            in = !(f & (PF_STATIC | PF_SEL | PF_AFF));                /* NewPodDefaultFilterFunc */
        } else {
            in = pair0[p] == q;                                         /* NewPodAffinityFilterFunc */
            for (uint32_t k = 0; k < nx; ++k) in |= xp[op + k] == q;
        }
        op += nx;
        if (!in || (f & PF_DS) || pod_node[p] == NONE) continue;        /* NodePodsRemaining skips DS */
        occ[pod_node[p]]++;
    }
    int64_t cand = 0, del = 0, rem = 0, ql = 0;
    for (int64_t i = 0; i < n_nodes; ++i) {
        const uint32_t f = nflags[i];
        int member = 0;
        for (uint32_t k = 0; k <= xlbl(f); ++k) member |= (k == 0 ? label0[i] : xl[ql + k - 1]) == q;
        ql += xlbl(f);
        if (!member || node_class(f, dry[group], tn, tg, n_trk, i, group) != 1) continue;
        ++cand;
        if (no_delete[i] || taint_s[i] == INT64_MIN) continue;
        const i128 d = (i128)now_ns - (i128)taint_s[i] * 1000000000;
        const int64_t age = d > (i128)INT64_MAX ? INT64_MAX : d < (i128)INT64_MIN ? INT64_MIN : (int64_t)d;
        if (age > soft_ns && (occ[i] == 0 || age > hard_ns) && !dry[group]) {
            if (del < cap) out[del] = i;
            ++del;
            rem += occ[i];
        }
    }
    res[0] = cand; res[1] = del; res[2] = rem;
    free(occ);
    return del;
}

/* Every group's two orderings at once (the full-size config-5 check): one pass buckets
 * each (node, group) membership of nodes [lo, hi) by (group, class) — classes 0
 * untainted (oldest first) and 1 tainted (newest first), cordoned dropped — and each
 * bucket is sorted as orc_order sorts.  off[2G + 1] (bucket g * 2 + which), idx[off[2G]].
 * Two calls: idx == NULL only counts (fills off). */
int64_t orc_order_all(int64_t n_nodes, const uint32_t* nflags, const uint32_t* label0, const int64_t* created,
                      const uint32_t* xl, const int32_t* tn, const int32_t* tg, int64_t n_trk, int64_t lo, int64_t hi,
                      const uint8_t* dry, const uint32_t* gpair, uint32_t n_gp, int32_t G, int64_t* off, int64_t* idx) {
    PairIdx px;
    if (pair_idx(&px, gpair, n_gp, G, -1)) return -1;
    int64_t* cnt = (int64_t*)calloc((size_t)2 * G + 1, sizeof(int64_t));
    KI* v = NULL;
    if (!cnt) { pair_idx_free(&px); return -1; }
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {
            if (!idx) break;
            v = (KI*)malloc(sizeof(KI) * (size_t)(off[2 * G] + 1));
            if (!v) { free(cnt); pair_idx_free(&px); return -1; }
            for (int64_t b = 0; b < 2 * (int64_t)G; ++b) cnt[b] = off[b];
        }
        uint64_t q = 0;
        for (int64_t i = 0; i < lo && i < n_nodes; ++i) q += xlbl(nflags[i]);
        for (int64_t i = lo; i < hi; ++i) {
            const uint32_t f = nflags[i];
            const uint32_t nx = xlbl(f);
            for (uint32_t k = 0; k <= nx; ++k) {
                const uint32_t pr = k == 0 ? label0[i] : xl[q++];
                for (int32_t g = first_group(&px, pr); g >= 0; g = px.nxt[g]) {
                    const int c = node_class(f, dry[g], tn, tg, n_trk, i, g);
                    if (c > 1) continue;
                    const int64_t b = 2 * (int64_t)g + c;
                    if (pass == 0) { cnt[b]++; continue; }
                    v[cnt[b]].key = c == 0 ? created[i] : -created[i];
                    v[cnt[b]].idx = i;
                    cnt[b]++;
                }
            }
        }
        if (pass == 0) {
            off[0] = 0;
            for (int64_t b = 0; b < 2 * (int64_t)G; ++b) off[b + 1] = off[b] + cnt[b];
        }
    }
    if (v) {
        for (int64_t b = 0; b < 2 * (int64_t)G; ++b) {
            qsort(v + off[b], (size_t)(off[b + 1] - off[b]), sizeof(KI), cmp_ki);
            for (int64_t k = off[b]; k < off[b + 1]; ++k) idx[k] = v[k].idx;
        }
        free(v);
    }
    free(cnt);
    pair_idx_free(&px);
    return off[2 * G];
}
