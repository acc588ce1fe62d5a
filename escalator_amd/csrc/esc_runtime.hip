// esc_runtime.hip — host runtime behind the C ABI (include/escalator_hip.h).
//
// One esc_ctx per process and GPU.  The context owns the device-resident snapshot
// (pod shard replicas + full node table), the per-workgroup partial buffers, the
// exchanged per-group words and the decision buffers, one HIP stream (or the caller's)
// and an optional hipGraph of the whole decision step.  The only host<->device
// traffic per decision is the launch (a graph replay for one rank) and the copy of the
// per-group decisions back to pinned host memory.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <type_traits>
#include <string>
#include <vector>

#include "esc_internal.h"
#include "esc_kernels.h"
#include "esc_multi.h"

#ifndef ESC_MEASURE
#define ESC_MEASURE 0   // 1: the measurement library (Makefile ABLATIONS=1) reads its knobs
#endif

using namespace esc;

namespace {

constexpr int LDS_BYTES = 160 * 1024;
constexpr int POD_WINDOW_MAX = LDS_BYTES / 16;      // groups whose pod partials fit in LDS
static_assert(POD_WINDOW_MAX % 2 == 0 && FC_COL % 2 == 0, "K1's 16-B partial-row stores need even window starts");
constexpr int MAX_STAGES = 10;
constexpr int32_t HTOT_MAX_GROUPS = 1024;   // K4 writes the totals records to host memory (<= 104 KB)

#define HIP_TRY(x)                                              \
    do {                                                        \
        hipError_t e_ = (x);                                    \
        if (e_ != hipSuccess) return fail_hip(e_, #x);          \
    } while (0)

thread_local char g_last_error[256];

template <class T>
hipError_t dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T));
}

template <class T>
void dfree(T*& p) {
    if (p) hipFree(p);
    p = nullptr;
}

struct PodBuf {
    uint32_t* kb = nullptr;                      // K blocks (tile-major K section)
    uint32_t *flags = nullptr, *cpu0 = nullptr, *pair0 = nullptr, *xp = nullptr, *xc_base = nullptr,
             *xp_base = nullptr, *big = nullptr;
    int64_t *mem0 = nullptr, *xc_cpu = nullptr, *xc_mem = nullptr;
    PodClass* cls = nullptr;
    void release() {
        dfree(kb); dfree(flags); dfree(cpu0); dfree(pair0); dfree(xp); dfree(xc_base); dfree(xp_base); dfree(big);
        dfree(mem0); dfree(xc_cpu); dfree(xc_mem); dfree(cls);
    }
};

struct NodeBuf {
    // node table (snapshot order)
    uint32_t *flags = nullptr, *label0 = nullptr, *xl = nullptr, *xl_off = nullptr, *trk_start = nullptr;
    int64_t *cpu = nullptr, *mem = nullptr, *created = nullptr;
    int32_t *trk_node = nullptr, *trk_group = nullptr;
    // pair-major entries, pieces, tracker by group, K2 rows
    uint32_t *e_flags = nullptr, *e_node = nullptr, *piece_off = nullptr, *piece_pair = nullptr, *pp_off = nullptr;
    uint32_t* span_off = nullptr;                // K2 waves' piece ranges
    uint32_t* span_e = nullptr;                  // and their entry ranges
    int64_t *e_cpu = nullptr, *e_mem = nullptr, *rows = nullptr;
    uint4* e_pk = nullptr;                       // the entries packed 16 B each (NodeDev::e_pk)
    GroupNode* gnode = nullptr;
    void release() {
        dfree(gnode);
        dfree(flags); dfree(label0); dfree(xl); dfree(xl_off); dfree(trk_start); dfree(cpu); dfree(mem);
        dfree(created); dfree(trk_node); dfree(trk_group);
        dfree(e_flags); dfree(e_node); dfree(piece_off); dfree(piece_pair); dfree(pp_off); dfree(span_off); dfree(span_e);
        dfree(e_cpu); dfree(e_mem); dfree(rows); dfree(e_pk);
    }
};

}  // namespace

namespace esc {
int32_t fail_hip(hipError_t e, const char* what) {
    std::snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? ESC_E_NOMEM : ESC_E_HIP;
}

int32_t fail_comm(const char* what, const char* why) {
    std::snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, why);
    return ESC_E_COMM;
}

const RcclApi& rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = nullptr;
        for (const char* n : {"librccl.so", "librccl.so.1"})
            if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD)) != nullptr) break;
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!h) return a;
        auto sym = [&](auto& f, const char* name) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name)); };
        sym(a.get_unique_id, "ncclGetUniqueId");
        sym(a.init_rank, "ncclCommInitRank");
        sym(a.init_all, "ncclCommInitAll");
        sym(a.all_reduce, "ncclAllReduce");
        sym(a.reduce_scatter, "ncclReduceScatter");
        sym(a.group_start, "ncclGroupStart");
        sym(a.group_end, "ncclGroupEnd");
        sym(a.count, "ncclCommCount");
        sym(a.destroy, "ncclCommDestroy");
        sym(a.error_string, "ncclGetErrorString");
        a.ok = a.get_unique_id && a.init_rank && a.init_all && a.all_reduce && a.reduce_scatter && a.group_start &&
               a.group_end && a.count && a.destroy && a.error_string;
        return a;
    }();
    return api;
}
}  // namespace esc

namespace {

int bit_width(uint64_t v) {
    int b = 0;
    while (v) { ++b; v >>= 1; }
    return b;
}

}  // namespace

struct esc_ctx {
    int device = -1, rank = 0, world = 1;
    bool has_device = false;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int cu_count = 0;
    GroupIndex gi;
    std::vector<GroupParams> params;
    // device group tables
    uint8_t* d_dry = nullptr;
    GroupParams* d_params = nullptr;
    uint32_t *d_gpair = nullptr, *d_node_code = nullptr, *d_code_list = nullptr;
    uint32_t* d_gslot = nullptr;
    // snapshot
    std::vector<PodBuf> pods;
    int n_replicas = 1, cur = 0;
    int64_t k_weight = 0;
    int64_t n_pods = 0, k_tiles = 0, c_tiles = 0, n_xc = 0, n_xp = 0, pod_offset = 0, n_big = 0;
    int32_t n_cls = 0;
    bool pods_loaded = false;
    NodeBuf nodes;
    int64_t n_nodes = 0, n_xl = 0, n_trk = 0, node_lo = 0, node_hi = 0;
    int64_t n_entries = 0, n_pieces = 0, pc_lo = 0, pc_hi = 0, node_bytes = 0, n_spans = 0;
    int64_t ts_min = 0, ts_max = 0;
    bool nodes_loaded = false;
    // every node's allocatable cpu is in [0, 2^32): K2 reads the packed 16-B entries (node
    // events that break it switch K2 back to the three entry arrays, dropping the graphs)
    bool e_pk_ok = false;
    uint32_t q_lo = 0, q_hi = 0;                              // the group pairs this rank owns (§7)
    std::vector<uint32_t> q_bounds;                           // every rank's first owned pair, + n_gp
    std::vector<int64_t> pair_live;                           // group pair -> live node entries
    // work
    int nblk = 0;
    uint64_t* d_pod_part = nullptr;
    uint32_t *d_col_off = nullptr, *d_col_groups = nullptr;   // K3: groups by pod slot column
    int k3_ablate = 0;                                        // ESC_K3_ABLATE (timing-only knob)
    bool tail_trace = false;                                  // ESC_TAIL_TRACE (measurement library)
    uint64_t* d_ttrace = nullptr;                             // tail + node-groups block timestamps
    int64_t ttrace_cap = 0, ttrace_tail = 0, ttrace_ng = 0;   // words; blocks of the last traced step
    int64_t* d_wide_pod = nullptr;
    uint32_t* d_k1_ticket = nullptr;                          // K1 dynamic shares (next chunk, done)
    int64_t* d_k1seg = nullptr;                               // K1 work plan [nblk][K1_SEGS][2]
    // Compact K1 flush: the pod-slot columns each workgroup's share touches
    // (bitmap of touch_tw u32 per workgroup, kept current by pod upserts), as per-workgroup
    // {column, entry} lists and per-column entry ranges on the device.
    bool touch_on = false;
    bool full_flush = false;                                  // ESC_K1_FULL_FLUSH=1 (measurement knob)
    int touch_tw = 0;
    std::vector<uint32_t> h_touch;
    std::vector<std::array<int64_t, 3>> h_tile_wg;            // {first tile, end tile, workgroup}, sorted
    uint32_t* d_touch = nullptr;
    uint2* d_wg_cols = nullptr;
    uint32_t* d_wg_off = nullptr;
    uint32_t* d_col_rows = nullptr;
    std::vector<double> k1_share;                             // calibrated K1 shares (esc_k1_calibrate)
    int k1_cap = 0;                                           // K1 chunks per workgroup at most (0: static)
    uint64_t* d_k1_trace = nullptr;                           // K1 per-workgroup timestamps (esc_k1_trace)
    int64_t* d_trk_acc = nullptr;                             // [G][TA_K] dry-mode tracked sums
    int64_t* d_pwords = nullptr;                              // active exchange buffer [world * own_cap][PW_K]
    int64_t* own_pwords = nullptr;                            // the context-owned one
    int64_t* d_nwords = nullptr;                              // [G][NW_K] node words (exact for owned groups),
                                                              // right after own_pwords (one allocation)
    // Owner-major exchange rows: group g's pod words at row h_xs[g] = owner *
    // own_cap + its index among the owner's groups, so one ncclReduceScatter hands every
    // owner the exact sums of its own groups; h_own = this rank's groups (ascending).
    int32_t own_cap = 0, own_first = 0;
    bool own_seq = true;                                      // h_own is own_first + i
    std::vector<uint32_t> h_own, h_xs;
    uint32_t *d_own = nullptr, *d_xs = nullptr;
    esc_group_decision* d_dec = nullptr;                     // full records (device)
    DecCompact* d_cdec = nullptr;                             // compact records (device; no zero-copy)
    DecCompact* h_cdec = nullptr;                             // compact records (pinned host)
    DecCompact* h_cdec_dev = nullptr;                         // device view of h_cdec (zero-copy)
    bool zero_copy = true;                                    // K3/K4 write compact decisions to h_cdec
    bool order_in_step = false;                               // K5 ordering inside every decision
    // selections delivered with the decision (esc_set_selections, SelOut): K4 writes every
    // decided group's taint / untaint nodes into h_sel (pinned, zero-copy) as [header, nodes]
    // runs, their offsets into the compact records
    int32_t sel_slack = -1, sel_group_cap = 0;
    uint32_t *h_sel = nullptr, *h_sel_dev = nullptr;
    int64_t sel_words = 0;
    bool want_metrics = false;                                // K4 also writes the gauges
    esc_group_metrics* d_metrics = nullptr;
    int64_t* bound_pwords = nullptr;                          // caller-bound exchange buffer
    int64_t bound_words = 0;                                  // its size: xw_count when bound
    void* comm = nullptr;                                     // RCCL communicator (esc_comm_init)
    bool work_ready = false;
    // An informer-event batch that failed after its first write (a HIP error mid-apply)
    // leaves host mirrors and device arrays half-updated: decisions and reaping are refused
    // (ESC_E_STATE) until the snapshot is reloaded (STALE_PODS: esc_load_pods, STALE_NODES:
    // esc_load_nodes).  ADVICE r4.
    uint32_t stale = 0;
    // world > 1: a shard step's node groups run with K4 after the exchange (esc_decide); a
    // reduce not followed by a decide leaves them pending (the tail's tracker sums unread)
    bool ng_pending = false;
    bool force_wide = false;
    int k1_variant = 0;                                       // ESC_K1_VARIANT (measurement knob)
    // K pods of a class are laid out in order of pair0 / pod_sort (0: input order), so that a
    // K1 workgroup's share touches few pod-slot columns; ESC_POD_SORT
    uint32_t pod_sort = FC_COL;   // one K3 column per bucket (exact pair order serialises K1's LDS atomics: 0.65 ms)
    // graph
    bool use_graph = false;
    std::vector<hipGraphExec_t> graphs;                       // esc_run: whole decision (world 1)
    std::vector<hipGraphExec_t> rgraphs;                      // esc_reduce: the shard's step (world > 1)
    // timing
    bool timing = false;
    hipEvent_t ev[MAX_STAGES] = {};
    hipEvent_t k1t_ev[2] = {};                                // esc_k1_time's own pair (stage events stay readable)
    double stage_ms[MAX_STAGES] = {};
    int n_stage_ev = 0;
    bool pending = false;
    // K5 ordering: the age index (built at load) and the per-decision partition
    uint64_t* d_mkeys[2] = {nullptr, nullptr};               // index build: (group | creation offset)
    uint32_t* d_mvals[2] = {nullptr, nullptr};               //              (node | flags << 28)
    int64_t mcap = 0;                                         // their capacity (memberships)
    bool age_built = false;
    bool age_ok = false;                                      // the last build succeeded (its regions are valid)
    uint32_t *d_hist = nullptr, *d_tot = nullptr;
    // The index's small tables live in ONE allocation, filled by ONE upload per build
    // (build_age_index): sorted starts d_seg, region starts / lengths, chunk tables, the
    // listing's status words, the error word and listed total, the groups' tie flags.
    uint8_t* d_itab = nullptr;
    size_t itab_cap = 0;
    uint32_t *d_total = nullptr, *d_ierr = nullptr;           // (views into d_itab)
    uint32_t* d_g_tie = nullptr;                              // [G] equal creation times in the group (RegionSink::tie)
    uint64_t* d_lstat = nullptr;                              // single-pass listing status words
    int64_t* d_seg = nullptr;
    int64_t n_memb = 0;
    int order_src = 0;
    // group order of the memberships (per-decision 3-way split by class inside each group)
    uint32_t* d_g_memb = nullptr;                             // K5 regions: membership words
    uint32_t *d_grp_off = nullptr, *d_gch_off = nullptr;
    uint64_t* d_ostat = nullptr;                              // k_ord_split status words (x2)
    int ord_parity = 0;                                       // which status array the next ordering uses
    // A look-back that gave up (k_ord_split, OrdFail) sets the pinned word h_oerr; the host
    // reads it after its stream waits: esc_sync reports it once as ESC_E_ORDER and clears it,
    // and esc_group_order refuses (ESC_E_ORDER) until the next ordering is enqueued.
    uint32_t *h_oerr = nullptr, *h_oerr_dev = nullptr;
    bool ord_failed = false;
    // fault injection, measurement library only (esc_debug_*: tests/test_gpu_faults.py): the
    // next n ordering / listing launches give up their look-back at once, the next n event
    // patch applications fail after their host-side writes
    int lb_fail_order = 0, lb_fail_list = 0, fail_patches = 0;
    uint32_t *d_pstart = nullptr, *d_plen = nullptr;
    uint32_t* d_ord = nullptr;                                // K5 output, in the group regions
    OrdChunk* d_pchunks = nullptr;                            // packed chunks of small groups
    int64_t n_pchunks = 0, n_psmall = 0;                      // all / those <= ORD_PCHUNK (first)
    std::vector<uint32_t> h_pstart, h_plen;                   // group regions: start, memberships
    std::vector<uint32_t> h_pcap;                             // every group's region capacity (owned or not)
    std::vector<uint32_t> h_gch_off;                          // group -> its split chunks (big groups)
    int64_t n_gpad = 0;                                       // padded group-order length
    OrdChunk* d_chunks = nullptr;
    int64_t n_chunks = 0;
    uint64_t sort_div = 1;
    int sort_R = 1;
    bool age_exact = false;                                   // this snapshot needs the exact 64-bit keys
    bool sorted = false;
    std::vector<int64_t> h_created;                           // [lo, hi) creation times (tie order)
    // node informer events (§8f rank 1): capacity and host mirrors for in-place add / delete
    int64_t n_cap = 0, xl_used = 0, xl_cap = 0, age_n = -1;
    std::vector<uint32_t> h_label0, h_xl_off, h_xl;           // node labels (pair ids)
    std::vector<uint32_t> h_e_node;                           // pair-major entry -> node (NONE: spare)
    std::vector<uint32_t> pair_next, pair_end;                // group pair -> next spare entry, range end
    std::vector<uint32_t> pair_lo;                            // group pair -> its first entry
    uint32_t nodes_piece_lo(uint32_t q) const { return pair_lo[q]; }
    std::vector<uint32_t> h_gn;                               // group regions' nodes (lazy mirror of d_g_memb)
    // per-function drop-ins: the list reducer (esc_list.hip); esc_order_by_creation runs
    // on a one-group list context
    esc_ctx* list_ctx = nullptr;
    esc::ListReducer* lred = nullptr;
    // single-process multi-device context (esc_ctx_create_multi): every call dispatches to
    // its per-device contexts (esc_multi.hip); null for a per-device context
    esc::esc_multi_state* multi = nullptr;
    // incremental snapshot (§8f rank 1): where each loaded pod lives, free K slots
    double spare_frac = 0.0;                                  // esc_set_spare
    hvec<int32_t> pod_cls;                                    // by pod id: K class index, -1 C, -2 absent
    hvec<int64_t> pod_pos;                                    // K: position in its class; C: base-array index
    std::vector<std::vector<int64_t>> cls_free;               // per K class: free positions
    std::vector<PodClass> h_cls;
    std::vector<int> h_cls_of;                                // signature id -> class index (-1: none)
    std::vector<uint32_t> h_cflags;                           // C-section flags (deletes keep the counts)
    std::vector<int64_t> c_free;                              // free C slots (C-array index), room in h_cflags
    std::vector<uint32_t> h_cused;                            // a C slot's pod's own records | pairs << 16
    std::vector<uint32_t> h_xc_base, h_xp_base;               // C tiles' record / pair offsets
    int64_t live_pods = 0, live_xc = 0, live_xp = 0;
    int64_t live_pk_pods = 0, live_pk_xc = 0;   // of them in packed K classes (either size)
    int64_t live_p8_pods = 0, live_p8_xp = 0;   // of them in packed small K classes, their extra pairs
    int64_t c_tiles_loaded = 0;                 // C tiles of loaded pods (the spare C tiles excluded)
    // node state mirrors for esc_nodes_update
    std::vector<uint32_t> h_nflags;
    std::vector<int64_t> h_ncpu, h_nmem;
    std::vector<uint32_t> ne_off, ne_pos;                     // node -> its pair-major entry positions
    // The reaping occupancy words, maintained by pod / node events once esc_load_placement
    // counted them (K6 no longer runs per call): d_occ at one rank; with several ranks the
    // maintained local words are d_occ_local and d_occ is the exchange buffer.
    uint32_t* d_occ_local = nullptr;
    uint32_t* d_ne_off = nullptr;                             // device copies of ne_off / ne_pos
    uint32_t* d_ne_pos = nullptr;
    int64_t ne_dev_nodes = -1, ne_dev_pos = -1;
    std::vector<GroupNode> h_gnode;
    // dry-mode taintTracker mirror (§8f rank 4): (node << 32 | group), sorted, unique
    std::vector<uint64_t> h_trk;
    int64_t trk_cap = 0;                                      // device capacity of trk_node/_group
    // scale-down reaping (§8f rank 2): pods bound to nodes, per-node taint times
    bool placed = false;                                      // pod binding current
    bool node_removal = false;                                // taint times / no-delete loaded
    PodRef* d_refs = nullptr;
    uint32_t* d_e_pair = nullptr;
    uint32_t *d_nrun_off = nullptr, *d_nrun_len = nullptr, *d_occ = nullptr, *d_rm_off = nullptr,
             *d_rm_list = nullptr;                             // d_occ: [2][n_entries] (pair, default)
    // host mirror of the placement: runs per node (capacity offsets, lengths), the pod at
    // each run position, each pod's node and run position (pod events keep them current)
    std::vector<uint32_t> h_run_off, h_run_len, h_pod_node;
    std::vector<int32_t> h_run_pod;
    std::vector<int64_t> h_pod_rpos;
    int64_t *d_taint_s = nullptr, *d_soft = nullptr, *d_hard = nullptr;
    uint8_t* d_no_delete = nullptr;
    RmRec* d_rm_out = nullptr;
    std::vector<uint32_t> h_rm_off;                           // [G + 1]
    RmRec* h_rm = nullptr;                                    // K7 results (pinned copy)
    uint8_t* h_istage = nullptr;                              // age-index build uploads (pinned)
    size_t istage_cap = 0;
    int64_t* h_words = nullptr;                               // esc_results' pod + node words (pinned)
    size_t words_cap = 0;
    // Small contexts (G <= HTOT_MAX_GROUPS): K4 writes every decided group's totals record
    // straight to pinned host memory with its decision (<= 104 KB over PCIe), so esc_results
    // copies nothing; tot_dec = the last enqueued step decided (the records are current).
    esc_group_totals* h_tot = nullptr;
    esc_group_totals* h_tot_dev = nullptr;
    bool tot_dec = false;
    std::vector<int64_t> h_soft, h_hard;                      // grace periods last uploaded
    bool rm_valid = false;                                    // esc_try_remove results current
    int64_t rm_nodes = -1;                                    // node count the reaping buffers are sized for
};

namespace esc {
const GroupIndex* ctx_group_index(const esc_ctx* ctx) { return &ctx->gi; }
esc_multi_state* ctx_multi(const esc_ctx* c) { return c->multi; }
void ctx_set_multi(esc_ctx* c, esc_multi_state* m) { c->multi = m; }
hipStream_t ctx_stream(const esc_ctx* c) { return c->stream; }
int ctx_device(const esc_ctx* c) { return c->device; }
}

namespace {

// A kb_write_pod / kb_write_free put into the host copy of the K blocks.
void put_kb(uint32_t* kb, int width, int64_t at, uint64_t v) {
    if (width == 8) reinterpret_cast<int64_t*>(kb)[at] = (int64_t)v;
    else if (width == 4) kb[at] = (uint32_t)v;
    else reinterpret_cast<uint16_t*>(kb)[at] = (uint16_t)v;
}

// Host threads for the load-time layout passes: ESC_HOST_THREADS, else OMP_NUM_THREADS (the
// GPU box sets 16, its CPU share per GPU), else min(16, hardware threads).
int host_threads() {
    int n = 0;
    for (const char* e : {"ESC_HOST_THREADS", "OMP_NUM_THREADS"})
        if (const char* v = std::getenv(e)) { n = std::atoi(v); if (n > 0) break; }
    if (n <= 0) n = std::min<int>(16, std::max(1u, std::thread::hardware_concurrency()));
    return std::max(1, std::min(n, 64));
}

// f(t, lo, hi) over T contiguous chunks of [0, n), one host thread each (in order for T = 1)
template <class F>
void par_chunks(int64_t n, int T, F&& f) {
    if (T <= 1 || n < 4096) {
        f(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { f(t, n * t / T, n * (t + 1) / T); });
    for (auto& x : th) x.join();
}

// Spare C slots (esc_load_pods with esc_set_spare): room per slot, slots per 64-pod tile.
constexpr int CS_SLOTS = 16, CS_XREG = 4, CS_XINIT = 2, CS_REC = CS_XREG + CS_XINIT + 1, CS_XP = 6;
static_assert(CS_SLOTS * CS_REC <= 128 && CS_SLOTS * CS_XP <= 128, "a spare C tile stays on K1's C path");
constexpr uint32_t CS_FLAGS = ESC_PF_DAEMONSET | ESC_PF_HAS_OVH | (uint32_t)CS_XREG << ESC_PF_XREG_SHIFT |
                              (uint32_t)CS_XINIT << ESC_PF_XINIT_SHIFT | (uint32_t)CS_XP << ESC_PF_XPAIR_SHIFT;

// K class of a pod: its record signature (at most 3 extra container
// records and 3 extra pairs; -1: the C section) | packed << 7: 1 when its values fit the
// packed block (kp_fits), 2 when they also fit the packed small block (kp8_fits, in a context
// with fewer than KP8_PAIR_NONE group pairs).  xc_cpu / xc_mem: the pod's own records (null
// when it has none).
int pod_class_id(uint32_t f, uint32_t cpu0, int64_t mem0, uint32_t pair0, const int64_t* xc_cpu,
                 const int64_t* xc_mem, uint32_t n_gp) {
    const uint32_t xr = pf_xreg(f), xi = pf_xinit(f), ov = (f & ESC_PF_HAS_OVH) ? 1u : 0u, np = pf_xpair(f);
    if (xr + xi + ov > 3 || np > 3) return -1;
    const int sig = (int)(((xr * 4 + xi) * 2 + ov) * 4 + np);
    if (!kp_fits(f, cpu0, mem0, pair0, xc_cpu, xc_mem)) return sig;
    return sig | (n_gp < KP8_PAIR_NONE && kp8_fits(cpu0, mem0) ? 2 : 1) * POD_SIG_IDS;
}

// A node's allocatable cpu fits K2's packed entry (NodeDev::e_pk).
bool entry_cpu_packs(int64_t cpu) { return cpu >= 0 && cpu <= (int64_t)0xFFFFFFFF; }

// K1 partial row stride: the pod slots (one per group pair + the default filter's)
// rounded up to whole K3 columns.
int64_t slot_stride(const esc_ctx* c) { return ((int64_t)c->gi.n_gp + 1 + FC_COL - 1) / FC_COL * FC_COL; }

// The exchange buffer (SUM across ranks, reduce-scattered to the owners): the pods' words
// in owner-major rows, [world][own_cap][PW_K].
int64_t xw_count(const esc_ctx* c) { return (int64_t)c->world * c->own_cap * PW_K; }
int64_t* own_xwords(const esc_ctx* c) { return c->d_pwords + (int64_t)c->rank * c->own_cap * PW_K; }
GroupList own_list(const esc_ctx* c) {
    return GroupList{c->own_seq ? nullptr : c->d_own, (int32_t)c->h_own.size(), c->own_first};
}

GroupDev group_dev(const esc_ctx* c) {
    GroupDev g;
    g.dry = c->d_dry;
    g.params = c->d_params;
    g.gpair = c->d_gpair;
    g.node_code = c->d_node_code;
    g.code_list = c->d_code_list;
    g.gslot = c->d_gslot;
    g.xs = c->world > 1 ? c->d_xs : nullptr;
    g.metrics = c->want_metrics ? c->d_metrics : nullptr;
    g.htot = c->h_tot_dev;
    g.n_gp = c->gi.n_gp;
    g.sp = slot_stride(c);
    g.G = c->gi.G;
    g.default_group = c->gi.default_group < 0 ? NONE : (uint32_t)c->gi.default_group;
    return g;
}

PodDev pod_dev(const esc_ctx* c, int replica) {
    const PodBuf& b = c->pods[replica];
    PodDev p;
    p.kb = b.kb;
    p.flags = b.flags; p.cpu0 = b.cpu0; p.mem0 = b.mem0; p.pair0 = b.pair0;
    p.xc_cpu = b.xc_cpu; p.xc_mem = b.xc_mem; p.xp = b.xp;
    p.xc_base = b.xc_base; p.xp_base = b.xp_base;
    p.cls = b.cls;
    p.seg = (c->k1_variant == 5 || c->k1_variant == 6 || c->k1_variant == 7 || c->k1_variant == 14) ? nullptr
                                                                                                    : c->d_k1seg;
    p.wg_cols = c->touch_on ? c->d_wg_cols : nullptr;
    p.wg_off = c->touch_on ? c->d_wg_off : nullptr;
    p.n_cls = c->n_cls;
    p.k_tiles = c->k_tiles;
    p.k_weight = c->k_weight;
    p.c_tiles = c->c_tiles;
    return p;
}

NodeDev node_dev(const esc_ctx* c) {
    NodeDev n;
    n.gnode = c->nodes.gnode;
    n.flags = c->nodes.flags; n.label0 = c->nodes.label0; n.cpu = c->nodes.cpu; n.mem = c->nodes.mem;
    n.created = c->nodes.created; n.xl = c->nodes.xl; n.xl_off = c->nodes.xl_off;
    n.trk_node = c->nodes.trk_node; n.trk_group = c->nodes.trk_group; n.trk_start = c->nodes.trk_start;
    n.n_trk = c->n_trk;
    n.lo = c->node_lo; n.hi = c->node_hi;
    n.e_flags = c->nodes.e_flags; n.e_cpu = c->nodes.e_cpu; n.e_mem = c->nodes.e_mem; n.e_node = c->nodes.e_node;
    n.e_pk = c->e_pk_ok ? c->nodes.e_pk : nullptr;
    n.piece_off = c->nodes.piece_off; n.piece_pair = c->nodes.piece_pair; n.pp_off = c->nodes.pp_off;
    n.n_pieces = c->n_pieces; n.pc_lo = c->pc_lo; n.pc_hi = c->pc_hi;
    n.span_off = c->nodes.span_off; n.span_e = c->nodes.span_e; n.n_spans = c->n_spans;
    n.q_lo = c->q_lo; n.q_hi = c->q_hi;
    return n;
}

void params_from(GroupParams& p, const esc_group_spec& s, const esc_group_state* st) {
    p.min_nodes = s.min_nodes; p.max_nodes = s.max_nodes;
    p.taint_upper = s.taint_upper_pct; p.taint_lower = s.taint_lower_pct; p.scale_up = s.scale_up_pct;
    p.slow_rate = s.slow_removal_rate; p.fast_rate = s.fast_removal_rate;
    p.dry = s.dry_mode ? 1 : 0;
    p.locked = st ? st->locked : 0;
    p.requested = st ? st->requested_nodes : 0;
    p.cached_cpu = st ? st->cached_cpu_m : 0;
    p.cached_mem = st ? st->cached_mem_b : 0;
}

void drop_graphs(esc_ctx* c) {
    for (auto& g : c->graphs)
        if (g) hipGraphExecDestroy(g);
    c->graphs.clear();
    for (auto& g : c->rgraphs)
        if (g) hipGraphExecDestroy(g);
    c->rgraphs.clear();
}

int32_t enqueue_step(esc_ctx* c, int r, bool decide, bool copy_out);

// The look-back bound of the next K5 launch (ordering or listing): LOOKBACK_SPINS, except
// for launches a measurement-library test set to give up at once (esc_debug_lookback_fail,
// tests/test_gpu_faults.py).
uint32_t lb_spins(int& fail_next) {
    if (fail_next > 0) {
        --fail_next;
        return 0;
    }
    return LOOKBACK_SPINS;
}
OrdFail ord_fail(esc_ctx* c) { return OrdFail{c->h_oerr_dev, lb_spins(c->lb_fail_order)}; }

// K4's selection target for a deciding launch (null out: off, or no ordering in the step to
// select from)
SelOut sel_out(const esc_ctx* c) {
    SelOut s{};
    if (c->sel_slack < 0 || !c->h_sel || !c->order_in_step || !c->d_ord || !c->d_seg || !c->d_g_tie) return s;
    s.ord = c->d_ord;
    s.seg = c->d_seg;
    s.tie = c->d_g_tie;
    s.out = c->h_sel_dev;
    s.cap_words = c->sel_words;
    s.slack = c->sel_slack;
    s.group_cap = c->sel_group_cap;
    return s;
}

void release_selections(esc_ctx* c) {
    if (c->h_sel) hipHostFree(c->h_sel);
    c->h_sel = c->h_sel_dev = nullptr;
    c->sel_words = 0;
}

// After a wait on the context's stream: a split ordering that gave up since the last check
// latches ord_failed (clearing the host word for the next one); true when it was new.
bool order_gave_up(esc_ctx* c) {
    if (!c->h_oerr || !*reinterpret_cast<volatile uint32_t*>(c->h_oerr)) return false;
    *reinterpret_cast<volatile uint32_t*>(c->h_oerr) = 0;
    c->ord_failed = true;
    return true;
}

// K5 per-decision ordering (classify + stable split of every group's age-ordered
// memberships) on stream st: the two-pass kernels and the packed small / mid-size groups.
hipError_t enqueue_order(esc_ctx* c, hipStream_t st) {
    const hipError_t e = launch_order(node_dev(c), c->d_chunks, c->n_chunks, c->d_gch_off, c->d_grp_off, c->d_g_memb,
                                      c->d_ostat, c->ord_parity, c->d_ord, c->d_seg, ord_fail(c), st);
    c->ord_parity ^= 1;
    c->ord_failed = false;
    if (e != hipSuccess) return e;
    return launch_order_packed(node_dev(c), c->d_pchunks, c->n_pchunks, c->n_psmall, c->d_grp_off, c->d_dry, c->d_g_memb,
                               c->d_ord, c->d_seg, st);
}

// Replays (capturing on first use) the per-replica graph of enqueue_step(r, decide, decide)
// on the context's stream: one launch instead of the step's kernels, events and waits.
// With the ordering in the step there is one graph per (replica, ordering parity): the
// split ordering alternates two status arrays (k_ord_split), and a graph holds its launch's.
int32_t replay_step(esc_ctx* c, std::vector<hipGraphExec_t>& gs, int r, bool decide) {
    const int nrep = (int)c->pods.size();
    if ((int)gs.size() != 2 * nrep) {
        for (auto& g : gs)
            if (g) hipGraphExecDestroy(g);
        gs.assign(2 * (size_t)nrep, nullptr);
    }
    const bool ord = c->order_in_step;
    const int k = 2 * r + (ord ? c->ord_parity : 0);
    if (!gs[k]) {
        hipGraph_t graph = nullptr;
        HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        const int32_t rc = enqueue_step(c, r, decide, decide);          // flips the parity (ord)
        hipError_t e = hipStreamEndCapture(c->stream, &graph);
        if (rc) { if (graph) hipGraphDestroy(graph); return rc; }
        if (e != hipSuccess) return fail_hip(e, "hipStreamEndCapture");
        e = hipGraphInstantiate(&gs[k], graph, nullptr, nullptr, 0);
        hipGraphDestroy(graph);
        if (e != hipSuccess) return fail_hip(e, "hipGraphInstantiate");
    } else if (ord) {
        c->ord_parity ^= 1;
        c->ord_failed = false;
    }
    HIP_TRY(hipGraphLaunch(gs[k], c->stream));
    return ESC_OK;
}

void release_work(esc_ctx* c) {
    dfree(c->d_k1seg); dfree(c->d_pod_part); dfree(c->d_wide_pod); dfree(c->d_k1_ticket); dfree(c->d_trk_acc);
    dfree(c->d_k1_trace);
    dfree(c->d_ttrace);
    c->ttrace_cap = 0;
    dfree(c->d_touch); dfree(c->d_wg_cols); dfree(c->d_wg_off); dfree(c->d_col_rows);
    c->touch_on = false;
    dfree(c->own_pwords); c->d_nwords = nullptr; dfree(c->d_dec); dfree(c->d_cdec); dfree(c->d_metrics);
    dfree(c->d_own); dfree(c->d_xs);
    c->d_pwords = nullptr;
    if (c->h_cdec) hipHostFree(c->h_cdec);
    c->h_cdec = nullptr;
    c->h_cdec_dev = nullptr;
    if (c->h_tot) hipHostFree(c->h_tot);
    c->h_tot = c->h_tot_dev = nullptr;
    c->tot_dec = false;
    c->work_ready = false;
    drop_graphs(c);
}

void release_placement(esc_ctx* c) {
    dfree(c->d_refs); dfree(c->d_e_pair); dfree(c->d_nrun_off); dfree(c->d_nrun_len); dfree(c->d_occ); dfree(c->d_rm_off);
    dfree(c->d_occ_local); dfree(c->d_ne_off); dfree(c->d_ne_pos);
    c->ne_dev_nodes = c->ne_dev_pos = -1;
    dfree(c->d_rm_list); dfree(c->d_taint_s); dfree(c->d_soft); dfree(c->d_hard); dfree(c->d_no_delete);
    dfree(c->d_rm_out);
    if (c->h_rm) { hipHostFree(c->h_rm); c->h_rm = nullptr; }
    c->h_soft.clear();
    c->h_hard.clear();
    c->placed = c->node_removal = c->rm_valid = false;
}

void release_sort(esc_ctx* c) {
    drop_graphs(c);                                     // captured steps hold the index's buffers
    for (int i = 0; i < 2; ++i) { dfree(c->d_mkeys[i]); dfree(c->d_mvals[i]); }
    c->mcap = 0;
    c->age_built = false;
    dfree(c->d_g_memb);
    dfree(c->d_ostat); dfree(c->d_ord);
    c->n_pchunks = 0;
    c->n_chunks = 0;
    c->n_gpad = 0;
    dfree(c->d_hist); dfree(c->d_tot);
    dfree(c->d_itab);
    c->itab_cap = 0;
    c->d_seg = nullptr; c->d_grp_off = c->d_gch_off = c->d_pstart = c->d_plen = nullptr;
    c->d_chunks = c->d_pchunks = nullptr; c->d_lstat = nullptr; c->d_total = c->d_ierr = c->d_g_tie = nullptr;
    c->n_memb = 0;
    c->sorted = false;
}

// The age index: every group membership of this rank's node range, in
// (group, creation time, snapshot index) order, with its flags — one LSD radix sort of
// (group << R | creation offset) keys (the offsets divided by the largest of 1e9 / 1e6 /
// 1e3 that divides them all — an exact order-preserving transform) over the memberships
// listed in snapshot order (stable: equal times keep index order), carrying (node | flags)
// as the value, so no pass gathers at random.  Built once per snapshot.
int32_t build_age_index(esc_ctx* c) {
    const GroupDev g = group_dev(c);
    const NodeDev n = node_dev(c);
    hipStream_t st = c->stream;
    const int64_t nl = c->node_hi - c->node_lo;
    if (c->age_built && c->age_n != nl) release_sort(c);   // the range grew (esc_nodes_add)
    const bool fresh = !c->age_built;
    // until this build succeeds the regions are not an ordering's input: orderings, steps with
    // the ordering inside and region patches are refused (ESC_E_STATE) or skipped
    c->age_ok = false;
    if (fresh) {
        c->age_n = nl;
        c->age_exact = false;
        c->h_gn.clear();
        if (nl) {                                    // creation-time range of the node range
            c->ts_min = *std::min_element(c->h_created.begin(), c->h_created.end());
            c->ts_max = *std::max_element(c->h_created.begin(), c->h_created.end());
        }
        uint64_t div = 1;
        for (uint64_t d : {1000000000ull, 1000000ull, 1000ull}) {
            bool ok = true;
            for (int64_t i = 0; i < nl && ok; ++i) ok = ((uint64_t)(c->h_created[i] - c->ts_min)) % d == 0;
            if (ok) { div = d; break; }
        }
        c->sort_div = div;
        c->sort_R = std::max(1, bit_width((uint64_t)(c->ts_max - c->ts_min) / div));
        if (c->sort_R + bit_width((uint64_t)std::max<int32_t>(g.G - 1, 1)) > 64) return ESC_E_LIMIT;
        if (c->node_hi >= ((int64_t)1 << 28)) return ESC_E_LIMIT;   // node | flags << 28 sort values
        HIP_TRY(dalloc(&c->d_tot, 256));
        c->age_built = true;
    }
    // Every group's membership count is the live entry count of its pair (the host's), so
    // the total and the sorted groups' starts need no round trip; the device's own counts
    // are compared with them on a fresh build (and on every build with ESC_CHECK_INDEX=1).
    std::vector<int64_t> starts((size_t)g.G + 1, 0);
    for (int32_t q = 0; q < g.G; ++q) {
        const uint32_t gp = c->gi.gpair[q];
        starts[q + 1] = starts[q] + ((gp >= c->q_lo && gp < c->q_hi) ? c->pair_live[gp] : 0);
    }
    if (starts[g.G] > (int64_t)0xFFFFFFFF) return ESC_E_LIMIT;
    const uint32_t total = (uint32_t)starts[g.G];
    static const bool check_env = std::getenv("ESC_CHECK_INDEX") && std::atoi(std::getenv("ESC_CHECK_INDEX")) != 0;
    const bool check = fresh || check_env;
    c->n_memb = total;
    if ((int64_t)total > c->mcap || !c->d_hist) {
        for (int i = 0; i < 2; ++i) {
            dfree(c->d_mkeys[i]); dfree(c->d_mvals[i]);
            HIP_TRY(dalloc(&c->d_mkeys[i], std::max<int64_t>(total, 1)));
            HIP_TRY(dalloc(&c->d_mvals[i], std::max<int64_t>(total, 1)));
        }
        c->mcap = std::max<int64_t>(total, 1);
        dfree(c->d_hist);
        HIP_TRY(dalloc(&c->d_hist, std::max(sort_hist_words(c->mcap), sort_hist_words(1) * 4)));
    }
    // every group's region: its memberships (oldest first), then padding to whole quads plus
    // the spare slots node additions take (esc_set_spare); the per-decision output uses the
    // same positions (grp_off = region starts)
    // Every group's length and capacity come from the host's live entry counts, identically on
    // every rank (node additions check the capacity of every group they touch, owned or not,
    // so that all ranks accept or refuse a batch alike); only the groups of the
    // pairs this rank owns get a device region.
    std::vector<uint32_t> gch_off(g.G + 1), pstart(g.G + 1, 0), plen(std::max<int32_t>(g.G, 1), 0),
        pcap(std::max<int32_t>(g.G, 1), 0);
    for (int32_t q = 0; q < g.G; ++q) {
        const uint32_t gp = c->gi.gpair[q];
        const bool own = gp >= c->q_lo && gp < c->q_hi;
        const int64_t len = c->pair_live[gp];
        const int64_t spare = c->spare_frac > 0 ? (int64_t)std::ceil((double)len * c->spare_frac) + 4 : 0;
        const int64_t cap = (len + spare + 3) & ~(int64_t)3;
        if (cap >= (int64_t)0xFFFFFFFF) return ESC_E_LIMIT;
        plen[q] = (uint32_t)len;
        pcap[q] = (uint32_t)cap;
        const int64_t reg = own ? cap : 0;
        if ((int64_t)pstart[q] + reg >= (int64_t)0xFFFFFFFF) return ESC_E_LIMIT;
        pstart[q + 1] = pstart[q] + (uint32_t)reg;
    }
    // chunks: a group whose region exceeds ORD_CHUNK is split (two-pass kernels, chunk
    // prefix across the group); smaller groups are packed whole, several per chunk,
    // and ordered in one pass (k_ord_packed)
    std::vector<OrdChunk> chunks, pchunks, pbig;
    // a packed chunk covers the groups [g0, g1] (the empty ones between included: the kernel
    // finds a quad's group in that table, <= ORD_GCAP of them)
    uint32_t pk_lo = 0, pk_hi = 0, qk_lo = 0, qk_hi = 0, pk_g0 = 0, pk_g1 = 0, qk_g0 = 0, qk_g1 = 0;
    auto flush_small = [&]() {
        if (pk_hi > pk_lo) pchunks.push_back({pk_lo, pk_hi, pk_g0, pk_g1 - pk_g0 + 1});
        pk_lo = pk_hi;
    };
    auto flush_mid = [&]() {
        if (qk_hi > qk_lo) pbig.push_back({qk_lo, qk_hi, qk_g0, qk_g1 - qk_g0 + 1});
        qk_lo = qk_hi;
    };
    for (int32_t q = 0; q < g.G; ++q) {
        const uint32_t reg = pstart[q + 1] - pstart[q];
        gch_off[q] = (uint32_t)chunks.size();
        if (reg == 0) continue;
        if (reg > (uint32_t)ORD_CHUNK) {
            flush_small();
            flush_mid();
            pk_lo = pk_hi = qk_lo = qk_hi = pstart[q + 1];
            for (int64_t a = 0; a < reg; a += ORD_CHUNK)
                chunks.push_back({pstart[q] + (uint32_t)a, pstart[q] + (uint32_t)std::min<int64_t>(reg, a + ORD_CHUNK),
                                  (uint32_t)q, c->params[q].dry ? ORD_CHUNK_DRY : 0u});
            continue;
        }
        if (reg > (uint32_t)ORD_PCHUNK) {          // mid-size: packed up to ORD_CHUNK
            flush_small();
            if (qk_hi - qk_lo + reg > (uint32_t)ORD_CHUNK || qk_hi != pstart[q] ||
                (qk_hi > qk_lo && (uint32_t)q - qk_g0 + 1 > ORD_GCAP))
                flush_mid();
            if (qk_hi == qk_lo) { qk_lo = qk_hi = pstart[q]; qk_g0 = (uint32_t)q; }
            qk_hi = pstart[q + 1];
            qk_g1 = (uint32_t)q;
            pk_lo = pk_hi = pstart[q + 1];
            continue;
        }
        flush_mid();                               // a pending mid-size chunk ends here (it was
                                                   // dropped before round 6: test_packed_chunk_mix)
        if (pk_hi - pk_lo + reg > (uint32_t)ORD_PCHUNK || pk_hi != pstart[q] ||
            (pk_hi > pk_lo && (uint32_t)q - pk_g0 + 1 > ORD_GCAP))
            flush_small();
        if (pk_hi == pk_lo) { pk_lo = pk_hi = pstart[q]; pk_g0 = (uint32_t)q; }
        pk_hi = pstart[q + 1];
        pk_g1 = (uint32_t)q;
        qk_lo = qk_hi = pstart[q + 1];
    }
    flush_small();
    flush_mid();
    c->n_psmall = (int64_t)pchunks.size();
    pchunks.insert(pchunks.end(), pbig.begin(), pbig.end());
    gch_off[g.G] = (uint32_t)chunks.size();
    const int64_t npad = pstart[g.G];
    if (fresh || npad != c->n_gpad) {
        drop_graphs(c);                                 // captured steps hold the old regions
        dfree(c->d_g_memb); dfree(c->d_ord);
        HIP_TRY(dalloc(&c->d_g_memb, npad)); HIP_TRY(dalloc(&c->d_ord, npad));
    }
    c->n_gpad = npad;
    // no clearing: the sort's last pass fills every group's [start, start + len), k_region_pad the
    // rest of its region
    if (fresh || (int64_t)chunks.size() != c->n_chunks) {
        dfree(c->d_ostat);
        HIP_TRY(dalloc(&c->d_ostat, 2 * chunks.size() + 1));
        HIP_TRY(hipMemsetAsync(c->d_ostat, 0, (2 * chunks.size() + 1) * 8, st));
        c->ord_failed = false;
        c->ord_parity = 0;
        drop_graphs(c);                                 // captured steps hold the old status words
    }
    c->n_chunks = (int64_t)chunks.size();
    c->n_pchunks = (int64_t)pchunks.size();
    // The host-made tables, the listing's status words (zero), the error word and listed total
    // (zero) and the tie flags (coarse keys: zero, k_age_fix sets them; exact keys: every group)
    // are laid out in the pinned staging area exactly as in d_itab and go up as ONE copy per
    // attempt (round 5: seven queued copies and three fills, ~10 stream operations of a few µs
    // each); the build waits once, at its end, for the error word and total read back.
    const int gbits = bit_width((uint64_t)std::max<int32_t>(g.G - 1, 1));
    const size_t Gw = (size_t)std::max<int32_t>(g.G, 1);
    struct Part { void** view; const void* src; size_t src_bytes; size_t bytes; size_t at; };   // src: copied, else zero
    void* v_seg = nullptr; void* v_grp = nullptr; void* v_gch = nullptr; void* v_ps = nullptr; void* v_pl = nullptr;
    void* v_ch = nullptr; void* v_pch = nullptr; void* v_st = nullptr; void* v_err = nullptr; void* v_tie = nullptr;
    // d_seg: the G + 1 sorted starts the sort's last pass reads, room for the 4G + 1 segment
    // bounds k_region_pad and the orderings write over them
    Part parts[] = {{&v_seg, starts.data(), starts.size() * 8, (4 * (size_t)g.G + 1) * 8, 0},
                    {&v_grp, pstart.data(), pstart.size() * 4, pstart.size() * 4, 0},
                    {&v_gch, gch_off.data(), gch_off.size() * 4, gch_off.size() * 4, 0},
                    {&v_ps, pstart.data(), pstart.size() * 4, pstart.size() * 4, 0},
                    {&v_pl, plen.data(), plen.size() * 4, plen.size() * 4, 0},
                    {&v_ch, chunks.data(), chunks.size() * sizeof(OrdChunk), std::max<size_t>(chunks.size(), 1) * sizeof(OrdChunk), 0},
                    {&v_pch, pchunks.data(), pchunks.size() * sizeof(OrdChunk),
                     std::max<size_t>(pchunks.size(), 1) * sizeof(OrdChunk), 0},
                    {&v_st, nullptr, 0, memb_status_words(nl) * 8, 0},
                    {&v_err, nullptr, 0, 8, 0},                          // error word, listed total
                    {&v_tie, nullptr, 0, Gw * 4, 0}};
    size_t bytes = 0;
    for (Part& q : parts) { q.at = bytes; bytes += (q.bytes + 255) & ~(size_t)255; }
    const size_t rb_at = bytes;                              // the read-back words (error, total)
    const size_t stage = bytes + 256;
    if (bytes > c->itab_cap) {
        drop_graphs(c);                                      // captured steps hold the old tables
        HIP_TRY(hipStreamSynchronize(st));
        dfree(c->d_itab);
        c->itab_cap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->d_itab), bytes));
        c->itab_cap = bytes;
    }
    if (stage > c->istage_cap) {
        HIP_TRY(hipStreamSynchronize(st));                  // the previous build's copies are done
        if (c->h_istage) hipHostFree(c->h_istage);
        c->h_istage = nullptr;
        c->istage_cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_istage), stage));
        c->istage_cap = stage;
    }
    for (Part& q : parts) *q.view = c->d_itab + q.at;
    int64_t* const new_seg = static_cast<int64_t*>(v_seg);
    if (new_seg != c->d_seg || static_cast<OrdChunk*>(v_pch) != c->d_pchunks || static_cast<OrdChunk*>(v_ch) != c->d_chunks ||
        static_cast<uint32_t*>(v_tie) != c->d_g_tie)
        drop_graphs(c);                                      // the layout moved: captured steps hold the old views
    c->d_seg = new_seg;
    c->d_grp_off = static_cast<uint32_t*>(v_grp);
    c->d_gch_off = static_cast<uint32_t*>(v_gch);
    c->d_pstart = static_cast<uint32_t*>(v_ps);
    c->d_plen = static_cast<uint32_t*>(v_pl);
    c->d_chunks = static_cast<OrdChunk*>(v_ch);
    c->d_pchunks = static_cast<OrdChunk*>(v_pch);
    c->d_lstat = static_cast<uint64_t*>(v_st);
    c->d_ierr = static_cast<uint32_t*>(v_err);
    c->d_total = c->d_ierr + 1;
    c->d_g_tie = static_cast<uint32_t*>(v_tie);
    auto stage_tables = [&](bool coarse) {
        for (Part& q : parts) {
            uint8_t* h = c->h_istage + q.at;
            if (q.view == &v_tie && !coarse) {
                for (size_t k = 0; k < Gw; ++k) reinterpret_cast<uint32_t*>(h)[k] = 1u;
                continue;
            }
            if (q.src_bytes) std::memcpy(h, q.src, q.src_bytes);
            if (q.bytes > q.src_bytes) std::memset(h + q.src_bytes, 0, q.bytes - q.src_bytes);
        }
    };
    volatile uint32_t* h_err = reinterpret_cast<volatile uint32_t*>(c->h_istage + rb_at);
    // the listing and the sort; its last pass writes the regions at the host's sorted starts.
    // Keys: 32-bit coarse keys — the group in the top gbits, the creation offset's top
    // (32 - gbits) bits — when the groups leave at least 16 bits of time: four 8-bit LSD
    // passes over 8-B (key, value) pairs instead of six over 12-B ones; if offset bits were
    // dropped, k_age_fix orders the runs of equal coarse keys by the exact time, and a run
    // too long for it sends the build back to the exact 64-bit keys.
    for (int attempt = 0;; ++attempt) {
        const bool coarse = !c->age_exact && gbits <= 16;
        const int cshift = coarse ? std::max(0, c->sort_R - (32 - gbits)) : -1;
        if (attempt) HIP_TRY(hipStreamSynchronize(st));      // (the staging is rewritten)
        stage_tables(coarse);
        HIP_TRY(hipMemcpyAsync(c->d_itab, c->h_istage, bytes, hipMemcpyHostToDevice, st));
        RegionSink sink{c->d_seg, c->d_pstart, c->d_plen, c->d_g_memb, c->d_ierr,
                        g.G, coarse ? 32 - gbits : c->sort_R, coarse ? (cshift > 0 ? 1 : 2) : 0, lb_spins(c->lb_fail_list),
                        c->d_g_tie};
        HIP_TRY(launch_age_sort(n, g, c->d_lstat, c->d_total, c->n_memb, c->mcap, c->ts_min, c->sort_div, c->sort_R,
                                gbits, cshift, c->d_mkeys, c->d_mvals, c->d_hist, c->d_tot, sink, st));
        HIP_TRY(launch_region_pad(c->d_pstart, c->d_plen, g.G, c->d_g_memb, c->d_seg, st));
        // the error word (the listing's bounded look-back, region counts, the run fix-up) and
        // the listed total, read at the build's one wait
        h_err[0] = 0;
        h_err[1] = 0;
        HIP_TRY(hipMemcpyAsync(c->h_istage + rb_at, c->d_ierr, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        const uint32_t err = h_err[0];
        if (check && nl && h_err[1] != total) return fail_hip(hipErrorUnknown, "age index: membership total");
        if (err & 1u) return fail_hip(hipErrorUnknown, "age index: membership count");
        if (!(err & 2u)) break;
        if (attempt) return fail_hip(hipErrorUnknown, "age index: exact rebuild");
        c->age_exact = true;                        // a long run of equal coarse keys: exact keys
    }
    c->h_pstart.swap(pstart);
    c->h_plen.swap(plen);
    c->h_pcap.swap(pcap);
    c->h_gch_off.swap(gch_off);
    c->sorted = false;
    c->age_ok = true;
    return ESC_OK;
}

// K1 work plan: every workgroup's K tiles as at most K1_SEGS runs of one
// class, balanced in work weight (16-B loads), with at most two class boundaries per
// workgroup.  A class run restarts the workgroup's load pipeline (its first tiles' full
// latency, every wave at once), so the old weight-range shares, which let a workgroup
// cross every small class in its range (up to 4 runs at 12.5M pods), set the launch's
// tail.  Classes lighter than one share ("small") are each placed whole into one
// workgroup, beside a chunk of a large class that does not end there; large classes are
// cut at tile boundaries following the cumulative weight target, so rounding never drifts.
//
// `share` (calibrated, esc_k1_calibrate): workgroup k's fraction of the weight; empty = equal.
std::vector<int64_t> plan_k1(const std::vector<PodClass>& cls, int64_t W, int64_t nblk,
                             const std::vector<double>& share);

// Largest pod count one workgroup of `plan` sees (K runs + its C tiles).
int64_t plan_worst(const esc_ctx* c, const std::vector<int64_t>& plan, int64_t nblk) {
    int64_t worst = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t pods = ((c->c_tiles + nblk - 1) / nblk) * CTILE;
        for (int k = 0; k < K1_SEGS; ++k) {
            const int64_t* e = &plan[((size_t)b * K1_SEGS + k) * 2];
            if (e[1]) pods += (e[1] - (e[0] & ((1ll << 48) - 1))) * TILE;
        }
        worst = std::max(worst, pods);
    }
    return worst;
}

std::vector<int64_t> plan_k1(const std::vector<PodClass>& cls, int64_t W, int64_t nblk,
                             const std::vector<double>& share) {
    std::vector<int64_t> seg((size_t)nblk * K1_SEGS * 2, 0);
    if (W <= 0 || nblk <= 0) return seg;
    std::vector<int64_t> cut(nblk + 1, 0);                // cumulative weight targets
    const bool eq = (int64_t)share.size() != nblk;
    double acc = 0;
    for (int64_t k = 0; k < nblk; ++k) {
        acc += eq ? 1.0 / (double)nblk : share[k];
        cut[k + 1] = eq ? (int64_t)((__int128)W * (k + 1) / nblk) : (int64_t)std::llround(acc * (double)W);
    }
    cut[nblk] = W;
    std::vector<int> big, small;
    for (int i = 0; i < (int)cls.size(); ++i) {
        const int64_t w = (cls[i].t1 - cls[i].t0) * (int64_t)cls[i].wt;
        if (w == 0) continue;
        (w * nblk < W ? small : big).push_back(i);
    }
    std::sort(small.begin(), small.end(), [&](int a, int b) {
        return (cls[a].t1 - cls[a].t0) * cls[a].wt > (cls[b].t1 - cls[b].t0) * cls[b].wt;
    });
    size_t bi = 0, si = 0;
    int64_t toff = 0, cum = 0;
    const int64_t n_small = (int64_t)small.size();
    for (int64_t k = 0; k < nblk; ++k) {
        int ns = 0;
        auto add = [&](int ci, int64_t a, int64_t b) {
            int64_t* e = &seg[((size_t)k * K1_SEGS + ns) * 2];
            e[0] = a | ((int64_t)ci << 48);
            e[1] = b;
            ++ns;
        };
        const int64_t end = cut[k + 1];
        // spread the small classes over the grid, one per workgroup, where the large stream
        // has no boundary inside this workgroup
        if (si < small.size() && k >= (int64_t)si * nblk / std::max<int64_t>(n_small, 1)) {
            const PodClass& q = cls[small[si]];
            const int64_t wq = (q.t1 - q.t0) * q.wt;
            bool fits = bi >= big.size();
            if (!fits) {
                const PodClass& c = cls[big[bi]];
                fits = (c.t1 - c.t0 - toff) * (int64_t)c.wt >= end - cum - wq;
            }
            if (fits || k + 1 == nblk || nblk - k <= n_small - (int64_t)si) {
                add(small[si], q.t0, q.t1);
                cum += wq;
                ++si;
            }
        }
        while (bi < big.size() && (cum < end || k + 1 == nblk) && ns < K1_SEGS) {
            const PodClass& c = cls[big[bi]];
            const int64_t rem = c.t1 - c.t0 - toff;
            int64_t take = k + 1 == nblk ? rem : std::min(rem, (end - cum + c.wt / 2) / (int64_t)c.wt);
            if (take <= 0) break;
            add(big[bi], c.t0 + toff, c.t0 + toff + take);
            toff += take;
            cum += take * (int64_t)c.wt;
            if (toff == c.t1 - c.t0) { ++bi; toff = 0; }
        }
        while (k + 1 == nblk && si < small.size() && ns < K1_SEGS) {   // leftovers (never in practice)
            const PodClass& q = cls[small[si++]];
            add((int)(&q - cls.data()), q.t0, q.t1);
        }
    }
    // a grid smaller than the class count can leave tiles unplanned: no plan then (K1 falls
    // back to the weight-range shares)
    if (bi < big.size() || si < small.size()) seg.clear();
    return seg;
}

// The group pairs [lo, hi) rank `rank` of `world` owns: pair q (weight =
// its node entries + OWN_PAD, for the per-pair work that does not scale with entries) goes
// to rank floor(S_q * world / W), S_q the weight of the pairs before q and W the total —
// contiguous ranges in pair order, balanced by weight, computed from the whole table, so
// every rank derives the same split (escalator_amd/layout.py owner_ranges restates it).
constexpr int64_t OWN_PAD = 64;
void owned_pairs(const std::vector<int64_t>& cnt, int32_t world, int32_t rank, uint32_t& lo, uint32_t& hi) {
    const uint32_t n = (uint32_t)cnt.size();
    lo = 0;
    hi = n;
    if (world <= 1) return;
    __int128 W = 0;
    for (int64_t x : cnt) W += x + OWN_PAD;
    __int128 S = 0;
    lo = hi = n;
    bool have_lo = false;
    for (uint32_t q = 0; q < n; ++q) {
        const int64_t r = (int64_t)(S * world / W);
        if (!have_lo && r >= rank) { lo = q; have_lo = true; }
        if (r >= (int64_t)rank + 1) { hi = q; break; }
        S += cnt[q] + OWN_PAD;
    }
    if (!have_lo) lo = hi;
}

// Live node entries per group pair of a packed node table (the weights of owned_pairs).
std::vector<int64_t> pair_counts(const esc_ctx* c, const esc_node_soa* s) {
    const uint32_t n_gp = c->gi.n_gp;
    std::vector<int64_t> cnt(n_gp, 0);
    int64_t x = 0;
    for (int64_t i = 0; i < s->n_nodes; ++i) {
        if (s->label0[i] < n_gp) ++cnt[s->label0[i]];
        const uint32_t nx = nf_xlbl(s->flags[i]);
        for (uint32_t k = 0; k < nx; ++k)
            if (s->xl_pair[x + k] < n_gp) ++cnt[s->xl_pair[x + k]];
        x += nx;
    }
    return cnt;
}

// Pod accumulator slots: one per group pair + one for the default filter.
int64_t pod_slots(const esc_ctx* c) { return (int64_t)c->gi.n_gp + 1; }

// Compact K1 flush lists from the touch bitmap: per column its entries (one per workgroup
// touching it, in workgroup order), per workgroup its {column, entry} list (fixed stride of
// n_col entries) and length.
int32_t touch_upload(esc_ctx* c) {
    const int64_t nblk = c->nblk, tw = c->touch_tw, n_col = slot_stride(c) / FC_COL;
    std::vector<uint32_t> col_rows(n_col + 1, 0), wg_cnt(nblk, 0);
    std::vector<uint2> cols((size_t)nblk * n_col, make_uint2(0xFFFFFFFFu, 0u));
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t w = 0; w < tw; ++w)
            for (uint32_t x = c->h_touch[b * tw + w]; x; x &= x - 1) {
                const int64_t col = w * 32 + __builtin_ctz(x);
                if (col < n_col) ++col_rows[col + 1];
            }
    for (int64_t k = 0; k < n_col; ++k) col_rows[k + 1] += col_rows[k];
    std::vector<uint32_t> next(col_rows.begin(), col_rows.end() - 1);
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t w = 0; w < tw; ++w)
            for (uint32_t x = c->h_touch[b * tw + w]; x; x &= x - 1) {
                const int64_t col = w * 32 + __builtin_ctz(x);
                if (col < n_col) cols[b * n_col + wg_cnt[b]++] = make_uint2((uint32_t)col, next[col]++);
            }
    HIP_TRY(hipMemcpy(c->d_col_rows, col_rows.data(), col_rows.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_wg_off, wg_cnt.data(), wg_cnt.size() * 4, hipMemcpyHostToDevice));
    if (!cols.empty()) HIP_TRY(hipMemcpy(c->d_wg_cols, cols.data(), cols.size() * sizeof(uint2), hipMemcpyHostToDevice));
    return ESC_OK;
}

// (Re)computes the touched columns of the current K1 plan (after ensure_work and every plan
// change of esc_k1_calibrate): k_touch on the device, the lists on the host.  Off (every
// row flushed whole) without a static plan (dynamic shares) or with ESC_K1_FULL_FLUSH.
int32_t touch_refresh(esc_ctx* c, const std::vector<int64_t>& plan) {
    const PodDev p0 = pod_dev(c, 0);
    const bool on = !plan.empty() && p0.seg && !c->full_flush && c->nblk > 0 && !c->pods.empty();
    if (on != c->touch_on) drop_graphs(c);             // the captured steps hold the flush mode
    c->touch_on = false;
    if (!on) return ESC_OK;
    c->h_tile_wg.clear();
    for (int64_t b = 0; b < c->nblk; ++b)
        for (int k = 0; k < K1_SEGS; ++k) {
            const int64_t* e = &plan[((size_t)b * K1_SEGS + k) * 2];
            if (e[1] == 0) break;
            c->h_tile_wg.push_back({e[0] & ((1ll << 48) - 1), e[1], b});
        }
    std::sort(c->h_tile_wg.begin(), c->h_tile_wg.end());
    c->h_touch.assign((size_t)c->nblk * c->touch_tw, 0);
    HIP_TRY(launch_touch(p0, group_dev(c), c->nblk, c->touch_tw, c->d_touch, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_touch.data(), c->d_touch, c->h_touch.size() * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (int32_t rc = touch_upload(c)) return rc;
    c->touch_on = true;
    return ESC_OK;
}

// Marks the columns a pod written into K slot q of class ci adds to (esc_pods_upsert);
// true when its workgroup did not touch one of them yet (the lists need an upload).
bool touch_mark(esc_ctx* c, int32_t ci, int64_t q, uint32_t f, uint32_t pair0, const uint32_t* xp) {
    if (!c->touch_on || (f & ESC_PF_DAEMONSET)) return false;
    const int64_t t = c->h_cls[ci].t0 + q / TILE;
    auto it = std::upper_bound(c->h_tile_wg.begin(), c->h_tile_wg.end(), std::array<int64_t, 3>{t, INT64_MAX, INT64_MAX});
    if (it == c->h_tile_wg.begin() || t >= (it - 1)->at(1)) return false;   // a tile no workgroup streams (none)
    uint32_t* row = c->h_touch.data() + (size_t)(it - 1)->at(2) * c->touch_tw;
    bool grew = false;
    auto mark = [&](uint32_t slot) {
        const uint32_t col = slot / FC_COL, bit = 1u << (col & 31);
        if (!(row[col >> 5] & bit)) { row[col >> 5] |= bit; grew = true; }
    };
    const uint32_t n_gp = c->gi.n_gp;
    if (pair0 < n_gp) mark(pair0);
    for (uint32_t k = 0; k < pf_xpair(f); ++k)
        if (xp[k] < n_gp) mark(xp[k]);
    return grew;
}

// The same for a pod written into C slot d (K1 and k_touch give workgroup b the C tiles
// [b * per, (b + 1) * per), per = ceil(c_tiles / nblk)).
bool touch_mark_c(esc_ctx* c, int64_t d, uint32_t f, uint32_t pair0, const uint32_t* xp) {
    if (!c->touch_on || (f & ESC_PF_DAEMONSET) || c->nblk <= 0) return false;
    const int64_t per = (c->c_tiles + c->nblk - 1) / c->nblk, b = (d / CTILE) / std::max<int64_t>(per, 1);
    uint32_t* row = c->h_touch.data() + (size_t)b * c->touch_tw;
    bool grew = false;
    auto mark = [&](uint32_t slot) {
        const uint32_t col = slot / FC_COL, bit = 1u << (col & 31);
        if (!(row[col >> 5] & bit)) { row[col >> 5] |= bit; grew = true; }
    };
    const uint32_t n_gp = c->gi.n_gp;
    if (pair0 < n_gp) mark(pair0);
    for (uint32_t k = 0; k < pf_xpair(f); ++k)
        if (xp[k] < n_gp) mark(xp[k]);
    return grew;
}

// The rank owning group g's node side: the one whose pair range holds the group's pair
// (q_bounds from esc_load_nodes).
int32_t group_owner_rank(const esc_ctx* c, int32_t g) {
    if (c->world <= 1 || c->q_bounds.size() < 2) return 0;
    const uint32_t q = c->gi.gpair[(size_t)g];
    return (int32_t)(std::upper_bound(c->q_bounds.begin(), c->q_bounds.end() - 1, q) - c->q_bounds.begin()) - 1;
}

constexpr uint32_t STALE_PODS = 1, STALE_NODES = 2;

// The apply phase of an event batch (its checks passed): on failure the context is marked
// stale (esc_ctx::stale) until the matching reload.
template <class F>
int32_t guarded(esc_ctx* c, uint32_t bit, F&& apply) {
    const uint32_t was = c->stale;
    const int32_t rc = apply();
    c->stale = rc == ESC_OK ? was : (was | bit);
    return rc;
}

// Grid geometry for the current snapshot.
int32_t ensure_work(esc_ctx* c) {
    if (c->work_ready) return ESC_OK;
    const int32_t G = c->gi.G;
    const int64_t S = pod_slots(c);
    const int gw = (int)std::min<int64_t>(S, POD_WINDOW_MAX);
    const int lds = (gw + FC_COL - 1) / FC_COL * FC_COL * 16;   // K1's two LDS halves, whole columns each
    const int max_blocks = c->k1_variant == 2 ? 2 : 4;   // 2048 threads per CU
    const int per_cu = std::max(1, std::min(max_blocks, LDS_BYTES / std::max(lds, 1)));
    int64_t nblk = c->cu_count * per_cu;
    // every workgroup takes 1/nblk of the K tiles' weight + ceil(c_tiles/nblk) C tiles;
    // keep that within PODS_PER_BLOCK_MAX (exactness of the packed LDS partials)
    int64_t cap = 0;
    auto block_pods = [&](int64_t b) {
        // a weight share holds at most share / (lightest tile weight) + one partial tile
        // per class; with dynamic shares a workgroup takes up to K1_CHUNK_CAP chunks of
        // 1 / (b * K1_CHUNKS) each
        const int64_t nch = b * K1_CHUNKS;
        return cap * ((c->k_weight + nch - 1) / nch / K_TILE_WEIGHT_MIN + c->n_cls + 1) * TILE +
               ((c->c_tiles + b - 1) / b) * CTILE;
    };
    // the static share (cap K1_CHUNKS: one share) sets the grid
    cap = K1_CHUNKS;
    while (block_pods(nblk) > PODS_PER_BLOCK_MAX) nblk *= 2;
    c->k1_cap = 0;
    nblk = std::min<int64_t>(nblk, std::max(c->k_tiles, c->c_tiles));
    std::vector<int64_t> plan;
    for (;;) {            // the plan's own per-workgroup pod counts must keep the LDS words exact
        if ((int64_t)c->k1_share.size() != nblk) c->k1_share.clear();
        plan = plan_k1(c->h_cls, c->k_weight, std::max<int64_t>(nblk, 1), c->k1_share);
        if (plan.empty()) break;
        if (plan_worst(c, plan, nblk) <= PODS_PER_BLOCK_MAX || nblk >= std::max(c->k_tiles, c->c_tiles)) break;
        nblk *= 2;
    }
    c->nblk = (int)nblk;
    if (!plan.empty()) {
        HIP_TRY(dalloc(&c->d_k1seg, plan.size()));
        HIP_TRY(hipMemcpy(c->d_k1seg, plan.data(), plan.size() * 8, hipMemcpyHostToDevice));
    }
    HIP_TRY(dalloc(&c->d_k1_trace, (size_t)std::max<int64_t>(nblk, 1) * 8));
    HIP_TRY(hipMemset(c->d_k1_trace, 0, (size_t)std::max<int64_t>(nblk, 1) * 64));
    const int64_t SP = slot_stride(c), n_col = SP / FC_COL;
    HIP_TRY(dalloc(&c->d_pod_part, (size_t)std::max<int64_t>(nblk, 1) * 2 * SP));
    HIP_TRY(dalloc(&c->d_wide_pod, (size_t)S * WP_K));
    HIP_TRY(dalloc(&c->d_k1_ticket, 2));
    HIP_TRY(hipMemset(c->d_k1_ticket, 0, 2 * sizeof(uint32_t)));
    HIP_TRY(hipMemset(c->d_wide_pod, 0, (size_t)S * WP_K * sizeof(int64_t)));
    HIP_TRY(dalloc(&c->d_trk_acc, (size_t)G * TA_K));
    HIP_TRY(hipMemset(c->d_trk_acc, 0, (size_t)G * TA_K * sizeof(int64_t)));
    {   // owner-major exchange rows: every rank derives the same split
        std::vector<std::vector<uint32_t>> lists((size_t)c->world);
        for (int32_t g = 0; g < G; ++g) lists[(size_t)group_owner_rank(c, g)].push_back((uint32_t)g);
        size_t cap = 1;
        for (const auto& l : lists) cap = std::max(cap, l.size());
        c->own_cap = (int32_t)cap;
        c->h_xs.assign((size_t)G, 0);
        for (int32_t r = 0; r < c->world; ++r)
            for (size_t i = 0; i < lists[(size_t)r].size(); ++i) c->h_xs[lists[(size_t)r][i]] = (uint32_t)(r * cap + i);
        c->h_own = lists[(size_t)c->rank];
        c->own_first = c->h_own.empty() ? 0 : (int32_t)c->h_own[0];
        c->own_seq = true;
        for (size_t i = 0; i < c->h_own.size(); ++i) c->own_seq &= c->h_own[i] == (uint32_t)c->own_first + i;
        HIP_TRY(dalloc(&c->d_xs, (size_t)G));
        HIP_TRY(dalloc(&c->d_own, std::max<size_t>(c->h_own.size(), 1)));
        HIP_TRY(hipMemcpy(c->d_xs, c->h_xs.data(), (size_t)G * 4, hipMemcpyHostToDevice));
        if (!c->h_own.empty()) HIP_TRY(hipMemcpy(c->d_own, c->h_own.data(), c->h_own.size() * 4, hipMemcpyHostToDevice));
    }
    // the pod words, then (at a 256-B boundary) the node words: esc_results reads both with
    // one copy when they are adjacent
    const size_t pw_span = ((size_t)xw_count(c) + 31) & ~(size_t)31;
    HIP_TRY(dalloc(&c->own_pwords, pw_span + (size_t)G * NW_K));
    HIP_TRY(hipMemset(c->own_pwords, 0, (pw_span + (size_t)G * NW_K) * 8));
    c->d_nwords = c->own_pwords + pw_span;
    c->d_pwords = c->bound_pwords ? c->bound_pwords : c->own_pwords;
    HIP_TRY(dalloc(&c->d_dec, (size_t)G));
    HIP_TRY(dalloc(&c->d_metrics, (size_t)G));
    HIP_TRY(hipMemset(c->d_metrics, 0, (size_t)G * sizeof(esc_group_metrics)));
    HIP_TRY(dalloc(&c->d_cdec, (size_t)G));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_cdec), (size_t)G * sizeof(DecCompact)));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_cdec_dev), c->h_cdec, 0));
    if (G <= HTOT_MAX_GROUPS) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_tot), (size_t)G * sizeof(esc_group_totals)));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_tot_dev), c->h_tot, 0));
    }
    // compact flush: every workgroup may touch every column at most once, so the lists and
    // the entries fit the full-row buffers' sizes
    c->touch_tw = (int)((n_col + 31) / 32);
    HIP_TRY(dalloc(&c->d_touch, (size_t)std::max<int64_t>(nblk, 1) * c->touch_tw));
    HIP_TRY(dalloc(&c->d_wg_cols, (size_t)std::max<int64_t>(nblk, 1) * n_col));
    HIP_TRY(dalloc(&c->d_wg_off, (size_t)nblk + 1));
    HIP_TRY(dalloc(&c->d_col_rows, (size_t)n_col + 1));
    c->work_ready = true;
    return touch_refresh(c, plan);
}

// Enqueue one step for replica r on the context's stream, three launches in order:
//   K1  the pod pass (LDS windows of pod slots; the exact paths when needed),
//   tail k_step_tail: the K3 fold into the pod words + K2 (node piece rows, dry-mode
//        tracker entries) + the K5 ordering of the packed small groups when the ordering is
//        in the step,
//   D   k_node_groups: the node words, then K4 + the decisions when `decide` (one rank;
//        after an exchange esc_decide launches K4 alone).
// (Fusing D into the tail, and K2 into K1, measured slower: DESIGN.md §8e.)
// The ordering's remaining kernels (split groups, mid-size packed chunks) follow the tail.
// Everything is on one stream: K1 fills every CU's LDS, so nothing overlaps it usefully,
// and a cross-stream join cost ~10 us per step.  With timing on each
// stage has its own events.  Decisions go straight to pinned host memory (zero-copy)
// unless disabled, in which case a copy follows.
// Timing mode: one more stage boundary on the context's stream (esc_exchange and esc_decide
// append theirs to enqueue_step's, so a sharded step reads K1 / tail / orderings / node
// groups / exchange / decide).
int32_t stage_mark(esc_ctx* c) {
    if (!c->timing || c->n_stage_ev >= MAX_STAGES - 1) return ESC_OK;
    HIP_TRY(hipEventRecord(c->ev[c->n_stage_ev++], c->stream));
    return ESC_OK;
}

int32_t enqueue_step(esc_ctx* c, int r, bool decide, bool copy_out) {
    const GroupDev g = group_dev(c);
    const NodeDev n = node_dev(c);
    hipStream_t st = c->stream;
    int e = 0;
    auto mark = [&]() -> int32_t {
        if (c->timing) HIP_TRY(hipEventRecord(c->ev[e++], st));
        return ESC_OK;
    };
    DecCompact* cdec = c->zero_copy ? c->h_cdec_dev : c->d_cdec;
    c->tot_dec = decide;                                 // K4's host totals records (small contexts)
    if (int32_t rc = mark()) return rc;
    int nblk = 0;
    if (c->force_wide) {
        if (c->k_tiles + c->c_tiles) HIP_TRY(launch_wide_pods(pod_dev(c, r), g, c->d_wide_pod, st));
    } else if (c->nblk) {
        const PodDev p = pod_dev(c, r);
        const int32_t S = (int32_t)pod_slots(c);
        for (int32_t g0 = 0; g0 < S; g0 += POD_WINDOW_MAX) {           // LDS windows of pod slots
            const int32_t gw = std::min(POD_WINDOW_MAX, S - g0);
            const K1Diag diag{c->d_k1_trace};
            HIP_TRY(launch_pod_reduce(p, g, g0, gw, c->nblk, c->k1_variant, c->d_pod_part, c->d_wide_pod,
                                      c->d_k1_ticket, c->k1_cap, diag, st));
        }
        HIP_TRY(launch_pod_bigtiles(p, g, c->pods[r].big, c->n_big, c->d_wide_pod, st));
        nblk = c->nblk;
    }
    if (int32_t rc = mark()) return rc;
    FoldPlan f;
    f.part = c->d_pod_part;
    f.nblk = nblk;
    f.sp = slot_stride(c);
    f.n_col = f.sp / FC_COL;
    f.col_off = c->d_col_off;
    f.col_groups = c->d_col_groups;
    f.col_rows = nblk && c->touch_on ? c->d_col_rows : nullptr;
    f.ablate = c->k3_ablate;
    const bool ord = c->order_in_step;
    uint64_t* ng_trace = nullptr;
#if ESC_MEASURE
    if (c->tail_trace) {                             // block timestamps of the tail and node groups
        const int64_t nt = f.n_col + tail_span_blocks(n) + tail_trk_blocks(n) + (ord ? c->n_psmall : 0);
        const int64_t nn = (own_list(c).n + 63) / 64;
        if (3 * nt + 2 * nn > c->ttrace_cap) {
            dfree(c->d_ttrace);
            c->ttrace_cap = 0;
            HIP_TRY(dalloc(&c->d_ttrace, (size_t)(3 * nt + 2 * nn)));
            c->ttrace_cap = 3 * nt + 2 * nn;
        }
        c->ttrace_tail = nt;
        c->ttrace_ng = decide ? nn : 0;
        f.trace = c->d_ttrace;
        ng_trace = c->d_ttrace + 3 * nt;
    }
#endif
    HIP_TRY(launch_step_tail(g, n, f, true, c->d_wide_pod, c->d_pwords, c->nodes.rows, c->d_trk_acc, c->d_pchunks,
                             ord ? c->n_psmall : 0, c->d_grp_off, c->d_g_memb, c->d_ord, c->d_seg, st));
    if (int32_t rc = mark()) return rc;
    if (ord) {                                       // split groups, mid-size packed chunks
        HIP_TRY(launch_order(n, c->d_chunks, c->n_chunks, c->d_gch_off, c->d_grp_off, c->d_g_memb, c->d_ostat,
                             c->ord_parity, c->d_ord, c->d_seg, ord_fail(c), st));
        c->ord_parity ^= 1;
        c->ord_failed = false;
        HIP_TRY(launch_order_packed(n, c->d_pchunks + c->n_psmall, c->n_pchunks - c->n_psmall, 0, c->d_grp_off,
                                    c->d_dry, c->d_g_memb, c->d_ord, c->d_seg, st));
    }
    if (int32_t rc = mark()) return rc;
    // D reads and resets the tracker sums the tail accumulated (once per step), for this
    // rank's own groups, and decides them (K4).  A sharded step (no decide) stops before D:
    // the node groups do not depend on the exchange, so they run with K4 after it in ONE
    // launch (esc_decide) — one kernel boundary less on the rank's critical path.
    if (decide) {
        HIP_TRY(launch_node_groups(g, n, own_list(c), c->nodes.rows, c->d_trk_acc, c->d_nwords,
                                   NGDecide{c->d_pwords, c->d_dec, cdec, sel_out(c), ng_trace}, st));
        if (int32_t rc = mark()) return rc;
    }
    if (copy_out && !c->zero_copy) {
        HIP_TRY(hipMemcpyAsync(c->h_cdec, c->d_cdec, (size_t)g.G * sizeof(DecCompact), hipMemcpyDeviceToHost, st));
        if (int32_t rc = mark()) return rc;
    }
    c->n_stage_ev = e;
    return ESC_OK;
}

// fit = false: the exchange-buffer queries, which must still report the new size when a
// bound buffer no longer fits.
int32_t check_ready(esc_ctx* c, bool fit = true) {
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->pods_loaded || !c->nodes_loaded || c->stale) return ESC_E_STATE;
    hipSetDevice(c->device);          // a multi-device host drives several contexts from one thread
    if (int32_t rc = ensure_work(c)) return rc;
    // a node reload can change the owner split and so the exchange words (own_cap): a
    // caller-bound buffer sized before it may be too small, so nothing runs on it until the
    // caller binds one of the new size
    if (fit && c->bound_pwords && xw_count(c) > c->bound_words) return ESC_E_STATE;
    if (c->order_in_step && !c->age_ok) return ESC_E_STATE;   // the age index build failed: rebuild
    return ESC_OK;
}

}  // namespace

namespace esc {
int32_t ctx_stage_mark(esc_ctx* c) { return stage_mark(c); }
}  // namespace esc

// ======================================================================= C ABI
extern "C" {

int32_t esc_abi_version(void) { return ESC_ABI_VERSION; }

const char* esc_strerror(int32_t code) {
    switch (code) {
        case ESC_OK: return "ok";
        case ESC_E_INVAL: return "invalid argument";
        case ESC_E_HIP: return g_last_error[0] ? g_last_error : "HIP runtime error";
        case ESC_E_NOMEM: return "out of memory";
        case ESC_E_LIMIT: return "input exceeds an encoding limit";
        case ESC_E_STATE: return "call order violated";
        case ESC_E_NODEV: return "no gfx950 device available";
        case ESC_E_COMM: return g_last_error[0] ? g_last_error : "RCCL unavailable or a collective failed";
        case ESC_E_ORDER: return "an ordering's bounded look-back gave up (that ordering is invalid; the next one runs afresh)";
        default: return "unknown error";
    }
}

const char* esc_status_string(int32_t status) {
    switch (status) {
        case ESC_ST_OK: return "";
        case ESC_ST_ERR_MIN_NODES: return "node count less than the minimum";
        case ESC_ST_ERR_MAX_NODES: return "node count larger than the maximum";
        case ESC_ST_ERR_DIV_ZERO: return "cannot divide by zero in percent calculation";
        case ESC_ST_ERR_NEG_DELTA: return "negative scale up delta";
        case ESC_ST_ERR_OVERFLOW: return "int64 overflow (Quantity inf.Dec regime, not emulated)";
        case ESC_ST_ERR_TAINT_MIN: return "the number of nodes is less than specified minimum. Taking no action";
        case ESC_ST_NOT_OWNED: return "decided on the group's owner rank";
        default: return "unknown status";
    }
}

int32_t esc_taint_error(int64_t n_untainted, int32_t min_nodes, char* buf, int32_t buf_len) {
    if (!buf || buf_len <= 0) return ESC_E_INVAL;
    std::snprintf(buf, (size_t)buf_len, "the number of nodes(%lld) is less than specified minimum of %d. Taking no action",
                  (long long)n_untainted, (int)min_nodes);
    return ESC_OK;
}

int32_t esc_ctx_create(const esc_group_spec* groups, int32_t n_groups, int32_t device, int32_t rank,
                       int32_t world, esc_ctx** out) {
    if (!out || !groups || n_groups <= 0 || world < 1 || rank < 0 || rank >= world) return ESC_E_INVAL;
    if ((uint32_t)n_groups > NODE_GROUP_MASK) return ESC_E_LIMIT;   // ids share a word with flag bits
    esc_ctx* c = new (std::nothrow) esc_ctx();
    if (!c) return ESC_E_NOMEM;
    c->rank = rank;
    c->world = world;
#if ESC_MEASURE
    // measurement knobs: read by the measurement library only (Makefile ABLATIONS=1,
    // libescalator_hip_measure.so); the product library's results depend on its inputs alone
    if (const char* v = std::getenv("ESC_K1_VARIANT")) c->k1_variant = std::atoi(v);
    if (const char* v = std::getenv("ESC_POD_SORT")) c->pod_sort = (uint32_t)std::max(0, std::atoi(v));
    if (const char* v = std::getenv("ESC_K1_FULL_FLUSH")) c->full_flush = std::atoi(v) != 0;
    if (const char* v = std::getenv("ESC_K3_ABLATE")) c->k3_ablate = std::atoi(v);
    if (const char* v = std::getenv("ESC_TAIL_TRACE")) c->tail_trace = std::atoi(v) != 0;
#endif
    c->gi.build(groups, n_groups);
    c->params.resize(n_groups);
    for (int32_t g = 0; g < n_groups; ++g) params_from(c->params[g], groups[g], nullptr);
    c->pods.resize(1);
    *out = c;
    if (device < 0) return ESC_OK;                         // host-only: packer + scalar math
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess || device >= n_dev) { *out = nullptr; delete c; return ESC_E_NODEV; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        *out = nullptr;
        delete c;
        return ESC_E_NODEV;
    }
    c->device = device;
    c->has_device = true;
    c->cu_count = prop.multiProcessorCount;
    int32_t rc = ESC_OK;
    auto fail = [&](int32_t r) { esc_ctx_destroy(c); *out = nullptr; return r; };
    if (hipSetDevice(device) != hipSuccess) return fail(ESC_E_HIP);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return fail(ESC_E_HIP);
    c->own_stream = true;
    for (int i = 0; i < MAX_STAGES; ++i)
        if (hipEventCreate(&c->ev[i]) != hipSuccess) return fail(ESC_E_HIP);
    for (int i = 0; i < 2; ++i)
        if (hipEventCreate(&c->k1t_ev[i]) != hipSuccess) return fail(ESC_E_HIP);

#if ESC_MEASURE
    if (const char* v = std::getenv("ESC_NO_ZEROCOPY")) c->zero_copy = std::atoi(v) == 0;
#endif
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_oerr), sizeof(uint32_t)) != hipSuccess) return fail(ESC_E_NOMEM);
    *c->h_oerr = 0;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_oerr_dev), c->h_oerr, 0) != hipSuccess) return fail(ESC_E_HIP);
    const size_t G = (size_t)n_groups;
    if (dalloc(&c->d_dry, G) || dalloc(&c->d_params, G)) return fail(ESC_E_NOMEM);
    const GroupIndex& gi = c->gi;
    if (dalloc(&c->d_gpair, G) || dalloc(&c->d_node_code, gi.n_gp) ||
        dalloc(&c->d_code_list, gi.code_list.size()) ||
        dalloc(&c->d_gslot, G))
        return fail(ESC_E_NOMEM);
    // each group's pod slot in K3: the default group reads the default filter's slot
    // n_gp, every other group its pair's slot
    std::vector<uint32_t> gslot(G);
    for (int32_t g = 0; g < n_groups; ++g) gslot[g] = g == gi.default_group ? gi.n_gp : gi.gpair[g];
    if (hipMemcpy(c->d_gslot, gslot.data(), G * 4, hipMemcpyHostToDevice)) return fail(ESC_E_HIP);
    {   // K3: the groups of every column of FC_COL pod slots, ordered by (slot, group)
        const int64_t n_col = slot_stride(c) / FC_COL;
        std::vector<uint32_t> off((size_t)n_col + 1, 0), order(G);
        for (size_t g = 0; g < G; ++g) { order[g] = (uint32_t)g; ++off[gslot[g] / FC_COL + 1]; }
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return gslot[a] < gslot[b]; });
        for (int64_t k = 0; k < n_col; ++k) off[k + 1] += off[k];
        if (dalloc(&c->d_col_off, off.size()) || dalloc(&c->d_col_groups, G)) return fail(ESC_E_NOMEM);
        if (hipMemcpy(c->d_col_off, off.data(), off.size() * 4, hipMemcpyHostToDevice) ||
            hipMemcpy(c->d_col_groups, order.data(), G * 4, hipMemcpyHostToDevice))
            return fail(ESC_E_HIP);
    }
    if (hipMemcpy(c->d_gpair, gi.gpair.data(), G * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(c->d_node_code, gi.node_code.data(), gi.n_gp * 4, hipMemcpyHostToDevice) ||
        (!gi.code_list.empty() &&
         hipMemcpy(c->d_code_list, gi.code_list.data(), gi.code_list.size() * 4, hipMemcpyHostToDevice)))
        return fail(ESC_E_HIP);
    std::vector<uint8_t> dry(G);
    for (size_t g = 0; g < G; ++g) dry[g] = (uint8_t)c->params[g].dry;
    if (hipMemcpy(c->d_dry, dry.data(), G, hipMemcpyHostToDevice) ||
        hipMemcpy(c->d_params, c->params.data(), G * sizeof(GroupParams), hipMemcpyHostToDevice))
        return fail(ESC_E_HIP);
    (void)rc;
    return ESC_OK;
}

int32_t esc_ctx_destroy(esc_ctx* c) {
    if (!c) return ESC_OK;
    if (c->multi) esc::multi_destroy(c);                    // the devices' contexts and communicators
    if (c->list_ctx) esc_ctx_destroy(c->list_ctx);
    list_reducer_free(c->lred);
    if (c->has_device) {
        hipSetDevice(c->device);
        if (c->stream) hipStreamSynchronize(c->stream);
        if (c->comm && rccl().ok) rccl().destroy(reinterpret_cast<ncclComm_t>(c->comm));
        c->comm = nullptr;
        release_work(c);
        release_sort(c);
        release_placement(c);
        for (auto& b : c->pods) b.release();
        c->nodes.release();
        dfree(c->d_dry); dfree(c->d_params);
        dfree(c->d_gpair); dfree(c->d_node_code); dfree(c->d_code_list); dfree(c->d_gslot);
        dfree(c->d_col_off); dfree(c->d_col_groups);
        for (int i = 0; i < MAX_STAGES; ++i)
            if (c->ev[i]) hipEventDestroy(c->ev[i]);
        for (int i = 0; i < 2; ++i)
            if (c->k1t_ev[i]) hipEventDestroy(c->k1t_ev[i]);
        if (c->h_istage) hipHostFree(c->h_istage);
        c->h_istage = nullptr;
        if (c->h_words) hipHostFree(c->h_words);
        c->h_words = nullptr;
        if (c->h_oerr) hipHostFree(c->h_oerr);
        c->h_oerr = c->h_oerr_dev = nullptr;
        release_selections(c);
        if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    }
    delete c;
    return ESC_OK;
}

int32_t esc_ctx_set_stream(esc_ctx* c, void* hip_stream) {
    if (c && c->multi) return ESC_E_STATE;              // the devices' contexts own their streams
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    drop_graphs(c);
    if (hip_stream) {
        c->stream = reinterpret_cast<hipStream_t>(hip_stream);
        c->own_stream = false;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return ESC_E_HIP;
        c->own_stream = true;
    }
    return ESC_OK;
}

int32_t esc_ctx_num_groups(const esc_ctx* c) { return c ? c->gi.G : 0; }

uint32_t esc_ctx_pair_id(const esc_ctx* c, const char* key, const char* value) {
    if (!c) return NONE;
    return c->gi.pair_id(key, value);
}

int32_t esc_ctx_num_group_pairs(const esc_ctx* c) { return c ? (int32_t)c->gi.n_gp : 0; }

int32_t esc_set_replicas(esc_ctx* c, int32_t n) {
    if (c && c->multi) return esc::multi_set_replicas(c, n);
    if (!c || n < 1 || n > 64) return ESC_E_INVAL;
    c->n_replicas = n;              // applies from the next esc_load_pods
    return ESC_OK;
}

int32_t esc_load_pods(esc_ctx* c, const esc_pod_soa* p, int64_t global_offset) {
    if (c && c->multi) return esc::multi_load_pods(c, p, global_offset);
    if (!c || !p || p->n_pods < 0) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    const int64_t n = p->n_pods;
    if (n > 0 && (!p->flags || !p->cpu0 || !p->mem0 || !p->pair0)) return ESC_E_INVAL;
    if ((p->n_xc > 0 && (!p->xc_cpu || !p->xc_mem)) || (p->n_xp > 0 && !p->xp_pair)) return ESC_E_INVAL;
    if (p->n_xc >= (int64_t)0xFFFFFFFF || p->n_xp >= (int64_t)0xFFFFFFFF) return ESC_E_LIMIT;
    // The host layout runs in T chunks of the pods, one host thread each: per
    // chunk counts, then exact prefixes over the chunks, so every pod lands where the
    // one-pass sequential layout put it.
    const int T = n >= (1 << 16) ? host_threads() : 1;
    const int64_t TT = (n >= (1 << 16) && T > 1) ? T : 1;
    // (1) records and extra pairs of each chunk: its pods' offsets into xc / xp
    std::vector<uint64_t> ch_c(TT + 1, 0), ch_p(TT + 1, 0);
    par_chunks(n, (int)TT, [&](int t, int64_t lo, int64_t hi) {
        uint64_t a = 0, b = 0;
        for (int64_t i = lo; i < hi; ++i) { a += pf_xctr(p->flags[i]); b += pf_xpair(p->flags[i]); }
        ch_c[t + 1] = a;
        ch_p[t + 1] = b;
    });
    for (int64_t t = 0; t < TT; ++t) { ch_c[t + 1] += ch_c[t]; ch_p[t + 1] += ch_p[t]; }
    if ((int64_t)ch_c[TT] != p->n_xc || (int64_t)ch_p[TT] != p->n_xp) return ESC_E_INVAL;
    // (2) validate the pair lists (ascending, unique, < ESC_PAIR_LIMIT: a pod matches each
    // group at most once); the class of every pod: pods with at most 3 extra
    // container records and at most 3 extra pairs go to homogeneous K classes, one per record
    // signature, in 256-pod tiles whose records sit in per-tile rows; the rest go to 64-pod C
    // tiles with per-tile record offsets.  Sums are order-independent, so the placement
    // changes no result.  Padding pods carry ESC_PF_DAEMONSET, padding records are 0 and
    // padding pairs NONE.  class id = record signature | packed << 7 (the pod's values fit the
    // packed block, esc_kernels.h kp_fits; the packed class is listed first so that K1
    // streams it first)
    hvec<int16_t> pid(n);
    std::vector<std::vector<int64_t>> ch_cnt(TT, std::vector<int64_t>(POD_CLASS_IDS, 0));
    std::vector<int64_t> ch_nc(TT + 1, 0);
    std::vector<uint64_t> ch_sc(TT + 1, 0), ch_sp(TT + 1, 0);
    std::vector<int32_t> ch_rc(TT, ESC_OK);
    par_chunks(n, (int)TT, [&](int t, int64_t lo, int64_t hi) {
        uint64_t rc = ch_c[t], sp = ch_p[t];
        auto& cn = ch_cnt[t];
        for (int64_t i = lo; i < hi; ++i) {
            const uint32_t f = p->flags[i];
            const uint32_t nx = pf_xpair(f), nc = pf_xctr(f);
            uint32_t last = p->pair0[i];
            if (last == NONE ? nx != 0 : last >= ESC_PAIR_LIMIT) { ch_rc[t] = ESC_E_INVAL; return; }
            for (uint32_t k = 0; k < nx; ++k) {
                const uint32_t q = p->xp_pair[sp + k];
                if (q >= ESC_PAIR_LIMIT || q <= last) { ch_rc[t] = ESC_E_INVAL; return; }
                last = q;
            }
            const int id = pod_class_id(f, p->cpu0[i], p->mem0[i], p->pair0[i], p->xc_cpu ? p->xc_cpu + rc : nullptr,
                                        p->xc_mem ? p->xc_mem + rc : nullptr, c->gi.n_gp);
            pid[i] = (int16_t)id;
            if (id >= 0) {
                ++cn[id];
            } else {
                ++ch_nc[t + 1];
                ch_sc[t + 1] += nc;
                ch_sp[t + 1] += nx;
            }
            rc += nc;
            sp += nx;
        }
    });
    for (int32_t r : ch_rc)
        if (r) return r;
    std::vector<int64_t> cnt(POD_CLASS_IDS, 0);
    for (int64_t t = 0; t < TT; ++t) {
        for (int id = 0; id < POD_CLASS_IDS; ++id) cnt[id] += ch_cnt[t][id];
        ch_nc[t + 1] += ch_nc[t];
        ch_sc[t + 1] += ch_sc[t];
        ch_sp[t + 1] += ch_sp[t];
    }
    const int64_t n_c = ch_nc[TT];
    const uint64_t sc_c = ch_sc[TT], sp_c = ch_sp[TT];
    std::vector<PodClass> cls;
    std::vector<int> cls_of(POD_CLASS_IDS, -1);
    int64_t kt = 0, kbw = 0, kw = 0;
    for (int ord = 0; ord < POD_CLASS_IDS; ++ord) {
        const int id = POD_CLASS_IDS - POD_SIG_IDS * (ord / POD_SIG_IDS + 1) + ord % POD_SIG_IDS;   // small, packed, plain
        const int sig = id % POD_SIG_IDS;
        // with spare slots requested every signature the K layout can hold gets a class, so
        // that inserts of shapes absent at load still land in place
        const bool holdable = (sig / 32) + ((sig / 8) % 4) + ((sig / 4) % 2) <= 3;
        if (!cnt[id] && !(c->spare_frac > 0 && holdable)) continue;
        PodClass k;
        std::memset(&k, 0, sizeof k);
        k.nxp = (uint32_t)(sig % 4);
        k.ovh = (uint32_t)((sig / 4) % 2);
        k.xinit = (uint32_t)((sig / 8) % 4);
        k.xreg = (uint32_t)(sig / 32);
        k.packed = (uint32_t)(id / POD_SIG_IDS);
        const int64_t want = cnt[id] + (c->spare_frac > 0 ? std::max<int64_t>(1, (int64_t)(cnt[id] * c->spare_frac)) : 0);
        const int64_t R = k.xreg + k.xinit + k.ovh, tiles = (want + TILE - 1) / TILE;
        k.t0 = kt;
        k.t1 = kt + tiles;
        k.kind = (uint32_t)(k.packed * 16 + R * 4 + k.nxp);
        k.wt = k_tile_weight((uint32_t)R, k.nxp, k.packed);
        k.kb0 = kbw;
        k.w0 = kw;
        kw += tiles * k.wt;
        kt += tiles;
        kbw += tiles * (int64_t)k.wt * KB_UNIT;
        cls_of[id] = (int)cls.size();
        cls.push_back(k);
    }
    // spare C slots (esc_set_spare): tiles of CS_SLOTS free slots, each with room for a pod of
    // up to CS_XREG regular and CS_XINIT init containers, an overhead and CS_XP extra pairs
    // (the tile's other slots hold nothing, so no tile passes the C path's 128 records of a
    // kind); an upsert of a pod outside the K classes (or of a full K class) takes one
    const int64_t n_cs = c->spare_frac > 0 ? std::max<int64_t>(CS_SLOTS, (int64_t)std::ceil((double)n_c * c->spare_frac)) : 0;
    const int64_t c_real = (n_c + CTILE - 1) / CTILE, cs_tiles = (n_cs + CS_SLOTS - 1) / CS_SLOTS;
    const int64_t k_tiles = kt, c_tiles = c_real + cs_tiles;
    const int64_t c0 = k_tiles * TILE, npad = c_tiles * CTILE;   // C arrays: the C section only
    // C record arrays; one element of padding (K1 clamps its unconditional C record loads)
    const int64_t nxc_dev = (int64_t)sc_c + cs_tiles * CS_SLOTS * CS_REC + 1, nxp_dev = (int64_t)sp_c + cs_tiles * CS_SLOTS * CS_XP + 1;
    if (nxc_dev >= (int64_t)0xFFFFFFFF || nxp_dev >= (int64_t)0xFFFFFFFF) return ESC_E_LIMIT;
    std::vector<uint32_t> hf(npad, ESC_PF_DAEMONSET), hc(npad, 0), hp(npad, NONE);
    std::vector<int64_t> hm(npad, 0), hxc(nxc_dev, 0), hxm(nxc_dev, 0);
    std::vector<uint32_t> hxp(nxp_dev, NONE);
    // (3) K blocks, every tile first as padding (daemonset-flagged pods with no pairs,
    // records 0), tiles split over the threads
    hvec<uint32_t> hkb((size_t)std::max<int64_t>(kbw, 1));
    {
        std::vector<std::pair<int, int64_t>> tl;          // (class, first tile) of each class
        for (int ci = 0; ci < (int)cls.size(); ++ci) tl.emplace_back(ci, cls[ci].t0);
        par_chunks(k_tiles, (int)TT, [&](int, int64_t lo, int64_t hi) {
            int ci = 0;
            for (int64_t t = lo; t < hi; ++t) {
                while (cls[ci].t1 <= t) ++ci;
                const PodClass& k = cls[ci];
                const int64_t blk = kb_block(k, t);
                std::memset(hkb.data() + blk, 0, (size_t)k.wt * KB_UNIT * 4);
                for (int64_t sl = 0; sl < TILE; ++sl)
                    kb_write_free(k, blk, sl, [&](int width, int64_t at, uint64_t v) { put_kb(hkb.data(), width, at, v); });
                if (!k.packed) std::fill(hkb.begin() + blk + KB_PAIR0, hkb.begin() + blk + KB_PAIR0 + TILE, NONE);
                const int64_t x0 = kb_xp_row0(k, blk);     // no pairs (u32 or u16 NONE)
                std::fill(hkb.begin() + x0, hkb.begin() + x0 + kb_xp_words(k), NONE);
            }
        });
    }
    std::vector<uint32_t> xc_base(c_tiles + 1, 0), xp_base(c_tiles + 1, 0);
    hvec<int32_t> pod_cls(n);
    hvec<int64_t> pod_pos(n);
    // (4) positions inside each class: counting sort by bucket = pair0 / pod_sort (NONE and
    // pairs no group selects last); input order inside a bucket, so chunk t's pods of a
    // (class, bucket) follow every earlier chunk's
    const uint32_t sw = c->pod_sort, n_gp = c->gi.n_gp;
    const int64_t nbk = sw ? (int64_t)(n_gp / sw) + 2 : 1;
    auto bucket = [&](uint32_t q0) -> int64_t { return sw ? (q0 < n_gp ? (int64_t)(q0 / sw) : nbk - 1) : 0; };
    std::vector<int> dense(POD_CLASS_IDS, -1);
    int n_dense = 0;
    for (int id = 0; id < POD_CLASS_IDS; ++id)
        if (cnt[id]) dense[id] = n_dense++;
    const int64_t nb_all = (int64_t)n_dense * nbk;
    std::vector<std::vector<int64_t>> ch_next(TT, std::vector<int64_t>(nb_all, 0));
    par_chunks(n, (int)TT, [&](int t, int64_t lo, int64_t hi) {
        auto& v = ch_next[t];
        for (int64_t i = lo; i < hi; ++i)
            if (pid[i] >= 0) ++v[dense[pid[i]] * nbk + bucket(p->pair0[i])];
    });
    for (int64_t a = 0; a < n_dense; ++a) {              // class-local starts, bucket-major, chunk order
        int64_t acc = 0;
        for (int64_t bk = 0; bk < nbk; ++bk)
            for (int64_t t = 0; t < TT; ++t) {
                int64_t& x = ch_next[t][a * nbk + bk];
                const int64_t v = x;
                x = acc;
                acc += v;
            }
    }
    par_chunks(n, (int)TT, [&](int t, int64_t lo, int64_t hi) {
        auto& next = ch_next[t];
        int64_t ic = ch_nc[t];
        uint64_t rc = ch_c[t], rp = ch_p[t];               // the pod's records in the input
        uint64_t oc = ch_sc[t], op = ch_sp[t];             // C record cursors
        for (int64_t i = lo; i < hi; ++i) {
            const uint32_t f = p->flags[i];
            const uint32_t nx = pf_xpair(f), nc = pf_xctr(f);
            const int id = pid[i];
            if (id >= 0) {
                const PodClass& k = cls[cls_of[id]];
                const int64_t q = next[dense[id] * nbk + bucket(p->pair0[i])]++, sl = q % TILE;
                pod_cls[i] = cls_of[id];
                pod_pos[i] = q;
                const int64_t blk = kb_block(k, k.t0 + q / TILE);
                kb_write_pod(k, blk, sl, f, p->cpu0[i], p->mem0[i], p->pair0[i], nc ? p->xc_cpu + rc : nullptr,
                             nc ? p->xc_mem + rc : nullptr, nx ? p->xp_pair + rp : nullptr,
                             [&](int width, int64_t at, uint64_t v) { put_kb(hkb.data(), width, at, v); });
            } else {
                if (ic % CTILE == 0) { xc_base[ic / CTILE] = (uint32_t)oc; xp_base[ic / CTILE] = (uint32_t)op; }
                const int64_t d = ic++;                   // C-array index (slot c0 + d)
                pod_cls[i] = -1;
                pod_pos[i] = c0 + d;
                for (uint32_t j = 0; j < nc; ++j) { hxc[oc + j] = p->xc_cpu[rc + j]; hxm[oc + j] = p->xc_mem[rc + j]; }
                for (uint32_t j = 0; j < nx; ++j) hxp[op + j] = p->xp_pair[rp + j];
                oc += nc;
                op += nx;
                hf[d] = f; hc[d] = p->cpu0[i]; hm[d] = p->mem0[i]; hp[d] = p->pair0[i];
            }
            rc += nc;
            rp += nx;
        }
    });
    {
        uint64_t oc = sc_c, op = sp_c;
        for (int64_t t = c_real; t < c_tiles; ++t) {         // spare C tiles: free slots with room
            xc_base[t] = (uint32_t)oc;
            xp_base[t] = (uint32_t)op;
            for (int l = 0; l < CS_SLOTS; ++l) {
                hf[t * CTILE + l] = CS_FLAGS;
                for (int k = 0; k < CS_REC; ++k) {       // neutral records: 0 added, init keys absent
                    const bool init = k >= CS_XREG && k < CS_XREG + CS_XINIT;
                    hxc[oc + k] = hxm[oc + k] = init ? INT64_MIN : 0;
                }
                oc += CS_REC;
                op += CS_XP;                             // hxp is NONE already
            }
        }
        xc_base[c_tiles] = (uint32_t)oc;
        xp_base[c_tiles] = (uint32_t)op;
    }
    // C tiles with more extra records than a wave holds in registers go to k_pod_bigtiles.
    std::vector<uint32_t> big;
    for (int64_t t = 0; t < c_tiles; ++t)
        if (xc_base[t + 1] - xc_base[t] > 128 || xp_base[t + 1] - xp_base[t] > 128) big.push_back((uint32_t)t);
    const int64_t n_cls = (int64_t)cls.size();
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    drop_graphs(c);
    release_work(c);
    release_sort(c);
    release_placement(c);
    for (auto& b : c->pods) b.release();
    c->pods.assign(c->n_replicas, PodBuf());
    for (int r = 0; r < c->n_replicas; ++r) {
        PodBuf& b = c->pods[r];
        HIP_TRY(dalloc(&b.kb, std::max<int64_t>(kbw, 4)));
        HIP_TRY(dalloc(&b.flags, npad)); HIP_TRY(dalloc(&b.cpu0, npad)); HIP_TRY(dalloc(&b.mem0, npad));
        HIP_TRY(dalloc(&b.pair0, npad)); HIP_TRY(dalloc(&b.xc_cpu, nxc_dev)); HIP_TRY(dalloc(&b.xc_mem, nxc_dev));
        HIP_TRY(dalloc(&b.xp, nxp_dev)); HIP_TRY(dalloc(&b.xc_base, c_tiles + 1)); HIP_TRY(dalloc(&b.xp_base, c_tiles + 1));
        HIP_TRY(dalloc(&b.big, big.size())); HIP_TRY(dalloc(&b.cls, n_cls));
        const hipMemcpyKind kind = r == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
        const PodBuf& a = c->pods[0];
        auto src = [&](const void* host, const void* dev) { return r == 0 ? host : dev; };
        if (kbw) HIP_TRY(hipMemcpy(b.kb, src(hkb.data(), a.kb), kbw * 4, kind));
        if (npad) {
            HIP_TRY(hipMemcpy(b.flags, src(hf.data(), a.flags), npad * 4, kind));
            HIP_TRY(hipMemcpy(b.cpu0, src(hc.data(), a.cpu0), npad * 4, kind));
            HIP_TRY(hipMemcpy(b.mem0, src(hm.data(), a.mem0), npad * 8, kind));
            HIP_TRY(hipMemcpy(b.pair0, src(hp.data(), a.pair0), npad * 4, kind));
        }
        HIP_TRY(hipMemcpy(b.xc_cpu, src(hxc.data(), a.xc_cpu), nxc_dev * 8, kind));
        HIP_TRY(hipMemcpy(b.xc_mem, src(hxm.data(), a.xc_mem), nxc_dev * 8, kind));
        HIP_TRY(hipMemcpy(b.xp, src(hxp.data(), a.xp), nxp_dev * 4, kind));
        HIP_TRY(hipMemcpy(b.xc_base, src(xc_base.data(), a.xc_base), (c_tiles + 1) * 4, kind));
        HIP_TRY(hipMemcpy(b.xp_base, src(xp_base.data(), a.xp_base), (c_tiles + 1) * 4, kind));
        if (!big.empty()) HIP_TRY(hipMemcpy(b.big, src(big.data(), a.big), big.size() * 4, kind));
        if (n_cls) HIP_TRY(hipMemcpy(b.cls, src(cls.data(), a.cls), n_cls * sizeof(PodClass), kind));
    }
    // incremental-update bookkeeping: slot map, free K positions (padding and spare)
    c->pod_cls.swap(pod_cls);
    c->pod_pos.swap(pod_pos);
    c->h_cls = cls;
    c->h_cls_of = cls_of;
    c->cls_free.assign(cls.size(), {});
    for (int id = 0; id < POD_CLASS_IDS; ++id) {
        const int ci = cls_of[id];
        if (ci < 0) continue;
        auto& fr = c->cls_free[ci];
        for (int64_t q = (cls[ci].t1 - cls[ci].t0) * TILE - 1; q >= cnt[id]; --q) fr.push_back(q);
    }
    c->h_cflags.assign(hf.begin(), hf.end());
    c->h_xc_base = xc_base;
    c->h_xp_base = xp_base;
    c->c_free.clear();
    for (int64_t t = c_tiles - 1; t >= c_real; --t)
        for (int l = CS_SLOTS - 1; l >= 0; --l) c->c_free.push_back(t * CTILE + l);
    c->h_cused.assign(npad, 0);
    for (int64_t d = 0; d < npad; ++d)
        if (!(hf[d] & ESC_PF_DAEMONSET) || d < n_c) c->h_cused[d] = pf_xctr(hf[d]) | pf_xpair(hf[d]) << 16;
    c->live_pods = n;
    c->live_xc = p->n_xc;
    c->live_xp = p->n_xp;
    c->live_pk_pods = c->live_pk_xc = c->live_p8_pods = c->live_p8_xp = 0;
    for (int id = POD_SIG_IDS; id < POD_CLASS_IDS; ++id) {
        if (cls_of[id] < 0) continue;
        c->live_pk_pods += cnt[id];
        c->live_pk_xc += cnt[id] * (int64_t)kb_nrec(cls[cls_of[id]]);
        if (id >= 2 * POD_SIG_IDS) { c->live_p8_pods += cnt[id]; c->live_p8_xp += cnt[id] * (int64_t)cls[cls_of[id]].nxp; }
    }
    c->n_pods = n;
    c->k_tiles = k_tiles;
    c->k_weight = kw;
    c->n_cls = (int32_t)n_cls;
    c->c_tiles = c_tiles;
    c->c_tiles_loaded = c_real;
    c->n_big = (int64_t)big.size();
    c->n_xc = p->n_xc;
    c->n_xp = p->n_xp;
    c->pod_offset = global_offset;
    c->cur = 0;
    c->pods_loaded = true;
    c->stale &= ~STALE_PODS;                          // a failed pod event's half-writes are gone
    return ESC_OK;
}

int32_t esc_load_nodes(esc_ctx* c, const esc_node_soa* s, int64_t lo, int64_t hi) {
    if (c && c->multi) return esc::multi_load_nodes(c, s, lo, hi);
    // every rank holds the whole table; its share is the pairs it owns
    if (!c || !s || s->n_nodes < 0 || lo != 0 || hi != s->n_nodes) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    const int64_t n = s->n_nodes;
    if (n >= (int64_t)0x7FFFFFFF) return ESC_E_LIMIT;
    if (n > 0 && (!s->flags || !s->label0 || !s->cpu || !s->mem || !s->created_ns)) return ESC_E_INVAL;
    if ((s->n_xl > 0 && !s->xl_pair) || (s->n_trk > 0 && (!s->trk_node || !s->trk_group))) return ESC_E_INVAL;
    const uint32_t G = (uint32_t)c->gi.G;
    std::vector<uint32_t> xl_off(std::max<int64_t>(n, 1));
    uint64_t sx = 0;
    int64_t tmin = 0, tmax = 0;
    for (int64_t i = 0; i < n; ++i) {
        xl_off[i] = (uint32_t)sx;
        const uint32_t nx = nf_xlbl(s->flags[i]);
        uint32_t last = s->label0[i];                // label pairs ascending, unique
        if (last == NONE ? nx != 0 : last >= ESC_PAIR_LIMIT) return ESC_E_INVAL;
        if (sx + nx > (uint64_t)s->n_xl) return ESC_E_INVAL;
        for (uint32_t k = 0; k < nx; ++k) {
            const uint32_t q = s->xl_pair[sx + k];
            if (q >= ESC_PAIR_LIMIT || q <= last) return ESC_E_INVAL;
            last = q;
        }
        sx += nx;
        if (i >= lo && i < hi) {
            if (i == lo || s->created_ns[i] < tmin) tmin = s->created_ns[i];
            if (i == lo || s->created_ns[i] > tmax) tmax = s->created_ns[i];
        }
    }
    if ((int64_t)sx != s->n_xl) return ESC_E_INVAL;
    for (int64_t i = 0; i < s->n_trk; ++i) {
        if (s->trk_node[i] < 0 || s->trk_node[i] >= n || s->trk_group[i] < 0 || (uint32_t)s->trk_group[i] >= G)
            return ESC_E_INVAL;
        if (i && (s->trk_node[i] < s->trk_node[i - 1] ||
                  (s->trk_node[i] == s->trk_node[i - 1] && s->trk_group[i] <= s->trk_group[i - 1])))
            return ESC_E_INVAL;                      // must be sorted by (node, group), unique
    }
    // Pair-major entries: one per (label pair, node) of the whole table, sorted by
    // (pair, node) — the group-independent index K2 streams.  Pieces are
    // runs of entries of one pair that never cross a multiple of PIECE_ALIGN (256) entries,
    // so K2's spans (whole pieces, <= NODE_SPAN entries) come out full: cut only
    // at pairs, spans averaged 72 % of NODE_SPAN at config 4 (a pair's run seldom fits
    // beside the previous one), 1 460 tail blocks of mostly-masked loads instead of ~1 060
    // (round 6); a pair cut in two is summed from both rows by k_node_groups, as any
    // multi-piece pair.  This rank reduces the pieces that start in its 1/world share of
    // the entries.
    std::vector<uint64_t> ent;
    ent.reserve((size_t)n + (size_t)s->n_xl);
    const uint32_t n_gp0 = c->gi.n_gp;
    std::vector<int64_t> pair_cnt(n_gp0, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (s->flags[i] & ESC_NF_ABSENT) return ESC_E_INVAL;   // the context owns that bit
        if (s->label0[i] == NONE) continue;
        ent.push_back(((uint64_t)s->label0[i] << 32) | (uint64_t)i);
        if (s->label0[i] < n_gp0) ++pair_cnt[s->label0[i]];
        const uint32_t nx = nf_xlbl(s->flags[i]);
        for (uint32_t k = 0; k < nx; ++k) {
            const uint32_t q = s->xl_pair[xl_off[i] + k];
            ent.push_back(((uint64_t)q << 32) | (uint64_t)i);
            if (q < n_gp0) ++pair_cnt[q];
        }
    }
    // spare entries (esc_set_spare): after each group pair's entries, flagged ESC_NF_ABSENT,
    // taken in order by added nodes (whose indices are above every loaded one, so a
    // pair's entries stay in snapshot order)
    const double sf = c->spare_frac;
    for (uint32_t q = 0; q < n_gp0 && sf > 0; ++q) {
        const int64_t sp = (int64_t)std::ceil((double)pair_cnt[q] * sf) + 4;
        for (int64_t k = 0; k < sp; ++k) ent.push_back(((uint64_t)q << 32) | 0xFFFFFFFFull);
    }
    std::sort(ent.begin(), ent.end());
    const int64_t E = (int64_t)ent.size();
    if (E >= (int64_t)0xFFFFFFFF) return ESC_E_LIMIT;
    std::vector<uint32_t> e_flags(std::max<int64_t>(E, 1)), e_node(std::max<int64_t>(E, 1));
    std::vector<int64_t> e_cpu(std::max<int64_t>(E, 1)), e_mem(std::max<int64_t>(E, 1));
    std::vector<uint32_t> piece_off, piece_pair;
    for (int64_t k = 0; k < E; ++k) {
        const uint32_t q = (uint32_t)(ent[k] >> 32), i = (uint32_t)ent[k];
        if (k == 0 || q != piece_pair.back() || k % PIECE_ALIGN == 0) {
            piece_off.push_back((uint32_t)k);
            piece_pair.push_back(q);
        }
        if (i == NONE) {                             // spare entry
            e_flags[k] = ESC_NF_ABSENT;
            e_node[k] = NONE;
            e_cpu[k] = e_mem[k] = 0;
            continue;
        }
        e_flags[k] = s->flags[i];
        e_node[k] = i;
        e_cpu[k] = s->cpu[i];
        e_mem[k] = s->mem[i];
    }
    const int64_t n_pieces = (int64_t)piece_pair.size();
    piece_off.push_back((uint32_t)E);
    // node -> its entry positions (esc_nodes_update patches the entries' copies)
    std::vector<uint32_t> ne_off((size_t)n + 1, 0), ne_pos((size_t)std::max<int64_t>(E, 1));
    for (int64_t k = 0; k < E; ++k)
        if ((uint32_t)ent[k] != NONE) ++ne_off[(uint32_t)ent[k] + 1];
    for (int64_t i = 0; i < n; ++i) ne_off[i + 1] += ne_off[i];
    {
        std::vector<uint32_t> fill(ne_off.begin(), ne_off.end() - 1);
        for (int64_t k = 0; k < E; ++k)
            if ((uint32_t)ent[k] != NONE) ne_pos[fill[(uint32_t)ent[k]]++] = (uint32_t)k;
    }
    ne_pos.resize(ne_off[n]);
    const uint32_t n_gp = c->gi.n_gp;
    std::vector<uint32_t> pp_off((size_t)n_gp + 1);
    for (uint32_t q = 0; q <= n_gp; ++q)
        pp_off[q] = (uint32_t)(std::lower_bound(piece_pair.begin(), piece_pair.end(), q) - piece_pair.begin());
    // This rank's share of the index: the pieces of the group pairs it owns, a
    // contiguous pair range balanced by entry count, the same split on every rank.  Its K2
    // streams only those, its node words are exact for those groups and zero for the others
    // (the SUM exchange carries them), and its K5 orders those groups.  The whole table stays
    // resident on every rank: allNodes[0] and the reaping read it.
    uint32_t q_lo = 0, q_hi = n_gp;
    owned_pairs(pair_cnt, c->world, c->rank, q_lo, q_hi);
    const int64_t pc_lo = pp_off[q_lo], pc_hi = pp_off[q_hi];
    bool pk_ok = true;                               // K2's packed entries (NodeDev::e_pk)
    for (int64_t i = 0; i < n && pk_ok; ++i) pk_ok = entry_cpu_packs(s->cpu[i]);
    // algorithmic bytes K2 streams per decision: per piece its pair and offset, per entry 16 B
    // packed (flags, cpu, memory in one record) or 20 B (the three arrays)
    const int64_t per_entry = pk_ok ? 16 : 20;
    int64_t node_bytes = 0;
    for (int64_t p = pc_lo; p < pc_hi; ++p) {
        node_bytes += 8;                             // piece_pair + piece_off
        if (piece_pair[p] < n_gp) node_bytes += per_entry * (int64_t)(piece_off[p + 1] - piece_off[p]);
    }
    // K2 spans: consecutive whole pieces of the group pairs (a prefix: pieces are pair-sorted
    // and ids >= n_gp come last), <= NODE_SPAN entries (or one larger piece) and <= 63
    // pieces per wave
    std::vector<uint32_t> span_off(1, (uint32_t)pc_lo);
    {
        int64_t p_end = pc_lo, acc = 0;
        while (p_end < pc_hi && piece_pair[p_end] < n_gp) ++p_end;
        int64_t np = 0;
        for (int64_t p = pc_lo; p < p_end; ++p) {
            const int64_t len = (int64_t)piece_off[p + 1] - piece_off[p];
            if (acc > 0 && (acc + len > NODE_SPAN || np == 63)) { span_off.push_back((uint32_t)p); acc = 0; np = 0; }
            acc += len;
            ++np;
        }
        if (p_end > pc_lo) span_off.push_back((uint32_t)p_end);
    }
    // dry-mode tracker: each tracked node's first entry (the (node, group) list is node-sorted)
    std::vector<uint32_t> trk_start(std::max<int64_t>(n + (sf > 0 ? (int64_t)std::ceil((double)n * sf) + 64 : 0), 1),
                                    NONE);
    for (int64_t k = s->n_trk - 1; k >= 0; --k) trk_start[s->trk_node[k]] = (uint32_t)k;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    drop_graphs(c);
    release_work(c);
    release_sort(c);
    release_placement(c);
    c->nodes.release();
    // capacity for added nodes (esc_nodes_add): table slots and extra-label words
    const int64_t n_cap = n + (sf > 0 ? (int64_t)std::ceil((double)n * sf) + 64 : 0);
    const int64_t xl_cap = s->n_xl + (sf > 0 ? (int64_t)std::ceil((double)s->n_xl * sf) + 256 : 0);
    if (n_cap >= (int64_t)0x7FFFFFFF) return ESC_E_LIMIT;
    NodeBuf& b = c->nodes;
    HIP_TRY(dalloc(&b.flags, n_cap)); HIP_TRY(dalloc(&b.label0, n_cap)); HIP_TRY(dalloc(&b.cpu, n_cap));
    HIP_TRY(dalloc(&b.mem, n_cap)); HIP_TRY(dalloc(&b.created, n_cap)); HIP_TRY(dalloc(&b.xl, xl_cap));
    HIP_TRY(dalloc(&b.xl_off, n_cap)); HIP_TRY(dalloc(&b.trk_node, s->n_trk)); HIP_TRY(dalloc(&b.trk_group, s->n_trk));
    if (n_cap > n) {                                 // free slots: absent, no labels
        std::vector<uint32_t> fa(n_cap - n, ESC_NF_ABSENT), la(n_cap - n, NONE);
        HIP_TRY(hipMemcpy(b.flags + n, fa.data(), fa.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.label0 + n, la.data(), la.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(b.cpu + n, 0, (n_cap - n) * 8)); HIP_TRY(hipMemset(b.mem + n, 0, (n_cap - n) * 8));
        HIP_TRY(hipMemset(b.created + n, 0, (n_cap - n) * 8)); HIP_TRY(hipMemset(b.xl_off + n, 0, (n_cap - n) * 4));
    }
    if (n) {
        HIP_TRY(hipMemcpy(b.flags, s->flags, n * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.label0, s->label0, n * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.cpu, s->cpu, n * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.mem, s->mem, n * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.created, s->created_ns, n * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.xl_off, xl_off.data(), n * 4, hipMemcpyHostToDevice));
    }
    if (s->n_xl) HIP_TRY(hipMemcpy(b.xl, s->xl_pair, s->n_xl * 4, hipMemcpyHostToDevice));
    if (s->n_trk) {
        HIP_TRY(hipMemcpy(b.trk_node, s->trk_node, s->n_trk * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.trk_group, s->trk_group, s->n_trk * 4, hipMemcpyHostToDevice));
    }
    HIP_TRY(dalloc(&b.trk_start, trk_start.size()));
    HIP_TRY(hipMemcpy(b.trk_start, trk_start.data(), trk_start.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(dalloc(&b.e_flags, e_flags.size())); HIP_TRY(dalloc(&b.e_node, e_node.size()));
    HIP_TRY(dalloc(&b.e_cpu, e_cpu.size())); HIP_TRY(dalloc(&b.e_mem, e_mem.size()));
    HIP_TRY(hipMemcpy(b.e_flags, e_flags.data(), e_flags.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b.e_node, e_node.data(), e_node.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b.e_cpu, e_cpu.data(), e_cpu.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b.e_mem, e_mem.data(), e_mem.size() * 8, hipMemcpyHostToDevice));
    {   // the packed copy K2 reads (kept current by entry_patch even when not in use)
        std::vector<uint4> pk(e_flags.size());
        for (size_t k = 0; k < pk.size(); ++k)
            pk[k] = make_uint4(e_flags[k], (uint32_t)e_cpu[k], (uint32_t)(uint64_t)e_mem[k],
                               (uint32_t)((uint64_t)e_mem[k] >> 32));
        HIP_TRY(dalloc(&b.e_pk, pk.size()));
        HIP_TRY(hipMemcpy(b.e_pk, pk.data(), pk.size() * sizeof(uint4), hipMemcpyHostToDevice));
    }
    c->e_pk_ok = pk_ok;
    HIP_TRY(dalloc(&b.piece_off, piece_off.size())); HIP_TRY(dalloc(&b.piece_pair, std::max<size_t>(piece_pair.size(), 1)));
    HIP_TRY(dalloc(&b.pp_off, pp_off.size()));
    HIP_TRY(hipMemcpy(b.piece_off, piece_off.data(), piece_off.size() * 4, hipMemcpyHostToDevice));
    if (n_pieces) HIP_TRY(hipMemcpy(b.piece_pair, piece_pair.data(), piece_pair.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b.pp_off, pp_off.data(), pp_off.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(dalloc(&b.span_off, span_off.size()));
    HIP_TRY(hipMemcpy(b.span_off, span_off.data(), span_off.size() * 4, hipMemcpyHostToDevice));
    {
        std::vector<uint32_t> span_e(span_off.size());
        for (size_t w = 0; w < span_off.size(); ++w) span_e[w] = piece_off[span_off[w]];
        HIP_TRY(dalloc(&b.span_e, span_e.size()));
        HIP_TRY(hipMemcpy(b.span_e, span_e.data(), span_e.size() * 4, hipMemcpyHostToDevice));
    }
    HIP_TRY(dalloc(&b.rows, (size_t)std::max<int64_t>(n_pieces, 1) * NR_K));
    {   // per-group facts fixed by this snapshot: this rank's pieces of the group's pair and
        // allNodes[0] (controller.go:207-211) = the pair's first entry (lowest node index)
        std::vector<GroupNode> gn(G);
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t q = c->gi.gpair[g], p0 = pp_off[q], p1 = pp_off[q + 1];
            GroupNode& x = gn[g];
            x.plo = std::max<int64_t>(p0, pc_lo);
            x.phi = std::min<int64_t>(p1, pc_hi);
            if (x.phi < x.plo) x.phi = x.plo;
            const bool any = p1 > p0 && e_node[piece_off[p0]] != NONE;     // not only spare entries
            x.first = any ? (int64_t)e_node[piece_off[p0]] : INT64_MAX;
            x.first_cpu = any ? s->cpu[x.first] : 0;
            x.first_mem = any ? s->mem[x.first] : 0;
        }
        HIP_TRY(dalloc(&b.gnode, gn.size()));
        HIP_TRY(hipMemcpy(b.gnode, gn.data(), gn.size() * sizeof(GroupNode), hipMemcpyHostToDevice));
        c->h_gnode.swap(gn);
    }
    // host mirrors for node events (table slots up to the capacity)
    c->pair_next.assign(n_gp, 0);
    c->pair_end.assign(n_gp, 0);
    c->pair_lo.assign(n_gp, 0);
    for (uint32_t q = 0; q < n_gp; ++q) {
        const uint32_t a = piece_off[pp_off[q]], z = piece_off[pp_off[q + 1]];
        c->pair_end[q] = z;
        c->pair_lo[q] = a;
        c->pair_next[q] = a + (uint32_t)pair_cnt[q];
    }
    c->h_e_node.swap(e_node);
    c->h_e_node.resize(E);
    c->ne_off.swap(ne_off);
    c->ne_pos.swap(ne_pos);
    c->h_nflags.assign(s->flags, s->flags + n);
    c->h_ncpu.assign(s->cpu, s->cpu + n);
    c->h_nmem.assign(s->mem, s->mem + n);
    c->h_label0.assign(s->label0, s->label0 + n);
    c->h_xl_off.assign(xl_off.begin(), xl_off.begin() + n);
    c->h_xl.assign(s->xl_pair, s->xl_pair + s->n_xl);
    c->h_nflags.resize(n_cap, ESC_NF_ABSENT);
    c->h_ncpu.resize(n_cap, 0);
    c->h_nmem.resize(n_cap, 0);
    c->h_label0.resize(n_cap, NONE);
    c->h_xl_off.resize(n_cap, 0);
    c->n_cap = n_cap;
    c->xl_used = s->n_xl;
    c->xl_cap = xl_cap;
    c->q_lo = q_lo;
    c->q_hi = q_hi;
    c->q_bounds.assign((size_t)c->world + 1, n_gp);
    for (int32_t r = 0; r < c->world; ++r) {
        uint32_t a = 0, b = 0;
        owned_pairs(pair_cnt, c->world, r, a, b);
        c->q_bounds[r] = a;
    }
    c->pair_live = pair_cnt;
    c->h_gn.clear();
    c->n_entries = E;
    c->n_pieces = n_pieces;
    c->n_spans = (int64_t)span_off.size() - 1;
    c->pc_lo = pc_lo;
    c->pc_hi = pc_hi;
    c->node_bytes = node_bytes;
    c->n_nodes = n;
    c->n_xl = s->n_xl;
    c->n_trk = s->n_trk;
    c->trk_cap = s->n_trk;
    c->h_trk.resize(s->n_trk);
    for (int64_t k = 0; k < s->n_trk; ++k) c->h_trk[k] = ((uint64_t)(uint32_t)s->trk_node[k] << 32) | (uint32_t)s->trk_group[k];
    c->node_lo = lo;
    c->node_hi = hi;
    c->ts_min = tmin;
    c->ts_max = tmax;
    c->h_created.assign(s->created_ns + lo, s->created_ns + hi);
    c->nodes_loaded = true;
    c->stale &= ~STALE_NODES;
    return build_age_index(c);
}

int32_t esc_stream_bytes(const esc_ctx* c, int64_t* pod_bytes, int64_t* node_bytes) {
    if (c && c->multi) return esc::multi_stream_bytes(c, pod_bytes, node_bytes);
    if (!c || !pod_bytes || !node_bytes) return ESC_E_INVAL;
    if (!c->pods_loaded || !c->nodes_loaded) return ESC_E_STATE;
    // K1: flags 4 + cpu0 4 + mem0 8 + pair0 4 per pod, 16 per extra container record,
    // 4 per extra pair, 8 per C tile (record offsets); a pod of a packed class 12 B + 8 per
    // record, of a packed small class 8 B + 8 per record + 2 per extra pair (esc_kernels.h,
    // kp_*, kp8_*); K2:
    // see esc_load_nodes
    *pod_bytes = c->live_pods * 20 + c->live_xc * 16 + c->live_xp * 4 + c->c_tiles_loaded * 8 - c->live_pk_pods * 8 -
                 c->live_pk_xc * 8 - c->live_p8_pods * 4 - c->live_p8_xp * 2;
    *node_bytes = c->node_bytes;
    return ESC_OK;
}

int32_t esc_set_state(esc_ctx* c, const esc_group_state* st) {
    if (c && c->multi) return esc::multi_set_state(c, st);
    if (!c) return ESC_E_INVAL;
    for (int32_t g = 0; g < c->gi.G; ++g) params_from(c->params[g], c->gi.groups[g].spec, st ? st + g : nullptr);
    if (!c->has_device) return ESC_OK;
    hipSetDevice(c->device);
    HIP_TRY(hipMemcpyAsync(c->d_params, c->params.data(), c->params.size() * sizeof(GroupParams),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ESC_OK;
}

int32_t esc_set_metrics(esc_ctx* c, int32_t enable) {
    if (c && c->multi) return esc::multi_each(c, esc_set_metrics, enable);
    if (!c) return ESC_E_INVAL;
    c->want_metrics = enable != 0;
    drop_graphs(c);
    return ESC_OK;
}

int32_t esc_metrics_results(esc_ctx* c, esc_group_metrics* out) {
    if (c && c->multi) return esc::multi_metrics_results(c, out);
    if (!c || !out) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->work_ready || !c->want_metrics) return ESC_E_STATE;
    int32_t rc = esc_sync(c);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(out, c->d_metrics, (size_t)c->gi.G * sizeof(esc_group_metrics), hipMemcpyDeviceToHost));
    return ESC_OK;
}

int32_t esc_use_graph(esc_ctx* c, int32_t enable) {
    if (c && c->multi) return esc::multi_each(c, esc_use_graph, enable);
    if (!c) return ESC_E_INVAL;
    c->use_graph = enable != 0;
    if (!c->use_graph) drop_graphs(c);
    return ESC_OK;
}

int32_t esc_force_wide(esc_ctx* c, int32_t enable) {
    if (c && c->multi) return esc::multi_each(c, esc_force_wide, enable);
    if (!c) return ESC_E_INVAL;
    c->force_wide = enable != 0;
    drop_graphs(c);
    return ESC_OK;
}

int32_t esc_set_timing(esc_ctx* c, int32_t enable) {
    if (c && c->multi) return esc::multi_each(c, esc_set_timing, enable);
    if (!c) return ESC_E_INVAL;
    c->timing = enable != 0;
    drop_graphs(c);
    return ESC_OK;
}

int32_t esc_stage_times(esc_ctx* c, double* ms, int32_t n) {
    if (c && c->multi) return esc_stage_times(esc::multi_sub(c, 0), ms, n);
    if (!c || !ms || n <= 0) return ESC_E_INVAL;
    for (int i = 0; i < n && i < MAX_STAGES; ++i) ms[i] = c->stage_ms[i];
    return ESC_OK;
}

// K1 share calibration.  The K1 workgroups stream equal bytes at unequal rates, and the
// rates are a stable property of the grid position on a device: at 100 M pods the slowest
// workgroup's K phase took 1.14x the mean (odd XCDs ~5 % slower than even ones, plus a
// within-XCD spread), and the per-workgroup durations correlate 0.9-0.98 between
// decisions and 0.96-0.99 between processes (profiles/r02_v8/k1_trace_stability_*.json).
// Each round runs three decisions and averages every workgroup's start offset, K phase and
// tail (trace words 0, 1, 3), then moves each share half-way to the one that would end every
// workgroup at the same time under its measured streaming rate (round 5: balancing END
// times, so the XCDs' dispatch stagger and the flush are paid for too — balancing the K
// phases alone left the slowest workgroup ~2.5 us after the mean at a rank's shard); the
// plan with the lowest slowest-workgroup end seen is kept.  The grid and the per-workgroup pod bound
// do not change, and sums are order-independent, so every result is unchanged; the graphs
// read the plan from device memory, so they stay valid.
int32_t esc_k1_calibrate(esc_ctx* c, int32_t rounds) {
    if (c && c->multi) return esc::multi_k1_calibrate(c, rounds);
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (rounds < 0) return ESC_E_INVAL;
    hipSetDevice(c->device);
    const int64_t nblk = c->nblk;
    if (!c->d_k1seg || nblk <= 1 || c->force_wide || rounds == 0) return ESC_OK;   // nothing to balance
    std::vector<uint64_t> tr((size_t)nblk * 8);
    std::vector<double> share = c->k1_share, best;
    if ((int64_t)share.size() != nblk) share.assign(nblk, 1.0 / (double)nblk);
    double best_max = 0;
    auto upload = [&](const std::vector<double>& sh) -> int32_t {
        std::vector<int64_t> plan = plan_k1(c->h_cls, c->k_weight, nblk, sh);
        if (plan.empty() || plan_worst(c, plan, nblk) > PODS_PER_BLOCK_MAX) return 1;
        HIP_TRY(hipMemcpy(c->d_k1seg, plan.data(), plan.size() * 8, hipMemcpyHostToDevice));
        c->k1_share = sh;
        return touch_refresh(c, plan);
    };
#ifndef ESC_CAL_REPS
#define ESC_CAL_REPS 8       // (timing builds may override; r05cal2: 8 decisions per round, 0.7 steps)
#endif
#ifndef ESC_CAL_STEP
#define ESC_CAL_STEP 0.7
#endif
    constexpr int REPS = ESC_CAL_REPS;                   // decisions averaged per round (noise ~1-4 %)
    for (int32_t r = 0; r <= rounds; ++r) {
        // per workgroup: its start offset from the grid's first start (the XCDs are dispatched
        // ~1.4 us apart, the same XCD order every launch), its K phase, and what follows it
        // (C tiles, the compact flush), averaged over REPS decisions
        std::vector<double> st(nblk, 0.0), kp(nblk, 0.0), tl(nblk, 0.0);
        for (int k = 0; k < REPS; ++k) {
            rc = c->world == 1 ? esc_run(c) : esc_reduce(c);
            if (!rc) rc = esc_sync(c);
            if (rc) return rc;
            HIP_TRY(hipMemcpy(tr.data(), c->d_k1_trace, tr.size() * 8, hipMemcpyDeviceToHost));
            uint64_t t0 = tr[0];
            for (int64_t b = 0; b < nblk; ++b) t0 = std::min<uint64_t>(t0, tr[b * 8 + 0]);
            for (int64_t b = 0; b < nblk; ++b) {
                const double d = (double)(int64_t)(tr[b * 8 + 1] - tr[b * 8 + 0]);
                if (!(d > 0)) return ESC_OK;            // no K phase measured: keep the plan
                st[b] += (double)(int64_t)(tr[b * 8 + 0] - t0) / REPS;
                kp[b] += d / REPS;
                tl[b] += std::max(0.0, (double)(int64_t)(tr[b * 8 + 3] - tr[b * 8 + 1])) / REPS;
            }
        }
        // the grid ends with its last workgroup: balance END times (start + K phase + tail),
        // not K phases — a workgroup of a late XCD or with a long flush gets less weight
        double mx = 0, rsum = 0, rfix = 0;
        for (int64_t b = 0; b < nblk; ++b) {
            mx = std::max(mx, st[b] + kp[b] + tl[b]);    // (the REPS-mean end of the latest workgroup)
            const double rate = share[b] / kp[b];        // share per tick while streaming
            rsum += rate;
            rfix += rate * (st[b] + tl[b]);
        }
        if (best.empty() || mx < best_max) { best = share; best_max = mx; }
        if (r == rounds) break;
        // shares that would end every workgroup at the same time T under the measured rates
        // (sum = 1), half-way from the current ones (the rates move with the tiles a share
        // takes)
        const double T = (1.0 + rfix) / rsum;
        std::vector<double> next(nblk);
        double sum = 0;
        for (int64_t b = 0; b < nblk; ++b) {
            const double want = std::max(0.25 * share[b], share[b] / kp[b] * (T - st[b] - tl[b]));
            sum += (next[b] = (1.0 - ESC_CAL_STEP) * share[b] + ESC_CAL_STEP * want);
        }
        for (double& x : next) x /= sum;
        if (upload(next) != ESC_OK) break;               // outside the exactness bound: stop here
        share = next;
    }
    if (best != c->k1_share) {
        rc = upload(best);
        if (rc < 0) return rc;
    }
    return ESC_OK;
}

int32_t esc_k1_flush_entries(const esc_ctx* c, int64_t* entries, int64_t* full) {
    if (!c || !entries || !full) return ESC_E_INVAL;
    if (c->multi) {
        int64_t e = 0, f = 0;
        for (int i = 0; esc::multi_sub(const_cast<esc_ctx*>(c), i); ++i) {
            int64_t a, b;
            if (int32_t rc = esc_k1_flush_entries(esc::multi_sub(const_cast<esc_ctx*>(c), i), &a, &b)) return rc;
            e += a;
            f += b;
        }
        *entries = e;
        *full = f;
        return ESC_OK;
    }
    if (!c->work_ready) return ESC_E_STATE;
    const int64_t n_col = slot_stride(c) / FC_COL;
    *full = (int64_t)c->nblk * n_col;
    int64_t e = 0;
    for (uint32_t x : c->h_touch) e += __builtin_popcount(x);
    *entries = c->touch_on ? e : *full;
    return ESC_OK;
}

int32_t esc_k1_trace(esc_ctx* c, uint64_t* out, int64_t cap, int64_t* n_out) {
    if (c && c->multi) return esc_k1_trace(esc::multi_sub(c, 0), out, cap, n_out);
    if (!c || !n_out || cap < 0 || (cap > 0 && !out)) return ESC_E_INVAL;
    if (!c->d_k1_trace) return ESC_E_STATE;
    *n_out = c->nblk;
    hipSetDevice(c->device);
    const int64_t w = std::min<int64_t>(cap, (int64_t)c->nblk * 8);
    if (w > 0) HIP_TRY(hipMemcpy(out, c->d_k1_trace, (size_t)w * 8, hipMemcpyDeviceToHost));
    return ESC_OK;
}

int32_t esc_k1_time(esc_ctx* c, int32_t reps, double* ms_per_launch) {
    if (c && c->multi) return esc_k1_time(esc::multi_sub(c, 0), reps, ms_per_launch);
    if (!ms_per_launch || reps < 1) return ESC_E_INVAL;
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (c->force_wide || !c->nblk) return ESC_E_STATE;
    hipSetDevice(c->device);
    hipStream_t st = c->stream;
    const GroupDev g = group_dev(c);
    const int32_t S = (int32_t)pod_slots(c);
    const int nrep = (int)c->pods.size();
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipEventRecord(c->k1t_ev[0], st));
    // every K1 launch of a step (its LDS windows and the big C tiles, so the pod bytes the
    // roofline divides are all timed); no trace, so esc_k1_trace keeps the last decision's.
    // The launches rotate over the replicas as the decisions do: a shard small enough for
    // the 256 MB Infinity Cache, launched on one replica back to back, is read from the
    // cache, not HBM (round 5, a rank of 8's 124 MB: 29.7-30.0 us on one replica, 30.7-31.1
    // rotating)
    for (int32_t k = 0; k < reps; ++k) {
        const int r = (c->cur + k) % nrep;
        const PodDev p = pod_dev(c, r);
        for (int32_t g0 = 0; g0 < S; g0 += POD_WINDOW_MAX) {
            const K1Diag diag{nullptr};
            HIP_TRY(launch_pod_reduce(p, g, g0, std::min(POD_WINDOW_MAX, S - g0), c->nblk, c->k1_variant, c->d_pod_part,
                                      c->d_wide_pod, c->d_k1_ticket, c->k1_cap, diag, st));
        }
        HIP_TRY(launch_pod_bigtiles(p, g, c->pods[r].big, c->n_big, c->d_wide_pod, st));
    }
    HIP_TRY(hipEventRecord(c->k1t_ev[1], st));
    // the exact-path accumulators K1 added to without a fold: back to zero for the next step
    HIP_TRY(hipMemsetAsync(c->d_wide_pod, 0, (size_t)pod_slots(c) * WP_K * sizeof(int64_t), st));
    HIP_TRY(hipStreamSynchronize(st));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->k1t_ev[0], c->k1t_ev[1]));
    *ms_per_launch = (double)ms / reps;
    return ESC_OK;
}

int32_t esc_reduce(esc_ctx* c) {
    if (c && c->multi) return ESC_E_STATE;             // the exchange is internal: esc_step
    int32_t rc = check_ready(c);
    if (rc) return rc;
    hipSetDevice(c->device);
    if (c->ng_pending) {                               // the previous reduce was not decided:
        // its node groups consume its tracker sums now (no decisions), so no step's sums mix
        HIP_TRY(launch_node_groups(group_dev(c), node_dev(c), own_list(c), c->nodes.rows, c->d_trk_acc, c->d_nwords,
                                   NGDecide{nullptr, nullptr, nullptr}, c->stream));
    }
    c->ng_pending = true;
    c->tot_dec = false;              // the host totals records are the last decide's (a replayed
                                     // graph does not run enqueue_step, which also says so: ADVICE r5)
    const int r = c->cur;
    c->cur = (c->cur + 1) % (int)c->pods.size();
    c->pending = true;
    if (c->order_in_step) { c->order_src = 0; c->sorted = true; }
    if (!c->use_graph || c->timing) return enqueue_step(c, r, false, false);
    return replay_step(c, c->rgraphs, r, false);
}

int32_t esc_exchange_buffers(esc_ctx* c, void** sum_buf, int64_t* sum_count, void** min_buf, int64_t* min_count) {
    if (c && c->multi) return ESC_E_STATE;
    int32_t rc = check_ready(c, false);
    if (rc) return rc;
    if (sum_buf) *sum_buf = c->d_pwords;
    if (sum_count) *sum_count = xw_count(c);
    // allNodes[0] is resolved from the whole node table every rank holds, so the
    // first-member words need no MIN exchange in this build
    if (min_buf) *min_buf = nullptr;
    if (min_count) *min_count = 0;
    return ESC_OK;
}

int32_t esc_exchange_slice(const esc_ctx* c, int64_t* offset, int64_t* count) {
    if (c && c->multi) return ESC_E_STATE;
    if (!c || !offset || !count) return ESC_E_INVAL;
    if (!c->work_ready) return ESC_E_STATE;
    *offset = (int64_t)c->rank * c->own_cap * PW_K;
    *count = (int64_t)c->own_cap * PW_K;
    return ESC_OK;
}

int32_t esc_exchange_rows(const esc_ctx* c, const esc_node_soa* s, int32_t world, uint32_t* rows, int32_t* own_rows) {
    if (!c || !s || !rows || !own_rows || world < 1) return ESC_E_INVAL;
    const int32_t G = c->gi.G;
    std::vector<uint32_t> qb((size_t)world + 1);
    if (int32_t rc = esc_node_owner_ranges(c, s, world, qb.data())) return rc;
    std::vector<int32_t> n((size_t)world, 0), owner((size_t)G);
    for (int32_t g = 0; g < G; ++g) {
        const uint32_t q = c->gi.gpair[(size_t)g];
        owner[(size_t)g] = world == 1 ? 0 : (int32_t)(std::upper_bound(qb.begin(), qb.end() - 1, q) - qb.begin()) - 1;
        ++n[(size_t)owner[(size_t)g]];
    }
    const int32_t cap = std::max(1, *std::max_element(n.begin(), n.end()));
    std::fill(n.begin(), n.end(), 0);
    for (int32_t g = 0; g < G; ++g) rows[g] = (uint32_t)(owner[(size_t)g] * cap + n[(size_t)owner[(size_t)g]]++);
    *own_rows = cap;
    return ESC_OK;
}

int32_t esc_bind_exchange_buffers(esc_ctx* c, void* sum_buf, void* min_buf) {
    if (c && c->multi) return ESC_E_STATE;
    if (!c || (!sum_buf && min_buf)) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (min_buf) return ESC_E_INVAL;                  // min_count is 0: nothing to MIN-exchange
    if (sum_buf) {
        // the buffer holds sum_count words as esc_exchange_buffers reports them now: record
        // that, so a reload that grows them is refused instead of overrunning it
        c->bound_pwords = nullptr;
        if (int32_t rc = check_ready(c, false)) return rc;
        c->bound_words = xw_count(c);
    }
    c->bound_pwords = reinterpret_cast<int64_t*>(sum_buf);
    if (c->work_ready) c->d_pwords = c->bound_pwords ? c->bound_pwords : c->own_pwords;
    drop_graphs(c);
    return ESC_OK;
}

int32_t esc_exchange_download(esc_ctx* c, int64_t* sum_out, int64_t* min_out) {
    if (c && c->multi) return ESC_E_STATE;
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (!sum_out) return ESC_E_INVAL;
    (void)min_out;                                   // min_count is 0: nothing to MIN-exchange
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(sum_out, c->d_pwords, (size_t)xw_count(c) * 8, hipMemcpyDeviceToHost));
    return ESC_OK;
}

int32_t esc_exchange_upload(esc_ctx* c, const int64_t* sum_in, const int64_t* min_in) {
    if (c && c->multi) return ESC_E_STATE;
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (!sum_in) return ESC_E_INVAL;
    (void)min_in;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(c->d_pwords, sum_in, (size_t)xw_count(c) * 8, hipMemcpyHostToDevice));
    return stage_mark(c);                               // timing mode: the host-staged exchange's end
}

int32_t esc_decide(esc_ctx* c) {
    if (c && c->multi) return ESC_E_STATE;
    int32_t rc = check_ready(c);
    if (rc) return rc;
    hipSetDevice(c->device);
    // node groups + K4 over this rank's own groups: their node words from K2's piece rows
    // (the tracker sums of the step), their exchanged pod words (the rank's slice, rows xs[g])
    if (!c->ng_pending) return ESC_E_STATE;            // nothing reduced since the last decide
    uint64_t* ng_trace = nullptr;
#if ESC_MEASURE
    if (c->tail_trace && c->d_ttrace) {                // after the reduce's tail blocks (esc_debug_tail_trace)
        const int64_t nn = (own_list(c).n + 63) / 64;
        if (3 * c->ttrace_tail + 2 * nn <= c->ttrace_cap) {
            ng_trace = c->d_ttrace + 3 * c->ttrace_tail;
            c->ttrace_ng = nn;
        }
    }
#endif
    HIP_TRY(launch_node_groups(group_dev(c), node_dev(c), own_list(c), c->nodes.rows, c->d_trk_acc, c->d_nwords,
                               NGDecide{c->d_pwords, c->d_dec, c->zero_copy ? c->h_cdec_dev : c->d_cdec, sel_out(c), ng_trace},
                               c->stream));
    c->ng_pending = false;
    c->tot_dec = true;
    if (!c->zero_copy)
        HIP_TRY(hipMemcpyAsync(c->h_cdec, c->d_cdec, (size_t)c->gi.G * sizeof(DecCompact), hipMemcpyDeviceToHost,
                               c->stream));
    if (int32_t rc = stage_mark(c)) return rc;
    c->pending = true;
    return ESC_OK;
}

int32_t esc_run(esc_ctx* c) {
    if (c && c->multi) return esc::multi_step(c);
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (c->world != 1) return ESC_E_STATE;            // multi-rank: reduce, exchange, decide
    hipSetDevice(c->device);
    const int r = c->cur;
    const int nrep = (int)c->pods.size();
    c->cur = (c->cur + 1) % nrep;
    c->pending = true;
    (void)nrep;
    c->tot_dec = true;
    if (c->order_in_step) { c->order_src = 0; c->sorted = true; }
    if (!c->use_graph || c->timing) return enqueue_step(c, r, true, true);
    return replay_step(c, c->graphs, r, true);
}

int32_t esc_set_order_in_step(esc_ctx* c, int32_t enable) {
    if (c && c->multi) return esc::multi_each(c, esc_set_order_in_step, enable);
    if (!c) return ESC_E_INVAL;
    c->order_in_step = enable != 0;
    drop_graphs(c);
    return ESC_OK;
}

#if ESC_MEASURE
// Fault injection (measurement library only; not in the header): the next n_order ordering
// and n_list listing launches give up their look-back at once; the next n apply phases of
// informer events fail after their host-side writes.
int32_t esc_debug_lookback_fail(esc_ctx* c, int32_t n_order, int32_t n_list) {
    if (!c || c->multi) return ESC_E_INVAL;
    c->lb_fail_order = std::max(0, n_order);
    c->lb_fail_list = std::max(0, n_list);
    drop_graphs(c);                                     // captured launches hold their bound
    return ESC_OK;
}
// [n_tail, n_ng, the tail's {start, end, role} per block, the node groups' {start, end}]
// of the last step traced (ESC_TAIL_TRACE=1; s_memrealtime ticks, 100 MHz).
int32_t esc_debug_tail_trace(esc_ctx* c, uint64_t* out, int64_t cap, int64_t* n_out) {
    if (!c || c->multi || !out || !n_out) return ESC_E_INVAL;
    if (!c->d_ttrace) return ESC_E_STATE;
    const int64_t w = 3 * c->ttrace_tail + 2 * c->ttrace_ng;
    *n_out = w + 2;
    if (cap < w + 2) return ESC_E_LIMIT;
    HIP_TRY(hipStreamSynchronize(c->stream));
    out[0] = (uint64_t)c->ttrace_tail;
    out[1] = (uint64_t)c->ttrace_ng;
    HIP_TRY(hipMemcpy(out + 2, c->d_ttrace, (size_t)w * 8, hipMemcpyDeviceToHost));
    return ESC_OK;
}
int32_t esc_debug_fail_patches(esc_ctx* c, int32_t n) {
    if (!c || c->multi) return ESC_E_INVAL;
    c->fail_patches = std::max(0, n);
    return ESC_OK;
}
#endif

int32_t esc_set_selections(esc_ctx* c, int32_t slack, int32_t group_cap) {
    if (c && c->multi) {
        for (int i = 0; esc::multi_sub(c, i); ++i)
            if (int32_t rc = esc_set_selections(esc::multi_sub(c, i), slack, group_cap)) return rc;
        return ESC_OK;
    }
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (group_cap <= 0) group_cap = 256;
    if ((uint32_t)group_cap > SEL_COUNT_MASK) return ESC_E_LIMIT;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));          // queued decisions may still write the buffer
    drop_graphs(c);                                     // captured steps hold the old target
    release_selections(c);
    // every block of 64 groups has a slot for its groups' runs at their largest (header +
    // group_cap nodes; k_node_groups): no decision overflows it
    const int64_t words = (((int64_t)c->gi.G + 63) / 64) * 64 * ((int64_t)group_cap + 1);
    if (slack >= 0 && words > (int64_t)0xFFFFFFFE) return ESC_E_LIMIT;   // 32-bit run offsets
    c->sel_slack = slack < 0 ? -1 : slack;
    c->sel_group_cap = group_cap;
    if (slack < 0) return ESC_OK;
    c->sel_words = words;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_sel), (size_t)c->sel_words * 4));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_sel_dev), c->h_sel, 0));
    for (int32_t g = 0; c->h_cdec && g < c->gi.G; ++g) c->h_cdec[g].sel = SEL_NONE;
    return ESC_OK;
}

namespace {
// Group g's selection in the last decision (after a wait): which (ESC_SEL_*), its nodes.
int32_t group_selection(const esc_ctx* c, int32_t g, int32_t* which, const uint32_t** nodes, int64_t* n) {
    *which = ESC_SEL_NONE;
    *nodes = nullptr;
    *n = 0;
    if (c->multi) {
        int32_t owner = 0;
        if (int32_t rc = esc_group_owner(c, g, &owner)) return rc;
        return group_selection(esc::multi_sub(c, owner), g, which, nodes, n);
    }
    if (c->world > 1 && group_owner_rank(c, g) != c->rank) return ESC_OK;   // decided on its owner
    const uint32_t at = c->h_cdec[g].sel;
    if (at == SEL_NONE) return ESC_OK;
    if (at == SEL_OVERFLOW || (int64_t)at >= c->sel_words) {   // not delivered: the walk reads esc_group_order
        *which = ESC_SEL_CUT;
        return ESC_OK;
    }
    const uint32_t h = c->h_sel[at];
    const uint32_t w = (h >> 28) & 3u;
    if (w == 0) return ESC_OK;
    *which = (int32_t)w - 1;
    if (h & SEL_TIE) {                                  // a long tie run: no nodes delivered
        *which |= ESC_SEL_CUT;
        return ESC_OK;
    }
    if (h & SEL_CUT) *which |= ESC_SEL_CUT;
    *nodes = c->h_sel + at + 1;
    *n = h & SEL_COUNT_MASK;
    return ESC_OK;
}
}  // namespace

int32_t esc_selections(esc_ctx* c, int32_t* which, int64_t* offsets, int64_t* idx, int64_t cap, int64_t* n_total) {
    if (!c || !which || !offsets || !n_total || cap < 0 || (cap > 0 && !idx)) return ESC_E_INVAL;
    esc_ctx* c0 = c->multi ? esc::multi_sub(c, 0) : c;
    if (!c0 || !c0->has_device) return ESC_E_NODEV;
    if (c0->sel_slack < 0 || !c0->h_cdec) return ESC_E_STATE;
    if (int32_t rc = esc_sync(c); rc != ESC_OK && rc != ESC_E_ORDER) return rc;
    // the ordering the selections come from gave up: they are invalid, as its orderings
    bool failed = false;
    for (int i = 0; c->multi ? esc::multi_sub(c, i) != nullptr : i < 1; ++i)
        failed |= (c->multi ? esc::multi_sub(c, i) : c)->ord_failed;
    if (failed) return ESC_E_ORDER;
    const int32_t G = c0->gi.G;
    int64_t total = 0;
    offsets[0] = 0;
    for (int32_t g = 0; g < G; ++g) {
        const uint32_t* nodes = nullptr;
        int64_t n = 0;
        if (int32_t rc = group_selection(c, g, &which[g], &nodes, &n)) return rc;
        if (idx && total + n <= cap)
            for (int64_t k = 0; k < n; ++k) idx[total + k] = nodes[k];
        total += n;
        offsets[g + 1] = total;
    }
    *n_total = total;
    return idx && total > cap ? ESC_E_LIMIT : ESC_OK;
}

// ------------------------------------------------- RCCL exchange (§8e) inside the library
int32_t esc_comm_unique_id(void* id_out) {
    if (!id_out) return ESC_E_INVAL;
    if (!rccl().ok) return fail_comm("esc_comm_unique_id", "librccl not found");
    ncclUniqueId id;
    const ncclResult_t r = rccl().get_unique_id(&id);
    if (r != ncclSuccess) return fail_comm("ncclGetUniqueId", rccl().error_string(r));
    static_assert(sizeof(ncclUniqueId) == ESC_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id_out, &id, sizeof id);
    return ESC_OK;
}

int32_t esc_comm_init(esc_ctx* c, const void* id, int32_t rank, int32_t world) {
    if (c && c->multi) return ESC_E_STATE;              // esc_ctx_create_multi made its communicators
    if (!c || !id) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (rank != c->rank || world != c->world || c->comm) return ESC_E_STATE;
    if (!rccl().ok) return fail_comm("esc_comm_init", "librccl not found");
    hipSetDevice(c->device);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = rccl().init_rank(&comm, world, uid, rank);
    if (r != ncclSuccess) return fail_comm("ncclCommInitRank", rccl().error_string(r));
    c->comm = comm;
    return ESC_OK;
}

int32_t esc_exchange(esc_ctx* c) {
    if (c && c->multi) return ESC_E_STATE;
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (!c->comm) return ESC_E_STATE;
    hipSetDevice(c->device);
    // int64 SUM is exact in any order (the pod words are split lo32 / hi): one in-place
    // reduce-scatter leaves every owner the sums of its own groups' rows; the
    // node words never travel (each owner computed its own)
    const ncclResult_t r = rccl().reduce_scatter(c->d_pwords, own_xwords(c), (size_t)c->own_cap * PW_K, ncclInt64,
                                                 ncclSum, reinterpret_cast<ncclComm_t>(c->comm), c->stream);
    if (r != ncclSuccess) return fail_comm("ncclReduceScatter", rccl().error_string(r));
    if (int32_t rc = stage_mark(c)) return rc;
    c->pending = true;
    return ESC_OK;
}

int32_t esc_step(esc_ctx* c) {
    if (c && c->multi) return esc::multi_step(c);
    int32_t rc = check_ready(c);
    if (rc) return rc;
    if (!c->comm) return c->world == 1 ? esc_run(c) : ESC_E_STATE;
    if ((rc = esc_reduce(c)) != ESC_OK) return rc;
    if ((rc = esc_exchange(c)) != ESC_OK) return rc;
    return esc_decide(c);
}

int32_t esc_sync(esc_ctx* c) {
    if (c && c->multi) return esc::multi_sync(c);
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->timing && c->pending && c->n_stage_ev > 1) {
        float ms = 0;
        for (int i = 0; i + 1 < c->n_stage_ev; ++i) {
            HIP_TRY(hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]));
            c->stage_ms[i] = ms;
        }
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[c->n_stage_ev - 1]));
        c->stage_ms[MAX_STAGES - 1] = ms;
    }
    c->pending = false;
    // an ordering whose look-back gave up: reported once (its orderings stay refused by
    // esc_group_order until the next ordering), the next decision orders afresh
    return order_gave_up(c) ? ESC_E_ORDER : ESC_OK;
}

int32_t esc_results(esc_ctx* c, esc_group_totals* totals, esc_group_decision* decisions) {
    if (c && c->multi) return esc::multi_results(c, totals, decisions);
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->work_ready) return ESC_E_STATE;
    int32_t rc = esc_sync(c);
    if (rc && rc != ESC_E_ORDER) return rc;           // a failed ordering leaves totals and decisions valid
    const int32_t G = c->gi.G;
    // With several ranks a rank decides its own groups only: the others'
    // records come back zeroed, flagged ESC_TF_NOT_OWNED / ESC_ST_NOT_OWNED.
    auto mine = [&](int32_t g) { return c->world == 1 || group_owner_rank(c, g) == c->rank; };
    if (decisions) {
        // the compact records -> esc_group_decision (cached capacity: allNodes[0]'s allocatable
        // when the group has nodes, else the state's, controller.go:207-211)
        for (int32_t g = 0; g < G; ++g) {
            const DecCompact& x = c->h_cdec[g];
            esc_group_decision& d = decisions[g];
            if (!mine(g)) {
                std::memset(&d, 0, sizeof d);
                d.status = ESC_ST_NOT_OWNED;
                continue;
            }
            if (x.wide) {                                // delta / n_to_taint beyond int32
                HIP_TRY(hipMemcpy(&d, c->d_dec + g, sizeof d, hipMemcpyDeviceToHost));
                continue;
            }
            d.cpu_pct = x.cpu_pct;
            d.mem_pct = x.mem_pct;
            d.delta = x.delta;
            d.n_to_taint = x.n_to_taint;
            const GroupNode& gn = c->h_gnode[g];
            d.cached_cpu_m = gn.first != INT64_MAX ? gn.first_cpu : c->params[g].cached_cpu;
            d.cached_mem_b = gn.first != INT64_MAX ? gn.first_mem : c->params[g].cached_mem;
            d.status = x.status;
            d.branch = x.branch;
            d.taint_status = x.taint_status;
            d.reserved = 0;
        }
    }
    if (totals && c->h_tot && c->tot_dec) {
        // small contexts: K4 wrote every decided group's record to pinned memory (the answer
        // a controller's CalculatePodsRequestsTotal takes from the batched decision)
        for (int32_t g = 0; g < G; ++g) {
            if (mine(g)) {
                totals[g] = c->h_tot[g];
                continue;
            }
            std::memset(&totals[g], 0, sizeof totals[g]);
            totals[g].first_node = -1;
            totals[g].flags = ESC_TF_NOT_OWNED;
        }
    } else if (totals) {
        // both word arrays into one pinned buffer, one queued copy (two when the pod words are
        // a bound buffer) and one wait
        const size_t nwp = (size_t)(c->d_nwords - c->own_pwords), nwn = (size_t)G * NW_K;   // nwp >= xw_count
        if (nwp + nwn > c->words_cap) {
            if (c->h_words) hipHostFree(c->h_words);
            c->h_words = nullptr;
            c->words_cap = 0;
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_words), (nwp + nwn) * 8));
            c->words_cap = nwp + nwn;
        }
        if (c->d_pwords == c->own_pwords) {              // adjacent (the context's own pod words)
            HIP_TRY(hipMemcpyAsync(c->h_words, c->d_pwords, (nwp + nwn) * 8, hipMemcpyDeviceToHost, c->stream));
        } else {
            HIP_TRY(hipMemcpyAsync(c->h_words, c->d_pwords, (size_t)xw_count(c) * 8, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipMemcpyAsync(c->h_words + nwp, c->d_nwords, nwn * 8, hipMemcpyDeviceToHost, c->stream));
        }
        HIP_TRY(hipStreamSynchronize(c->stream));
        const int64_t* w = c->h_words;
        const int64_t* nw = c->h_words + nwp;
        for (int32_t g = 0; g < G; ++g) {
            if (!mine(g)) {
                std::memset(&totals[g], 0, sizeof totals[g]);
                totals[g].first_node = -1;
                totals[g].flags = ESC_TF_NOT_OWNED;
                continue;
            }
            const int64_t* x = w + (size_t)(c->world > 1 ? c->h_xs[(size_t)g] : (uint32_t)g) * PW_K;
            const int64_t* y = nw + (size_t)g * NW_K;
            esc_group_totals& t = totals[g];
            auto join = [&](int k, int64_t& out) {
                const __int128 v = ((__int128)x[k + 1] << 32) + (__int128)x[k];
                out = (int64_t)v;
                return v >= (__int128)INT64_MIN && v <= (__int128)INT64_MAX;
            };
            t.flags = y[NW_FLAGS];
            if (!join(PW_CPU_LO, t.pod_cpu_m)) t.flags |= ESC_TF_POD_OVERFLOW;
            if (!join(PW_MEM_LO, t.pod_mem_b)) t.flags |= ESC_TF_POD_OVERFLOW;
            t.n_pods = x[PW_N];
            t.node_cpu_m = y[NW_CPU];
            t.node_mem_b = y[NW_MEM];
            t.n_untainted = y[NW_N_UNT];
            t.n_tainted = y[NW_N_TAINT];
            t.n_cordoned = y[NW_N_CORD];
            t.n_nodes = t.n_untainted + t.n_tainted + t.n_cordoned;
            const int64_t first = c->h_gnode[g].first;
            t.first_node = first == INT64_MAX ? -1 : first;
            t.first_cpu_m = t.first_node >= 0 ? c->h_ncpu[t.first_node] : 0;
            t.first_mem_b = t.first_node >= 0 ? c->h_nmem[t.first_node] : 0;
        }
    }
    return ESC_OK;
}

// ------------------------------------------------ incremental snapshot (§8f rank 1)
}  // extern "C"

namespace {

struct Patches {
    std::vector<uint64_t> where, what;
    void add(uint32_t target, int64_t idx, uint64_t v) {
        where.push_back(((uint64_t)target << 60) | (uint64_t)idx);
        what.push_back(v);
    }
};

// Applies a batch (last write per element wins) to `targets` of every replica.
int32_t apply_patches(esc_ctx* c, Patches& P, const std::vector<PatchTargets>& targets) {
    const int64_t n = (int64_t)P.where.size();
    if (n == 0) return ESC_OK;
    std::vector<int64_t> ord(n);
    for (int64_t i = 0; i < n; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return P.where[a] < P.where[b]; });
    std::vector<uint64_t> w, v;
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = ord[k];
        if (k + 1 < n && P.where[ord[k + 1]] == P.where[i]) continue;      // a later write wins
        w.push_back(P.where[i]);
        v.push_back(P.what[i]);
    }
    uint64_t *dw = nullptr, *dv = nullptr;
    HIP_TRY(dalloc(&dw, w.size()));
    HIP_TRY(dalloc(&dv, v.size()));
    int32_t rc = ESC_OK;
    if (hipMemcpy(dw, w.data(), w.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dv, v.data(), v.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
        rc = ESC_E_HIP;
#if ESC_MEASURE
    if (!rc && c->fail_patches > 0) {                  // injected (esc_debug_fail_patches)
        --c->fail_patches;
        rc = fail_hip(hipErrorUnknown, "injected patch failure");
    }
#endif
    for (const PatchTargets& t : targets)
        if (!rc && launch_patch(t, dw, dv, (int64_t)w.size(), c->stream) != hipSuccess) rc = ESC_E_HIP;
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = ESC_E_HIP;
    dfree(dw);
    dfree(dv);
    return rc;
}

// C-section arrays (C index) and the K blocks as 4- and 8-byte words
enum : uint32_t { PT_FLAGS = 0, PT_CPU0 = 1, PT_PAIR0 = 2, PT_XP = 3, PT_KB32 = 4, PT_MEM0 = 6, PT_XC_CPU = 7,
                  PT_XC_MEM = 8, PT_KB64 = 9, PT_KB16 = 12 };
// the K-block patch target of a kb_write_pod / kb_write_free put of the given width
uint32_t pt_kb(int width) { return width == 8 ? PT_KB64 : (width == 4 ? PT_KB32 : PT_KB16); }

std::vector<PatchTargets> pod_targets(esc_ctx* c) {
    std::vector<PatchTargets> v;
    for (PodBuf& b : c->pods) {
        PatchTargets t{};
        t.u32[PT_FLAGS] = b.flags; t.u32[PT_CPU0] = b.cpu0; t.u32[PT_PAIR0] = b.pair0; t.u32[PT_XP] = b.xp;
        t.i64[PT_MEM0 - 6] = b.mem0; t.i64[PT_XC_CPU - 6] = b.xc_cpu; t.i64[PT_XC_MEM - 6] = b.xc_mem;
        t.u32[PT_KB32] = b.kb; t.i64[PT_KB64 - 6] = reinterpret_cast<int64_t*>(b.kb);
        t.u16[PT_KB16 - 12] = reinterpret_cast<uint16_t*>(b.kb);
        v.push_back(t);
    }
    return v;
}

// Removes pod `id` from the snapshot (its slot becomes padding: daemonset-flagged, which
// every kernel skips; a C pod keeps its record counts so its tile's offsets stay valid).
void remove_pod(esc_ctx* c, int64_t id, Patches& P) {
    const int32_t ci = c->pod_cls[id];
    if (ci == -2) return;
    if (ci == -1) {
        const int64_t d = c->pod_pos[id] - c->k_tiles * TILE;    // C-array index
        uint32_t& f = c->h_cflags[d];
        c->live_xc -= c->h_cused[d] & 0xFFFF;
        c->live_xp -= c->h_cused[d] >> 16;
        c->h_cused[d] = 0;
        f |= ESC_PF_DAEMONSET;
        P.add(PT_FLAGS, d, f);
        c->c_free.push_back(d);                           // its room (counts) stays: reusable
    } else {
        const PodClass& k = c->h_cls[ci];
        const int64_t q = c->pod_pos[id];
        kb_write_free(k, kb_block(k, k.t0 + q / TILE), q % TILE,
                      [&](int width, int64_t at, uint64_t v) { P.add(pt_kb(width), at, v); });
        c->cls_free[ci].push_back(q);
        c->live_xc -= k.xreg + k.xinit + k.ovh;
        c->live_xp -= k.nxp;
        if (k.packed) { --c->live_pk_pods; c->live_pk_xc -= k.xreg + k.xinit + k.ovh; }
        if (k.packed == 2) { --c->live_p8_pods; c->live_p8_xp -= k.nxp; }
    }
    c->pod_cls[id] = -2;
    --c->live_pods;
}

// Device slot of live pod `id` in the resident layout (K section: class tiles; C section:
// its position).
int64_t pod_slot(const esc_ctx* c, int64_t id) {
    const int32_t ci = c->pod_cls[id];
    const int64_t d = c->pod_pos[id];
    return ci >= 0 ? (c->h_cls[ci].t0 + d / TILE) * TILE + d % TILE : d;
}

RemovalDev removal_dev(const esc_ctx* c, int64_t now_ns);

// The maintained occupancy words (see esc_ctx::d_occ_local) as K6 / the deltas address them.
RemovalDev occ_dev(const esc_ctx* c) {
    RemovalDev r = removal_dev(c, 0);
    uint32_t* o = c->d_occ_local ? c->d_occ_local : c->d_occ;
    r.occ_pair = o;
    r.occ_def = o + std::max<int64_t>(c->n_entries, 0);
    return r;
}

// Device copy of the node -> entries map (node slots up to n_cap, entries up to n_entries).
int32_t ensure_ne_dev(esc_ctx* c) {
    const int64_t nn = (int64_t)c->ne_off.size() - 1, np = (int64_t)c->ne_pos.size();
    if (nn == c->ne_dev_nodes && np == c->ne_dev_pos) return ESC_OK;
    if (!c->d_ne_off) {
        HIP_TRY(dalloc(&c->d_ne_off, (size_t)std::max<int64_t>(c->n_cap, nn) + 1));
        HIP_TRY(dalloc(&c->d_ne_pos, (size_t)std::max<int64_t>(c->n_entries, std::max<int64_t>(np, 1))));
    }
    std::vector<uint32_t> off(c->ne_off);
    off.resize((size_t)std::max<int64_t>(c->n_cap, nn) + 1, c->ne_off.back());   // free slots: no entries
    HIP_TRY(hipMemcpy(c->d_ne_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    if (np) HIP_TRY(hipMemcpy(c->d_ne_pos, c->ne_pos.data(), (size_t)np * 4, hipMemcpyHostToDevice));
    c->ne_dev_nodes = nn;
    c->ne_dev_pos = np;
    return ESC_OK;
}

// K6 over every live entry into the maintained words (esc_load_placement).
int32_t occ_recount(esc_ctx* c) {
    if (int32_t rc = ensure_ne_dev(c)) return rc;
    HIP_TRY(launch_occupancy(node_dev(c), group_dev(c), occ_dev(c), c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ESC_OK;
}

// The PodRefs now at run positions pos (on nodes node) added to (+1) or removed from (-1)
// the maintained occupancy words: called before the runs change for the pods an event
// moves or drops, and after for the pods it binds or rewrites.
int32_t occ_delta(esc_ctx* c, const std::vector<uint32_t>& pos, const std::vector<uint32_t>& node, int sign) {
    if (!c->placed || pos.empty()) return ESC_OK;
    if (int32_t rc = ensure_ne_dev(c)) return rc;
    uint32_t *dp = nullptr, *dn = nullptr;
    HIP_TRY(dalloc(&dp, pos.size()));
    HIP_TRY(dalloc(&dn, node.size()));
    hipError_t e = hipMemcpy(dp, pos.data(), pos.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dn, node.data(), node.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = launch_occ_delta(group_dev(c), occ_dev(c), c->d_ne_off, c->d_ne_pos, dp, dn, (int64_t)pos.size(), sign, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree(dp);
    dfree(dn);
    HIP_TRY(e);
    return ESC_OK;
}

// (position, node) of every bound pod among ids
void bound_of(const esc_ctx* c, const int64_t* ids, int64_t n, std::vector<uint32_t>& pos, std::vector<uint32_t>& node) {
    pos.clear();
    node.clear();
    for (int64_t i = 0; i < n; ++i) {
        const int64_t id = ids[i];
        if (id >= 0 && id < (int64_t)c->h_pod_rpos.size() && c->h_pod_rpos[id] >= 0) {
            pos.push_back((uint32_t)c->h_pod_rpos[id]);
            node.push_back(c->h_pod_node[id]);
        }
    }
}

RemovalDev removal_dev(const esc_ctx* c, int64_t now_ns) {
    RemovalDev r;
    r.e_pair = c->d_e_pair; r.n_entries = c->n_entries;
    r.taint_s = c->d_taint_s; r.no_delete = c->d_no_delete;
    r.nrun_off = c->d_nrun_off; r.nrun_len = c->d_nrun_len; r.refs = c->d_refs;
    r.xp = c->pods[c->cur].xp;
    r.occ_pair = c->d_occ; r.occ_def = c->d_occ + std::max<int64_t>(c->n_entries, 0);
    r.soft_ns = c->d_soft; r.hard_ns = c->d_hard;
    r.rm_off = c->d_rm_off; r.rm_list = c->d_rm_list; r.out = c->d_rm_out; r.now_ns = now_ns;
    return r;
}

// Placement upkeep under pod events (§8f rank 2): a bound pod's PodRef lives in its node's
// run; removal swaps the run's last PodRef into the hole, binding appends.  `touched`
// collects pods whose PodRef must be (re)written (new position or new slot), `runs` the
// nodes whose run length changed; sync_placement writes both after the pod data patches.
void run_remove(esc_ctx* c, int64_t id, std::vector<int64_t>& touched, std::vector<uint32_t>& runs) {
    if (id >= (int64_t)c->h_pod_rpos.size() || c->h_pod_rpos[id] < 0) return;
    const uint32_t j = c->h_pod_node[id];
    const int64_t pos = c->h_pod_rpos[id], last = (int64_t)c->h_run_off[j] + c->h_run_len[j] - 1;
    if (pos != last) {
        const int32_t moved = c->h_run_pod[last];
        c->h_run_pod[pos] = moved;
        c->h_pod_rpos[moved] = pos;
        touched.push_back(moved);
    }
    c->h_run_pod[last] = -1;
    --c->h_run_len[j];
    runs.push_back(j);
    c->h_pod_rpos[id] = -1;
    c->h_pod_node[id] = NONE;
}

bool run_append(esc_ctx* c, int64_t id, uint32_t j, std::vector<int64_t>& touched, std::vector<uint32_t>& runs) {
    if (c->h_run_len[j] >= c->h_run_off[j + 1] - c->h_run_off[j]) return false;
    const int64_t pos = (int64_t)c->h_run_off[j] + c->h_run_len[j]++;
    c->h_run_pod[pos] = (int32_t)id;
    c->h_pod_rpos[id] = pos;
    c->h_pod_node[id] = j;
    touched.push_back(id);
    runs.push_back(j);
    return true;
}

int32_t sync_placement(esc_ctx* c, std::vector<int64_t>& touched, std::vector<uint32_t>& runs) {
    std::sort(touched.begin(), touched.end());
    touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
    std::vector<uint32_t> pos, slot;
    for (int64_t id : touched)
        if (id < (int64_t)c->h_pod_rpos.size() && c->h_pod_rpos[id] >= 0 && c->pod_cls[id] != -2) {
            pos.push_back((uint32_t)c->h_pod_rpos[id]);
            slot.push_back((uint32_t)pod_slot(c, id));
        }
    if (!pos.empty()) {
        uint32_t *dp = nullptr, *ds = nullptr;
        HIP_TRY(dalloc(&dp, pos.size()));
        HIP_TRY(dalloc(&ds, slot.size()));
        hipError_t e = hipMemcpy(dp, pos.data(), pos.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(ds, slot.data(), slot.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = launch_podref_fill(pod_dev(c, c->cur), ds, dp, (int64_t)pos.size(), c->d_refs, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        dfree(dp);
        dfree(ds);
        HIP_TRY(e);
    }
    if (!runs.empty()) {
        Patches P;
        for (uint32_t j : runs) P.add(0, j, c->h_run_len[j]);
        PatchTargets t{};
        t.u32[0] = c->d_nrun_len;
        int32_t rc = apply_patches(c, P, {t});
        if (rc) return rc;
    }
    c->rm_valid = false;
    return ESC_OK;
}

// ---- node events: host views of the node memberships and the K5 group regions
// Groups of node j (its label pairs through the node codes, dry bit included), as the
// kernels' node_groups lists them.
void node_membs(const esc_ctx* c, int64_t j, std::vector<uint32_t>& out) {
    out.clear();
    if (c->h_nflags[j] & ESC_NF_ABSENT) return;
    auto add = [&](uint32_t q) {
        if (q >= c->gi.n_gp) return;
        const uint32_t code = c->gi.node_code[q];
        if (code < CODE_MULTI) out.push_back(code);
        else if (code != NONE) {
            const uint32_t* l = c->gi.code_list.data() + (code & ~CODE_MULTI);
            for (uint32_t k = 1; k <= l[0]; ++k) out.push_back(l[k]);
        }
    };
    add(c->h_label0[j]);
    const uint32_t nx = nf_xlbl(c->h_nflags[j]);
    for (uint32_t k = 0; k < nx; ++k) add(c->h_xl[c->h_xl_off[j] + k]);
}

// Groups of a node given its label pairs (before it is in the mirrors).
void node_membs_from(const esc_ctx* c, uint32_t label0, uint32_t nx, const uint32_t* xl, std::vector<uint32_t>& out) {
    out.clear();
    auto add = [&](uint32_t q) {
        if (q >= c->gi.n_gp) return;
        const uint32_t code = c->gi.node_code[q];
        if (code < CODE_MULTI) out.push_back(code);
        else if (code != NONE) {
            const uint32_t* l = c->gi.code_list.data() + (code & ~CODE_MULTI);
            for (uint32_t k = 1; k <= l[0]; ++k) out.push_back(l[k]);
        }
    };
    add(label0);
    for (uint32_t k = 0; k < nx; ++k) add(xl[k]);
}

// The K5 copy of node j's flags for membership mb: a dry group's copy carries "tracked by
// this group" in the tracker bit (as k_memb_expand lists it).
uint32_t memb_flags(const esc_ctx* c, int64_t j, uint32_t mb) {
    const uint32_t f = c->h_nflags[j];
    if (!(mb & NODE_DRY_BIT)) return f;
    const uint64_t key = ((uint64_t)(uint32_t)j << 32) | (mb & NODE_GROUP_MASK);
    const bool tr = (f & ESC_NF_TRACKED) && std::binary_search(c->h_trk.begin(), c->h_trk.end(), key);
    return (f & ~ESC_NF_TRACKED) | (tr ? ESC_NF_TRACKED : 0u);
}

int64_t created_of(const esc_ctx* c, uint32_t j) { return c->h_created[(int64_t)j - c->node_lo]; }

// Does this rank own group g's node side (its pair in [q_lo, q_hi))?
bool owns_group(const esc_ctx* c, uint32_t g) {
    const uint32_t q = c->gi.gpair[g];
    return q >= c->q_lo && q < c->q_hi;
}

// Host mirror of the regions' node ids (fetched once, then kept in step with every patch).
int32_t ensure_gn(esc_ctx* c) {
    if ((int64_t)c->h_gn.size() == c->n_gpad) return ESC_OK;
    c->h_gn.resize(c->n_gpad);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->n_gpad) HIP_TRY(hipMemcpy(c->h_gn.data(), c->d_g_memb, c->n_gpad * 4, hipMemcpyDeviceToHost));
    for (uint32_t& x : c->h_gn) x &= MEMB_NODE_MASK;             // the node ids (the flags live on the device)
    return ESC_OK;
}

// Position of node j's membership in group g's region (regions are ordered by creation
// time, ties by index), or -1.
int64_t region_pos(const esc_ctx* c, uint32_t g, uint32_t j) {
    const uint32_t a = c->h_pstart[g], z = a + c->h_plen[g];
    const int64_t t = created_of(c, j);
    const uint32_t* b = c->h_gn.data();
    const uint32_t* it = std::lower_bound(b + a, b + z, j, [&](uint32_t x, uint32_t y) {
        const int64_t tx = created_of(c, x);
        return tx < t || (tx == t && x < y);
    });
    return (it != b + z && *it == j) ? (int64_t)(it - b) : -1;
}

enum : uint32_t { NT_FLAGS = 0, NT_EFLAGS = 1, NT_LABEL0 = 2, NT_XLOFF = 3, NT_ENODE = 4, NT_XL = 5, NT_CPU = 6,
                  NT_MEM = 7, NT_ECPU = 8, NT_EMEM = 9, NT_CREATED = 10, NT_EPK = 11 };

// Pair-major entry e's flags, cpu and memory: the three arrays and the packed record (as two
// 8-B words: flags | cpu << 32, memory).  A cpu the record cannot hold switches K2 to the
// arrays for the rest of the snapshot (the captured steps hold the packed pointer).
void entry_patch(esc_ctx* c, Patches& P, uint32_t e, uint32_t f, int64_t cpu, int64_t mem) {
    P.add(NT_EFLAGS, e, f);
    P.add(NT_ECPU, e, (uint64_t)cpu);
    P.add(NT_EMEM, e, (uint64_t)mem);
    P.add(NT_EPK, 2 * (int64_t)e, (uint64_t)f | (uint64_t)(uint32_t)cpu << 32);
    P.add(NT_EPK, 2 * (int64_t)e + 1, (uint64_t)mem);
    if (c->e_pk_ok && !entry_cpu_packs(cpu) && !(f & ESC_NF_ABSENT)) {
        c->e_pk_ok = false;
        drop_graphs(c);
    }
}

PatchTargets node_targets(esc_ctx* c) {
    PatchTargets t{};
    t.u32[NT_FLAGS] = c->nodes.flags; t.u32[NT_EFLAGS] = c->nodes.e_flags; t.u32[NT_LABEL0] = c->nodes.label0;
    t.u32[NT_XLOFF] = c->nodes.xl_off; t.u32[NT_ENODE] = c->nodes.e_node; t.u32[NT_XL] = c->nodes.xl;
    t.i64[NT_CPU - 6] = c->nodes.cpu; t.i64[NT_MEM - 6] = c->nodes.mem;
    t.i64[NT_ECPU - 6] = c->nodes.e_cpu; t.i64[NT_EMEM - 6] = c->nodes.e_mem;
    t.i64[NT_EPK - 6] = reinterpret_cast<int64_t*>(c->nodes.e_pk);
    t.i64[NT_CREATED - 6] = c->nodes.created;
    return t;
}

// K5 region copies of the memberships of nodes `ids` (their flags, as the split reads them).
int32_t patch_regions(esc_ctx* c, const std::vector<int64_t>& ids) {
    if (!c->n_gpad) return ESC_OK;
    int32_t rc = ensure_gn(c);
    if (rc) return rc;
    Patches P;
    std::vector<uint32_t> mb;
    for (int64_t j : ids) {
        const bool gone = (c->h_nflags[j] & ESC_NF_ABSENT) != 0;
        if (gone) {                                                   // the memberships it had
            uint32_t f = c->h_nflags[j];
            c->h_nflags[j] &= ~ESC_NF_ABSENT;
            node_membs(c, j, mb);
            c->h_nflags[j] = f;
        } else {
            node_membs(c, j, mb);
        }
        for (uint32_t m : mb) {
            if (!owns_group(c, m & NODE_GROUP_MASK)) continue;          // another rank's K5 region
            const int64_t pos = region_pos(c, m & NODE_GROUP_MASK, (uint32_t)j);
            if (pos < 0) return ESC_E_HIP;                            // mirror out of step: never expected
            P.add(0, pos, memb_word((uint32_t)j, gone ? ESC_NF_ABSENT : memb_flags(c, j, m)));
        }
    }
    PatchTargets t{};
    t.u32[0] = c->d_g_memb;
    return apply_patches(c, P, {t});
}

// allNodes[0] (controller.go:207-211) of a group with pair q: its lowest live member,
// over every entry of the pair (a relabelled node's entry sits after the others, so the
// pair's entries are not always in index order).
void pair_first(const esc_ctx* c, uint32_t q, GroupNode& x) {
    const uint32_t a = c->pair_lo[q], z = c->pair_next.empty() ? a : c->pair_next[q];
    x.first = INT64_MAX;
    x.first_cpu = x.first_mem = 0;
    for (uint32_t e = a; e < z; ++e) {
        const uint32_t j = c->h_e_node[e];
        if (j != NONE && (int64_t)j < x.first && !(c->h_nflags[j] & ESC_NF_ABSENT)) x.first = j;
    }
    if (x.first != INT64_MAX) {
        x.first_cpu = c->h_ncpu[x.first];
        x.first_mem = c->h_nmem[x.first];
    }
}

// Patch targets of the K5 regions: membership word (node | flags), the groups' tie flags.
PatchTargets region_targets(esc_ctx* c) {
    PatchTargets t{};
    t.u32[0] = c->d_g_memb;
    t.u32[1] = c->d_g_tie;
    return t;
}

// Node events, K5 regions: insert the nodes `add_by_g[g]` into the regions of the groups g
// (owned by this rank) at their place by (creation time, index); every touched region is
// rewritten from its first insertion on (one scatter for all of them, into R).
void regions_insert(esc_ctx* c, std::unordered_map<uint32_t, std::vector<uint32_t>>& add_by_g, Patches& R) {
    auto less = [&](uint32_t x, uint32_t y) {
        const int64_t tx = created_of(c, x), ty = created_of(c, y);
        return tx < ty || (tx == ty && x < y);
    };
    for (auto& kv : add_by_g) {
        const uint32_t g = kv.first;
        std::vector<uint32_t>& nw = kv.second;
        if (nw.empty()) continue;
        std::sort(nw.begin(), nw.end(), less);
        const uint32_t a = c->h_pstart[g], len = c->h_plen[g];
        uint32_t* run = c->h_gn.data() + a;
        const uint32_t from = (uint32_t)(std::upper_bound(run, run + len, nw.front(), less) - run);
        std::vector<uint32_t> merged(len - from + nw.size());
        std::merge(run + from, run + len, nw.begin(), nw.end(), merged.begin(), less);
        std::copy(merged.begin(), merged.end(), run + from);
        c->h_plen[g] = len + (uint32_t)nw.size();
        // equal creation times side by side from the insertion on: the group's selections take
        // the tie rule from now on (RegionSink::tie; a removal never clears the flag)
        bool tie = false;
        for (size_t k = 0; k < merged.size() && !tie; ++k) {
            const int64_t prev = k ? (int64_t)merged[k - 1] : (from ? (int64_t)run[from - 1] : -1);
            tie = prev >= 0 && created_of(c, (uint32_t)prev) == created_of(c, merged[k]);
        }
        if (tie) R.add(1, g, 1);
        const uint32_t mbit = (uint32_t)g | (c->params[g].dry ? NODE_DRY_BIT : 0u);
        for (size_t k = 0; k < merged.size(); ++k) {
            const int64_t pos = (int64_t)a + from + (int64_t)k;
            R.add(0, pos, memb_word(merged[k], (c->h_nflags[merged[k]] & ESC_NF_ABSENT) ? ESC_NF_ABSENT
                                                                                       : memb_flags(c, merged[k], mbit)));
        }
    }
}

// Node events, K5 regions: take node j's membership out of group g's region (owned by this
// rank; found by the node's CURRENT creation time): the region's tail moves up one slot and
// its last slot becomes padding (MEMB_PAD_WORD, absent), as k_region_pad writes it.
bool region_remove(esc_ctx* c, uint32_t g, uint32_t j, Patches& R) {
    const int64_t pos = region_pos(c, g, j);
    if (pos < 0) return false;
    const uint32_t a = c->h_pstart[g], len = c->h_plen[g];
    const int64_t last = (int64_t)a + len - 1;
    uint32_t* gn = c->h_gn.data();
    const uint32_t mbit = (uint32_t)g | (c->params[g].dry ? NODE_DRY_BIT : 0u);
    for (int64_t k = pos; k < last; ++k) {
        gn[k] = gn[k + 1];
        R.add(0, k, memb_word(gn[k], (c->h_nflags[gn[k]] & ESC_NF_ABSENT) ? ESC_NF_ABSENT : memb_flags(c, gn[k], mbit)));
    }
    gn[last] = 0;
    R.add(0, last, MEMB_PAD_WORD);
    c->h_plen[g] = len - 1;
    return true;
}

// Writes the host mirrors (h_nflags / h_ncpu / h_nmem) of nodes `ids` to the device:
// the node table, the nodes' pair-major K2 entries, allNodes[0]'s cached allocatable,
// and the K5 region copies (looked up by creation time: no re-listing).
int32_t patch_nodes(esc_ctx* c, const std::vector<int64_t>& ids) {
    c->rm_valid = false;
    Patches P;
    bool first_changed = false;
    for (int64_t j : ids) {
        const uint32_t f = c->h_nflags[j];
        const uint64_t cpu = (uint64_t)c->h_ncpu[j], mem = (uint64_t)c->h_nmem[j];
        P.add(NT_FLAGS, j, f);
        P.add(NT_CPU, j, cpu);
        P.add(NT_MEM, j, mem);
        for (uint32_t e = c->ne_off[j]; e < c->ne_off[j + 1]; ++e) {
            if (c->h_e_node[c->ne_pos[e]] != (uint32_t)j) continue;   // an entry a relabel retired
            entry_patch(c, P, c->ne_pos[e], f, (int64_t)cpu, (int64_t)mem);
        }
    }
    for (GroupNode& g : c->h_gnode)                  // allNodes[0]'s allocatable (controller.go:208)
        if (g.first != INT64_MAX && (g.first_cpu != c->h_ncpu[g.first] || g.first_mem != c->h_nmem[g.first])) {
            g.first_cpu = c->h_ncpu[g.first];
            g.first_mem = c->h_nmem[g.first];
            first_changed = true;
        }
    int32_t rc = apply_patches(c, P, {node_targets(c)});
    if (rc) return rc;
    if (first_changed)
        HIP_TRY(hipMemcpy(c->nodes.gnode, c->h_gnode.data(), c->h_gnode.size() * sizeof(GroupNode), hipMemcpyHostToDevice));
    rc = patch_regions(c, ids);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->sorted = false;
    return ESC_OK;
}

// The tracker list (sorted (node << 32 | group)) and its per-node first-entry index on the
// device; graphs are dropped (K2's grid and NodeDev carry n_trk).
int32_t write_tracker(esc_ctx* c, std::vector<uint64_t>& next) {
    const int64_t nt = (int64_t)next.size();
    NodeBuf& b = c->nodes;
    if (nt > c->trk_cap) {
        const int64_t cap = std::max<int64_t>({nt, 2 * c->trk_cap, 1024});
        dfree(b.trk_node); dfree(b.trk_group);
        b.trk_node = nullptr; b.trk_group = nullptr;
        HIP_TRY(dalloc(&b.trk_node, cap)); HIP_TRY(dalloc(&b.trk_group, cap));
        c->trk_cap = cap;
    }
    std::vector<int32_t> tn(std::max<int64_t>(nt, 1)), tg(std::max<int64_t>(nt, 1));
    std::vector<uint32_t> ts(std::max<int64_t>(c->n_cap, 1), NONE);
    for (int64_t k = nt - 1; k >= 0; --k) {
        tn[k] = (int32_t)(next[k] >> 32);
        tg[k] = (int32_t)(uint32_t)next[k];
        ts[tn[k]] = (uint32_t)k;
    }
    if (nt) {
        HIP_TRY(hipMemcpy(b.trk_node, tn.data(), nt * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(b.trk_group, tg.data(), nt * 4, hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemcpy(b.trk_start, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
    c->h_trk.swap(next);
    c->n_trk = nt;
    drop_graphs(c);
    return ESC_OK;
}

}  // namespace

extern "C" {

int32_t esc_set_spare(esc_ctx* c, double fraction) {
    if (c && c->multi) { for (int i = 0; esc::multi_sub(c, i); ++i) if (int32_t rc = esc_set_spare(esc::multi_sub(c, i), fraction)) return rc; return ESC_OK; }
    if (!c || !(fraction >= 0.0) || fraction > 4.0) return ESC_E_INVAL;
    c->spare_frac = fraction;                      // applies from the next esc_load_pods
    return ESC_OK;
}

}  // extern "C"

namespace {
// esc_pods_upsert in two phases, so that a multi-device context can check every device's
// share of a batch before it applies any (all or nothing across devices too).
struct UpsertPlan {
    std::vector<int64_t> rof, pof;   // each pod's first record / extra pair in the batch
    std::vector<int32_t> tgt;        // its K class, or -1: the C slot cslot
    std::vector<int64_t> cslot;
};

// Does C slot room `cf` (counts of a slot's flags) hold a pod with flags f?  Its records
// and pairs take the slot's first positions of each kind, the rest stay neutral.
bool c_room(uint32_t cf, uint32_t f) {
    return pf_xreg(f) <= pf_xreg(cf) && pf_xinit(f) <= pf_xinit(cf) && (!(f & ESC_PF_HAS_OVH) || (cf & ESC_PF_HAS_OVH)) &&
           pf_xpair(f) <= pf_xpair(cf);
}

bool touch_mark_c(esc_ctx* c, int64_t d, uint32_t f, uint32_t pair0, const uint32_t* xp);

// Writes pod i of the batch into C slot d (its room: the slot's flags' counts; the pod's
// records and pairs first of each kind, the rest neutral — 0 for added records, absent keys
// for init containers, NONE for pairs).  True when K1's touched columns grew.
bool upsert_c(esc_ctx* c, int64_t id, int64_t d, const esc_pod_soa* p, int64_t i, int64_t rof, int64_t pof, Patches& P) {
    const int64_t c0 = c->k_tiles * TILE;
    if (!(c->pod_cls[id] == -1 && c->pod_pos[id] - c0 == d)) {
        remove_pod(c, id, P);
        auto it = std::find(c->c_free.begin(), c->c_free.end(), d);
        if (it != c->c_free.end()) c->c_free.erase(it);
        c->pod_cls[id] = -1;
        c->pod_pos[id] = c0 + d;
    } else {
        --c->live_pods;                                   // re-added below
        c->live_xc -= c->h_cused[d] & 0xFFFF;
        c->live_xp -= c->h_cused[d] >> 16;
    }
    const uint32_t f = p->flags[i], cf = c->h_cflags[d];
    const uint32_t nf = (cf & ~KP_POD_FLAGS) | (f & KP_POD_FLAGS);
    const int64_t t = d / CTILE;
    uint32_t ro = c->h_xc_base[t], po = c->h_xp_base[t];
    for (int64_t k = t * CTILE; k < d; ++k) { ro += pf_xctr(c->h_cflags[k]); po += pf_xpair(c->h_cflags[k]); }
    P.add(PT_FLAGS, d, nf);
    P.add(PT_CPU0, d, p->cpu0[i]);
    P.add(PT_MEM0, d, (uint64_t)p->mem0[i]);
    P.add(PT_PAIR0, d, p->pair0[i]);
    const uint32_t xr = pf_xreg(f), xi = pf_xinit(f), ov = (f & ESC_PF_HAS_OVH) ? 1u : 0u;
    auto rec = [&](uint32_t at, bool have, int64_t src, int64_t neutral) {
        P.add(PT_XC_CPU, at, (uint64_t)(have ? p->xc_cpu[src] : neutral));
        P.add(PT_XC_MEM, at, (uint64_t)(have ? p->xc_mem[src] : neutral));
    };
    uint32_t o = ro;
    for (uint32_t k = 0; k < pf_xreg(cf); ++k) rec(o++, k < xr, rof + k, 0);
    for (uint32_t k = 0; k < pf_xinit(cf); ++k) rec(o++, k < xi, rof + xr + k, INT64_MIN);
    if (cf & ESC_PF_HAS_OVH) rec(o++, ov != 0, rof + xr + xi, 0);
    const uint32_t nx = pf_xpair(f);
    for (uint32_t k = 0; k < pf_xpair(cf); ++k) P.add(PT_XP, po + k, k < nx ? p->xp_pair[pof + k] : NONE);
    c->h_cflags[d] = nf;
    c->h_cused[d] = (xr + xi + ov) | nx << 16;
    ++c->live_pods;
    c->live_xc += xr + xi + ov;
    c->live_xp += nx;
    return touch_mark_c(c, d, f, p->pair0[i], nx ? p->xp_pair + pof : nullptr);
}

int32_t upsert_plan(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p, UpsertPlan& u) {
    if (!c || !p || p->n_pods < 0 || (p->n_pods > 0 && (!ids || !p->flags || !p->cpu0 || !p->mem0 || !p->pair0)))
        return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->pods_loaded) return ESC_E_STATE;
    const int64_t n = p->n_pods;
    // validate the batch and that every pod fits in place (all or nothing)
    std::vector<int64_t> need(c->h_cls.size(), 0), rof(n), pof(n), cslot(n, -1);
    std::vector<int32_t> tgt(n);
    std::vector<char> taken(c->c_free.size(), 0);          // free C slots this batch takes
    const int64_t c0 = c->k_tiles * TILE;
    uint64_t sc = 0, sp = 0;
    std::vector<int64_t> seen(ids, ids + n);
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) return ESC_E_INVAL;   // one event per id
    for (int64_t i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= ((int64_t)1 << 31)) return ESC_E_INVAL;
        const uint32_t f = p->flags[i], nx = pf_xpair(f), nc = pf_xctr(f);
        uint32_t last = p->pair0[i];
        if (last == NONE ? nx != 0 : last >= ESC_PAIR_LIMIT) return ESC_E_INVAL;
        if (sp + nx > (uint64_t)p->n_xp || sc + nc > (uint64_t)p->n_xc) return ESC_E_INVAL;
        for (uint32_t k = 0; k < nx; ++k) {
            const uint32_t q = p->xp_pair[sp + k];
            if (q >= ESC_PAIR_LIMIT || q <= last) return ESC_E_INVAL;
            last = q;
        }
        rof[i] = (int64_t)sc;
        pof[i] = (int64_t)sp;
        sc += nc;
        sp += nx;
        const int sid = pod_class_id(f, p->cpu0[i], p->mem0[i], p->pair0[i], nc ? p->xc_cpu + sc - nc : nullptr,
                                     nc ? p->xc_mem + sc - nc : nullptr, c->gi.n_gp);
        int ci = sid < 0 ? -1 : c->h_cls_of[sid];
        const int64_t id = ids[i];
        const bool known = id < (int64_t)c->pod_cls.size();
        if (ci >= 0 && !(known && c->pod_cls[id] == ci)) {
            if (need[ci] < (int64_t)c->cls_free[ci].size()) ++need[ci];
            else ci = -1;                                  // its class is full: a C slot
        }
        tgt[i] = ci;
        if (ci >= 0) continue;
        // a C slot: its own (when it has room), else a free one with room
        if (known && c->pod_cls[id] == -1 && c_room(c->h_cflags[c->pod_pos[id] - c0], f)) {
            cslot[i] = c->pod_pos[id] - c0;
            continue;
        }
        for (int64_t k = (int64_t)c->c_free.size() - 1; k >= 0 && cslot[i] < 0; --k)
            if (!taken[k] && c_room(c->h_cflags[c->c_free[k]], f)) {
                taken[k] = 1;
                cslot[i] = c->c_free[k];
            }
        if (cslot[i] < 0) {                                // no room in place: reload
            return ESC_E_LIMIT;
        }
    }
    u.rof.swap(rof);
    u.pof.swap(pof);
    u.tgt.swap(tgt);
    u.cslot.swap(cslot);
    return ESC_OK;
}

int32_t upsert_apply(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p, const UpsertPlan& u) {
    const int64_t n = p->n_pods;
    const std::vector<int64_t>& rof = u.rof;
    const std::vector<int64_t>& pof = u.pof;
    const std::vector<int32_t>& tgt = u.tgt;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->rm_valid = false;
    // A bound pod keeps its node and its run position; its occupancy contribution is taken
    // out while the device still holds its OLD record: a PodRef with more than 3 extra pairs
    // reads them through the pod's xp offset, which the patches below rewrite (or hand to
    // another pod of this batch).  The same order as esc_pods_delete.
    std::vector<uint32_t> bpos, bnode;
    if (c->placed) {
        bound_of(c, ids, n, bpos, bnode);
        if (int32_t r2 = occ_delta(c, bpos, bnode, -1)) return r2;
    }
    Patches P;
    bool touch_grew = false;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t id = ids[i];
        if (id >= (int64_t)c->pod_cls.size()) {
            c->pod_cls.resize(id + 1, -2);
            c->pod_pos.resize(id + 1, 0);
        }
        const int32_t ci = tgt[i];
        if (ci < 0) {
            touch_grew |= upsert_c(c, id, u.cslot[i], p, i, rof[i], pof[i], P);
            continue;
        }
        if (c->pod_cls[id] != ci) {
            remove_pod(c, id, P);
            c->pod_cls[id] = ci;
            c->pod_pos[id] = c->cls_free[ci].back();
            c->cls_free[ci].pop_back();
        } else {
            --c->live_pods;                           // re-added below
            const PodClass& k = c->h_cls[ci];
            c->live_xc -= k.xreg + k.xinit + k.ovh;
            c->live_xp -= k.nxp;
            if (k.packed) { --c->live_pk_pods; c->live_pk_xc -= k.xreg + k.xinit + k.ovh; }
        if (k.packed == 2) { --c->live_p8_pods; c->live_p8_xp -= k.nxp; }
        }
        const PodClass& k = c->h_cls[ci];
        const int64_t q = c->pod_pos[id], sl = q % TILE;
        const int64_t blk = kb_block(k, k.t0 + q / TILE);
        const uint32_t f = p->flags[i], R = kb_nrec(k);
        kb_write_pod(k, blk, sl, f, p->cpu0[i], p->mem0[i], p->pair0[i], R ? p->xc_cpu + rof[i] : nullptr,
                     R ? p->xc_mem + rof[i] : nullptr, k.nxp ? p->xp_pair + pof[i] : nullptr,
                     [&](int width, int64_t at, uint64_t v) { P.add(pt_kb(width), at, v); });
        touch_grew |= touch_mark(c, ci, q, f, p->pair0[i], k.nxp ? p->xp_pair + pof[i] : nullptr);
        ++c->live_pods;
        c->live_xc += R;
        c->live_xp += k.nxp;
        if (k.packed) { ++c->live_pk_pods; c->live_pk_xc += R; }
        if (k.packed == 2) { ++c->live_p8_pods; c->live_p8_xp += k.nxp; }
    }
    int32_t rc = apply_patches(c, P, pod_targets(c));
    if (!rc && touch_grew) rc = touch_upload(c);
    if (rc || !c->placed) return rc;
    // its PodRef follows the new record (and slot), and the occupancy with it
    std::vector<int64_t> touched(ids, ids + n);
    std::vector<uint32_t> runs;
    if (int32_t r2 = sync_placement(c, touched, runs)) return r2;
    return occ_delta(c, bpos, bnode, +1);
}

// esc_pods_bind's checks (ids, nodes, room in the runs) without applying anything.
int32_t bind_check(esc_ctx* c, const int64_t* ids, const uint32_t* pod_node, int64_t n) {
    if (!c || n < 0 || (n > 0 && (!ids || !pod_node))) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->placed) return ESC_E_STATE;
    std::vector<int64_t> seen(ids, ids + n);
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) return ESC_E_INVAL;
    std::unordered_map<uint32_t, int64_t> need;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t id = ids[i];
        if (id < 0 || id >= (int64_t)c->pod_cls.size() || c->pod_cls[id] == -2) return ESC_E_INVAL;
        if (pod_node[i] != NONE && ((int64_t)pod_node[i] >= c->n_nodes || (c->h_nflags[pod_node[i]] & ESC_NF_ABSENT)))
            return ESC_E_INVAL;
        const uint32_t old = id < (int64_t)c->h_pod_node.size() ? c->h_pod_node[id] : NONE;
        if (old != NONE) --need[old];
        if (pod_node[i] != NONE) ++need[pod_node[i]];
    }
    for (const auto& kv : need)
        if (kv.second > 0 && c->h_run_len[kv.first] + kv.second > c->h_run_off[kv.first + 1] - c->h_run_off[kv.first])
            return ESC_E_LIMIT;
    return ESC_OK;
}
}  // namespace

namespace esc {
int32_t pods_upsert_check(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p) {
    UpsertPlan u;
    return upsert_plan(c, ids, p, u);
}
int32_t pods_bind_check(esc_ctx* c, const int64_t* ids, const uint32_t* pod_node, int64_t n) {
    return bind_check(c, ids, pod_node, n);
}
}  // namespace esc

extern "C" {

int32_t esc_pods_upsert(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p) {
    if (c && c->multi) return multi_pods_upsert(c, ids, p);
    UpsertPlan u;
    const int32_t rc = upsert_plan(c, ids, p, u);
    return rc ? rc : guarded(c, STALE_PODS, [&] { return upsert_apply(c, ids, p, u); });
}

int32_t esc_pods_delete(esc_ctx* c, const int64_t* ids, int64_t n) {
    if (c && c->multi) return esc::multi_pods_delete(c, ids, n);
    if (!c || n < 0 || (n > 0 && !ids)) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->pods_loaded) return ESC_E_STATE;
    for (int64_t i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= (int64_t)c->pod_cls.size()) return ESC_E_INVAL;
    return guarded(c, STALE_PODS, [&]() -> int32_t {
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    Patches P;
    std::vector<int64_t> touched;
    std::vector<uint32_t> runs;
    if (c->placed) {                                 // the deleted pods leave their nodes' occupancy
        std::vector<int64_t> live_ids;
        for (int64_t i = 0; i < n; ++i)
            if (c->pod_cls[ids[i]] != -2) live_ids.push_back(ids[i]);
        std::vector<uint32_t> bpos, bnode;
        bound_of(c, live_ids.data(), (int64_t)live_ids.size(), bpos, bnode);
        if (int32_t rc = occ_delta(c, bpos, bnode, -1)) return rc;
    }
    for (int64_t i = 0; i < n; ++i) {
        if (c->placed && c->pod_cls[ids[i]] != -2) run_remove(c, ids[i], touched, runs);   // leaves its node
        remove_pod(c, ids[i], P);
    }
    c->rm_valid = false;
    int32_t rc = apply_patches(c, P, pod_targets(c));
    if (rc || !c->placed) return rc;
    return sync_placement(c, touched, runs);
    });
}

// Spec.NodeName of pods (the informer's pod Update once the scheduler binds a pod, or a
// pod leaving its node): moves each pod's PodRef between node runs (node_state.go:10-39
// builds the same map per decision).  NONE = unbound.  All or nothing: ESC_E_LIMIT when a
// node's run has no room left (esc_load_placement again).
int32_t esc_pods_bind(esc_ctx* c, const int64_t* ids, const uint32_t* pod_node, int64_t n) {
    if (c && c->multi) return multi_pods_bind(c, ids, pod_node, n);
    if (int32_t rc = bind_check(c, ids, pod_node, n)) return rc;
    return guarded(c, STALE_PODS, [&]() -> int32_t {
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if ((int64_t)c->h_pod_node.size() < (int64_t)c->pod_cls.size()) {
        c->h_pod_node.resize(c->pod_cls.size(), NONE);
        c->h_pod_rpos.resize(c->pod_cls.size(), -1);
    }
    std::vector<int64_t> touched;
    std::vector<uint32_t> runs;
    std::vector<uint32_t> bpos, bnode;
    bound_of(c, ids, n, bpos, bnode);                // the pods leave their old nodes' occupancy
    if (int32_t rc = occ_delta(c, bpos, bnode, -1)) return rc;
    for (int64_t i = 0; i < n; ++i) run_remove(c, ids[i], touched, runs);      // removals first: room
    for (int64_t i = 0; i < n; ++i)
        if (pod_node[i] != NONE && !run_append(c, ids[i], pod_node[i], touched, runs)) return ESC_E_HIP;
    if (int32_t rc = sync_placement(c, touched, runs)) return rc;
    bound_of(c, ids, n, bpos, bnode);                // and join their new ones'
    return occ_delta(c, bpos, bnode, +1);
    });
}

int32_t esc_nodes_update(esc_ctx* c, const int64_t* ids, int64_t n, const uint32_t* flags, const int64_t* cpu,
                         const int64_t* mem) {
    if (c && c->multi) return esc::multi_nodes_update(c, ids, n, flags, cpu, mem);
    if (!c || n < 0 || (n > 0 && (!ids || !flags || !cpu || !mem))) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded) return ESC_E_STATE;
    // the tracker bit is the context's (esc_tracker_update), whatever the caller packed
    const uint32_t mutable_bits = ESC_NF_UNSCHED | ESC_NF_TAINTED | ESC_NF_TRACKED;
    for (int64_t i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= c->n_nodes || (c->h_nflags[ids[i]] & ESC_NF_ABSENT)) return ESC_E_INVAL;
        if ((flags[i] ^ c->h_nflags[ids[i]]) & ~mutable_bits) return ESC_E_INVAL;   // labels: reload
    }
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    // the host mirrors change first: a device write that fails after them leaves the
    // context stale until esc_load_nodes
    return guarded(c, STALE_NODES, [&]() -> int32_t {
        std::vector<int64_t> touched(ids, ids + n);
        for (int64_t i = 0; i < n; ++i) {
            const int64_t j = ids[i];
            c->h_nflags[j] = (flags[i] & ~ESC_NF_TRACKED) | (c->h_nflags[j] & ESC_NF_TRACKED);
            c->h_ncpu[j] = cpu[i];
            c->h_nmem[j] = mem[i];
        }
        return patch_nodes(c, touched);
    });
}

// Node informer events that add or delete nodes (pkg/k8s/cache.go:37-56 feeds the
// reference's node lister).  Added nodes take the next snapshot indices (listed after every
// loaded node, so allNodes[0] and each pair's entries keep snapshot order), spare entries
// of their label pairs (K2), and slots of their groups' K5 regions, inserted at their place
// by creation time; a deleted node's slot becomes ESC_NF_ABSENT everywhere (no kernel
// counts it) and its tracker entries are dropped.  All or nothing: ESC_E_LIMIT when the
// spare room (esc_set_spare before esc_load_nodes) does not hold the batch.
int32_t esc_nodes_add(esc_ctx* c, const esc_node_soa* s, int64_t* ids_out) {
    if (c && c->multi) return esc::multi_nodes_add(c, s, ids_out);
    if (!c || !s || s->n_nodes < 0 || (s->n_nodes > 0 && (!ids_out || !s->flags || !s->label0 || !s->cpu || !s->mem ||
                                                          !s->created_ns)))
        return ESC_E_INVAL;
    if (s->n_trk != 0 || (s->n_xl > 0 && !s->xl_pair)) return ESC_E_INVAL;   // trackers: esc_tracker_update
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded) return ESC_E_STATE;
    const int64_t n = s->n_nodes;
    if (n == 0) return ESC_OK;
    if (c->n_nodes + n > c->n_cap || c->xl_used + s->n_xl > c->xl_cap) return ESC_E_LIMIT;
    // validate, and count the spare room the batch needs (entries per pair, region slots)
    const uint32_t n_gp = c->gi.n_gp;
    std::vector<int64_t> xo(n);
    std::vector<uint32_t> need_e(n_gp, 0);
    std::unordered_map<uint32_t, uint32_t> need_r;
    std::vector<uint32_t> mb;
    uint64_t sx = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t f = s->flags[i], nx = nf_xlbl(f);
        if (f & (ESC_NF_TRACKED | ESC_NF_ABSENT)) return ESC_E_INVAL;
        uint32_t last = s->label0[i];
        if (last == NONE ? nx != 0 : last >= ESC_PAIR_LIMIT) return ESC_E_INVAL;
        if (sx + nx > (uint64_t)s->n_xl) return ESC_E_INVAL;
        for (uint32_t k = 0; k < nx; ++k) {
            const uint32_t q = s->xl_pair[sx + k];
            if (q >= ESC_PAIR_LIMIT || q <= last) return ESC_E_INVAL;
            last = q;
        }
        xo[i] = (int64_t)sx;
        auto count = [&](uint32_t q) {
            if (q >= n_gp) return;
            ++need_e[q];
        };
        count(s->label0[i]);
        for (uint32_t k = 0; k < nx; ++k) count(s->xl_pair[sx + k]);
        sx += nx;
    }
    if ((int64_t)sx != s->n_xl) return ESC_E_INVAL;
    for (uint32_t q = 0; q < n_gp; ++q)
        if (need_e[q] && c->pair_next[q] + need_e[q] > c->pair_end[q]) return ESC_E_LIMIT;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    // K5 regions: every rank checks the capacity of every group the batch touches (the host
    // knows them all), so that all ranks accept or refuse alike; it inserts into the regions
    // of the groups it owns
    const bool k5 = c->age_built && c->age_ok && !c->h_pcap.empty();
    if (k5 && c->n_gpad > 0) {
        int32_t rc = ensure_gn(c);
        if (rc) return rc;
    }
    // host mirrors of the new nodes (their memberships are read from these)
    const int64_t j0 = c->n_nodes;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t j = j0 + i;
        c->h_nflags[j] = s->flags[i];
        c->h_ncpu[j] = s->cpu[i];
        c->h_nmem[j] = s->mem[i];
        c->h_label0[j] = s->label0[i];
        c->h_xl_off[j] = (uint32_t)(c->xl_used + xo[i]);
    }
    if (k5) {
        for (int64_t i = 0; i < n; ++i) {
            node_membs_from(c, s->label0[i], nf_xlbl(s->flags[i]), s->xl_pair + xo[i], mb);
            for (uint32_t m : mb) ++need_r[m & NODE_GROUP_MASK];
        }
        for (const auto& kv : need_r)
            if ((int64_t)c->h_plen[kv.first] + kv.second > (int64_t)c->h_pcap[kv.first]) {
                for (int64_t i = 0; i < n; ++i) c->h_nflags[j0 + i] = ESC_NF_ABSENT;   // undo
                return ESC_E_LIMIT;
            }
    }
    // commit: node table, extra labels, pair-major entries, allNodes[0] (a failure from here
    // on leaves the context stale until esc_load_nodes)
    return guarded(c, STALE_NODES, [&]() -> int32_t {
        c->h_xl.insert(c->h_xl.end(), s->xl_pair, s->xl_pair + s->n_xl);
        Patches P;
        bool first_changed = false;
        std::vector<uint32_t> pairs;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t j = j0 + i;
            const uint32_t f = s->flags[i];
            P.add(NT_FLAGS, j, f);
            P.add(NT_LABEL0, j, s->label0[i]);
            P.add(NT_XLOFF, j, c->h_xl_off[j]);
            P.add(NT_CPU, j, (uint64_t)s->cpu[i]);
            P.add(NT_MEM, j, (uint64_t)s->mem[i]);
            P.add(NT_CREATED, j, (uint64_t)s->created_ns[i]);
            for (uint32_t k = 0; k < nf_xlbl(f); ++k) P.add(NT_XL, c->h_xl_off[j] + k, s->xl_pair[xo[i] + k]);
            pairs.clear();
            if (s->label0[i] < n_gp) pairs.push_back(s->label0[i]);
            for (uint32_t k = 0; k < nf_xlbl(f); ++k)
                if (s->xl_pair[xo[i] + k] < n_gp) pairs.push_back(s->xl_pair[xo[i] + k]);
            for (uint32_t q : pairs) {
                const uint32_t e = c->pair_next[q]++;
                ++c->pair_live[q];
                entry_patch(c, P, e, f, s->cpu[i], s->mem[i]);
                P.add(NT_ENODE, e, (uint32_t)j);
                c->h_e_node[e] = (uint32_t)j;
                c->ne_pos.push_back(e);
                const uint32_t code = c->gi.node_code[q];
                auto first_of = [&](uint32_t g) {
                    GroupNode& x = c->h_gnode[g];
                    if (x.first == INT64_MAX) {           // the group's first member (controller.go:208)
                        x.first = j;
                        x.first_cpu = s->cpu[i];
                        x.first_mem = s->mem[i];
                        first_changed = true;
                    }
                };
                if (code < CODE_MULTI) first_of(code & NODE_GROUP_MASK);
                else if (code != NONE) {
                    const uint32_t* l = c->gi.code_list.data() + (code & ~CODE_MULTI);
                    for (uint32_t k = 1; k <= l[0]; ++k) first_of(l[k] & NODE_GROUP_MASK);
                }
            }
            c->ne_off.push_back((uint32_t)c->ne_pos.size());
            ids_out[i] = j;
        }
        c->xl_used += s->n_xl;
        c->n_nodes += n;
        c->rm_valid = false;            // the placement stays: every table slot has a run and facts
        int32_t rc = apply_patches(c, P, {node_targets(c)});
        if (rc) return rc;
        if (first_changed)
            HIP_TRY(hipMemcpy(c->nodes.gnode, c->h_gnode.data(), c->h_gnode.size() * sizeof(GroupNode), hipMemcpyHostToDevice));
        for (int64_t i = 0; i < n; ++i) c->h_created.push_back(s->created_ns[i]);
        c->node_hi = c->n_nodes;
        if (k5) {
            // K5: insert each new membership at its place by (creation time, index) in its
            // group's region (the groups this rank owns; the others only count it); every group
            // touched is rewritten from its first insertion on
            std::unordered_map<uint32_t, std::vector<uint32_t>> add_by_g;
            for (int64_t i = 0; i < n; ++i) {
                node_membs(c, j0 + i, mb);
                for (uint32_t m : mb) {
                    const uint32_t g = m & NODE_GROUP_MASK;
                    if (owns_group(c, g)) add_by_g[g].push_back((uint32_t)(j0 + i));
                    else ++c->h_plen[g];
                }
            }
            Patches R;                                   // one scatter for every touched region
            regions_insert(c, add_by_g, R);
            PatchTargets t = region_targets(c);
            rc = apply_patches(c, R, {t});
            if (rc) return rc;
        }
        c->sorted = false;
        return ESC_OK;
    });
}

int32_t esc_nodes_delete(esc_ctx* c, const int64_t* ids, int64_t n) {
    if (c && c->multi) return esc::multi_nodes_delete(c, ids, n);
    if (!c || n < 0 || (n > 0 && !ids)) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded) return ESC_E_STATE;
    std::vector<int64_t> del(ids, ids + n);
    std::sort(del.begin(), del.end());
    if (std::adjacent_find(del.begin(), del.end()) != del.end()) return ESC_E_INVAL;
    for (int64_t j : del)
        if (j < 0 || j >= c->n_nodes || (c->h_nflags[j] & ESC_NF_ABSENT)) return ESC_E_INVAL;
    if (n == 0) return ESC_OK;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    // from the first write on, a failure leaves the context stale until esc_load_nodes
    return guarded(c, STALE_NODES, [&]() -> int32_t {
        // tracker entries of the deleted nodes go (a re-added name is re-tracked by the host)
        std::vector<uint64_t> next;
        next.reserve(c->h_trk.size());
        for (uint64_t k : c->h_trk)
            if (!std::binary_search(del.begin(), del.end(), (int64_t)(k >> 32))) next.push_back(k);
        if (next.size() != c->h_trk.size()) {
            int32_t rc = write_tracker(c, next);
            if (rc) return rc;
        }
        for (int64_t j : del) {
            auto drop = [&](uint32_t q) { if (q < c->gi.n_gp) --c->pair_live[q]; };   // live entries (owner split)
            drop(c->h_label0[j]);
            for (uint32_t k = 0; k < nf_xlbl(c->h_nflags[j]); ++k) drop(c->h_xl[c->h_xl_off[j] + k]);
            c->h_nflags[j] = (c->h_nflags[j] & ~ESC_NF_TRACKED) | ESC_NF_ABSENT;
        }
        // allNodes[0] of the groups whose first member went: the next live entry of the pair
        bool first_changed = false;
        for (int32_t g = 0; g < c->gi.G; ++g) {
            GroupNode& x = c->h_gnode[g];
            if (x.first == INT64_MAX || !(c->h_nflags[x.first] & ESC_NF_ABSENT)) continue;
            pair_first(c, c->gi.gpair[g], x);
            first_changed = true;
        }
        if (first_changed)
            HIP_TRY(hipMemcpy(c->nodes.gnode, c->h_gnode.data(), c->h_gnode.size() * sizeof(GroupNode), hipMemcpyHostToDevice));
        // the placement stays: a deleted node's entries are absent (K6 / K7 skip them) and its
        // pods' PodRefs stay in its run until they are rebound or deleted
        c->rm_valid = false;
        return patch_nodes(c, del);
    });
}

// Node informer Update events that change a node's LABELS or CREATION TIME (besides its
// flags and allocatable).  The reference re-reads every node's labels on every List
// (NewNodeLabelFilterFunc node_group.go:278-287 through FilteredNodesLister.List
// node_listers.go:33-48, fed by the informer cache.go:37-56), so a relabelled node simply
// moves between groups on the next scan.  Here the node keeps its snapshot index and:
//  - its pair-major entries of pairs it no longer carries are retired (absent, no node) and
//    entries of the group pairs it now carries are taken from their pairs' spare room (as
//    esc_nodes_add does); the node -> entries map follows;
//  - allNodes[0] of every group whose pair gained or lost the node is recomputed (lowest
//    live member);
//  - its K5 memberships leave the regions of the groups it left (the region closes up) and
//    join the regions of the groups it joined at their place by creation time (a creation
//    time change moves it in every region);
//  - with a placement loaded, its pods' occupancy contributions leave the old entries and
//    join the new ones (k_occ_delta).
// All or nothing: ESC_E_LIMIT when the spare entries, extra-label words or region slots do
// not hold the batch (nothing applied; reload).
namespace {

struct RelabelPlan {
    std::vector<std::vector<uint32_t>> old_m, new_m;          // memberships (group | dry bit)
    std::vector<int64_t> xo;                                  // each node's first new extra label
    std::vector<uint8_t> moved;                               // creation time changed
};

// group pairs (ids < n_gp) of a label set, ascending
void group_pairs(uint32_t n_gp, uint32_t label0, uint32_t nx, const uint32_t* xl, std::vector<uint32_t>& out) {
    out.clear();
    if (label0 < n_gp) out.push_back(label0);
    for (uint32_t k = 0; k < nx; ++k)
        if (xl[k] < n_gp) out.push_back(xl[k]);
}

// the group pair of pair-major entry e (NONE: a pair no group uses)
uint32_t entry_pair(const esc_ctx* c, uint32_t e) {
    const uint32_t n_gp = c->gi.n_gp;
    if (!n_gp || e >= c->pair_end[n_gp - 1]) return NONE;
    const uint32_t q = (uint32_t)(std::upper_bound(c->pair_lo.begin(), c->pair_lo.end(), e) - c->pair_lo.begin()) - 1;
    return e < c->pair_end[q] ? q : NONE;
}

// Node j's own retired entry of pair q (an entry it left earlier and nobody took since),
// or NONE: a relabel that brings j back to q reuses it instead of a spare entry, so label
// churn (A -> B -> A ...) does not use up the pair's spare room.
uint32_t retired_entry(const esc_ctx* c, int64_t j, uint32_t q) {
    for (uint32_t k = c->ne_off[j]; k < c->ne_off[j + 1]; ++k) {
        const uint32_t e = c->ne_pos[k];
        if (c->h_e_node[e] == NONE && entry_pair(c, e) == q) return e;
    }
    return NONE;
}

int32_t relabel_plan(esc_ctx* c, const int64_t* ids, const esc_node_soa* s, RelabelPlan& u) {
    if (!c || !s || s->n_nodes < 0 || (s->n_nodes > 0 && (!ids || !s->flags || !s->label0 || !s->cpu || !s->mem ||
                                                          !s->created_ns)))
        return ESC_E_INVAL;
    if (s->n_trk != 0 || (s->n_xl > 0 && !s->xl_pair)) return ESC_E_INVAL;   // trackers: esc_tracker_update
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded) return ESC_E_STATE;
    const int64_t n = s->n_nodes;
    std::vector<int64_t> seen(ids, ids + n);
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end()) return ESC_E_INVAL;
    const uint32_t n_gp = c->gi.n_gp;
    u.old_m.assign(n, {});
    u.new_m.assign(n, {});
    u.xo.assign(n, 0);
    u.moved.assign(n, 0);
    std::unordered_map<uint32_t, int64_t> need_e;
    std::unordered_map<uint32_t, int64_t> need_r;
    std::vector<uint32_t> oq, nq;
    uint64_t sx = 0, xl_grow = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t j = ids[i];
        if (j < 0 || j >= c->n_nodes || (c->h_nflags[j] & ESC_NF_ABSENT)) return ESC_E_INVAL;
        const uint32_t f = s->flags[i], nx = nf_xlbl(f);
        if (f & ESC_NF_ABSENT) return ESC_E_INVAL;
        uint32_t last = s->label0[i];
        if (last == NONE ? nx != 0 : last >= ESC_PAIR_LIMIT) return ESC_E_INVAL;
        if (sx + nx > (uint64_t)s->n_xl) return ESC_E_INVAL;
        for (uint32_t k = 0; k < nx; ++k) {
            const uint32_t q = s->xl_pair[sx + k];
            if (q >= ESC_PAIR_LIMIT || q <= last) return ESC_E_INVAL;
            last = q;
        }
        u.xo[i] = (int64_t)sx;
        if (nx > nf_xlbl(c->h_nflags[j])) xl_grow += nx;
        // entries: the group pairs the node gains
        group_pairs(n_gp, c->h_label0[j], nf_xlbl(c->h_nflags[j]), c->h_xl.data() + c->h_xl_off[j], oq);
        group_pairs(n_gp, s->label0[i], nx, s->xl_pair + sx, nq);
        for (uint32_t q : nq)
            if (!std::binary_search(oq.begin(), oq.end(), q) && retired_entry(c, j, q) == NONE) ++need_e[q];
        // K5 regions: memberships left / joined (all of them when the creation time moved)
        node_membs(c, j, u.old_m[i]);
        node_membs_from(c, s->label0[i], nx, s->xl_pair + sx, u.new_m[i]);
        u.moved[i] = s->created_ns[i] != created_of(c, (uint32_t)j);
        for (uint32_t m : u.old_m[i])
            if (u.moved[i] || std::find(u.new_m[i].begin(), u.new_m[i].end(), m) == u.new_m[i].end())
                --need_r[m & NODE_GROUP_MASK];
        for (uint32_t m : u.new_m[i])
            if (u.moved[i] || std::find(u.old_m[i].begin(), u.old_m[i].end(), m) == u.old_m[i].end())
                ++need_r[m & NODE_GROUP_MASK];
        sx += nx;
    }
    if ((int64_t)sx != s->n_xl) return ESC_E_INVAL;
    if (c->xl_used + (int64_t)xl_grow > c->xl_cap) return ESC_E_LIMIT;
    for (const auto& kv : need_e)
        if ((int64_t)c->pair_next[kv.first] + kv.second > (int64_t)c->pair_end[kv.first]) return ESC_E_LIMIT;
    if (c->age_built && c->age_ok && !c->h_pcap.empty())
        for (const auto& kv : need_r)
            if ((int64_t)c->h_plen[kv.first] + kv.second > (int64_t)c->h_pcap[kv.first]) return ESC_E_LIMIT;
    return ESC_OK;
}

int32_t relabel_apply(esc_ctx* c, const int64_t* ids, const esc_node_soa* s, const RelabelPlan& u) {
    const int64_t n = s->n_nodes;
    if (n == 0) return ESC_OK;
    const uint32_t n_gp = c->gi.n_gp;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->rm_valid = false;
    // the nodes' pods leave the occupancy words of their current entries
    std::vector<uint32_t> opos, onode;
    if (c->placed) {
        for (int64_t i = 0; i < n; ++i) {
            const uint32_t j = (uint32_t)ids[i];
            for (uint32_t p = c->h_run_off[j]; p < c->h_run_off[j] + c->h_run_len[j]; ++p) {
                opos.push_back(p);
                onode.push_back(j);
            }
        }
        if (int32_t rc = occ_delta(c, opos, onode, -1)) return rc;
    }
    // K5: memberships leave their regions while the creation times are the old ones
    const bool k5 = c->age_built && c->age_ok && !c->h_pcap.empty();
    Patches R;
    if (k5) {
        if (c->n_gpad > 0)
            if (int32_t rc = ensure_gn(c)) return rc;
        for (int64_t i = 0; i < n; ++i)
            for (uint32_t m : u.old_m[i]) {
                if (!u.moved[i] && std::find(u.new_m[i].begin(), u.new_m[i].end(), m) != u.new_m[i].end()) continue;
                const uint32_t g = m & NODE_GROUP_MASK;
                if (!owns_group(c, g)) { --c->h_plen[g]; continue; }
                if (!region_remove(c, g, (uint32_t)ids[i], R)) return fail_hip(hipErrorUnknown, "relabel: region mirror");
            }
    }
    // host mirrors, extra labels, pair-major entries, node -> entries map
    Patches P;
    std::vector<uint32_t> oq, nq, keep;
    std::vector<uint8_t> pair_touched(n_gp, 0);
    std::vector<std::pair<int64_t, std::vector<uint32_t>>> regrow;   // nodes whose entry list changed size
    std::vector<uint32_t> reused;                                       // retired entries taken back
    for (int64_t i = 0; i < n; ++i) {
        const int64_t j = ids[i];
        const uint32_t f = s->flags[i], nx = nf_xlbl(f), onx = nf_xlbl(c->h_nflags[j]);
        group_pairs(n_gp, s->label0[i], nx, s->xl_pair + u.xo[i], nq);
        keep.clear();
        std::vector<uint32_t> dead;                                       // retired entries in j's slots
        for (uint32_t k = c->ne_off[j]; k < c->ne_off[j + 1]; ++k) {
            const uint32_t e = c->ne_pos[k];
            if (c->h_e_node[e] != (uint32_t)j) { dead.push_back(e); continue; }   // retired earlier
            const uint32_t q = entry_pair(c, e);
            if (q != NONE && std::binary_search(nq.begin(), nq.end(), q)) { keep.push_back(e); continue; }
            c->h_e_node[e] = NONE;                                        // retired: absent, no node
            entry_patch(c, P, e, ESC_NF_ABSENT, 0, 0);
            P.add(NT_ENODE, e, NONE);
            dead.push_back(e);
            if (q != NONE) { --c->pair_live[q]; pair_touched[q] = 1; }
        }
        for (uint32_t q : nq) {
            bool have = false;
            for (uint32_t e : keep) have |= entry_pair(c, e) == q;
            if (have) continue;
            uint32_t e = NONE;                                            // j's own retired entry of q
            for (uint32_t d : dead)
                if (c->h_e_node[d] == NONE && entry_pair(c, d) == q) { e = d; break; }
            if (e != NONE) {
                dead.erase(std::remove(dead.begin(), dead.end(), e), dead.end());
                reused.push_back(e);
            } else {
                e = c->pair_next[q]++;                                    // a spare entry of the pair
            }
            c->h_e_node[e] = (uint32_t)j;
            P.add(NT_ENODE, e, (uint32_t)j);                               // flags / cpu / mem: patch_nodes
            keep.push_back(e);
            ++c->pair_live[q];
            pair_touched[q] = 1;
        }
        // the node's map: its live entries, then its retired ones (each once; patch_nodes
        // skips them, and a later relabel back to their pair takes them again)
        std::sort(dead.begin(), dead.end());
        dead.erase(std::unique(dead.begin(), dead.end()), dead.end());
        std::vector<uint32_t> list(keep);
        list.insert(list.end(), dead.begin(), dead.end());
        const uint32_t slots = c->ne_off[j + 1] - c->ne_off[j];
        if (list.size() <= slots && !list.empty() && (list.size() == slots || !dead.empty())) {
            // in place; spare slots repeat a retired entry
            for (uint32_t k = 0; k < slots; ++k)
                c->ne_pos[c->ne_off[j] + k] = k < list.size() ? list[k] : dead[0];
        } else {
            regrow.emplace_back(j, list);
        }
        // extra labels: in place, or appended when the node has more of them now
        if (nx > onx) {
            c->h_xl_off[j] = (uint32_t)c->xl_used;
            c->h_xl.resize((size_t)c->xl_used + nx);
            c->xl_used += nx;
        }
        for (uint32_t k = 0; k < nx; ++k) {
            c->h_xl[c->h_xl_off[j] + k] = s->xl_pair[u.xo[i] + k];
            P.add(NT_XL, c->h_xl_off[j] + k, s->xl_pair[u.xo[i] + k]);
        }
        c->h_label0[j] = s->label0[i];
        c->h_nflags[j] = (f & ~ESC_NF_TRACKED) | (c->h_nflags[j] & ESC_NF_TRACKED);
        c->h_ncpu[j] = s->cpu[i];
        c->h_nmem[j] = s->mem[i];
        c->h_created[j - c->node_lo] = s->created_ns[i];
        P.add(NT_LABEL0, j, s->label0[i]);
        P.add(NT_XLOFF, j, c->h_xl_off[j]);
        P.add(NT_CREATED, j, (uint64_t)s->created_ns[i]);
        if (u.moved[i] && c->age_built && c->age_ok &&
            (s->created_ns[i] < c->ts_min || s->created_ns[i] > c->ts_max ||
             (uint64_t)(s->created_ns[i] - c->ts_min) % c->sort_div != 0))
            c->age_n = -1;                          // outside the index's key range: the next build is fresh
    }
    if (!regrow.empty()) {                          // rebuild the node -> entries map
        std::sort(regrow.begin(), regrow.end());
        std::vector<uint32_t> off(c->ne_off.size()), pos;
        pos.reserve(c->ne_pos.size() + 16);
        size_t r = 0;
        for (size_t j = 0; j + 1 < c->ne_off.size(); ++j) {
            off[j] = (uint32_t)pos.size();
            if (r < regrow.size() && regrow[r].first == (int64_t)j) {
                pos.insert(pos.end(), regrow[r].second.begin(), regrow[r].second.end());
                ++r;
            } else {
                pos.insert(pos.end(), c->ne_pos.begin() + c->ne_off[j], c->ne_pos.begin() + c->ne_off[j + 1]);
            }
        }
        off.back() = (uint32_t)pos.size();
        c->ne_off.swap(off);
        c->ne_pos.swap(pos);
    }
    c->ne_dev_nodes = -1;                           // the device copy is re-sent before its next use
    // a reused entry's occupancy words restart at zero (a retired entry repeated in a node's
    // spare map slots may have collected counts nobody read); the +1 below re-adds its pods
    if (c->placed)
        for (uint32_t e : reused)
            for (uint32_t* w : {c->d_occ, c->d_occ_local})
                if (w) {
                    HIP_TRY(hipMemsetAsync(w + e, 0, 4, c->stream));
                    HIP_TRY(hipMemsetAsync(w + c->n_entries + e, 0, 4, c->stream));
                }
    // allNodes[0] of the groups whose pair gained or lost a node
    for (int32_t g = 0; g < c->gi.G; ++g)
        if (pair_touched[c->gi.gpair[g]]) pair_first(c, c->gi.gpair[g], c->h_gnode[g]);
    HIP_TRY(hipMemcpy(c->nodes.gnode, c->h_gnode.data(), c->h_gnode.size() * sizeof(GroupNode), hipMemcpyHostToDevice));
    if (int32_t rc = apply_patches(c, P, {node_targets(c)})) return rc;
    // K5: memberships join their regions at their (new) place
    if (k5) {
        std::unordered_map<uint32_t, std::vector<uint32_t>> add_by_g;
        for (int64_t i = 0; i < n; ++i)
            for (uint32_t m : u.new_m[i]) {
                if (!u.moved[i] && std::find(u.old_m[i].begin(), u.old_m[i].end(), m) != u.old_m[i].end()) continue;
                const uint32_t g = m & NODE_GROUP_MASK;
                if (owns_group(c, g)) add_by_g[g].push_back((uint32_t)ids[i]);
                else ++c->h_plen[g];
            }
        regions_insert(c, add_by_g, R);
        if (int32_t rc = apply_patches(c, R, {region_targets(c)})) return rc;
    }
    // node table flags / allocatable, the entries' copies (the new ones included), allNodes[0]'s
    // allocatable, the K5 flag copies
    std::vector<int64_t> touched(ids, ids + n);
    if (int32_t rc = patch_nodes(c, touched)) return rc;
    // the nodes' pods join the occupancy words of their entries now
    if (c->placed) return occ_delta(c, opos, onode, +1);
    return ESC_OK;
}

}  // namespace

int32_t esc_nodes_relabel(esc_ctx* c, const int64_t* ids, const esc_node_soa* s) {
    if (c && c->multi) return esc::multi_nodes_relabel(c, ids, s);
    RelabelPlan u;
    const int32_t rc = relabel_plan(c, ids, s, u);
    return rc ? rc : guarded(c, STALE_NODES, [&] { return relabel_apply(c, ids, s, u); });
}

}  // extern "C"

namespace esc {
int32_t nodes_relabel_check(esc_ctx* c, const int64_t* ids, const esc_node_soa* s) {
    RelabelPlan u;
    return relabel_plan(c, ids, s, u);
}
}  // namespace esc

extern "C" {

// Dry-mode taintTracker bookkeeping (§8f rank 4).  The reference keeps per group a slice
// of node names: taintOldestN appends in dry mode (scale_down.go:197-200), untaintNewestN
// deletes the first equal name (scale_up.go:146-158) and filterNodes does a linear name
// search per node (controller.go:126-138).  Here the tracker is the sorted (node, group)
// list the kernels binary-index through trk_start; an update rewrites that list (a few
// KB), and only the nodes whose ESC_NF_TRACKED bit flips are patched in the node table,
// the pair-major entries and the K5 membership list.
int32_t esc_tracker_update(esc_ctx* c, int32_t group, const int64_t* add, int64_t n_add, const int64_t* rm,
                           int64_t n_rm) {
    if (c && c->multi) return esc::multi_tracker_update(c, group, add, n_add, rm, n_rm);
    if (!c || n_add < 0 || n_rm < 0 || (n_add > 0 && !add) || (n_rm > 0 && !rm)) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded) return ESC_E_STATE;
    if (group < 0 || group >= c->gi.G) return ESC_E_INVAL;
    auto key = [&](int64_t j) { return ((uint64_t)(uint32_t)j << 32) | (uint32_t)group; };
    for (int64_t i = 0; i < n_rm; ++i) if (rm[i] < 0 || rm[i] >= c->n_nodes) return ESC_E_INVAL;
    for (int64_t i = 0; i < n_add; ++i)
        if (add[i] < 0 || add[i] >= c->n_nodes || (c->h_nflags[add[i]] & ESC_NF_ABSENT)) return ESC_E_INVAL;
    // removals first (absent names are ignored, as untaintNewestN's deleteIndex == -1), then
    // additions (a node already tracked by the group, or added twice, is refused: the
    // reference only appends untainted, i.e. untracked, nodes)
    std::vector<uint64_t> rk(n_rm), ak(n_add);
    for (int64_t i = 0; i < n_rm; ++i) rk[i] = key(rm[i]);
    for (int64_t i = 0; i < n_add; ++i) ak[i] = key(add[i]);
    std::sort(rk.begin(), rk.end());
    std::sort(ak.begin(), ak.end());
    if (std::adjacent_find(ak.begin(), ak.end()) != ak.end()) return ESC_E_INVAL;
    std::vector<uint64_t> kept;
    kept.reserve(c->h_trk.size() + ak.size());
    std::vector<int64_t> touched;
    for (uint64_t k : c->h_trk) {
        if (std::binary_search(rk.begin(), rk.end(), k)) touched.push_back((int64_t)(k >> 32));
        else kept.push_back(k);
    }
    for (uint64_t k : ak)
        if (std::binary_search(kept.begin(), kept.end(), k)) return ESC_E_INVAL;
    for (uint64_t k : ak) touched.push_back((int64_t)(k >> 32));
    std::vector<uint64_t> next(kept.size() + ak.size());
    std::merge(kept.begin(), kept.end(), ak.begin(), ak.end(), next.begin());
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    // the tracker list, then the flags: a failure after the first write leaves the context
    // stale until esc_load_nodes
    return guarded(c, STALE_NODES, [&]() -> int32_t {
        int32_t rc = write_tracker(c, next);
        if (rc) return rc;
        // ESC_NF_TRACKED = tracked by some group (controller.go:128 is per group; the kernels
        // confirm the group through the list)
        std::vector<int64_t> flip;
        std::sort(touched.begin(), touched.end());
        touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
        for (int64_t j : touched) {
            const uint64_t lo = (uint64_t)(uint32_t)j << 32;
            const auto it = std::lower_bound(c->h_trk.begin(), c->h_trk.end(), lo);
            const bool on = it != c->h_trk.end() && (*it >> 32) == (uint64_t)(uint32_t)j;
            const uint32_t f = on ? (c->h_nflags[j] | ESC_NF_TRACKED) : (c->h_nflags[j] & ~ESC_NF_TRACKED);
            if (f != c->h_nflags[j]) { c->h_nflags[j] = f; flip.push_back(j); }
        }
        c->sorted = false;
        c->rm_valid = false;
        if (!flip.empty()) return patch_nodes(c, touched);     // node table + entries + K5 copies
        // the K5 copies carry each dry membership's tracker bit: patch the touched nodes'
        rc = patch_regions(c, touched);
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        return ESC_OK;
    });
}

int32_t esc_tracker_list(const esc_ctx* c, int32_t group, int64_t* idx_out, int64_t cap, int64_t* n_out) {
    if (c && c->multi) return esc_tracker_list(esc::multi_sub(c, 0), group, idx_out, cap, n_out);
    if (!c || !n_out || cap < 0 || (cap > 0 && !idx_out)) return ESC_E_INVAL;
    if (group < 0 || group >= c->gi.G) return ESC_E_INVAL;
    int64_t m = 0;
    for (uint64_t k : c->h_trk)
        if ((int32_t)(uint32_t)k == group) {
            if (m < cap) idx_out[m] = (int64_t)(k >> 32);
            ++m;
        }
    *n_out = m;
    return ESC_OK;
}

// ------------------------------------------------ scale-down reaping (§8f rank 2)
// esc_load_placement: CreateNodeNameToInfoMap (node_state.go:10-39) as runs of PodRef per
// node (a host counting sort of the pods by node, then one gather of each pod's flags and
// pairs from the resident layout), plus the per-node GetToBeRemovedTime / no-delete facts.
int32_t esc_load_placement(esc_ctx* c, const uint32_t* pod_node, const int64_t* taint_s, const uint8_t* no_delete) {
    if (c && c->multi) return esc::multi_load_placement(c, pod_node, taint_s, no_delete);
    if (!c || !taint_s || !no_delete) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->pods_loaded || !c->nodes_loaded) return ESC_E_STATE;
    if (!pod_node && !c->placed) return ESC_E_STATE;
    const int64_t N = c->n_nodes, np = (int64_t)c->pod_cls.size();
    if (pod_node)
        for (int64_t i = 0; i < np; ++i)
            if (pod_node[i] != NONE && (int64_t)pod_node[i] >= N) return ESC_E_INVAL;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int32_t G = c->gi.G;
    // per-node arrays cover every table slot (n_cap), so that nodes added later
    // (esc_nodes_add) have facts (none until refreshed) and an empty run of their own
    const int64_t NC = std::max<int64_t>(c->n_cap, N);
    if (!c->d_taint_s || c->rm_nodes != NC) {
        // per-node facts and the per-entry occupancy words, sized for this node table
        dfree(c->d_taint_s); dfree(c->d_no_delete); dfree(c->d_occ); dfree(c->d_e_pair); dfree(c->d_occ_local);
        dfree(c->d_soft); dfree(c->d_hard); dfree(c->d_rm_out); dfree(c->d_rm_off); dfree(c->d_rm_list);
        HIP_TRY(dalloc(&c->d_taint_s, std::max<int64_t>(NC, 1)));
        HIP_TRY(dalloc(&c->d_no_delete, std::max<int64_t>(NC, 1)));
        if (NC > N) {
            const std::vector<int64_t> none(NC - N, INT64_MIN);
            HIP_TRY(hipMemcpy(c->d_taint_s + N, none.data(), (NC - N) * 8, hipMemcpyHostToDevice));
            HIP_TRY(hipMemset(c->d_no_delete + N, 0, NC - N));
        }
        HIP_TRY(dalloc(&c->d_occ, 2 * std::max<int64_t>(c->n_entries, 1)));
        if (c->world > 1) HIP_TRY(dalloc(&c->d_occ_local, 2 * std::max<int64_t>(c->n_entries, 1)));
        c->placed = false;                             // the occupancy words are recounted below
        HIP_TRY(dalloc(&c->d_soft, G)); HIP_TRY(dalloc(&c->d_hard, G));
        HIP_TRY(dalloc(&c->d_rm_out, G)); HIP_TRY(dalloc(&c->d_rm_off, G));
        // each group's deletable-node list can hold all of its pair's entries
        std::vector<uint32_t> poff(c->n_pieces + 1), ppo(c->gi.n_gp + 1), ppair(std::max<int64_t>(c->n_pieces, 1));
        HIP_TRY(hipMemcpy(poff.data(), c->nodes.piece_off, poff.size() * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(ppo.data(), c->nodes.pp_off, ppo.size() * 4, hipMemcpyDeviceToHost));
        if (c->n_pieces)
            HIP_TRY(hipMemcpy(ppair.data(), c->nodes.piece_pair, c->n_pieces * 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> epair(std::max<int64_t>(c->n_entries, 1), NONE);
        for (int64_t pc = 0; pc < c->n_pieces; ++pc)
            for (uint32_t e = poff[pc]; e < poff[pc + 1]; ++e) epair[e] = ppair[pc];
        HIP_TRY(dalloc(&c->d_e_pair, epair.size()));
        HIP_TRY(hipMemcpy(c->d_e_pair, epair.data(), epair.size() * 4, hipMemcpyHostToDevice));
        c->h_rm_off.assign(G + 1, 0);
        for (int32_t g = 0; g < G; ++g) {
            const uint32_t q = c->gi.gpair[g];
            c->h_rm_off[g + 1] = c->h_rm_off[g] + (poff[ppo[q + 1]] - poff[ppo[q]]);
        }
        HIP_TRY(dalloc(&c->d_rm_list, std::max<uint32_t>(c->h_rm_off[G], 1)));
        HIP_TRY(hipMemcpy(c->d_rm_off, c->h_rm_off.data(), (size_t)G * 4, hipMemcpyHostToDevice));
        if (c->h_rm) { hipHostFree(c->h_rm); c->h_rm = nullptr; }
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_rm), (size_t)std::max<int32_t>(G, 1) * sizeof(RmRec)));
        c->h_soft.clear();
        c->h_hard.clear();
        c->rm_nodes = NC;
    }
    if (N) {
        HIP_TRY(hipMemcpy(c->d_taint_s, taint_s, N * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_no_delete, no_delete, N, hipMemcpyHostToDevice));
    }
    if (pod_node) {
        // runs of PodRefs per node, each with spare room (esc_set_spare) for pods bound later
        std::vector<uint32_t> cnt(NC, 0);
        int64_t bound = 0, live = 0;
        for (int64_t i = 0; i < np; ++i)
            if (c->pod_cls[i] != -2 && pod_node[i] != NONE) { ++cnt[pod_node[i]]; ++bound; }
        for (int64_t j = 0; j < N; ++j) live += (c->h_nflags[j] & ESC_NF_ABSENT) ? 0 : 1;
        // room for pods bound later: a node's own count with the spare fraction on top, and at
        // least the mean pods per node with the spare fraction on top — what a lightly loaded
        // node, or a table slot with no node yet (added later), gets; the scheduler fills those
        const uint64_t cap_new = c->spare_frac > 0
            ? (uint64_t)std::ceil((double)bound / (double)std::max<int64_t>(live, 1) * (1.0 + c->spare_frac)) + 4 : 0;
        std::vector<uint32_t> off(NC + 1, 0);
        for (int64_t j = 0; j < NC; ++j) {
            const uint64_t own = cnt[j] + (c->spare_frac > 0 ? (uint64_t)std::ceil(cnt[j] * c->spare_frac) + 2 : 0);
            const uint64_t cap = j >= N ? cap_new : std::max(own, cap_new);
            if ((uint64_t)off[j] + cap >= 0xFFFFFFFFull) return ESC_E_LIMIT;
            off[j + 1] = off[j] + (uint32_t)cap;
        }
        const int64_t total = off[NC];
        std::vector<uint32_t> len(std::max<int64_t>(NC, 1), 0), slot(std::max<int64_t>(total, 1), 0);
        c->h_run_pod.assign(std::max<int64_t>(total, 1), -1);
        c->h_pod_node.assign(np, NONE);
        c->h_pod_rpos.assign(np, -1);
        for (int64_t i = 0; i < np; ++i) {
            if (c->pod_cls[i] == -2 || pod_node[i] == NONE) continue;
            const uint32_t j = pod_node[i];
            const uint32_t pos = off[j] + len[j]++;
            slot[pos] = (uint32_t)pod_slot(c, i);
            c->h_run_pod[pos] = (int32_t)i;
            c->h_pod_node[i] = j;
            c->h_pod_rpos[i] = pos;
        }
        dfree(c->d_refs); dfree(c->d_nrun_off); dfree(c->d_nrun_len);
        uint32_t* d_slot = nullptr;
        HIP_TRY(dalloc(&c->d_refs, std::max<int64_t>(total, 1)));
        HIP_TRY(dalloc(&c->d_nrun_off, NC + 1));
        HIP_TRY(dalloc(&c->d_nrun_len, std::max<int64_t>(NC, 1)));
        HIP_TRY(dalloc(&d_slot, slot.size()));
        HIP_TRY(hipMemcpy(d_slot, slot.data(), slot.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_nrun_off, off.data(), (NC + 1) * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_nrun_len, len.data(), len.size() * 4, hipMemcpyHostToDevice));
        const hipError_t e = launch_podref_fill(pod_dev(c, c->cur), d_slot, nullptr, total, c->d_refs, c->stream);
        const hipError_t e2 = hipStreamSynchronize(c->stream);
        dfree(d_slot);
        HIP_TRY(e);
        HIP_TRY(e2);
        c->h_run_off.swap(off);
        c->h_run_len.swap(len);
        if (int32_t rc = occ_recount(c)) return rc;
        c->placed = true;
    }
    c->node_removal = true;
    c->rm_valid = false;
    return ESC_OK;
}

// K6 (node occupancy by group filter over this rank's pods) — the first half of
// esc_try_remove; with several ranks the occupancy words are summed across ranks before K7.
int32_t esc_reap_occupancy(esc_ctx* c) {
    if (c && c->multi) return ESC_E_STATE;              // esc_try_remove exchanges internally
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->placed || !c->node_removal || c->stale) return ESC_E_STATE;
    hipSetDevice(c->device);
    // the words are current (events maintain them); with several ranks this rank's words
    // go into the exchange buffer the SUM works on
    if (c->d_occ_local && c->n_entries)
        HIP_TRY(hipMemcpyAsync(c->d_occ, c->d_occ_local, (size_t)(2 * c->n_entries) * 4, hipMemcpyDeviceToDevice, c->stream));
    c->rm_valid = false;
    return ESC_OK;
}

int32_t esc_reap_buffer(esc_ctx* c, void** buf, int64_t* n_words) {
    if (c && c->multi) return ESC_E_STATE;
    if (!c || !buf || !n_words) return ESC_E_INVAL;
    if (!c->placed) return ESC_E_STATE;
    *buf = c->d_occ;
    *n_words = 2 * c->n_entries;
    return ESC_OK;
}

int32_t esc_reap_download(esc_ctx* c, uint32_t* out) {
    if (c && c->multi) return ESC_E_STATE;
    if (!c || !out) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->placed) return ESC_E_STATE;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->n_entries) HIP_TRY(hipMemcpy(out, c->d_occ, 2 * c->n_entries * 4, hipMemcpyDeviceToHost));
    return ESC_OK;
}

int32_t esc_reap_upload(esc_ctx* c, const uint32_t* in) {
    if (c && c->multi) return ESC_E_STATE;
    if (!c || !in) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->placed) return ESC_E_STATE;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->n_entries) HIP_TRY(hipMemcpy(c->d_occ, in, 2 * c->n_entries * 4, hipMemcpyHostToDevice));
    return ESC_OK;
}

// K7 over the (summed) occupancy: the per-group reaping pass.
int32_t esc_reap_finish(esc_ctx* c, int64_t now_ns, const int64_t* soft_ns, const int64_t* hard_ns, esc_removal* out) {
    if (c && c->multi) return ESC_E_STATE;
    if (!c || !soft_ns || !hard_ns || !out) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->placed || !c->node_removal || c->stale) return ESC_E_STATE;
    const int32_t G = c->gi.G;
    hipSetDevice(c->device);
    // the grace periods are node-group options: uploaded when they change
    const bool same = (int32_t)c->h_soft.size() == G && (int32_t)c->h_hard.size() == G &&
                      std::memcmp(c->h_soft.data(), soft_ns, (size_t)G * 8) == 0 &&
                      std::memcmp(c->h_hard.data(), hard_ns, (size_t)G * 8) == 0;
    if (!same) {
        c->h_soft.assign(soft_ns, soft_ns + G);
        c->h_hard.assign(hard_ns, hard_ns + G);
        HIP_TRY(hipMemcpyAsync(c->d_soft, c->h_soft.data(), (size_t)G * 8, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->d_hard, c->h_hard.data(), (size_t)G * 8, hipMemcpyHostToDevice, c->stream));
    }
    // K7's per-group records come back by one DMA copy into pinned memory (one 32-B
    // record per group is too small a write for zero-copy over PCIe)
    HIP_TRY(launch_try_remove(node_dev(c), group_dev(c), removal_dev(c, now_ns), c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_rm, c->d_rm_out, (size_t)G * sizeof(RmRec), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int32_t g = 0; g < G; ++g) {
        const RmRec& s = c->h_rm[g];
        out[g].n_candidates = s.n_candidates;
        out[g].n_delete = s.n_delete;
        out[g].pods_remaining = s.pods_remaining;
        out[g].reserved = 0;
    }
    c->rm_valid = true;
    return ESC_OK;
}

// esc_try_remove: K6 (node occupancy by group filter) + the cross-rank SUM of the occupancy
// words over the context's RCCL communicator when there are several ranks + K7.
int32_t esc_try_remove(esc_ctx* c, int64_t now_ns, const int64_t* soft_ns, const int64_t* hard_ns, esc_removal* out) {
    if (c && c->multi) return esc::multi_try_remove(c, now_ns, soft_ns, hard_ns, out);
    if (!c || !soft_ns || !hard_ns || !out) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (c->world > 1 && !c->comm) return ESC_E_STATE;  // host-staged: esc_reap_occupancy / _download / _upload / _finish
    int32_t rc = esc_reap_occupancy(c);
    if (rc) return rc;
    if (c->world > 1) {
        hipSetDevice(c->device);
        const ncclResult_t r = rccl().all_reduce(c->d_occ, c->d_occ, (size_t)(2 * c->n_entries), ncclUint32, ncclSum,
                                                 reinterpret_cast<ncclComm_t>(c->comm), c->stream);
        if (r != ncclSuccess) return fail_comm("ncclAllReduce", rccl().error_string(r));
    }
    return esc_reap_finish(c, now_ns, soft_ns, hard_ns, out);
}

int32_t esc_removal_nodes(esc_ctx* c, int32_t g, int64_t* idx, int64_t cap, int64_t* n_out) {
    if (c && c->multi) return esc_removal_nodes(esc::multi_sub(c, 0), g, idx, cap, n_out);
    if (!c || !n_out || g < 0 || g >= c->gi.G || cap < 0 || (cap > 0 && !idx)) return ESC_E_INVAL;
    if (!c->rm_valid) return ESC_E_STATE;
    const int64_t n = c->h_rm[g].n_delete;
    *n_out = n;
    if (n > cap) return ESC_E_LIMIT;
    if (!n) return ESC_OK;
    std::vector<uint32_t> v(n);
    hipSetDevice(c->device);
    HIP_TRY(hipMemcpy(v.data(), c->d_rm_list + c->h_rm_off[g], n * 4, hipMemcpyDeviceToHost));
    // K7 lists them in entry order: snapshot order, except behind a relabelled node's entry
    std::sort(v.begin(), v.end());
    for (int64_t k = 0; k < n; ++k) idx[k] = v[k];
    return ESC_OK;
}

// ----------------------------------------------------------------- ordering
int32_t esc_sort_nodes(esc_ctx* c) {
    if (c && c->multi) return esc::multi_each(c, [](esc_ctx* x, int32_t) { return esc_sort_nodes(x); }, 0);
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded || !c->age_ok) return ESC_E_STATE;
    hipSetDevice(c->device);
    HIP_TRY(enqueue_order(c, c->stream));
    c->order_src = 0;
    c->sorted = true;
    return ESC_OK;
}

int32_t esc_build_age_index(esc_ctx* c) {
    if (c && c->multi) return esc::multi_each(c, [](esc_ctx* x, int32_t) { return esc_build_age_index(x); }, 0);
    if (!c) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->nodes_loaded) return ESC_E_STATE;
    hipSetDevice(c->device);
    return build_age_index(c);
}

int32_t esc_order_info(const esc_ctx* c, int64_t* n_memberships, int32_t* key_bits) {
    if (c && c->multi) return esc::multi_order_info(c, n_memberships, key_bits);
    if (!c || !n_memberships || !key_bits) return ESC_E_INVAL;
    if (!c->nodes_loaded) return ESC_E_STATE;
    *n_memberships = c->n_memb;
    *key_bits = c->sort_R;
    return ESC_OK;
}

int32_t esc_group_order(esc_ctx* c, int32_t group, int32_t which, int64_t* idx_out, int64_t cap, int64_t* n_out) {
    if (c && c->multi) return esc::multi_group_order(c, group, which, idx_out, cap, n_out);
    if (!c || group < 0 || group >= c->gi.G || (which != 0 && which != 1) || cap < 0 || (cap > 0 && !idx_out))
        return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    if (!c->sorted) return ESC_E_STATE;
    hipSetDevice(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    order_gave_up(c);
    if (c->ord_failed) return ESC_E_ORDER;          // this ordering's look-back gave up

    // class segments [s0, s1) (untainted, oldest first) and [s2, s3) (tainted, newest first)
    const int64_t so = 2 * which;
    int64_t seg[2];
    HIP_TRY(hipMemcpy(seg, c->d_seg + 4 * (int64_t)group + so, 16, hipMemcpyDeviceToHost));
    const int64_t cnt = seg[1] - seg[0];
    if (n_out) *n_out = cnt;
    const int64_t m = std::min(cnt, cap);
    if (m <= 0) return ESC_OK;
    const uint32_t* vals = c->d_ord;
    if (which == 0) {                                  // taintOldestN: the segment in age order
        std::vector<uint32_t> v(m);
        HIP_TRY(hipMemcpy(v.data(), vals + seg[0], m * 4, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < m; ++i) idx_out[i] = v[i];
        return ESC_OK;
    }
    // untaintNewestN: the segment is stored newest first; equal creation times keep
    // ascending snapshot index (the age index breaks ties that way, so the stored run is
    // descending), so read on until the tie run that straddles position m ends, then sort
    // each run of equal times by index.
    const int64_t lo_ts = c->node_lo;
    auto ts = [&](uint32_t i) { return c->h_created[(int64_t)i - lo_ts]; };
    int64_t take = std::min(cnt, m + 64);
    std::vector<uint32_t> v;
    for (;;) {
        v.resize(take);
        HIP_TRY(hipMemcpy(v.data(), vals + seg[0], take * 4, hipMemcpyDeviceToHost));
        if (take == cnt || ts(v[take - 1]) != ts(v[m - 1])) break;
        take = std::min(cnt, take * 2);
    }
    for (int64_t a = 0; a < m;) {
        int64_t b = a + 1;
        while (b < take && ts(v[b]) == ts(v[a])) ++b;
        std::sort(v.begin() + a, v.begin() + b);
        a = b;
    }
    for (int64_t i = 0; i < m; ++i) idx_out[i] = v[i];
    return ESC_OK;
}

// ---------------------------------------------------------------- drop-ins
namespace {

int32_t list_context(esc_ctx* c, esc_ctx** out) {
    if (!c->list_ctx) {
        esc_group_spec s;
        std::memset(&s, 0, sizeof s);
        s.name = "\x01list";
        s.label_key = "\x01list";
        s.label_value = "\x01list";
        int32_t rc = esc_ctx_create(&s, 1, c->device, 0, 1, &c->list_ctx);
        if (rc) return rc;
    }
    *out = c->list_ctx;
    return ESC_OK;
}

}  // namespace

int32_t esc_pods_requests_total(esc_ctx* c, const esc_pod_obj* pods, int64_t n, int64_t* mem_b, int64_t* cpu_m) {
    if (c && c->multi) return esc_pods_requests_total(esc::multi_sub(c, 0), pods, n, mem_b, cpu_m);
    if (!c || n < 0 || (n > 0 && !pods) || !mem_b || !cpu_m) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    return list_pods_requests_total(c->lred, c->device, c->stream, pods, n, mem_b, cpu_m);
}

int32_t esc_hbm_probe(esc_ctx* c, int64_t bytes, int32_t reps, double* read_gbps) {
    if (c && c->multi) return esc_hbm_probe(esc::multi_sub(c, 0), bytes, reps, read_gbps);
    if (!c || !read_gbps) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    return hbm_probe(c->device, c->stream, bytes, reps, read_gbps);
}

int32_t esc_nodes_capacity_total(esc_ctx* c, const esc_node_obj* nodes, int64_t n, int64_t* mem_b, int64_t* cpu_m) {
    if (c && c->multi) return esc_nodes_capacity_total(esc::multi_sub(c, 0), nodes, n, mem_b, cpu_m);
    if (!c || n < 0 || (n > 0 && !nodes) || !mem_b || !cpu_m) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    return list_nodes_capacity_total(c->lred, c->device, c->stream, nodes, n, mem_b, cpu_m);
}

int32_t esc_order_by_creation(esc_ctx* c, const int64_t* created_ns, int64_t n, int32_t oldest, int64_t n_take,
                              int64_t* idx_out) {
    if (c && c->multi) return esc_order_by_creation(esc::multi_sub(c, 0), created_ns, n, oldest, n_take, idx_out);
    if (!c || n < 0 || (n > 0 && !created_ns) || (n_take > 0 && !idx_out)) return ESC_E_INVAL;
    if (!c->has_device) return ESC_E_NODEV;
    esc_ctx* L = nullptr;
    int32_t rc = list_context(c, &L);
    if (rc) return rc;
    // all nodes in group 0; class 0 sorts oldest-first, class 1 (tainted) newest-first
    HostSnapshot s;
    s.nflags.assign(n, oldest ? 0u : ESC_NF_TAINTED);
    s.label0.assign(n, 0u);
    s.ncpu.assign(n, 0);
    s.nmem.assign(n, 0);
    s.created.assign(created_ns, created_ns + n);
    esc_pod_soa ps;
    esc_node_soa ns;
    s.view(&ps, &ns);
    rc = esc_load_pods(L, &ps, 0);
    if (!rc) rc = esc_load_nodes(L, &ns, 0, n);
    if (!rc) rc = esc_sort_nodes(L);
    int64_t cnt = 0;
    if (!rc) rc = esc_group_order(L, 0, oldest ? 0 : 1, idx_out, std::max<int64_t>(0, std::min(n_take, n)), &cnt);
    return rc;
}

// ------------------------------------------------------- sizes, ownership, communicators
int32_t esc_ctx_counts(const esc_ctx* c, int64_t* n_pod_ids, int64_t* n_nodes) {
    if (!c || !n_pod_ids || !n_nodes) return ESC_E_INVAL;
    if (c->multi) return esc::multi_counts(c, n_pod_ids, n_nodes);
    *n_pod_ids = c->pods_loaded ? (int64_t)c->pod_cls.size() : 0;
    *n_nodes = c->nodes_loaded ? c->n_nodes : 0;
    return ESC_OK;
}

int32_t esc_group_owner(const esc_ctx* c, int32_t group, int32_t* rank) {
    if (!c || !rank || group < 0 || group >= c->gi.G) return ESC_E_INVAL;
    if (c->multi) return esc_group_owner(esc::multi_sub(c, 0), group, rank);   // every device knows the split
    if (!c->nodes_loaded) return ESC_E_STATE;
    const uint32_t q = c->gi.gpair[group];
    *rank = (int32_t)(std::upper_bound(c->q_bounds.begin(), c->q_bounds.end() - 1, q) - c->q_bounds.begin()) - 1;
    return ESC_OK;
}

int32_t esc_node_owner_ranges(const esc_ctx* c, const esc_node_soa* s, int32_t world, uint32_t* q_bounds) {
    if (!c || !s || !q_bounds || world < 1 || s->n_nodes < 0) return ESC_E_INVAL;
    if (s->n_nodes > 0 && (!s->flags || !s->label0 || (s->n_xl > 0 && !s->xl_pair))) return ESC_E_INVAL;
    int64_t sx = 0;
    for (int64_t i = 0; i < s->n_nodes; ++i) sx += nf_xlbl(s->flags[i]);
    if (sx != s->n_xl) return ESC_E_INVAL;
    const std::vector<int64_t> cnt = pair_counts(c, s);
    for (int32_t r = 0; r < world; ++r) {
        uint32_t a = 0, b = 0;
        owned_pairs(cnt, world, r, a, b);
        q_bounds[r] = a;
    }
    q_bounds[world] = c->gi.n_gp;
    return ESC_OK;
}

int32_t esc_comm_size(const esc_ctx* c, int32_t* ranks) {
    if (!c || !ranks) return ESC_E_INVAL;
    if (c->multi) { *ranks = esc::multi_size(c); return ESC_OK; }
    if (!c->comm) return ESC_E_STATE;
    int n = 0;
    const ncclResult_t r = rccl().count(reinterpret_cast<ncclComm_t>(c->comm), &n);
    if (r != ncclSuccess) return fail_comm("ncclCommCount", rccl().error_string(r));
    *ranks = n;
    return ESC_OK;
}

// ------------------------------------------------------- scalar decision math
int32_t esc_calc_percent_usage(int64_t cpu_req_m, int64_t mem_req_b, int64_t cpu_cap_m, int64_t mem_cap_b,
                               int64_t n_untainted, double* cpu_pct, double* mem_pct) {
    if (!cpu_pct || !mem_pct) return ESC_E_INVAL;
    return percent_usage(cpu_req_m, mem_req_b, cpu_cap_m, mem_cap_b, n_untainted, cpu_pct, mem_pct);
}

int32_t esc_calc_scale_up_delta(int64_t n_untainted, double cpu_pct, double mem_pct, int64_t cpu_req_m,
                                int64_t mem_req_b, int64_t cached_cpu_m, int64_t cached_mem_b, int32_t scale_up_pct,
                                int64_t* delta) {
    if (!delta) return ESC_E_INVAL;
    return scale_up_delta(n_untainted, cpu_pct, mem_pct, cpu_req_m, mem_req_b, cached_cpu_m, cached_mem_b,
                          scale_up_pct, delta);
}

}  // extern "C"
