// esc_multi.hip — one process driving several MI355X (esc_ctx_create_multi).
//
// The reference is one Go binary whose RunOnce walks every node group on one goroutine
// (cmd/main.go:187, pkg/controller/controller.go:416-445).  A drop-in for it on an
// 8-GPU node is therefore ONE process and ONE context that fans out internally
// (SURVEY.md §8b): the context returned by esc_ctx_create_multi holds one per-device
// context per GPU (rank i of n: pods [lo_i, hi_i) of the loaded snapshot, the whole node
// table with the node side of the group pairs it owns) and a communicator set from
// ncclCommInitAll.  A decision enqueues every device's shard step, the in-place
// ncclReduceScatter(int64, SUM) of the exchange words inside ncclGroupStart / ncclGroupEnd
// (every device receives the sums of the groups it owns), and every device's
// K4 over its own groups, all from the calling thread; esc_results merges the owners'
// records.  The layer is a client of the
// per-device ABI (esc_reduce / esc_exchange_buffers / esc_decide ...): it adds the fan-out,
// the routing of pod ids to shards and the exchange.
//
// Exchange modes: RCCL when the devices are distinct (the default); a peer exchange —
// every device sums its own slice of everyone's words over peer-mapped memory with one
// kernel, ordered by HIP events — when ESC_EXCHANGE=peer is set or a device is listed twice
// (several shards on one GPU: how the fan-out, routing and exchange are exercised on a
// one-GPU machine).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "esc_internal.h"
#include "esc_kernels.h"
#include "esc_multi.h"

namespace esc {

struct esc_multi_state {
    std::vector<esc_ctx*> subs;              // per-device contexts, rank = index
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;           // RCCL communicators (empty: peer exchange)
    std::vector<int64_t> pod_lo;             // first input pod id of each device's shard
    // peer exchange: each device's summed words, and the events that order the reads
    std::vector<int64_t*> psum;
    int64_t psum_n = 0;
    std::vector<uint32_t*> psum32;
    int64_t psum32_n = 0;
    std::vector<hipEvent_t> ev_done, ev_read;
    // a node event applied on some devices but failed on a later one: the devices' node
    // tables differ, so decisions are refused (ESC_E_STATE) until the nodes are reloaded
    bool diverged = false;
};

namespace {

esc_multi_state& M(const esc_ctx* c) { return *ctx_multi(c); }
int nsub(const esc_ctx* c) { return (int)M(c).subs.size(); }

// f(i) for every device, each on its own host thread (loads and calibration are host- and
// PCIe-bound per device); the first non-zero status.
template <class F>
int32_t par(const esc_ctx* c, F&& f) {
    const int k = nsub(c);
    std::vector<int32_t> rc(k, ESC_OK);
    if (k == 1) return f(0);
    std::vector<std::thread> th;
    th.reserve(k);
    for (int i = 0; i < k; ++i) th.emplace_back([&, i] { rc[i] = f(i); });
    for (auto& t : th) t.join();
    for (int32_t r : rc)
        if (r) return r;
    return ESC_OK;
}

template <class F>
int32_t seq(const esc_ctx* c, F&& f) {
    for (int i = 0; i < nsub(c); ++i)
        if (int32_t rc = f(i)) return rc;
    return ESC_OK;
}

// The device whose shard holds input pod id `id` (ids past the loaded ones are inserts:
// the last device takes them).
int owner_of_pod(const esc_ctx* c, int64_t id) {
    const auto& lo = M(c).pod_lo;
    return (int)(std::upper_bound(lo.begin(), lo.end(), id) - lo.begin()) - 1;
}

// Sums every device's `words[j][off[i], off[i] + n)` into device i's own buffer over
// peer-mapped memory (off: the slice device i needs — its owned rows — or 0): the sums wait
// for every device's producer (ev_done), the write-backs for every sum (ev_read), so no
// buffer is rewritten while a peer still reads it.
template <class T>
int32_t peer_exchange(esc_ctx* c, const std::vector<T*>& words, const std::vector<int64_t>& off, int64_t n,
                      std::vector<T*>& tmp, int64_t& tmp_n, bool all_devices) {
    esc_multi_state& m = M(c);
    const int k = nsub(c);
    if (tmp_n < n) {
        for (int i = 0; i < k; ++i) {
            hipSetDevice(m.devices[i]);
            if (tmp[i]) hipFree(tmp[i]);
            tmp[i] = nullptr;
            if (hipMalloc(reinterpret_cast<void**>(&tmp[i]), (size_t)std::max<int64_t>(n, 1) * sizeof(T)) != hipSuccess)
                return ESC_E_NOMEM;
        }
        tmp_n = n;
    }
    std::vector<const T*> src(k);
    for (int i = 0; i < k; ++i) {
        hipSetDevice(m.devices[i]);
        if (hipEventRecord(m.ev_done[i], ctx_stream(m.subs[i])) != hipSuccess) return ESC_E_HIP;
    }
    const int n_dst = all_devices ? k : 1;
    for (int i = 0; i < n_dst; ++i) {
        hipSetDevice(m.devices[i]);
        hipStream_t st = ctx_stream(m.subs[i]);
        for (int j = 0; j < k; ++j)
            if (j != i && hipStreamWaitEvent(st, m.ev_done[j], 0) != hipSuccess) return ESC_E_HIP;
        for (int j = 0; j < k; ++j) src[j] = words[j] + off[i];
        hipError_t e;
        if constexpr (sizeof(T) == 8) e = launch_peer_sum64(reinterpret_cast<const int64_t* const*>(src.data()), k,
                                                             reinterpret_cast<int64_t*>(tmp[i]), n, st);
        else e = launch_peer_sum32(reinterpret_cast<const uint32_t* const*>(src.data()), k,
                                   reinterpret_cast<uint32_t*>(tmp[i]), n, st);
        if (e != hipSuccess) return fail_hip(e, "peer exchange");
        if (hipEventRecord(m.ev_read[i], st) != hipSuccess) return ESC_E_HIP;
    }
    for (int i = 0; i < k; ++i) {
        hipSetDevice(m.devices[i]);
        hipStream_t st = ctx_stream(m.subs[i]);
        for (int j = 0; j < n_dst; ++j)
            if (j != i && hipStreamWaitEvent(st, m.ev_read[j], 0) != hipSuccess) return ESC_E_HIP;
        if (i < n_dst && n > 0 &&
            hipMemcpyAsync(words[i] + off[i], tmp[i], (size_t)n * sizeof(T), hipMemcpyDeviceToDevice, st) != hipSuccess)
            return ESC_E_HIP;
    }
    return ESC_OK;
}

// Every device's slice of the SUM of the devices' pod words (esc_exchange_buffers, owner-
// major rows): a reduce-scatter, each device receiving the rows of the groups it owns.
int32_t exchange_words(esc_ctx* c) {
    esc_multi_state& m = M(c);
    const int k = nsub(c);
    std::vector<int64_t*> buf(k);
    std::vector<int64_t> off(k);
    int64_t n = 0;
    for (int i = 0; i < k; ++i) {
        void* b = nullptr;
        int64_t cnt = 0;
        if (int32_t rc = esc_exchange_buffers(m.subs[i], &b, &cnt, nullptr, nullptr)) return rc;
        if (int32_t rc = esc_exchange_slice(m.subs[i], &off[i], &n)) return rc;
        buf[i] = reinterpret_cast<int64_t*>(b);
    }
    // timing mode: every device's exchange ends a stage of its own (bench.py exchange_ms)
    auto marks = [&]() -> int32_t {
        for (int i = 0; i < k; ++i)
            if (int32_t rc = ctx_stage_mark(m.subs[i])) return rc;
        return ESC_OK;
    };
    if (m.comms.empty()) {
        if (int32_t rc = peer_exchange<int64_t>(c, buf, off, n, m.psum, m.psum_n, true)) return rc;
        return marks();
    }
    const RcclApi& r = rccl();
    ncclResult_t e = r.group_start();
    for (int i = 0; i < k && e == ncclSuccess; ++i) {
        hipSetDevice(m.devices[i]);
        e = r.reduce_scatter(buf[i], buf[i] + off[i], (size_t)n, ncclInt64, ncclSum, m.comms[i], ctx_stream(m.subs[i]));
    }
    const ncclResult_t e2 = r.group_end();
    if (e != ncclSuccess) return fail_comm("ncclReduceScatter", r.error_string(e));
    if (e2 != ncclSuccess) return fail_comm("ncclGroupEnd", r.error_string(e2));
    return marks();
}

// Pods of the batch that go to device i, as a packed SoA of their own.
struct PodBatch {
    std::vector<int64_t> ids;
    std::vector<uint32_t> flags, cpu0, pair0, xp;
    std::vector<int64_t> mem0, xc_cpu, xc_mem;
    esc_pod_soa view() const {
        esc_pod_soa s;
        s.n_pods = (int64_t)flags.size();
        s.flags = flags.data(); s.cpu0 = cpu0.data(); s.mem0 = mem0.data(); s.pair0 = pair0.data();
        s.xc_cpu = xc_cpu.data(); s.xc_mem = xc_mem.data(); s.n_xc = (int64_t)xc_cpu.size();
        s.xp_pair = xp.data(); s.n_xp = (int64_t)xp.size();
        return s;
    }
};

}  // namespace

void multi_destroy(esc_ctx* c) {
    esc_multi_state* m = ctx_multi(c);
    if (!m) return;
    for (size_t i = 0; i < m->subs.size(); ++i) {
        hipSetDevice(m->devices[i]);
        hipStreamSynchronize(ctx_stream(m->subs[i]));
    }
    for (ncclComm_t x : m->comms)
        if (x) rccl().destroy(x);
    for (size_t i = 0; i < m->subs.size(); ++i) {
        hipSetDevice(m->devices[i]);
        if (i < m->psum.size() && m->psum[i]) hipFree(m->psum[i]);
        if (i < m->psum32.size() && m->psum32[i]) hipFree(m->psum32[i]);
        if (i < m->ev_done.size() && m->ev_done[i]) hipEventDestroy(m->ev_done[i]);
        if (i < m->ev_read.size() && m->ev_read[i]) hipEventDestroy(m->ev_read[i]);
        esc_ctx_destroy(m->subs[i]);
    }
    delete m;
    ctx_set_multi(c, nullptr);
}

esc_ctx* multi_sub(const esc_ctx* c, int i) {
    const esc_multi_state* m = ctx_multi(c);
    return (m && i >= 0 && i < (int)m->subs.size()) ? m->subs[i] : nullptr;
}

int32_t multi_size(const esc_ctx* c) {
    const esc_multi_state& m = M(c);
    if (m.comms.empty()) return 0;                      // the peer exchange: no communicator
    int n = 0;
    return rccl().count(m.comms[0], &n) == ncclSuccess ? n : -1;
}

int32_t multi_each(esc_ctx* c, int32_t (*fn)(esc_ctx*, int32_t), int32_t arg) {
    return seq(c, [&](int i) { return fn(M(c).subs[i], arg); });
}

int32_t multi_set_replicas(esc_ctx* c, int32_t n) {
    return seq(c, [&](int i) { return esc_set_replicas(M(c).subs[i], n); });
}

// The snapshot's pods in n contiguous, balanced shards (rank order = input order).
int32_t multi_load_pods(esc_ctx* c, const esc_pod_soa* p, int64_t global_offset) {
    if (!p || p->n_pods < 0) return ESC_E_INVAL;
    const int64_t n = p->n_pods;
    if (n > 0 && !p->flags) return ESC_E_INVAL;
    const int k = nsub(c);
    std::vector<int64_t> lo(k + 1), xc(k + 1), xp(k + 1);
    for (int i = 0; i <= k; ++i) lo[i] = (int64_t)((__int128)n * i / k);
    int64_t oc = 0, op = 0;
    for (int i = 0, b = 0; i <= k; ++i) {
        for (; b < lo[i]; ++b) { oc += pf_xctr(p->flags[b]); op += pf_xpair(p->flags[b]); }
        xc[i] = oc;
        xp[i] = op;
    }
    if (xc[k] != p->n_xc || xp[k] != p->n_xp) return ESC_E_INVAL;
    const int32_t rc = par(c, [&](int i) {
        esc_pod_soa v;
        v.n_pods = lo[i + 1] - lo[i];
        v.flags = p->flags ? p->flags + lo[i] : nullptr;
        v.cpu0 = p->cpu0 ? p->cpu0 + lo[i] : nullptr;
        v.mem0 = p->mem0 ? p->mem0 + lo[i] : nullptr;
        v.pair0 = p->pair0 ? p->pair0 + lo[i] : nullptr;
        v.xc_cpu = p->xc_cpu ? p->xc_cpu + xc[i] : nullptr;
        v.xc_mem = p->xc_mem ? p->xc_mem + xc[i] : nullptr;
        v.n_xc = xc[i + 1] - xc[i];
        v.xp_pair = p->xp_pair ? p->xp_pair + xp[i] : nullptr;
        v.n_xp = xp[i + 1] - xp[i];
        return esc_load_pods(M(c).subs[i], &v, global_offset + lo[i]);
    });
    if (rc) return rc;
    M(c).pod_lo.assign(lo.begin(), lo.end() - 1);
    return ESC_OK;
}

int32_t multi_load_nodes(esc_ctx* c, const esc_node_soa* s, int64_t lo, int64_t hi) {
    const int32_t rc = par(c, [&](int i) { return esc_load_nodes(M(c).subs[i], s, lo, hi); });
    M(c).diverged = rc != ESC_OK && nsub(c) > 1;             // some devices may hold the new table
    return rc;
}

int32_t multi_stream_bytes(const esc_ctx* c, int64_t* pod_bytes, int64_t* node_bytes) {
    if (!pod_bytes || !node_bytes) return ESC_E_INVAL;
    *pod_bytes = *node_bytes = 0;
    return seq(c, [&](int i) {
        int64_t a = 0, b = 0;
        if (int32_t rc = esc_stream_bytes(M(c).subs[i], &a, &b)) return rc;
        *pod_bytes += a;
        *node_bytes += b;
        return (int32_t)ESC_OK;
    });
}

int32_t multi_set_state(esc_ctx* c, const esc_group_state* st) {
    return seq(c, [&](int i) { return esc_set_state(M(c).subs[i], st); });
}

// One decision: every device's shard step (K1, the fused tail, node groups: the exchange
// words), the SUM across the devices (RCCL group call, or the peer exchange), every
// device's K4.  Asynchronous like esc_run; esc_sync / esc_results wait.
int32_t multi_step(esc_ctx* c) {
    if (M(c).diverged) return ESC_E_STATE;
    if (int32_t rc = seq(c, [&](int i) { return esc_reduce(M(c).subs[i]); })) return rc;
    if (int32_t rc = exchange_words(c)) return rc;
    return seq(c, [&](int i) { return esc_decide(M(c).subs[i]); });
}

// Every device is waited for even when one reports (ESC_E_ORDER leaves the others' work
// queued otherwise); the first error is returned.
int32_t multi_sync(esc_ctx* c) {
    int32_t first = ESC_OK;
    for (int i = 0; i < nsub(c); ++i)
        if (int32_t rc = esc_sync(M(c).subs[i]); rc && !first) first = rc;
    return first;
}

// Every group's records from the device that owns it (each device decided its own groups).
int32_t multi_results(esc_ctx* c, esc_group_totals* t, esc_group_decision* d) {
    if (int32_t rc = multi_sync(c); rc && rc != ESC_E_ORDER) return rc;   // orderings apart, the records are valid
    const int k = nsub(c);
    if (k == 1) return esc_results(M(c).subs[0], t, d);
    const int32_t G = esc_ctx_num_groups(M(c).subs[0]);
    std::vector<esc_group_totals> tt((size_t)G);
    std::vector<esc_group_decision> dd((size_t)G);
    for (int i = 0; i < k; ++i) {
        if (int32_t rc = esc_results(M(c).subs[i], t ? tt.data() : nullptr, d ? dd.data() : nullptr)) return rc;
        for (int32_t g = 0; g < G; ++g) {
            int32_t owner = 0;
            if (int32_t rc = esc_group_owner(M(c).subs[i], g, &owner)) return rc;
            if (owner != i) continue;
            if (t) t[g] = tt[(size_t)g];
            if (d) d[g] = dd[(size_t)g];
        }
    }
    return ESC_OK;
}

int32_t multi_metrics_results(esc_ctx* c, esc_group_metrics* out) {
    const int k = nsub(c);
    if (k == 1) return esc_metrics_results(M(c).subs[0], out);
    const int32_t G = esc_ctx_num_groups(M(c).subs[0]);
    std::vector<esc_group_metrics> mm((size_t)G);
    for (int i = 0; i < k; ++i) {
        if (int32_t rc = esc_metrics_results(M(c).subs[i], mm.data())) return rc;
        for (int32_t g = 0; g < G; ++g) {
            int32_t owner = 0;
            if (int32_t rc = esc_group_owner(M(c).subs[i], g, &owner)) return rc;
            if (owner == i) out[g] = mm[(size_t)g];
        }
    }
    return ESC_OK;
}

int32_t multi_k1_calibrate(esc_ctx* c, int32_t rounds) {
    return par(c, [&](int i) { return esc_k1_calibrate(M(c).subs[i], rounds); });
}

// ---------------------------------------------------------------- informer events
int32_t multi_pods_upsert(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p) {
    if (!p || p->n_pods < 0 || (p->n_pods > 0 && (!ids || !p->flags || !p->cpu0 || !p->mem0 || !p->pair0)))
        return ESC_E_INVAL;
    const int k = nsub(c);
    if (M(c).pod_lo.empty()) return ESC_E_STATE;
    std::vector<PodBatch> b(k);
    int64_t oc = 0, op = 0;
    for (int64_t i = 0; i < p->n_pods; ++i) {
        const uint32_t f = p->flags[i], nc = pf_xctr(f), nx = pf_xpair(f);
        if (oc + nc > p->n_xc || op + nx > p->n_xp) return ESC_E_INVAL;
        if (ids[i] < 0) return ESC_E_INVAL;
        const int s = owner_of_pod(c, ids[i]);
        PodBatch& x = b[s];
        x.ids.push_back(ids[i] - M(c).pod_lo[s]);
        x.flags.push_back(f);
        x.cpu0.push_back(p->cpu0[i]);
        x.mem0.push_back(p->mem0[i]);
        x.pair0.push_back(p->pair0[i]);
        for (uint32_t r = 0; r < nc; ++r) { x.xc_cpu.push_back(p->xc_cpu[oc + r]); x.xc_mem.push_back(p->xc_mem[oc + r]); }
        for (uint32_t r = 0; r < nx; ++r) x.xp.push_back(p->xp_pair[op + r]);
        oc += nc;
        op += nx;
    }
    if (oc != p->n_xc || op != p->n_xp) return ESC_E_INVAL;
    // every device's share checked before any is applied: all or nothing across devices
    for (int s = 0; s < k; ++s) {
        if (b[s].ids.empty()) continue;
        const esc_pod_soa v = b[s].view();
        if (int32_t rc = pods_upsert_check(M(c).subs[s], b[s].ids.data(), &v)) return rc;
    }
    for (int s = 0; s < k; ++s) {
        if (b[s].ids.empty()) continue;
        const esc_pod_soa v = b[s].view();
        if (int32_t rc = esc_pods_upsert(M(c).subs[s], b[s].ids.data(), &v)) return rc;
    }
    return ESC_OK;
}

int32_t multi_pods_delete(esc_ctx* c, const int64_t* ids, int64_t n) {
    if (n < 0 || (n > 0 && !ids)) return ESC_E_INVAL;
    const int k = nsub(c);
    if (M(c).pod_lo.empty()) return ESC_E_STATE;
    std::vector<std::vector<int64_t>> b(k);
    for (int64_t i = 0; i < n; ++i) {
        if (ids[i] < 0) return ESC_E_INVAL;
        const int s = owner_of_pod(c, ids[i]);
        b[s].push_back(ids[i] - M(c).pod_lo[s]);
    }
    for (int s = 0; s < k; ++s) {                             // ids known to their device: checked first
        int64_t np = 0, nn = 0;
        if (int32_t rc = esc_ctx_counts(M(c).subs[s], &np, &nn)) return rc;
        for (int64_t id : b[s])
            if (id >= np) return ESC_E_INVAL;
    }
    for (int s = 0; s < k; ++s)
        if (!b[s].empty())
            if (int32_t rc = esc_pods_delete(M(c).subs[s], b[s].data(), (int64_t)b[s].size())) return rc;
    return ESC_OK;
}

int32_t multi_pods_bind(esc_ctx* c, const int64_t* ids, const uint32_t* pod_node, int64_t n) {
    if (n < 0 || (n > 0 && (!ids || !pod_node))) return ESC_E_INVAL;
    const int k = nsub(c);
    if (M(c).pod_lo.empty()) return ESC_E_STATE;
    std::vector<std::vector<int64_t>> bi(k);
    std::vector<std::vector<uint32_t>> bn(k);
    for (int64_t i = 0; i < n; ++i) {
        if (ids[i] < 0) return ESC_E_INVAL;
        const int s = owner_of_pod(c, ids[i]);
        bi[s].push_back(ids[i] - M(c).pod_lo[s]);
        bn[s].push_back(pod_node[i]);
    }
    for (int s = 0; s < k; ++s)
        if (!bi[s].empty())
            if (int32_t rc = pods_bind_check(M(c).subs[s], bi[s].data(), bn[s].data(), (int64_t)bi[s].size())) return rc;
    for (int s = 0; s < k; ++s)
        if (!bi[s].empty())
            if (int32_t rc = esc_pods_bind(M(c).subs[s], bi[s].data(), bn[s].data(), (int64_t)bi[s].size())) return rc;
    return ESC_OK;
}

// Node events reach every device (each holds the whole node table); their checks depend
// on that table only, so the devices accept or refuse a batch alike: device
// 0's refusal leaves every device untouched.  A failure on a later device (a HIP error after
// device 0 applied the batch) leaves the tables different: the context is marked diverged
// and refuses decisions until esc_load_nodes.
template <class F>
int32_t node_event(esc_ctx* c, F&& f) {
    esc_multi_state& m = M(c);
    if (m.diverged) return ESC_E_STATE;
    for (int i = 0; i < nsub(c); ++i)
        if (int32_t rc = f(i)) {
            if (i > 0) m.diverged = true;
            return i > 0 ? (int32_t)ESC_E_STATE : rc;
        }
    return ESC_OK;
}

int32_t multi_nodes_update(esc_ctx* c, const int64_t* ids, int64_t n, const uint32_t* flags, const int64_t* cpu,
                           const int64_t* mem) {
    return node_event(c, [&](int i) { return esc_nodes_update(M(c).subs[i], ids, n, flags, cpu, mem); });
}

int32_t multi_nodes_relabel(esc_ctx* c, const int64_t* ids, const esc_node_soa* s) {
    if (M(c).diverged) return ESC_E_STATE;
    if (int32_t rc = nodes_relabel_check(M(c).subs[0], ids, s)) return rc;   // nothing applied anywhere
    return node_event(c, [&](int i) { return esc_nodes_relabel(M(c).subs[i], ids, s); });
}

int32_t multi_nodes_add(esc_ctx* c, const esc_node_soa* s, int64_t* ids_out) {
    if (!s || s->n_nodes < 0 || (s->n_nodes > 0 && !ids_out)) return ESC_E_INVAL;
    std::vector<int64_t> tmp((size_t)std::max<int64_t>(s->n_nodes, 1));
    return node_event(c, [&](int i) {
        int64_t* out = i == 0 ? ids_out : tmp.data();
        const int32_t rc = esc_nodes_add(M(c).subs[i], s, out);
        if (rc == ESC_OK && i > 0 && s->n_nodes > 0 && std::memcmp(out, ids_out, (size_t)s->n_nodes * 8) != 0)
            return (int32_t)ESC_E_STATE;                      // the devices' tables diverged: never expected
        return rc;
    });
}

int32_t multi_nodes_delete(esc_ctx* c, const int64_t* ids, int64_t n) {
    return node_event(c, [&](int i) { return esc_nodes_delete(M(c).subs[i], ids, n); });
}

int32_t multi_tracker_update(esc_ctx* c, int32_t group, const int64_t* add, int64_t n_add, const int64_t* rm,
                             int64_t n_rm) {
    return node_event(c, [&](int i) { return esc_tracker_update(M(c).subs[i], group, add, n_add, rm, n_rm); });
}

// ------------------------------------------------------------------------ reaping
int32_t multi_load_placement(esc_ctx* c, const uint32_t* pod_node, const int64_t* taint_s, const uint8_t* no_delete) {
    if (M(c).pod_lo.empty()) return ESC_E_STATE;
    return seq(c, [&](int i) {
        return esc_load_placement(M(c).subs[i], pod_node ? pod_node + M(c).pod_lo[i] : nullptr, taint_s, no_delete);
    });
}

// TryRemoveTaintedNodes over the pod shards: every device's K6 counts its pods per tainted
// node, the occupancy words are summed across the devices, K7 runs on device 0.
int32_t multi_try_remove(esc_ctx* c, int64_t now_ns, const int64_t* soft, const int64_t* hard, esc_removal* out) {
    if (!soft || !hard || !out) return ESC_E_INVAL;
    esc_multi_state& m = M(c);
    const int k = nsub(c);
    std::vector<uint32_t*> buf(k);
    int64_t n = 0;
    for (int i = 0; i < k; ++i) {
        if (int32_t rc = esc_reap_occupancy(m.subs[i])) return rc;
        void* b = nullptr;
        if (int32_t rc = esc_reap_buffer(m.subs[i], &b, &n)) return rc;
        buf[i] = reinterpret_cast<uint32_t*>(b);
    }
    if (m.comms.empty()) {
        if (int32_t rc = peer_exchange<uint32_t>(c, buf, std::vector<int64_t>((size_t)k, 0), n, m.psum32, m.psum32_n,
                                                 false))
            return rc;
    } else {
        const RcclApi& r = rccl();
        ncclResult_t e = r.group_start();
        for (int i = 0; i < k && e == ncclSuccess; ++i) {
            hipSetDevice(m.devices[i]);
            e = r.all_reduce(buf[i], buf[i], (size_t)n, ncclUint32, ncclSum, m.comms[i], ctx_stream(m.subs[i]));
        }
        const ncclResult_t e2 = r.group_end();
        if (e != ncclSuccess) return fail_comm("ncclAllReduce", r.error_string(e));
        if (e2 != ncclSuccess) return fail_comm("ncclGroupEnd", r.error_string(e2));
    }
    return esc_reap_finish(m.subs[0], now_ns, soft, hard, out);
}

// ----------------------------------------------------------------------- ordering
int32_t multi_order_info(const esc_ctx* c, int64_t* n_memb, int32_t* key_bits) {
    if (!n_memb || !key_bits) return ESC_E_INVAL;
    int64_t total = 0;
    const int32_t rc = seq(c, [&](int i) {
        int64_t x = 0;
        if (int32_t r = esc_order_info(M(c).subs[i], &x, key_bits)) return r;
        total += x;
        return (int32_t)ESC_OK;
    });
    *n_memb = total;
    return rc;
}

// A group's orderings live on the device that owns its pair.
int32_t multi_group_order(esc_ctx* c, int32_t group, int32_t which, int64_t* idx, int64_t cap, int64_t* n_out) {
    int32_t owner = 0;
    if (int32_t rc = esc_group_owner(c, group, &owner)) return rc;
    return esc_group_order(M(c).subs[owner], group, which, idx, cap, n_out);
}

int32_t multi_counts(const esc_ctx* c, int64_t* n_pod_ids, int64_t* n_nodes) {
    const esc_multi_state& m = M(c);
    int64_t np = 0, nn = 0;
    if (int32_t rc = esc_ctx_counts(m.subs.back(), &np, &nn)) return rc;
    *n_pod_ids = m.pod_lo.empty() ? 0 : m.pod_lo.back() + np;
    return esc_ctx_counts(m.subs[0], &np, n_nodes);
}

}  // namespace esc

using namespace esc;

extern "C" int32_t esc_ctx_create_multi(const esc_group_spec* groups, int32_t n_groups, const int32_t* devices,
                                        int32_t n_dev, esc_ctx** out) {
    if (!out || !devices || n_dev < 1 || n_dev > 16) return ESC_E_INVAL;
    *out = nullptr;
    esc_ctx* c = nullptr;
    int32_t rc = esc_ctx_create(groups, n_groups, -1, 0, 1, &c);   // host side: groups, pair ids, packer
    if (rc) return rc;
    esc_multi_state* m = new (std::nothrow) esc_multi_state();
    if (!m) { esc_ctx_destroy(c); return ESC_E_NOMEM; }
    ctx_set_multi(c, m);
    auto fail = [&](int32_t r) { esc_ctx_destroy(c); return r; };   // destroys m and its devices too
    m->devices.assign(devices, devices + n_dev);
    m->subs.assign(n_dev, nullptr);
    for (int i = 0; i < n_dev; ++i)
        if ((rc = esc_ctx_create(groups, n_groups, devices[i], i, n_dev, &m->subs[i])) != ESC_OK) {
            m->subs.resize(i);
            return fail(rc);
        }
    std::vector<int> d(m->devices);
    std::sort(d.begin(), d.end());
    const bool distinct = std::adjacent_find(d.begin(), d.end()) == d.end();
    const char* mode = std::getenv("ESC_EXCHANGE");
    const bool peer = !distinct || (mode && std::strcmp(mode, "peer") == 0);
    if (!peer) {
        if (!rccl().ok) return fail(fail_comm("esc_ctx_create_multi", "librccl not found"));
        m->comms.assign(n_dev, nullptr);
        const ncclResult_t r = rccl().init_all(m->comms.data(), n_dev, m->devices.data());
        if (r != ncclSuccess) {
            m->comms.clear();
            return fail(fail_comm("ncclCommInitAll", rccl().error_string(r)));
        }
    } else {
        for (int i = 0; i < n_dev; ++i)                     // peer mappings between distinct devices
            for (int j = 0; j < n_dev; ++j)
                if (m->devices[i] != m->devices[j]) {
                    hipSetDevice(m->devices[i]);
                    const hipError_t e = hipDeviceEnablePeerAccess(m->devices[j], 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(fail_hip(e, "peer access"));
                    (void)hipGetLastError();
                }
        m->psum.assign(n_dev, nullptr);
        m->psum32.assign(n_dev, nullptr);
        m->ev_done.assign(n_dev, nullptr);
        m->ev_read.assign(n_dev, nullptr);
        for (int i = 0; i < n_dev; ++i) {
            hipSetDevice(m->devices[i]);
            if (hipEventCreateWithFlags(&m->ev_done[i], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&m->ev_read[i], hipEventDisableTiming) != hipSuccess)
                return fail(ESC_E_HIP);
        }
    }
    *out = c;
    return ESC_OK;
}
