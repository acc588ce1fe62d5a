// esc_pack.cpp — K0 host packer / interner.
//
// Replaces the object walk each group's lister performs on every scan
// (FilteredPodsLister.List pkg/k8s/pod_listers.go:33, FilteredNodesLister.List
// pkg/k8s/node_listers.go:33) by ONE pass that turns *v1.Pod / *v1.Node field copies
// into the struct-of-arrays the kernels stream:
//   - (key,value) strings whose key some group filters on are interned to pair ids
//     (node_group.go:226-247, :280); which groups a pair selects is resolved on the
//     device (K1/K2) through the context's pair tables;
//   - the group-independent predicates PodIsDaemonSet (util.go:11), PodIsStatic
//     (util.go:21) and the default filter's selector/affinity tests
//     (node_group.go:271-273) become flag bits;
//   - container requests become the (inline + extra records) encoding that
//     ComputePodResourceRequest (scheduler/types.go:72-89) is evaluated on by K1.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <set>
#include <string_view>
#include <thread>

#include "esc_internal.h"

using namespace esc;

void GroupIndex::build(const esc_group_spec* specs, int32_t n) {
    G = n;
    groups.resize(n);
    default_group = -1;
    for (int32_t g = 0; g < n; ++g) {
        GroupSpecCopy& c = groups[g];
        c.name = specs[g].name ? specs[g].name : "";
        c.key = specs[g].label_key ? specs[g].label_key : "";
        c.value = specs[g].label_value ? specs[g].label_value : "";
        c.spec = specs[g];
        // pkg/controller/client.go:59 — the lister choice is by name; names are map keys
        // in the reference (controller.go:93), so at most one "default" exists.
        if (c.name == "default" && default_group < 0) default_group = g;
    }
    // Re-point after the vector is final (no reallocation below).
    for (auto& c : groups) { c.spec.name = c.name.c_str(); c.spec.label_key = c.key.c_str(); c.spec.label_value = c.value.c_str(); }
    pair_ids.clear();
    keys.clear();
    gpair.assign(n, NONE);
    std::vector<std::vector<uint32_t>> node_groups;   // per pair id, ascending
    for (int32_t g = 0; g < n; ++g) {
        keys[groups[g].key] = 1;
        const std::string k = pair_key(groups[g].key.c_str(), groups[g].value.c_str());
        auto it = pair_ids.find(k);
        uint32_t id;
        if (it == pair_ids.end()) {
            id = (uint32_t)pair_ids.size();
            pair_ids.emplace(k, id);
            node_groups.emplace_back();
        } else {
            id = it->second;
        }
        gpair[g] = id;
        // node entries carry the dry-mode bit (node classes depend on it, controller.go:115-117)
        node_groups[id].push_back((uint32_t)g | (groups[g].spec.dry_mode ? NODE_DRY_BIT : 0u));
    }
    n_gp = (uint32_t)pair_ids.size();
    fast_pairs = PairTable();
    fast_keys = PairTable();
    for (int32_t g = 0; g < n; ++g) {
        if (fast_pairs.find(groups[g].key.c_str(), groups[g].value.c_str()) == NONE)
            fast_pairs.insert(groups[g].key.c_str(), groups[g].value.c_str(), gpair[g]);
        if (fast_keys.find(groups[g].key.c_str(), "") == NONE) fast_keys.insert(groups[g].key.c_str(), "", 1);
    }
    code_list.clear();
    auto encode = [&](const std::vector<uint32_t>& gs) -> uint32_t {
        if (gs.empty()) return NONE;
        if (gs.size() == 1) return gs[0];
        const uint32_t off = (uint32_t)code_list.size();
        code_list.push_back((uint32_t)gs.size());
        code_list.insert(code_list.end(), gs.begin(), gs.end());
        return CODE_MULTI | off;
    };
    node_code.resize(n_gp);
    for (uint32_t i = 0; i < n_gp; ++i) node_code[i] = encode(node_groups[i]);
}

void HostSnapshot::view(esc_pod_soa* p, esc_node_soa* n) const {
    if (p) {
        p->n_pods = (int64_t)flags.size();
        p->flags = flags.data(); p->cpu0 = cpu0.data(); p->mem0 = mem0.data(); p->pair0 = pair0.data();
        p->xc_cpu = xc_cpu.data(); p->xc_mem = xc_mem.data(); p->n_xc = (int64_t)xc_cpu.size();
        p->xp_pair = xp.data(); p->n_xp = (int64_t)xp.size();
    }
    if (n) {
        n->n_nodes = (int64_t)nflags.size();
        n->flags = nflags.data(); n->label0 = label0.data(); n->cpu = ncpu.data(); n->mem = nmem.data();
        n->created_ns = created.data(); n->xl_pair = xl.data(); n->n_xl = (int64_t)xl.size();
        n->trk_node = trk_node.data(); n->trk_group = trk_group.data(); n->n_trk = (int64_t)trk_node.size();
    }
}

struct esc_packer {
    const GroupIndex* gi = nullptr;
    bool list_mode = false;
    bool finished = false;
    HostSnapshot s;
    std::vector<std::string> node_names;
    std::vector<std::vector<std::string>> trackers;
    PairTable other_pairs;                                   // group-key values no group selects
};

namespace {

inline int64_t req_or(int32_t has, int64_t v, int64_t absent) { return has ? v : absent; }

// Pair id of (key, value) for a key some group uses: the group pair's id, or a
// packer-local id >= n_gp for a value no group selects (the numbering rule of
// include/escalator_hip.h).  Returns false when the id space is exhausted.
bool intern(esc_packer* pk, const char* k, size_t kl, uint64_t ks, const char* v, uint32_t& id) {
    size_t vl;
    const uint64_t h = PairTable::value_hash(ks, v, vl);
    v = v ? v : "";
    id = pk->gi->fast_pairs.find_h(h, k, kl, v, vl);
    if (id != NONE) return true;
    id = pk->other_pairs.find_h(h, k, kl, v, vl);
    if (id != NONE) return true;
    const uint64_t nid = (uint64_t)pk->gi->n_gp + pk->other_pairs.size();
    if (nid >= ESC_PAIR_LIMIT) return false;
    id = (uint32_t)nid;
    pk->other_pairs.insert_h(h, k, kl, v, vl, id);
    return true;
}

void sort_unique(std::vector<uint32_t>& v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
}

// One pod into `s` (HostSnapshot or a parallel part: the same member names); `in(k, kl,
// key_state, v, id)` interns a pair.  `pairs` is scratch.
template <class Out, class Intern>
int32_t pack_pod(const GroupIndex* gi, bool list_mode, const esc_pod_obj& o, Out& s, Intern&& in,
                 std::vector<uint32_t>& pairs) {
    uint32_t f = 0;
    pairs.clear();
    if (!list_mode) {
        for (int32_t i = 0; i < o.n_owner_kinds; ++i)                        // util.go:12-16
            if (o.owner_kinds[i] && std::strcmp(o.owner_kinds[i], "DaemonSet") == 0) { f |= ESC_PF_DAEMONSET; break; }
        if (o.has_config_source && o.config_source && std::strcmp(o.config_source, "file") == 0)
            f |= ESC_PF_STATIC;                                              // util.go:22-23
        if (o.n_node_selector > 0) f |= ESC_PF_HAS_SEL;                      // node_group.go:271
        if (o.has_affinity && (o.has_node_affinity || o.has_pod_affinity || o.has_pod_anti_affinity))
            f |= ESC_PF_AFF_BLOCK;                                           // node_group.go:271-273
        // The (key, value) pairs NewPodAffinityFilterFunc can match on (node_group.go:226-249):
        // Spec.NodeSelector entries and the values of "In" expressions of the required
        // node-affinity terms, for keys some group filters on.  As a set: a group counts
        // a pod once however many routes match.  K1 resolves pair -> groups.
        for (int32_t i = 0; i < o.n_node_selector; ++i) {
            const esc_kv& kv = o.node_selector[i];
            size_t kl;
            const uint64_t ks = PairTable::key_state(kv.key, kl);
            const char* k = kv.key ? kv.key : "";
            if (!gi->is_key_s(ks, k, kl)) continue;
            uint32_t id;
            if (!in(k, kl, ks, kv.value, id)) return ESC_E_LIMIT;
            pairs.push_back(id);
        }
        if (o.has_affinity && o.has_node_affinity && o.has_required) {     // unwrapNodeSelectorTerms :208
            for (int32_t e = 0; e < o.n_exprs; ++e) {
                const esc_selector_expr& x = o.exprs[e];
                if (!x.op || std::strcmp(x.op, "In") != 0) continue;         // only In (:241)
                size_t kl;
                const uint64_t ks = PairTable::key_state(x.key, kl);
                const char* k = x.key ? x.key : "";
                if (!gi->is_key_s(ks, k, kl)) continue;
                for (int32_t v = 0; v < x.n_values; ++v) {
                    uint32_t id;
                    if (!in(k, kl, ks, x.values[v], id)) return ESC_E_LIMIT;
                    pairs.push_back(id);
                }
            }
        }
        sort_unique(pairs);
    } else {
        pairs.push_back(0);                                                  // the list group's pair
    }
    if (pairs.size() > 1 + ESC_PF_PAIR_MASK) return ESC_E_LIMIT;   // > 64 distinct pairs
    const uint32_t pair0 = pairs.empty() ? NONE : pairs[0];
    for (size_t i = 1; i < pairs.size(); ++i) s.xp.push_back(pairs[i]);
    f |= (uint32_t)(pairs.empty() ? 0 : pairs.size() - 1) << ESC_PF_XPAIR_SHIFT;

    // Containers: the first regular container is inline when its cpu fits u32.
    uint32_t cpu0 = 0;
    int64_t mem0 = 0;
    int32_t first_extra = 0;
    if (o.n_containers > 0) {
        const esc_request& c = o.containers[0];
        int64_t cpu = req_or(c.has_cpu, c.cpu_m, 0);
        if (cpu >= 0 && cpu <= 0xFFFFFFFFll) {
            cpu0 = (uint32_t)cpu;
            mem0 = req_or(c.has_mem, c.mem_b, 0);
            first_extra = 1;
        }
    }
    const int32_t n_xreg = o.n_containers - first_extra;
    if (n_xreg > (int32_t)ESC_PF_CNT_MASK || o.n_init_containers > (int32_t)ESC_PF_CNT_MASK) return ESC_E_LIMIT;
    for (int32_t i = first_extra; i < o.n_containers; ++i) {             // Resource.Add types.go:14
        s.xc_cpu.push_back(req_or(o.containers[i].has_cpu, o.containers[i].cpu_m, 0));
        s.xc_mem.push_back(req_or(o.containers[i].has_mem, o.containers[i].mem_b, 0));
    }
    for (int32_t i = 0; i < o.n_init_containers; ++i) {                  // SetMaxResource types.go:30
        s.xc_cpu.push_back(req_or(o.init_containers[i].has_cpu, o.init_containers[i].cpu_m, INT64_MIN));
        s.xc_mem.push_back(req_or(o.init_containers[i].has_mem, o.init_containers[i].mem_b, INT64_MIN));
    }
    if (o.has_overhead && (o.overhead.has_cpu || o.overhead.has_mem)) {  // types.go:84-86
        s.xc_cpu.push_back(req_or(o.overhead.has_cpu, o.overhead.cpu_m, 0));
        s.xc_mem.push_back(req_or(o.overhead.has_mem, o.overhead.mem_b, 0));
        f |= ESC_PF_HAS_OVH;
    }
    f |= (uint32_t)n_xreg << ESC_PF_XREG_SHIFT;
    f |= (uint32_t)o.n_init_containers << ESC_PF_XINIT_SHIFT;
    s.flags.push_back(f);
    s.cpu0.push_back(cpu0);
    s.mem0.push_back(mem0);
    s.pair0.push_back(pair0);
    return ESC_OK;
}

template <class Out, class Intern>
int32_t pack_node(const GroupIndex* gi, bool list_mode, const esc_node_obj& o, Out& s,
                  std::vector<std::string>& names, Intern&& in, std::vector<uint32_t>& pairs) {
    uint32_t f = 0;
    pairs.clear();
    if (!list_mode) {
        if (o.unschedulable) f |= ESC_NF_UNSCHED;                            // controller.go:141
        for (int32_t i = 0; i < o.n_taints; ++i)                             // taint.go:81-85
            if (o.taint_keys[i] && std::strcmp(o.taint_keys[i], "atlassian.com/escalator") == 0) { f |= ESC_NF_TAINTED; break; }
        for (int32_t i = 0; i < o.n_labels; ++i) {                           // node_group.go:280
            size_t kl;
            const uint64_t ks = PairTable::key_state(o.labels[i].key, kl);
            const char* k = o.labels[i].key ? o.labels[i].key : "";
            if (!gi->is_key_s(ks, k, kl)) continue;                          // Labels[K] for group keys
            uint32_t id;
            if (!in(k, kl, ks, o.labels[i].value, id)) return ESC_E_LIMIT;
            pairs.push_back(id);
        }
        sort_unique(pairs);
    } else {
        pairs.push_back(0);
    }
    if (pairs.size() > 1 + ESC_PF_CNT_MASK) return ESC_E_LIMIT;
    s.label0.push_back(pairs.empty() ? NONE : pairs[0]);
    for (size_t i = 1; i < pairs.size(); ++i) s.xl.push_back(pairs[i]);
    f |= (uint32_t)(pairs.empty() ? 0 : pairs.size() - 1) << ESC_NF_XLBL_SHIFT;
    s.nflags.push_back(f);
    s.ncpu.push_back(req_or(o.allocatable.has_cpu, o.allocatable.cpu_m, 0));   // util.go:47 absent -> 0
    s.nmem.push_back(req_or(o.allocatable.has_mem, o.allocatable.mem_b, 0));
    s.created.push_back(o.created_unix_ns);
    names.emplace_back(o.name ? o.name : "");
    return ESC_OK;
}

// ---- the parallel packer (esc_packer_add_pods / _add_nodes over large slices)
// Objects are independent, so T threads each pack a contiguous chunk into a part of their
// own; the parts are then copied into the snapshot in chunk order.  The one shared piece of
// state is the interner of values no group selects (ids >= n_gp, numbered by first
// appearance): a part interns a value the packer does not know yet under a provisional id
// (PROV | its index in the part's new_keys), and the merge numbers the parts' new values in
// chunk order — exactly the sequential numbering — and rewrites the (rare) objects that used
// one, re-sorting their pair lists.  The output is identical to the sequential packer's.
constexpr uint32_t PROV = 0x80000000u;       // > every final id (< ESC_PAIR_LIMIT)
int64_t par_min() {                          // objects per call below which one thread packs
    const char* v = std::getenv("ESC_PACK_PAR_MIN");    // (tests lower it)
    return v ? std::max<int64_t>(1, std::atoll(v)) : (int64_t)1 << 16;
}

int host_threads() {
    int n = 0;
    for (const char* e : {"ESC_HOST_THREADS", "OMP_NUM_THREADS"})
        if (const char* v = std::getenv(e)) { n = std::atoi(v); if (n > 0) break; }
    if (n <= 0) n = std::min<int>(16, std::max(1u, std::thread::hardware_concurrency()));
    return std::max(1, std::min(n, 64));
}

struct Fix {                                  // an object whose pairs hold provisional ids
    int64_t item, xoff;                       // part-local index, its first extra pair
};

struct Part {
    // pods (HostSnapshot names)
    hvec<uint32_t> flags, cpu0, pair0, xp;
    hvec<int64_t> mem0, xc_cpu, xc_mem;
    // nodes
    hvec<uint32_t> nflags, label0, xl;
    hvec<int64_t> ncpu, nmem, created;
    std::vector<std::string> names;
    // the part's interner of values the packer did not know: (key, value) of each, in order
    std::vector<std::pair<std::string, std::string>> new_keys;
    PairTable local;
    std::vector<Fix> fix;
    int32_t rc = ESC_OK;
};

template <class F>
void run_parts(int64_t n, int T, F f) {
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { f(t, n * t / T, n * (t + 1) / T); });
    for (auto& x : th) x.join();
}

// the provisional-id interner of part P (the packer's known values are read-only meanwhile)
struct PartIntern {
    const esc_packer* pk;
    Part& P;
    bool used = false;
    bool operator()(const char* k, size_t kl, uint64_t ks, const char* v, uint32_t& id) {
        size_t vl;
        const uint64_t h = PairTable::value_hash(ks, v, vl);
        v = v ? v : "";
        id = pk->gi->fast_pairs.find_h(h, k, kl, v, vl);
        if (id != NONE) return true;
        id = pk->other_pairs.find_h(h, k, kl, v, vl);
        if (id != NONE) return true;
        id = P.local.find_h(h, k, kl, v, vl);
        if (id == NONE) {
            id = PROV | (uint32_t)P.new_keys.size();
            P.local.insert_h(h, k, kl, v, vl, id);
            P.new_keys.emplace_back(std::string(k, kl), std::string(v, vl));
        }
        used = true;
        return true;
    }
};

// Number the parts' new values in chunk order; remap[t][i] = final id of part t's value i.
int32_t merge_keys(esc_packer* pk, std::vector<Part>& parts, std::vector<std::vector<uint32_t>>& remap) {
    remap.assign(parts.size(), {});
    for (size_t t = 0; t < parts.size(); ++t)
        for (const auto& kv : parts[t].new_keys) {
            uint32_t id = pk->other_pairs.find(kv.first.c_str(), kv.second.c_str());
            if (id == NONE) {
                const uint64_t nid = (uint64_t)pk->gi->n_gp + pk->other_pairs.size();
                if (nid >= ESC_PAIR_LIMIT) return ESC_E_LIMIT;
                id = (uint32_t)nid;
                pk->other_pairs.insert(kv.first.c_str(), kv.second.c_str(), id);
            }
            remap[t].push_back(id);
        }
    return ESC_OK;
}

// The pair list (head + extras) of a fixed object with final ids, ascending again.
void refix(uint32_t& head, uint32_t* extra, uint32_t n_extra, const std::vector<uint32_t>& remap,
           std::vector<uint32_t>& tmp) {
    tmp.clear();
    if (head != NONE) tmp.push_back(head);
    tmp.insert(tmp.end(), extra, extra + n_extra);
    for (uint32_t& q : tmp)
        if (q != NONE && (q & PROV)) q = remap[q & ~PROV];
    std::sort(tmp.begin(), tmp.end());
    if (head != NONE) head = tmp[0];
    for (uint32_t k = 0; k < n_extra; ++k) extra[k] = tmp[k + 1];
}

template <class T, class A>
void append_at(hvec<T>& dst, size_t at, const std::vector<T, A>& src) {
    if (!src.empty()) std::memcpy(dst.data() + at, src.data(), src.size() * sizeof(T));
}

int32_t add_pods_parallel(esc_packer* pk, const esc_pod_obj* pods, int64_t n, int T) {
    std::vector<Part> parts(T);
    run_parts(n, T, [&](int t, int64_t lo, int64_t hi) {
        Part& P = parts[t];
        P.flags.reserve(hi - lo); P.cpu0.reserve(hi - lo); P.mem0.reserve(hi - lo); P.pair0.reserve(hi - lo);
        PartIntern in{pk, P};
        std::vector<uint32_t> scratch;
        for (int64_t i = lo; i < hi; ++i) {
            in.used = false;
            const int64_t xo = (int64_t)P.xp.size();
            const int32_t rc = pack_pod(pk->gi, pk->list_mode, pods[i], P, in, scratch);
            if (rc != ESC_OK) { P.rc = rc; return; }
            if (in.used) P.fix.push_back({i - lo, xo});
        }
    });
    for (const Part& P : parts)
        if (P.rc != ESC_OK) return P.rc;
    std::vector<std::vector<uint32_t>> remap;
    if (int32_t rc = merge_keys(pk, parts, remap)) return rc;
    HostSnapshot& s = pk->s;
    std::vector<size_t> b0(T + 1), bx(T + 1), bp(T + 1);
    b0[0] = s.flags.size(); bx[0] = s.xc_cpu.size(); bp[0] = s.xp.size();
    for (int t = 0; t < T; ++t) {
        b0[t + 1] = b0[t] + parts[t].flags.size();
        bx[t + 1] = bx[t] + parts[t].xc_cpu.size();
        bp[t + 1] = bp[t] + parts[t].xp.size();
    }
    s.flags.resize(b0[T]); s.cpu0.resize(b0[T]); s.mem0.resize(b0[T]); s.pair0.resize(b0[T]);
    s.xc_cpu.resize(bx[T]); s.xc_mem.resize(bx[T]); s.xp.resize(bp[T]);
    run_parts(T, T, [&](int t, int64_t, int64_t) {
        Part& P = parts[t];
        std::vector<uint32_t> tmp;
        for (const Fix& x : P.fix)
            refix(P.pair0[x.item], P.xp.data() + x.xoff, pf_xpair(P.flags[x.item]), remap[t], tmp);
        append_at(s.flags, b0[t], P.flags); append_at(s.cpu0, b0[t], P.cpu0);
        append_at(s.mem0, b0[t], P.mem0); append_at(s.pair0, b0[t], P.pair0);
        append_at(s.xc_cpu, bx[t], P.xc_cpu); append_at(s.xc_mem, bx[t], P.xc_mem);
        append_at(s.xp, bp[t], P.xp);
        P = Part();                                   // free the part early
    });
    return ESC_OK;
}

int32_t add_nodes_parallel(esc_packer* pk, const esc_node_obj* nodes, int64_t n, int T) {
    std::vector<Part> parts(T);
    run_parts(n, T, [&](int t, int64_t lo, int64_t hi) {
        Part& P = parts[t];
        PartIntern in{pk, P};
        std::vector<uint32_t> scratch;
        for (int64_t i = lo; i < hi; ++i) {
            in.used = false;
            const int64_t xo = (int64_t)P.xl.size();
            const int32_t rc = pack_node(pk->gi, pk->list_mode, nodes[i], P, P.names, in, scratch);
            if (rc != ESC_OK) { P.rc = rc; return; }
            if (in.used) P.fix.push_back({i - lo, xo});
        }
    });
    for (const Part& P : parts)
        if (P.rc != ESC_OK) return P.rc;
    std::vector<std::vector<uint32_t>> remap;
    if (int32_t rc = merge_keys(pk, parts, remap)) return rc;
    HostSnapshot& s = pk->s;
    std::vector<size_t> b0(T + 1), bl(T + 1);
    b0[0] = s.nflags.size(); bl[0] = s.xl.size();
    for (int t = 0; t < T; ++t) {
        b0[t + 1] = b0[t] + parts[t].nflags.size();
        bl[t + 1] = bl[t] + parts[t].xl.size();
    }
    s.nflags.resize(b0[T]); s.label0.resize(b0[T]); s.ncpu.resize(b0[T]); s.nmem.resize(b0[T]);
    s.created.resize(b0[T]); s.xl.resize(bl[T]);
    run_parts(T, T, [&](int t, int64_t, int64_t) {
        Part& P = parts[t];
        std::vector<uint32_t> tmp;
        for (const Fix& x : P.fix)
            refix(P.label0[x.item], P.xl.data() + x.xoff, nf_xlbl(P.nflags[x.item]), remap[t], tmp);
        append_at(s.nflags, b0[t], P.nflags); append_at(s.label0, b0[t], P.label0);
        append_at(s.ncpu, b0[t], P.ncpu); append_at(s.nmem, b0[t], P.nmem);
        append_at(s.created, b0[t], P.created); append_at(s.xl, bl[t], P.xl);
    });
    for (Part& P : parts)                             // names in order (one thread: strings)
        for (std::string& nm : P.names) pk->node_names.emplace_back(std::move(nm));
    return ESC_OK;
}

}  // namespace

// Implemented in esc_api.hip (needs the ctx layout).
namespace esc { const GroupIndex* ctx_group_index(const esc_ctx* ctx); }

extern "C" {

int32_t esc_packer_create(const esc_ctx* ctx, esc_packer** out) {
    if (!ctx || !out) return ESC_E_INVAL;
    esc_packer* pk = new (std::nothrow) esc_packer();
    if (!pk) return ESC_E_NOMEM;
    pk->gi = esc::ctx_group_index(ctx);
    pk->trackers.resize(pk->gi->G);
    *out = pk;
    return ESC_OK;
}

int32_t esc_packer_destroy(esc_packer* pk) { delete pk; return ESC_OK; }

int32_t esc_packer_set_list_mode(esc_packer* pk, int32_t list_mode) {
    if (!pk || !pk->s.flags.empty() || !pk->s.nflags.empty()) return ESC_E_STATE;
    pk->list_mode = list_mode != 0;
    return ESC_OK;
}

int32_t esc_packer_add_pods(esc_packer* pk, const esc_pod_obj* pods, int64_t n) {
    if (!pk || (n > 0 && !pods) || n < 0) return ESC_E_INVAL;
    if (pk->finished) return ESC_E_STATE;
    const int T = host_threads();
    if (n >= par_min() && T > 1) return add_pods_parallel(pk, pods, n, T);
    auto in = [pk](const char* k, size_t kl, uint64_t ks, const char* v, uint32_t& id) {
        return intern(pk, k, kl, ks, v, id);
    };
    std::vector<uint32_t> scratch;
    for (int64_t i = 0; i < n; ++i) {
        int32_t rc = pack_pod(pk->gi, pk->list_mode, pods[i], pk->s, in, scratch);
        if (rc != ESC_OK) return rc;
    }
    return ESC_OK;
}

int32_t esc_packer_add_nodes(esc_packer* pk, const esc_node_obj* nodes, int64_t n) {
    if (!pk || (n > 0 && !nodes) || n < 0) return ESC_E_INVAL;
    if (pk->finished) return ESC_E_STATE;
    const int T = host_threads();
    if (n >= par_min() && T > 1) return add_nodes_parallel(pk, nodes, n, T);
    auto in = [pk](const char* k, size_t kl, uint64_t ks, const char* v, uint32_t& id) {
        return intern(pk, k, kl, ks, v, id);
    };
    std::vector<uint32_t> scratch;
    for (int64_t i = 0; i < n; ++i) {
        int32_t rc = pack_node(pk->gi, pk->list_mode, nodes[i], pk->s, pk->node_names, in, scratch);
        if (rc != ESC_OK) return rc;
    }
    return ESC_OK;
}

int32_t esc_packer_set_tracker(esc_packer* pk, int32_t group, const char* const* names, int64_t n) {
    if (!pk || group < 0 || group >= pk->gi->G || n < 0 || (n > 0 && !names)) return ESC_E_INVAL;
    if (pk->finished) return ESC_E_STATE;
    auto& t = pk->trackers[group];
    t.clear();
    for (int64_t i = 0; i < n; ++i) t.emplace_back(names[i] ? names[i] : "");
    return ESC_OK;
}

int32_t esc_packer_view(esc_packer* pk, esc_pod_soa* pods, esc_node_soa* nodes) {
    if (!pk) return ESC_E_INVAL;
    if (!pk->finished) {
        // Resolve taintTracker names (controller.go:128-133) to (node, group) entries: the
        // (few) tracked names in a table, then one pass over the node names (a table of
        // every node name cost ~0.5 s at 1 M nodes in the reload path)
        std::unordered_map<std::string_view, std::vector<int32_t>> groups_of;
        for (int32_t g = 0; g < (int32_t)pk->trackers.size(); ++g)
            for (auto& nm : pk->trackers[g]) groups_of[std::string_view(nm)].push_back(g);
        if (!groups_of.empty()) {
            std::vector<std::pair<int32_t, int32_t>> ent;
            for (size_t i = 0; i < pk->node_names.size(); ++i) {
                auto it = groups_of.find(std::string_view(pk->node_names[i]));
                if (it == groups_of.end()) continue;
                for (int32_t g : it->second) ent.emplace_back((int32_t)i, g);
            }
            std::sort(ent.begin(), ent.end());
            ent.erase(std::unique(ent.begin(), ent.end()), ent.end());
            for (auto& e : ent) {
                pk->s.trk_node.push_back(e.first);
                pk->s.trk_group.push_back(e.second);
                pk->s.nflags[e.first] |= ESC_NF_TRACKED;
            }
        }
        pk->finished = true;
    }
    pk->s.view(pods, nodes);
    return ESC_OK;
}

}  // extern "C"
