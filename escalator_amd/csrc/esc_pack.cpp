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
#include <cstring>
#include <new>
#include <set>

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
    std::unordered_map<std::string, uint32_t> other_pairs;   // group-key values no group selects
};

namespace {

inline int64_t req_or(int32_t has, int64_t v, int64_t absent) { return has ? v : absent; }

// Pair id of (key, value) for a key some group uses: the group pair's id, or a
// packer-local id >= n_gp for a value no group selects (the numbering rule of
// include/escalator_hip.h).  Returns false when the id space is exhausted.
bool intern(esc_packer* pk, const char* k, const char* v, uint32_t& id) {
    id = pk->gi->pair_id(k, v);
    if (id != NONE) return true;
    const std::string key = GroupIndex::pair_key(k, v);
    auto it = pk->other_pairs.find(key);
    if (it != pk->other_pairs.end()) { id = it->second; return true; }
    const uint64_t nid = (uint64_t)pk->gi->n_gp + pk->other_pairs.size();
    if (nid >= ESC_PAIR_LIMIT) return false;
    id = (uint32_t)nid;
    pk->other_pairs.emplace(key, id);
    return true;
}

void sort_unique(std::vector<uint32_t>& v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
}

int32_t pack_pod(esc_packer* pk, const esc_pod_obj& o) {
    HostSnapshot& s = pk->s;
    uint32_t f = 0;
    std::vector<uint32_t> pairs;
    if (!pk->list_mode) {
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
            if (!pk->gi->is_key(kv.key)) continue;
            uint32_t id;
            if (!intern(pk, kv.key, kv.value, id)) return ESC_E_LIMIT;
            pairs.push_back(id);
        }
        if (o.has_affinity && o.has_node_affinity && o.has_required) {     // unwrapNodeSelectorTerms :208
            for (int32_t e = 0; e < o.n_exprs; ++e) {
                const esc_selector_expr& x = o.exprs[e];
                if (!x.op || std::strcmp(x.op, "In") != 0) continue;         // only In (:241)
                if (!pk->gi->is_key(x.key)) continue;
                for (int32_t v = 0; v < x.n_values; ++v) {
                    uint32_t id;
                    if (!intern(pk, x.key, x.values[v], id)) return ESC_E_LIMIT;
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

int32_t pack_node(esc_packer* pk, const esc_node_obj& o) {
    HostSnapshot& s = pk->s;
    uint32_t f = 0;
    std::vector<uint32_t> pairs;
    if (!pk->list_mode) {
        if (o.unschedulable) f |= ESC_NF_UNSCHED;                            // controller.go:141
        for (int32_t i = 0; i < o.n_taints; ++i)                             // taint.go:81-85
            if (o.taint_keys[i] && std::strcmp(o.taint_keys[i], "atlassian.com/escalator") == 0) { f |= ESC_NF_TAINTED; break; }
        for (int32_t i = 0; i < o.n_labels; ++i) {                           // node_group.go:280
            if (!pk->gi->is_key(o.labels[i].key)) continue;                  // Labels[K] for group keys
            uint32_t id;
            if (!intern(pk, o.labels[i].key, o.labels[i].value, id)) return ESC_E_LIMIT;
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
    pk->node_names.emplace_back(o.name ? o.name : "");
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
    for (int64_t i = 0; i < n; ++i) {
        int32_t rc = pack_pod(pk, pods[i]);
        if (rc != ESC_OK) return rc;
    }
    return ESC_OK;
}

int32_t esc_packer_add_nodes(esc_packer* pk, const esc_node_obj* nodes, int64_t n) {
    if (!pk || (n > 0 && !nodes) || n < 0) return ESC_E_INVAL;
    if (pk->finished) return ESC_E_STATE;
    for (int64_t i = 0; i < n; ++i) {
        int32_t rc = pack_node(pk, nodes[i]);
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
        // Resolve taintTracker names (controller.go:128-133) to (node, group) entries.
        std::unordered_map<std::string, std::vector<int64_t>> by_name;
        bool any = false;
        for (auto& t : pk->trackers) any |= !t.empty();
        if (any) {
            for (size_t i = 0; i < pk->node_names.size(); ++i) by_name[pk->node_names[i]].push_back((int64_t)i);
            std::vector<std::pair<int32_t, int32_t>> ent;
            for (int32_t g = 0; g < (int32_t)pk->trackers.size(); ++g)
                for (auto& nm : pk->trackers[g]) {
                    auto it = by_name.find(nm);
                    if (it == by_name.end()) continue;
                    for (int64_t idx : it->second) ent.emplace_back((int32_t)idx, g);
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
