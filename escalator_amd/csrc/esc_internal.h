// esc_internal.h — host-side structures shared by the runtime, the packer and the
// synthetic generator.
#pragma once

#include <stdint.h>
#include <string>
#include <unordered_map>
#include <vector>

#include "esc_common.h"

namespace esc {

// Owned copy of one NodeGroupOptions' hot-path fields.
struct GroupSpecCopy {
    std::string name, key, value;
    esc_group_spec spec;   // string pointers re-pointed at the members above
};

// (key,value) interning against the configured groups.  Each group selects exactly one
// (label_key, label_value) pair (node_group.go:290-303), so a pair maps to the set of
// groups sharing it.  The set is stored as a chain: head = lowest-index group with the
// pair, next[g] = next higher-index group with the same pair.  Pods use the chain that
// excludes the "default" group (its pods come from NewPodDefaultFilterFunc instead,
// client.go:58-64); nodes use the chain over all groups (node_group.go:301).
struct GroupIndex {
    int32_t G = 0;
    int32_t default_group = -1;
    std::vector<GroupSpecCopy> groups;
    std::unordered_map<std::string, uint32_t> pod_head, node_head;
    std::vector<uint32_t> pod_next, node_next;
    bool pod_chains = false, node_chains = false;

    static std::string pair_key(const char* k, const char* v) {
        std::string s(k ? k : "");
        s.push_back('\0');
        s.append(v ? v : "");
        return s;
    }
    void build(const esc_group_spec* specs, int32_t n);
    uint32_t head(const char* k, const char* v, int side) const {
        const auto& m = side == 0 ? pod_head : node_head;
        auto it = m.find(pair_key(k, v));
        return it == m.end() ? NONE : it->second;
    }
};

// Host-side packed snapshot (owned vectors) produced by the packer or the generator.
struct HostSnapshot {
    std::vector<uint32_t> flags, cpu0, pair0;
    std::vector<int64_t> mem0, xc_cpu, xc_mem;
    std::vector<uint32_t> xp;
    std::vector<uint32_t> nflags, label0, xl;
    std::vector<int64_t> ncpu, nmem, created;
    std::vector<int32_t> trk_node, trk_group;

    void view(esc_pod_soa* p, esc_node_soa* n) const;
};

}  // namespace esc
