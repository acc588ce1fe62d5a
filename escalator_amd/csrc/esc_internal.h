// esc_internal.h — host-side structures shared by the runtime, the packer and the
// synthetic generator.
#pragma once

#include <stdint.h>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <unordered_map>
#include <vector>

#include "esc_common.h"

namespace esc {

// Owned copy of one NodeGroupOptions' hot-path fields.
struct GroupSpecCopy {
    std::string name, key, value;
    esc_group_spec spec;   // string pointers re-pointed at the members above
};

// The groups' selector pairs and the pair -> groups tables the kernels resolve.
// Each group selects exactly one (label_key, label_value) pair (node_group.go:290-303);
// pair ids 0 .. n_gp-1 are the distinct group pairs in order of first appearance
// (the numbering rule of include/escalator_hip.h).  A pair may be shared by several
// groups, so each node-table entry is a "code": a single group id, NONE, or
// CODE_MULTI | offset of a [count, g...] list in `code_list` (node_group.go:301).
// Pods are accumulated per pair and joined to groups through `gpair` (the "default"
// group takes its pods from NewPodDefaultFilterFunc instead, client.go:58-64).
struct GroupIndex {
    int32_t G = 0;
    int32_t default_group = -1;
    std::vector<GroupSpecCopy> groups;
    std::unordered_map<std::string, uint32_t> pair_ids;   // group pair -> id
    std::unordered_map<std::string, int> keys;            // label keys some group uses
    uint32_t n_gp = 0;
    std::vector<uint32_t> gpair;                          // group -> pair id
    std::vector<uint32_t> node_code, code_list;

    static std::string pair_key(const char* k, const char* v) {
        std::string s(k ? k : "");
        s.push_back('\0');
        s.append(v ? v : "");
        return s;
    }
    void build(const esc_group_spec* specs, int32_t n);
    uint32_t pair_id(const char* k, const char* v) const {
        auto it = pair_ids.find(pair_key(k, v));
        return it == pair_ids.end() ? NONE : it->second;
    }
    bool is_key(const char* k) const { return keys.count(std::string(k ? k : "")) != 0; }
};

// std::vector whose resize() leaves new elements default-initialised (no zero fill): the
// host snapshot's arrays are written in full by their producers (the packer's parallel
// merge, the generator), so a 100 M-pod resize costs no single-threaded memset.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind { using other = DefaultInitAlloc<U>; };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) { ::new ((void*)p) U; }
    template <class U, class... A>
    void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T>
using hvec = std::vector<T, DefaultInitAlloc<T>>;

// Host-side packed snapshot (owned vectors) produced by the packer or the generator.
struct HostSnapshot {
    hvec<uint32_t> flags, cpu0, pair0;
    hvec<int64_t> mem0, xc_cpu, xc_mem;
    hvec<uint32_t> xp;
    hvec<uint32_t> nflags, label0, xl;
    hvec<int64_t> ncpu, nmem, created;
    hvec<int32_t> trk_node, trk_group;

    void view(esc_pod_soa* p, esc_node_soa* n) const;
};

// Per-call drop-ins over object slices (esc_list.hip): reusable pinned buffers and one
// small kernel per call, no snapshot layout (esc_pods_requests_total, util.go:27;
// esc_nodes_capacity_total, util.go:41).  stream: the context's hipStream_t.
struct ListReducer;
int32_t list_pods_requests_total(ListReducer*& r, int device, void* stream, const esc_pod_obj* pods, int64_t n,
                                 int64_t* mem_b, int64_t* cpu_m);
int32_t list_nodes_capacity_total(ListReducer*& r, int device, void* stream, const esc_node_obj* nodes, int64_t n,
                                  int64_t* mem_b, int64_t* cpu_m);
void list_reducer_free(ListReducer*& r);
// esc_hbm_probe's streaming read (esc_list.hip)
int32_t hbm_probe(int device, void* stream, int64_t bytes, int32_t reps, double* gbps);

}  // namespace esc
