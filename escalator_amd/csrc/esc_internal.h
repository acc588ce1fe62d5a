// esc_internal.h — host-side structures shared by the runtime, the packer and the
// synthetic generator.
#pragma once

#include <stdint.h>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <unordered_map>
#include <vector>

#include "esc_common.h"

namespace esc {

// Interning table for (key, value) label pairs (and bare keys): open addressing over a
// 64-bit hash of the bytes "key\0value", the strings kept in one arena.  A lookup hashes the
// caller's C strings in place — no std::string is built per lookup, which dominated the
// packer (several lookups per pod at 1-2 M objects/s on one thread with std::unordered_map).
class PairTable {
public:
    // FNV-1a over the key bytes and a separator (not a byte of either string): the state a
    // key's values continue from, so a key is hashed once for all of its values
    static uint64_t key_state(const char* k, size_t& kl) {
        uint64_t h = 0xcbf29ce484222325ull;
        const char* p = k ? k : "";
        for (; *p; ++p) h = (h ^ (uint8_t)*p) * 0x100000001b3ull;
        kl = (size_t)(p - (k ? k : ""));
        return (h ^ 0xFFu) * 0x100000001b3ull;
    }
    static uint64_t finish(uint64_t h) {
        h ^= h >> 33;
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
        return h;
    }
    static uint64_t value_hash(uint64_t ks, const char* v, size_t& vl) {
        const char* q = v ? v : "";
        for (; *q; ++q) ks = (ks ^ (uint8_t)*q) * 0x100000001b3ull;
        vl = (size_t)(q - (v ? v : ""));
        return finish(ks);
    }
    static uint64_t hash(const char* k, const char* v, size_t& kl, size_t& vl) {
        return value_hash(key_state(k, kl), v, vl);
    }
    // id of (k, v), or NONE
    uint32_t find(const char* k, const char* v) const {
        size_t kl, vl;
        const uint64_t h = hash(k, v, kl, vl);
        return find_h(h, k ? k : "", kl, v ? v : "", vl);
    }
    uint32_t find_h(uint64_t h, const char* k, size_t kl, const char* v, size_t vl) const {
        if (slots_.empty()) return NONE;
        for (size_t i = h & mask_;; i = (i + 1) & mask_) {
            const Slot& s = slots_[i];
            if (s.id == NONE) return NONE;
            if (s.h == h && s.kl == kl && s.vl == vl && std::memcmp(arena_.data() + s.off, k, kl) == 0 &&
                std::memcmp(arena_.data() + s.off + kl, v, vl) == 0)
                return s.id;
        }
    }
    // inserts (k, v) -> id (the caller checked it is absent)
    void insert_h(uint64_t h, const char* k, size_t kl, const char* v, size_t vl, uint32_t id) {
        if ((n_ + 1) * 2 > slots_.size()) grow();
        const size_t off = arena_.size();
        arena_.append(k, kl);
        arena_.append(v, vl);
        place(Slot{h, off, (uint32_t)kl, (uint32_t)vl, id});
        ++n_;
    }
    void insert(const char* k, const char* v, uint32_t id) {
        size_t kl, vl;
        const uint64_t h = hash(k, v, kl, vl);
        insert_h(h, k ? k : "", kl, v ? v : "", vl, id);
    }
    size_t size() const { return n_; }

private:
    struct Slot {
        uint64_t h = 0;
        size_t off = 0;
        uint32_t kl = 0, vl = 0, id = NONE;
    };
    void place(const Slot& x) {
        for (size_t i = x.h & mask_;; i = (i + 1) & mask_)
            if (slots_[i].id == NONE) { slots_[i] = x; return; }
    }
    void grow() {
        std::vector<Slot> old;
        old.swap(slots_);
        slots_.assign(std::max<size_t>(64, old.size() * 2), Slot{});
        mask_ = slots_.size() - 1;
        for (const Slot& x : old)
            if (x.id != NONE) place(x);
    }
    std::vector<Slot> slots_;
    std::string arena_;
    size_t mask_ = 0, n_ = 0;
};

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
    PairTable fast_pairs, fast_keys;                       // the same sets, for the packer's lookups
    void build(const esc_group_spec* specs, int32_t n);
    uint32_t pair_id(const char* k, const char* v) const { return fast_pairs.find(k, v); }
    bool is_key(const char* k) const { return fast_keys.find(k, "") != NONE; }
    // is_key given the key's hash state (PairTable::key_state)
    bool is_key_s(uint64_t ks, const char* k, size_t kl) const {
        return fast_keys.find_h(PairTable::finish(ks), k, kl, "", 0) != NONE;
    }
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
