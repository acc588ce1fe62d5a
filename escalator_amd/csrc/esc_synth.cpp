// esc_synth.cpp — deterministic synthetic cluster snapshots.
//
// Every pod and node is a pure function of (seed, global index) through a counter
// hash, so a rank can generate exactly its shard, and tests can regenerate any slice.
// The generator emits the packed SoA directly, with the same encoding the K0 packer
// produces from objects (esc_pack.cpp); the object-level semantics each record stands
// for are documented inline so the CPU oracle can be checked against the packer path
// on small cases (tests/test_pack_parity.py).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "esc_internal.h"

using namespace esc;

namespace {

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline uint64_t rnd(uint64_t seed, uint64_t stream, uint64_t idx, uint64_t k) {
    return mix64(seed ^ mix64(stream * 0x9E3779B97F4A7C15ull + idx) ^ (k * 0xD1B54A32D192ED03ull));
}

constexpr int64_t MiB = int64_t(1) << 20;
constexpr int64_t GiB = int64_t(1) << 30;
constexpr int64_t BASE_NS = 1704067200LL * 1000000000LL;   // 2024-01-01T00:00:00Z

enum KeyId { K_CUSTOMER = 0, K_POOL = 1 };

template <class F>
void parallel_for(int64_t n, int threads, F f) {
    if (threads <= 1 || n < 4096) { f(0, n, 0); return; }
    std::vector<std::thread> ts;
    int64_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
        if (lo >= hi) break;
        ts.emplace_back([=] { f(lo, hi, t); });
    }
    for (auto& t : ts) t.join();
}

}  // namespace

struct esc_synth {
    esc_synth_params p{};
    int64_t p_lo = 0, p_hi = 0;
    std::vector<std::string> names, keys, values;
    std::vector<esc_group_spec> specs;
    std::vector<esc_group_state> states;
    GroupIndex gi;
    // per-group derived tables
    std::vector<int32_t> canon, key_id;
    std::vector<uint32_t> pair_of;                      // pair id of the group's own pair
    std::vector<int32_t> nondefault, pool_groups;
    std::vector<int64_t> type_cpu, type_mem;
    uint64_t default_bp = 0;        // basis points of pods that carry no selector at all
    int64_t mem_mib_max = 16384;    // per-container memory request range (MiB)
    HostSnapshot s;
    // object-level form of the same snapshot (esc_synth_objects), built on first use
    struct Objects {
        bool built = false;
        std::vector<esc_pod_obj> pods;
        std::vector<esc_node_obj> nodes;
        std::vector<esc_kv> kvs;
        std::vector<esc_selector_expr> exprs;
        std::vector<const char*> vals;
        std::vector<esc_request> reqs;
        std::vector<std::string> values, node_names;
    } obj;
};

namespace {

struct PodDesc {
    uint32_t pred = 0;
    uint32_t heads[16];                                 // selected pair ids
    int nheads = 0;
    // the object-level routes of the heads (esc_synth_objects): nodeSelector pairs, the
    // "In" values of the required node-affinity term, and the other object facts
    uint32_t sel[4], aff[8];
    int nsel = 0, naff = 0;
    bool not_in = false, pod_aff = false, zone = false;
    void add_sel(uint32_t h) { if (nsel < 4) sel[nsel++] = h; add_head(h); }
    void add_aff(uint32_t h) { if (naff < 8) aff[naff++] = h; add_head(h); }
    int n_reg = 0, n_init = 0;
    bool ovh = false;
    int64_t cpu[4], mem[4], icpu = 0, imem = 0, ocpu = 0, omem = 0;
    void add_head(uint32_t h) {
        if (h == NONE) return;
        for (int i = 0; i < nheads; ++i) if (heads[i] == h) return;
        heads[nheads++] = h;
    }
};

// Pair id of a (group key, value) that no group selects: the generator's own interning
// of "other" values, above the group pairs (numbering rule, include/escalator_hip.h).
// `v` < n_groups stands for the value "g<v>", larger ones for values no group uses.
uint32_t other_pair(const esc_synth& S, int key, uint32_t v) {
    return S.gi.n_gp + (uint32_t)key * ((uint32_t)S.p.n_groups + 2000u) + v;
}

// The object-level pod that index i stands for.  Its fields map 1:1 onto esc_pod_obj:
// owner kind DaemonSet, config.source=file, a nodeSelector, a required node affinity
// term with one "In" expression (and sometimes an extra NotIn), containers with
// requests (an absent key is encoded as the packer encodes it).
void gen_pod(const esc_synth& S, int64_t i, PodDesc& d) {
    const uint64_t seed = S.p.seed;
    const int32_t nnd = (int32_t)S.nondefault.size();
    auto pick = [&](uint64_t k) { return S.nondefault[rnd(seed, 1, i, k) % (uint64_t)nnd]; };
    const uint64_t r = rnd(seed, 1, i, 0) % 10000;
    if (S.p.config == 1) {                              // 1 group, every non-DS pod selects it
        if (r < 500) d.pred |= ESC_PF_DAEMONSET;
        d.pred |= ESC_PF_HAS_SEL;
        d.add_sel(S.pair_of[0]);
    } else if (r < 500) {                               // daemonset with a selector
        d.pred |= ESC_PF_DAEMONSET | ESC_PF_HAS_SEL;
        if (nnd) d.add_sel(S.pair_of[pick(1)]);
    } else if (r < 550) {                               // static pod, no selector
        d.pred |= ESC_PF_STATIC;
    } else if (r < 550 + S.default_bp) {                // default-group pod (~one group's share)
    } else if (r < 570 + S.default_bp) {                // PodAffinity only: blocks default, no pairs
        d.pred |= ESC_PF_AFF_BLOCK;
        d.pod_aff = true;
    } else if (nnd) {
        const uint64_t sub = rnd(seed, 1, i, 2) % 100;
        const int32_t g1 = pick(3);
        const int32_t k1 = S.key_id[g1];
        auto aff_head = [&](int32_t gk) {               // (key(g1), value(gk)) is a group pair
            const int32_t c = S.canon[gk];              // iff key(gk) == key(g1)
            return S.key_id[c] == k1 ? S.pair_of[c] : other_pair(S, k1, (uint32_t)c);
        };
        if (sub < 70) {                                 // nodeSelector only
            d.pred |= ESC_PF_HAS_SEL;
            d.add_sel(S.pair_of[g1]);
        } else if (sub < 90) {                          // affinity In with 1-3 values
            d.pred |= ESC_PF_AFF_BLOCK;
            const int nv = 1 + (int)(rnd(seed, 1, i, 4) % 3);
            d.add_aff(aff_head(g1));
            if (nv > 1) d.add_aff(aff_head(pick(5)));
            if (nv > 2) d.add_aff(aff_head(pick(6)));
        } else {                                        // both (duplicate pair -> counted once)
            d.pred |= ESC_PF_HAS_SEL | ESC_PF_AFF_BLOCK;
            d.add_sel(S.pair_of[g1]);
            d.add_aff(aff_head(g1));
            d.add_aff(aff_head(pick(7)));
        }
        const uint64_t x = rnd(seed, 1, i, 8) % 1000;
        if (x < 10) { d.pred |= ESC_PF_AFF_BLOCK; d.not_in = true; }   // extra NotIn expression (ignored)
        if (x >= 100 && x < 150 && !S.pool_groups.empty()) {   // extra "pool" selector
            d.pred |= ESC_PF_HAS_SEL;
            int32_t gp = S.pool_groups[rnd(seed, 1, i, 9) % S.pool_groups.size()];
            d.add_sel(S.pair_of[S.canon[gp]]);
        }
        if (x >= 200 && x < 300) { d.pred |= ESC_PF_HAS_SEL; d.zone = true; }   // "zone" selector: no group key, not carried
        if (x >= 300 && x < 330)                                // a customer value no group has
            d.add_aff(other_pair(S, K_CUSTOMER, (uint32_t)S.p.n_groups + (uint32_t)(rnd(seed, 1, i, 11) % 1000)));
    }
    std::sort(d.heads, d.heads + d.nheads);
    // Containers: 90% one, 6% two, 3% three, 1% two + one init + overhead.
    const uint64_t c = rnd(seed, 1, i, 10) % 100;
    d.n_reg = c < 90 ? 1 : c < 96 ? 2 : c < 99 ? 3 : 2;
    if (c >= 99) { d.n_init = 1; d.ovh = true; }
    for (int k = 0; k < d.n_reg; ++k) {
        const uint64_t a = rnd(seed, 1, i, 16 + k);
        d.cpu[k] = (a % 100 == 0) ? 0 : 1 + (int64_t)((a >> 8) % 4000);          // 1%: no cpu key
        const uint64_t b = rnd(seed, 1, i, 24 + k);
        d.mem[k] = (b % 100 == 1) ? 0 : (1 + (int64_t)((b >> 8) % (uint64_t)S.mem_mib_max)) * MiB +
                                        (int64_t)((b >> 32) & 0xFFFFF);
    }
    if (d.n_init) {
        const uint64_t a = rnd(seed, 1, i, 32);
        d.icpu = 1 + (int64_t)(a % 8000);
        d.imem = (1 + (int64_t)((a >> 16) % 32768)) * MiB;
    }
    if (d.ovh) {
        const uint64_t a = rnd(seed, 1, i, 33);
        d.ocpu = (int64_t)(a % 250);
        d.omem = (int64_t)((a >> 16) % (64 * MiB));
    }
}

uint32_t pod_flags(const PodDesc& d) {
    uint32_t f = d.pred;
    f |= (uint32_t)(d.n_reg - 1) << ESC_PF_XREG_SHIFT;
    f |= (uint32_t)d.n_init << ESC_PF_XINIT_SHIFT;
    if (d.ovh) f |= ESC_PF_HAS_OVH;
    f |= (uint32_t)(d.nheads > 0 ? d.nheads - 1 : 0) << ESC_PF_XPAIR_SHIFT;
    return f;
}

// Bijection on [0, n) (4-round Feistel over the next even power of two + cycle walk).
uint64_t permute(uint64_t x, uint64_t n, uint64_t seed) {
    int bits = 2;
    while ((1ull << bits) < n) bits += 2;
    const int h = bits / 2;
    const uint64_t mask = (1ull << h) - 1;
    do {
        uint64_t L = x >> h, R = x & mask;
        for (int r = 0; r < 4; ++r) {
            uint64_t F = mix64(R ^ (seed + 0x9E37ull * (r + 1))) & mask;
            uint64_t t = L ^ F;
            L = R;
            R = t;
        }
        x = (L << h) | R;
    } while (x >= n);
    return x;
}

void build_groups(esc_synth& S) {
    const esc_synth_params& p = S.p;
    const int32_t G = p.n_groups;
    S.names.resize(G); S.keys.resize(G); S.values.resize(G);
    S.canon.resize(G); S.key_id.resize(G);
    S.specs.resize(G); S.states.resize(G);
    S.type_cpu.resize(G); S.type_mem.resize(G);
    const bool dflt = p.with_default && p.config != 1;
    const int64_t npg = std::max<int64_t>(1, p.n_nodes / std::max(1, G));
    for (int32_t g = 0; g < G; ++g) {
        const uint64_t h = rnd(p.seed, 3, g, 0);
        char buf[64];
        if (p.config == 1) {
            S.names[g] = "ref"; S.keys[g] = "customer"; S.values[g] = "ref";
            S.canon[g] = g; S.key_id[g] = K_CUSTOMER;
        } else if (dflt && g == 0) {
            S.names[g] = "default"; S.keys[g] = "customer"; S.values[g] = "default";
            S.canon[g] = g; S.key_id[g] = K_CUSTOMER;
        } else {
            std::snprintf(buf, sizeof buf, "ng-%d", g);
            S.names[g] = buf;
            int32_t c = g;
            if (g % 64 == 62 && g - 2 >= (dflt ? 1 : 0)) c = g - 2;   // shares its pair with g-2
            S.canon[g] = c;
            S.key_id[g] = (c % 8 == 7) ? K_POOL : K_CUSTOMER;
            S.keys[g] = S.key_id[g] == K_POOL ? "pool" : "customer";
            std::snprintf(buf, sizeof buf, "g%d", c);
            S.values[g] = buf;
        }
        esc_group_spec& sp = S.specs[g];
        std::memset(&sp, 0, sizeof sp);
        esc_group_state& st = S.states[g];
        std::memset(&st, 0, sizeof st);
        if (p.config == 1) {
            sp.min_nodes = 5; sp.max_nodes = 100;
            sp.taint_lower_pct = 40; sp.taint_upper_pct = 60; sp.scale_up_pct = 70;
            sp.fast_removal_rate = 4; sp.slow_removal_rate = 2;
            S.type_cpu[g] = 64000; S.type_mem[g] = 256 * GiB;
        } else {
            sp.taint_lower_pct = 20 + (int32_t)(h % 21);
            sp.taint_upper_pct = sp.taint_lower_pct + 20 + (int32_t)((h >> 8) % 11);
            sp.scale_up_pct = sp.taint_upper_pct + 10 + (int32_t)((h >> 16) % 21);
            sp.slow_removal_rate = 1 + (int32_t)((h >> 24) % 3);
            sp.fast_removal_rate = sp.slow_removal_rate + 1 + (int32_t)((h >> 28) % 4);
            sp.min_nodes = 1 + (int32_t)((h >> 32) % 3);
            sp.max_nodes = (int32_t)std::min<int64_t>(npg * 3 + 10, 2000000000);
            const uint64_t gate = (h >> 40) % 100;
            if (gate == 0) sp.min_nodes = (int32_t)std::min<int64_t>(npg * 2 + 5, 2000000000);  // ERR_MIN
            if (gate == 1) sp.max_nodes = (int32_t)(npg / 2);                                  // ERR_MAX
            if (p.config == 5) sp.min_nodes = (int32_t)(npg * 3 / 4);                          // clamp active
            sp.dry_mode = (g % 16 == 5) ? 1 : 0;
            int64_t cpu_mult = 1 + (int64_t)((h >> 48) % 16);
            S.type_cpu[g] = 48000 * cpu_mult / (p.config == 3 ? 4 : 1);
            S.type_mem[g] = 256 * GiB * (1 + (int64_t)((h >> 52) % 8)) / (p.config == 3 ? 4 : 1) -
                            (int64_t)((h >> 4) % GiB);
            if ((h >> 56) % 100 < 3) { st.locked = 1; st.requested_nodes = 1 + (int32_t)((h >> 60) % 5); }
            if ((h >> 44) % 2) { st.cached_cpu_m = S.type_cpu[g]; st.cached_mem_b = S.type_mem[g]; }
        }
        sp.name = S.names[g].c_str();
        sp.label_key = S.keys[g].c_str();
        sp.label_value = S.values[g].c_str();
    }
    // Keep every group's sums pinned (mem_sum * 1000 < 2^63): the default
    // group gets about one group's share of pods, and config 3 (10M pods over 100 groups)
    // halves the per-container memory range.
    S.default_bp = dflt ? std::max<uint64_t>(1, std::min<uint64_t>(1000, 10000 / (uint64_t)G)) : 1000;
    S.mem_mib_max = p.config == 3 ? 8192 : 16384;
    S.gi.build(S.specs.data(), G);
    S.pair_of.assign(G, NONE);
    for (int32_t g = 0; g < G; ++g) {
        S.pair_of[g] = S.gi.gpair[g];
        if (g != S.gi.default_group) S.nondefault.push_back(g);
        if (S.key_id[g] == K_POOL && S.canon[g] == g) S.pool_groups.push_back(g);
    }
}

void gen_pods(esc_synth& S) {
    const int64_t n = S.p_hi - S.p_lo;
    const int threads = std::max(1, S.p.n_threads);
    HostSnapshot& s = S.s;
    s.flags.resize(n); s.cpu0.resize(n); s.mem0.resize(n); s.pair0.resize(n);
    std::vector<int64_t> xc_cnt(n), xp_cnt(n);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k) {
            PodDesc d;
            gen_pod(S, S.p_lo + k, d);
            s.flags[k] = pod_flags(d);
            s.cpu0[k] = (uint32_t)d.cpu[0];
            s.mem0[k] = d.mem[0];
            s.pair0[k] = d.nheads ? d.heads[0] : NONE;
            xc_cnt[k] = (d.n_reg - 1) + d.n_init + (d.ovh ? 1 : 0);
            xp_cnt[k] = d.nheads > 1 ? d.nheads - 1 : 0;
        }
    });
    int64_t ac = 0, ap = 0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t c = xc_cnt[k], q = xp_cnt[k];
        xc_cnt[k] = ac; xp_cnt[k] = ap;
        ac += c; ap += q;
    }
    s.xc_cpu.resize(ac); s.xc_mem.resize(ac); s.xp.resize(ap);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k) {
            const uint32_t f = s.flags[k];
            if (pf_xctr(f) == 0 && pf_xpair(f) == 0) continue;
            PodDesc d;
            gen_pod(S, S.p_lo + k, d);
            int64_t o = xc_cnt[k];
            for (int r = 1; r < d.n_reg; ++r) { s.xc_cpu[o] = d.cpu[r]; s.xc_mem[o] = d.mem[r]; ++o; }
            if (d.n_init) { s.xc_cpu[o] = d.icpu; s.xc_mem[o] = d.imem; ++o; }
            if (d.ovh) { s.xc_cpu[o] = d.ocpu; s.xc_mem[o] = d.omem; ++o; }
            int64_t q = xp_cnt[k];
            for (int h = 1; h < d.nheads; ++h) s.xp[q++] = d.heads[h];
        }
    });
}

void gen_nodes(esc_synth& S) {
    const esc_synth_params& p = S.p;
    const int64_t n = p.n_nodes;
    const int32_t G = p.n_groups;
    HostSnapshot& s = S.s;
    s.nflags.resize(n); s.label0.resize(n); s.ncpu.resize(n); s.nmem.resize(n); s.created.resize(n);
    struct Extra { uint32_t g[6]; uint8_t n; };
    std::vector<Extra> extra(n);
    std::vector<uint8_t> trk(n, 0);
    const int threads = std::max(1, p.n_threads);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t j = lo; j < hi; ++j) {
            const uint64_t a = rnd(p.seed, 2, j, 0);
            const int32_t g = (int32_t)(a % (uint64_t)G);
            const int32_t c = S.canon[g];
            uint32_t f = 0;
            const uint64_t b = rnd(p.seed, 2, j, 1) % 1000;
            if (b < 30) f |= ESC_NF_UNSCHED;
            else if (b < 130) f |= ESC_NF_TAINTED;
            // label pairs (group keys only): the group's own pair, sometimes a "pool" pair
            // as well; 1% of nodes carry a customer value no group has instead.
            uint32_t grp[8];
            int ng = 0;
            const bool orphan = p.config != 1 && rnd(p.seed, 2, j, 8) % 100 == 0;
            grp[ng++] = orphan ? other_pair(S, K_CUSTOMER, (uint32_t)G + 1000 + (uint32_t)(j % 97))
                               : S.pair_of[c];
            if (p.config != 1 && S.key_id[c] != K_POOL && !S.pool_groups.empty() &&
                rnd(p.seed, 2, j, 2) % 10 == 0) {
                const int32_t gp = S.pool_groups[rnd(p.seed, 2, j, 3) % S.pool_groups.size()];
                grp[ng++] = S.pair_of[S.canon[gp]];
            }
            std::sort(grp, grp + ng);
            s.label0[j] = ng ? grp[0] : NONE;
            Extra& e = extra[j];
            e.n = (uint8_t)(ng > 1 ? ng - 1 : 0);
            for (int k = 1; k < ng; ++k) e.g[k - 1] = grp[k];
            f |= (uint32_t)e.n << ESC_NF_XLBL_SHIFT;
            // dry-mode taintTracker: 10% of the members of dry groups
            if (S.specs[g].dry_mode && rnd(p.seed, 2, j, 4) % 10 == 0) trk[j] = 1;
            int64_t cpu = S.type_cpu[g], mem = S.type_mem[g];
            if (p.config == 3) {                                      // multi-instance-type groups
                const int64_t k = 1 + (int64_t)(rnd(p.seed, 2, j, 5) % 4);
                cpu = cpu * k / 2 - 70 * k;
                mem = mem / 2 * k - (int64_t)(rnd(p.seed, 2, j, 6) % GiB);
            }
            s.ncpu[j] = cpu;
            s.nmem[j] = mem;
            s.created[j] = BASE_NS + (int64_t)permute((uint64_t)j, (uint64_t)n, p.seed) * 1000 +
                           (int64_t)(rnd(p.seed, 2, j, 7) % 1000);
            s.nflags[j] = f;
        }
    });
    for (int64_t j = 0; j < n; ++j) {
        for (int k = 0; k < extra[j].n; ++k) s.xl.push_back(extra[j].g[k]);
        if (trk[j]) {
            const int32_t g = (int32_t)(rnd(p.seed, 2, j, 0) % (uint64_t)G);
            s.trk_node.push_back((int32_t)j);
            s.trk_group.push_back(g);
            s.nflags[j] |= ESC_NF_TRACKED;
        }
    }
}

// (key, value) strings of pair id q (a group pair, or one of the generator's other values).
struct PairNames {
    std::vector<const char*> key, val;                 // group pairs
    const esc_synth* S;
    const char* k(uint32_t q) const {
        if (q < key.size()) return key[q];
        return ((q - key.size()) / ((uint32_t)S->p.n_groups + 2000u)) == K_POOL ? "pool" : "customer";
    }
    const char* v(uint32_t q) const {
        if (q < val.size()) return val[q];
        return S->obj.values[(q - val.size()) % ((uint32_t)S->p.n_groups + 2000u)].c_str();
    }
};

// The esc_pod_obj / esc_node_obj fields each generated record stands for (what the cgo
// shim copies out of *v1.Pod / *v1.Node): owner kinds, the config.source annotation, a
// nodeSelector, a required node-affinity term ("In" values per key, an ignored NotIn),
// PodAffinity, containers.  Packing them reproduces the generator's snapshot up to the
// numbering of values no group selects and to flag bits no filter reads differently
// (tests/test_pack_parity.py compares totals).
void build_objects(esc_synth& S) {
    auto& O = S.obj;
    const uint32_t G = (uint32_t)S.p.n_groups, nv = G + 2000u;
    O.values.resize(nv);
    for (uint32_t v = 0; v < nv; ++v) O.values[v] = (v < G ? "g" : "x") + std::to_string(v);
    PairNames pn;
    pn.S = &S;
    pn.key.assign(S.gi.n_gp, "");
    pn.val.assign(S.gi.n_gp, "");
    for (int32_t g = (int32_t)G - 1; g >= 0; --g) { pn.key[S.gi.gpair[g]] = S.keys[g].c_str(); pn.val[S.gi.gpair[g]] = S.values[g].c_str(); }
    static const char* const kind_ds[] = {"DaemonSet"};
    static const char* const kind_rs[] = {"ReplicaSet"};
    static const char* const taint_esc[] = {"atlassian.com/escalator"};
    const int64_t n = S.p_hi - S.p_lo;
    // pass 1: sizes
    std::vector<int64_t> nkv(n + 1, 0), nex(n + 1, 0), nva(n + 1, 0), nrq(n + 1, 0);
    parallel_for(n, std::max(1, S.p.n_threads), [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k) {
            PodDesc d;
            gen_pod(S, S.p_lo + k, d);
            nkv[k] = d.nsel + (d.zone ? 1 : 0);
            nex[k] = 3;                                         // In per key (<= 2 keys), NotIn
            nva[k] = d.naff + d.nsel + 1;                       // a selector key given twice moves here
            nrq[k] = d.n_reg + d.n_init;
        }
    });
    auto scan = [](std::vector<int64_t>& v) { int64_t a = 0; for (auto& x : v) { const int64_t t = x; x = a; a += t; } };
    scan(nkv); scan(nex); scan(nva); scan(nrq);
    const HostSnapshot& h = S.s;
    const int64_t nn = (int64_t)h.nflags.size();
    O.pods.assign(n, esc_pod_obj{});
    O.kvs.resize(std::max<int64_t>(nkv[n] + 2 * nn + (int64_t)h.xl.size(), 1));   // pods', then the nodes' labels
    O.exprs.resize(std::max<int64_t>(nex[n], 1));
    O.vals.resize(std::max<int64_t>(nva[n], 1));
    O.reqs.resize(std::max<int64_t>(nrq[n], 1));
    parallel_for(n, std::max(1, S.p.n_threads), [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k) {
            PodDesc d;
            gen_pod(S, S.p_lo + k, d);
            esc_pod_obj& o = O.pods[k];
            const bool ds = (d.pred & ESC_PF_DAEMONSET) != 0;
            o.owner_kinds = ds ? kind_ds : kind_rs;
            o.n_owner_kinds = 1;
            o.has_config_source = (d.pred & ESC_PF_STATIC) ? 1 : 0;
            o.config_source = o.has_config_source ? "file" : "";
            esc_kv* kv = O.kvs.data() + nkv[k];
            esc_selector_expr* ex = O.exprs.data() + nex[k];
            const char** va = O.vals.data() + nva[k];
            int nk = 0, ne = 0, nvv = 0;
            for (int i = 0; i < d.nsel; ++i) {                  // a key twice goes to the affinity term
                bool dup = false;
                for (int j = 0; j < nk; ++j) dup |= std::strcmp(kv[j].key, pn.k(d.sel[i])) == 0;
                if (dup) { d.aff[d.naff < 8 ? d.naff++ : 7] = d.sel[i]; continue; }
                kv[nk++] = esc_kv{pn.k(d.sel[i]), pn.v(d.sel[i])};
            }
            if (d.zone) kv[nk++] = esc_kv{"zone", "z1"};
            o.node_selector = kv;
            o.n_node_selector = nk;
            for (const char* key : {"customer", "pool"}) {      // one In expression per key
                const int first = nvv;
                for (int i = 0; i < d.naff; ++i)
                    if (std::strcmp(pn.k(d.aff[i]), key) == 0 && nvv < (int)(nva[k + 1] - nva[k])) va[nvv++] = pn.v(d.aff[i]);
                if (nvv > first) ex[ne++] = esc_selector_expr{key, "In", va + first, nvv - first, 0};
            }
            if (d.not_in && nvv < (int)(nva[k + 1] - nva[k])) {
                va[nvv] = "z9";
                ex[ne++] = esc_selector_expr{"zone", "NotIn", va + nvv, 1, 0};
                ++nvv;
            }
            o.exprs = ex;
            o.n_exprs = ne;
            o.has_affinity = (ne > 0 || d.pod_aff) ? 1 : 0;
            o.has_node_affinity = ne > 0 ? 1 : 0;
            o.has_required = ne > 0 ? 1 : 0;
            o.has_pod_affinity = d.pod_aff ? 1 : 0;
            esc_request* rq = O.reqs.data() + nrq[k];
            for (int i = 0; i < d.n_reg; ++i)
                rq[i] = esc_request{d.cpu[i], d.mem[i], d.cpu[i] != 0, d.mem[i] != 0};
            o.containers = rq;
            o.n_containers = d.n_reg;
            if (d.n_init) rq[d.n_reg] = esc_request{d.icpu, d.imem, 1, 1};
            o.init_containers = d.n_init ? rq + d.n_reg : nullptr;
            o.n_init_containers = d.n_init;
            o.has_overhead = d.ovh ? 1 : 0;
            o.overhead = esc_request{d.ocpu, d.omem, d.ovh ? 1 : 0, d.ovh ? 1 : 0};
        }
    });
    // nodes: name, label pairs (+ a zone label no group filters on), cordon, the escalator
    // taint, allocatable, creation time
    std::vector<int64_t> xo(nn + 1, 0);
    for (int64_t j = 0; j < nn; ++j) xo[j + 1] = xo[j] + nf_xlbl(h.nflags[j]);
    const int64_t kv0 = nkv[n];
    O.nodes.assign(nn, esc_node_obj{});
    O.node_names.resize(nn);
    for (int64_t j = 0; j < nn; ++j) O.node_names[j] = "node-" + std::to_string(j);
    for (int64_t j = 0, kp = kv0; j < nn; ++j) {
        esc_node_obj& o = O.nodes[j];
        o.name = O.node_names[j].c_str();
        esc_kv* kv = O.kvs.data() + kp;
        int nk = 0;
        if (h.label0[j] != NONE) kv[nk++] = esc_kv{pn.k(h.label0[j]), pn.v(h.label0[j])};
        for (int64_t x = xo[j]; x < xo[j + 1]; ++x) kv[nk++] = esc_kv{pn.k(h.xl[x]), pn.v(h.xl[x])};
        kv[nk++] = esc_kv{"zone", (j % 3 == 0) ? "z0" : (j % 3 == 1 ? "z1" : "z2")};
        kp += nk;
        o.labels = kv;
        o.n_labels = nk;
        o.unschedulable = (h.nflags[j] & ESC_NF_UNSCHED) ? 1 : 0;
        o.taint_keys = (h.nflags[j] & ESC_NF_TAINTED) ? taint_esc : nullptr;
        o.n_taints = (h.nflags[j] & ESC_NF_TAINTED) ? 1 : 0;
        o.allocatable = esc_request{h.ncpu[j], h.nmem[j], 1, 1};
        o.created_unix_ns = h.created[j];
    }
    O.built = true;
}

}  // namespace

extern "C" {

int32_t esc_synth_create(const esc_synth_params* p, int64_t p_lo, int64_t p_hi, esc_synth** out) {
    if (!p || !out || p->n_groups <= 0 || p->n_pods < 0 || p->n_nodes < 0) return ESC_E_INVAL;
    if (p_lo < 0 || p_hi > p->n_pods || p_lo > p_hi) return ESC_E_INVAL;
    if (p->n_nodes >= (int64_t)0x7FFFFFFF) return ESC_E_LIMIT;
    esc_synth* S = new (std::nothrow) esc_synth();
    if (!S) return ESC_E_NOMEM;
    S->p = *p;
    if (S->p.config < 1 || S->p.config > 5) S->p.config = 2;
    if (S->p.config == 1) S->p.n_groups = 1;
    S->p_lo = p_lo;
    S->p_hi = p_hi;
    try {
        build_groups(*S);
        gen_pods(*S);
        gen_nodes(*S);
    } catch (const std::bad_alloc&) {
        delete S;
        return ESC_E_NOMEM;
    }
    *out = S;
    return ESC_OK;
}

int32_t esc_synth_destroy(esc_synth* s) { delete s; return ESC_OK; }

int32_t esc_synth_groups(const esc_synth* s, const esc_group_spec** groups, int32_t* n) {
    if (!s || !groups || !n) return ESC_E_INVAL;
    *groups = s->specs.data();
    *n = (int32_t)s->specs.size();
    return ESC_OK;
}

int32_t esc_synth_states(const esc_synth* s, const esc_group_state** states) {
    if (!s || !states) return ESC_E_INVAL;
    *states = s->states.data();
    return ESC_OK;
}

int32_t esc_synth_view(const esc_synth* s, esc_pod_soa* pods, esc_node_soa* nodes) {
    if (!s) return ESC_E_INVAL;
    s->s.view(pods, nodes);
    return ESC_OK;
}

int32_t esc_synth_objects(esc_synth* s, const esc_pod_obj** pods, int64_t* n_pods, const esc_node_obj** nodes,
                          int64_t* n_nodes) {
    if (!s || !pods || !n_pods || !nodes || !n_nodes) return ESC_E_INVAL;
    if (!s->obj.built) {
        try {
            build_objects(*s);
        } catch (const std::bad_alloc&) {
            return ESC_E_NOMEM;
        }
    }
    *pods = s->obj.pods.data();
    *n_pods = (int64_t)s->obj.pods.size();
    *nodes = s->obj.nodes.data();
    *n_nodes = (int64_t)s->obj.nodes.size();
    return ESC_OK;
}

}  // extern "C"
