// esc_kernels.hip — gfx950 kernels of the scale-decision hot path.
//
//  K1 k_pod_reduce   : FilteredPodsLister.List (pod_listers.go:33) for EVERY group at once
//                      + ComputePodResourceRequest (scheduler/types.go:72) +
//                      CalculatePodsRequestsTotal (util.go:27).  One pass over the pod SoA,
//                      16-B-per-lane coalesced loads (4 pods per lane, 256 per wave), int64
//                      per-group partials privatised in LDS (ds_add_u64), flushed once per
//                      workgroup.  HBM-bound; no MFMA (nothing is a contraction).
//  K2 k_node_reduce  : FilteredNodesLister.List + filterNodes (controller.go:120) +
//                      CalculateNodesCapacityTotal(untainted) (util.go:41) + allNodes[0]
//                      (controller.go:208).  Group-tiled LDS privatisation.
//  K3 k_combine      : sums the per-workgroup partials into the exchanged int64 words;
//                      for one rank it also runs K4.
//  K4 k_decide       : calcPercentUsage / switch / calcScaleUpDelta / scaleDownTaint clamp
//                      (util.go:13-81, controller.go:233-351, scale_down.go:138-158).
//  K5 sort kernels   : segmented LSD radix sort for taintOldestN / untaintNewestN
//                      (scale_down.go:171, scale_up.go:118, sort.go:18,33).
// Wide variants      : exact any-range fallback with global atomics.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "esc_kernels.h"

namespace esc {

namespace {

constexpr int BLOCK = 1024;          // 16 waves per workgroup

__device__ __forceinline__ uint4 ld4(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ ulonglong2 ld2(const int64_t* p) {
    return *reinterpret_cast<const ulonglong2*>(p);
}

__device__ __forceinline__ void lds_add(uint64_t* a, uint64_t v) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a), (unsigned long long)v);
}
__device__ __forceinline__ void g_add(int64_t* a, int64_t v) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a), (unsigned long long)v);
}

// Effective request of one pod — ComputePodResourceRequest, scheduler/types.go:72-89:
// regular containers summed (Resource.Add, plain int64 += wraps), then max with every
// init container (SetMaxResource; an absent key is INT64_MIN so max() ignores it),
// then the overhead record added.  `o` walks the pod's extra records.
__device__ __forceinline__ void pod_request(uint32_t f, uint32_t cpu0, int64_t mem0,
                                            const int64_t* __restrict__ xc_cpu,
                                            const int64_t* __restrict__ xc_mem, uint32_t& o,
                                            int64_t& cpu, int64_t& mem) {
    uint64_t c = cpu0, m = (uint64_t)mem0;
    const uint32_t nreg = pf_xreg(f), ninit = pf_xinit(f);
    for (uint32_t r = 0; r < nreg; ++r, ++o) { c += (uint64_t)xc_cpu[o]; m += (uint64_t)xc_mem[o]; }
    for (uint32_t r = 0; r < ninit; ++r, ++o) {
        const int64_t ic = xc_cpu[o], im = xc_mem[o];
        c = ((int64_t)c >= ic) ? c : (uint64_t)ic;
        m = ((int64_t)m >= im) ? m : (uint64_t)im;
    }
    if (f & ESC_PF_HAS_OVH) { c += (uint64_t)xc_cpu[o]; m += (uint64_t)xc_mem[o]; ++o; }
    cpu = (int64_t)c;
    mem = (int64_t)m;
}

// ------------------------------------------------------------- wave primitives
// DPP lane movement (no LDS traffic).  Out-of-row sources and masked rows read 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, false);
}

// Inclusive prefix sum over the wave's 64 lanes: row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry row totals.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
    v += dpp<0x111, 0xF>(v);
    v += dpp<0x112, 0xF>(v);
    v += dpp<0x114, 0xF>(v);
    v += dpp<0x118, 0xF>(v);
    v += dpp<0x142, 0xA>(v);
    v += dpp<0x143, 0xC>(v);
    return v;
}

__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0; }

__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
    return __shfl(v, src, 64);
}

__device__ __forceinline__ int64_t imin64(int64_t a, int64_t b) { return a < b ? a : b; }

// ------------------------------------------------------- selector-pair matching
// NewPodAffinityFilterFunc / NewNodeLabelFilterFunc (node_group.go:218, :278) for all
// groups at once: a pair id selects the groups whose (label_key, label_value) it is;
// ids >= n_gp are values no group selects.
//  - pods: K1 accumulates per pair (LDS slot = pair id, plus one slot for the default
//    filter) and K3 joins each group to its pair's slot — the per-pod test
//    "(K_g, V_g) in pod pairs" evaluated for every group without a per-pod lookup;
//  - nodes: K2 resolves each label pair through the node code table (a group id, NONE,
//    or a list of the groups sharing the pair), since node classes depend on the group.
__device__ __forceinline__ uint32_t node_code(const GroupDev& G, uint32_t pair) {
    return pair < G.n_gp ? G.node_code[pair] : NONE;
}
// Membership entries carry the group's dry-mode bit (ESC_NODE_DRY_BIT) next to its id, so
// classifying a node needs no per-group load.
__device__ __forceinline__ uint32_t mg(uint32_t m) { return m & NODE_GROUP_MASK; }
__device__ __forceinline__ bool mdry(uint32_t m) { return (m & NODE_DRY_BIT) != 0; }

template <class F>
__device__ __forceinline__ void for_code(const GroupDev& G, uint32_t code, F&& emit) {
    if (code < CODE_MULTI) {
        emit(code);
    } else if (code != NONE) {                       // groups sharing one pair (rare)
        const uint32_t* l = G.code_list + (code & ~CODE_MULTI);
        const uint32_t n = l[0];
        for (uint32_t k = 1; k <= n; ++k) emit(l[k]);
    }
}

// ------------------------------------------------------------- accumulators
struct PodLds {          // fast path: LDS partials of a group window
    uint64_t* cc;        // cpu | count << 40
    uint64_t* mem;
    int32_t g0;
    uint32_t gw;
    __device__ __forceinline__ void add(uint32_t g, uint64_t vcc, uint64_t vmem) const {
        const uint32_t i = g - (uint32_t)g0;
        if (i < gw) { lds_add(cc + i, vcc); lds_add(mem + i, vmem); }
    }
};

struct PodWide {         // exact path: global int64 words, values split lo32/hi
    int64_t* w;
    __device__ __forceinline__ void add(uint32_t g, int64_t cpu, int64_t mem) const {
        int64_t* r = w + (int64_t)g * WP_K;
        g_add(r + WP_CPU_LO, (int64_t)((uint64_t)cpu & 0xFFFFFFFFull));
        g_add(r + WP_CPU_HI, cpu >> 32);
        g_add(r + WP_MEM_LO, (int64_t)((uint64_t)mem & 0xFFFFFFFFull));
        g_add(r + WP_MEM_HI, mem >> 32);
        g_add(r + WP_CNT, 1);
    }
};

// One pod's contribution to pod slot `g` (a pair id, or n_gp for the default filter):
// LDS when the effective request is inside the packed range, else the exact wide words
// (only for slots of this launch's window).
// ABLATE bit 0 (timing-only builds, wrong results) replaces the LDS atomics by a sink.
template <int ABLATE>
struct PodSink {
    PodLds acc;
    PodWide spill;
    __device__ __forceinline__ void add(uint32_t g, uint64_t cpu, uint64_t mem, bool in) const {
        if (in) {
            if constexpr (ABLATE & 1) asm volatile("" :: "v"(g), "v"(cpu), "v"(mem));
            else acc.add(g, cpu | (1ull << CNT_SHIFT), mem);
        } else if (g - (uint32_t)acc.g0 < acc.gw) {
            spill.add(g, (int64_t)cpu, (int64_t)mem);
        }
    }
};

__device__ __forceinline__ bool in_range(uint64_t cpu, uint64_t mem) {
    return cpu < (uint64_t)POD_CPU_LIMIT && mem < (uint64_t)POD_MEM_LIMIT;
}

// ------------------------------------------------------------------ S tiles
// 256 simple pods per wave, 4 per lane, 16-B loads per lane per array (20 B/pod).
struct STile {
    uint4 f, c, p;
    ulonglong2 m01, m23;
};
// (S tiles are pods with one container and at most one selector pair.)

__device__ __forceinline__ void s_load(const PodDev& P, int64_t t, uint32_t lane, STile& T) {
    const int64_t p0 = t * TILE + lane * PODS_PER_LANE;
    T.f = ld4(P.flags + p0);
    T.c = ld4(P.cpu0 + p0);
    T.m01 = ld2(P.mem0 + p0);
    T.m23 = ld2(P.mem0 + p0 + 2);
    T.p = ld4(P.pair0 + p0);
}

template <int ABLATE>
__device__ __forceinline__ void s_process(const GroupDev& G, const PodSink<ABLATE>& K, const STile& T) {
    const uint32_t fs[4] = {T.f.x, T.f.y, T.f.z, T.f.w};
    const uint32_t ps[4] = {T.p.x, T.p.y, T.p.z, T.p.w};
    const uint64_t cpu[4] = {T.c.x, T.c.y, T.c.z, T.c.w};
    const uint64_t mem[4] = {T.m01.x, T.m01.y, T.m23.x, T.m23.y};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (fs[j] & ESC_PF_DAEMONSET) continue;                      // node_group.go:221, :259
        const bool in = in_range(cpu[j], mem[j]);
        if (pf_default_ok(fs[j]) && G.default_group != NONE) K.add(G.n_gp, cpu[j], mem[j], in);
        if (ps[j] < G.n_gp) K.add(ps[j], cpu[j], mem[j], in);
    }
}

// ------------------------------------------------------------------ C tiles
// 64 pods with extra records per wave, one per lane.  The tile's records are contiguous
// ([xc_base[t], xc_base[t+1])), fetched coalesced (lane l holds records l and l+64) and
// handed to their pods with ds_bpermute; tiles with more than 128 records of a kind are
// listed at load and left to k_pod_bigtiles.
struct TileBases {
    uint32_t xcb, xcn, xpb, xpn;
};

typedef __attribute__((address_space(4))) const uint32_t cu32;   // constant: scalar loads

__device__ __forceinline__ TileBases tile_bases(const PodDev& P, int64_t t) {
    const cu32* xc = (const cu32*)P.xc_base;
    const cu32* xp = (const cu32*)P.xp_base;
    TileBases b;
    b.xcb = xc[t];
    b.xcn = xc[t + 1] - b.xcb;
    b.xpb = xp[t];
    b.xpn = xp[t + 1] - b.xpb;
    return b;
}

struct CTile {
    uint32_t f, c, p;
    uint64_t m;
    unsigned long long xcc0, xcm0, xcc1, xcm1;   // records l and l+64 (clamped: only the
    uint32_t xp0, xp1;                           // first xcn / xpn are meaningful)
    TileBases b;
};

// Every load is issued unconditionally (indices clamped into the tile's records; the
// record arrays carry one element of padding), so the compiler's vmcnt accounting can
// leave a second tile's loads in flight while the first is processed.
__device__ __forceinline__ void c_load(const PodDev& P, int64_t t, uint32_t lane, const TileBases& b, CTile& T) {
    const int64_t i = P.s_tiles * TILE + t * CTILE + lane;
    T.b = b;
    T.f = P.flags[i];
    T.c = P.cpu0[i];
    T.m = (uint64_t)P.mem0[i];
    T.p = P.pair0[i];
    const uint32_t lc = (b.xcn ? b.xcn : 1u) - 1u, lp = (b.xpn ? b.xpn : 1u) - 1u;
    const uint32_t c0 = b.xcb + min(lane, lc), c1 = b.xcb + min(lane + 64, lc);
    const uint32_t p0 = b.xpb + min(lane, lp), p1 = b.xpb + min(lane + 64, lp);
    T.xcc0 = (unsigned long long)P.xc_cpu[c0];
    T.xcm0 = (unsigned long long)P.xc_mem[c0];
    T.xcc1 = (unsigned long long)P.xc_cpu[c1];
    T.xcm1 = (unsigned long long)P.xc_mem[c1];
    T.xp0 = P.xp[p0];
    T.xp1 = P.xp[p1];
}

template <int ABLATE>
__device__ __forceinline__ void c_process(const GroupDev& G, const PodSink<ABLATE>& K, const CTile& T) {
    const uint32_t f = T.f;
    const uint32_t nxc = pf_xctr(f), nxp = pf_xpair(f);
    const uint32_t v = nxc | (nxp << 16);                 // tile totals <= 128 each
    const uint32_t ex = wave_incl_scan32(v) - v;
    const uint32_t oc = ex & 0xFFFF, op = ex >> 16;
    // ComputePodResourceRequest (types.go:72-89) over the pod's records in order:
    // regular extras add, init containers max, the overhead adds.
    uint64_t cpu = T.c, mem = T.m;
    const uint32_t nreg = pf_xreg(f), add_from = nreg + pf_xinit(f);
    for (uint32_t k = 0; wave_any(k < nxc); ++k) {
        const uint32_t rel = oc + k;
        unsigned long long c = shfl64(T.xcc0, (int)(rel & 63));
        unsigned long long m = shfl64(T.xcm0, (int)(rel & 63));
        if (T.b.xcn > 64) {                               // wave-uniform
            const unsigned long long c1 = shfl64(T.xcc1, (int)(rel & 63));
            const unsigned long long m1 = shfl64(T.xcm1, (int)(rel & 63));
            if (rel >= 64) { c = c1; m = m1; }
        }
        if (k < nxc) {
            if (k < nreg || k >= add_from) {
                cpu += c;
                mem += m;
            } else {
                cpu = ((int64_t)cpu >= (int64_t)c) ? cpu : c;
                mem = ((int64_t)mem >= (int64_t)m) ? mem : m;
            }
        }
    }
    const bool live = !(f & ESC_PF_DAEMONSET);            // node_group.go:221, :259
    const bool in = in_range(cpu, mem);
    if (live) {
        if (pf_default_ok(f) && G.default_group != NONE) K.add(G.n_gp, cpu, mem, in);
        if (T.p < G.n_gp) K.add(T.p, cpu, mem, in);
    }
    for (uint32_t k = 0; wave_any(k < nxp); ++k) {
        const uint32_t rel = op + k;
        uint32_t q = __shfl(T.xp0, (int)(rel & 63), 64);
        if (T.b.xpn > 64) {
            const uint32_t q1 = __shfl(T.xp1, (int)(rel & 63), 64);
            if (rel >= 64) q = q1;
        }
        if (live && k < nxp && q < G.n_gp) K.add(q, cpu, mem, in);
    }
}

// Exact (any-range) evaluation of one C tile from memory, one pod per lane.
__device__ __forceinline__ void c_tile_exact(const PodDev& P, const GroupDev& G, int64_t t, uint32_t lane,
                                             int64_t* __restrict__ wide) {
    const int64_t i = P.s_tiles * TILE + t * CTILE + lane;
    const uint32_t f = P.flags[i];
    const uint32_t nxc = pf_xctr(f), nxp = pf_xpair(f);
    uint32_t oc = P.xc_base[t] + wave_incl_scan32(nxc) - nxc;
    const uint32_t op = P.xp_base[t] + wave_incl_scan32(nxp) - nxp;
    if (f & ESC_PF_DAEMONSET) return;
    int64_t cpu, mem;
    pod_request(f, P.cpu0[i], P.mem0[i], P.xc_cpu, P.xc_mem, oc, cpu, mem);
    const PodWide acc{wide};
    if (pf_default_ok(f) && G.default_group != NONE) acc.add(G.n_gp, cpu, mem);
    if (P.pair0[i] < G.n_gp) acc.add(P.pair0[i], cpu, mem);
    for (uint32_t k = 0; k < nxp; ++k)
        if (P.xp[op + k] < G.n_gp) acc.add(P.xp[op + k], cpu, mem);
}

}  // namespace

// =====================================================================  K1 (fast)
// Each workgroup takes an equal share of the S tiles and of the C tiles; its waves
// interleave tiles (t = lo + wave, + waves).  16 waves per CU keep ~80 KB of tile loads
// in flight per CU; the per-group partials stay in LDS and are flushed once.
// ABLATE (timing-only builds): bit 0 LDS sink, bit 1 skip S tiles, bit 2 skip C tiles.
template <int THREADS, int ABLATE = 0>
__global__ __launch_bounds__(THREADS) void k_pod_reduce(PodDev P, GroupDev G, int32_t g0, uint32_t gw,
                                                        uint64_t* __restrict__ part,
                                                        int64_t* __restrict__ wide) {
    constexpr int NW = THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    for (uint32_t i = threadIdx.x; i < 2 * gw; i += THREADS) lds[i] = 0;
    __syncthreads();
    const PodSink<ABLATE> K{PodLds{lds, lds + gw, g0, gw}, PodWide{wide}};
    const uint32_t lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (!(ABLATE & 2)) {
        const int64_t per = (P.s_tiles + gridDim.x - 1) / gridDim.x;
        const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(lo + per, P.s_tiles);
        // Two tiles per wave iteration (10 KB in flight per wave); B's loads are issued
        // unconditionally (a repeat of A at the end) so they stay in flight during A.
        for (int64_t t = lo + wid; t < hi; t += 2 * NW) {
            const bool has_b = t + NW < hi;
            STile A, B;
            s_load(P, t, lane, A);
            s_load(P, has_b ? t + NW : t, lane, B);
            s_process<ABLATE>(G, K, A);
            if (has_b) s_process<ABLATE>(G, K, B);
        }
    }
    if (!(ABLATE & 4)) {
        const int64_t per = (P.c_tiles + gridDim.x - 1) / gridDim.x;
        const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(lo + per, P.c_tiles);
        // Two tiles per wave iteration: B's loads stay in flight while A is processed.
        // Offsets are scalar loads fetched one iteration ahead.
        int64_t t = lo + wid;
        TileBases na{0, 0, 0, 0}, nb{0, 0, 0, 0};
        if (t < hi) na = tile_bases(P, t);
        nb = (t + NW < hi) ? tile_bases(P, t + NW) : na;
        for (; t < hi; t += 2 * NW) {
            const bool has_b = t + NW < hi;               // wave-uniform
            CTile A, B;
            c_load(P, t, lane, na, A);
            c_load(P, has_b ? t + NW : t, lane, nb, B);   // a repeat of A when there is no B
            if (t + 2 * NW < hi) na = tile_bases(P, t + 2 * NW);
            nb = (t + 3 * NW < hi) ? tile_bases(P, t + 3 * NW) : na;
            if (A.b.xcn <= 128 && A.b.xpn <= 128) c_process<ABLATE>(G, K, A);
            if (has_b && B.b.xcn <= 128 && B.b.xpn <= 128) c_process<ABLATE>(G, K, B);
        }
    }
    __syncthreads();
    const int64_t S = G.n_gp + 1;
    uint64_t* out = part + (int64_t)blockIdx.x * 2 * S + g0;
    for (uint32_t i = threadIdx.x; i < gw; i += THREADS) {
        out[i] = lds[i];
        out[S + i] = lds[gw + i];
    }
}

// C tiles with more than 128 extra records of a kind (listed by the host at load):
// one wave per tile, records read from memory, exact wide accumulation.
__global__ __launch_bounds__(64) void k_pod_bigtiles(PodDev P, GroupDev G, const uint32_t* __restrict__ tiles,
                                                     int64_t* __restrict__ wide) {
    c_tile_exact(P, G, tiles[blockIdx.x], threadIdx.x, wide);
}

__global__ __launch_bounds__(256) void k_zero(int64_t* __restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0;
}

__global__ __launch_bounds__(256) void k_fill(uint64_t* __restrict__ p, int64_t n, uint64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// =====================================================================  K1 (wide)
// The whole shard through the exact accumulators (esc_force_wide; fallback testing).
__global__ __launch_bounds__(256) void k_pod_wide(PodDev P, GroupDev G, int64_t* __restrict__ wide) {
    const uint32_t lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const PodWide acc{wide};
    for (int64_t t = wave; t < P.s_tiles; t += nwaves) {
        for (int j = 0; j < PODS_PER_LANE; ++j) {
            const int64_t i = t * TILE + lane * PODS_PER_LANE + j;
            const uint32_t f = P.flags[i];
            if (f & ESC_PF_DAEMONSET) continue;
            const int64_t cpu = (int64_t)P.cpu0[i], mem = P.mem0[i];
            if (pf_default_ok(f) && G.default_group != NONE) acc.add(G.n_gp, cpu, mem);
            if (P.pair0[i] < G.n_gp) acc.add(P.pair0[i], cpu, mem);
        }
    }
    for (int64_t t = wave; t < P.c_tiles; t += nwaves) c_tile_exact(P, G, t, lane, wide);
}

// =====================================================================  K2 nodes
namespace {

// Is (node, group) in the group's dry-mode taintTracker (controller.go:128-133)?
__device__ __forceinline__ bool tracked(const NodeDev& N, int32_t node, int32_t g) {
    int64_t lo = 0, hi = N.n_trk;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t a = N.trk_node[mid], b = N.trk_group[mid];
        if (a < node || (a == node && b < g)) lo = mid + 1; else hi = mid;
    }
    return lo < N.n_trk && N.trk_node[lo] == node && N.trk_group[lo] == g;
}

// filterNodes classification (controller.go:125-150): 0 untainted, 1 tainted, 2 cordoned.
// Dry mode separates only tracker members; cordoned nodes are not split out there.
__device__ __forceinline__ int node_class(const NodeDev& N, uint32_t f, int64_t i, uint32_t m) {
    if (mdry(m)) return ((f & ESC_NF_TRACKED) && tracked(N, (int32_t)i, (int32_t)mg(m))) ? 1 : 0;
    if (f & ESC_NF_UNSCHED) return 2;
    return (f & ESC_NF_TAINTED) ? 1 : 0;
}

// Groups a node belongs to: NewNodeLabelFilterFunc (node_group.go:278) over its label
// pairs, resolved through the node pair table.
template <class F>
__device__ __forceinline__ void node_groups(const NodeDev& N, const GroupDev& G, uint32_t f, int64_t i,
                                            F&& emit) {
    for_code(G, node_code(G, N.label0[i]), emit);
    const uint32_t nx = nf_xlbl(f);
    if (nx) {
        const uint32_t q = N.xl_off[i];
        for (uint32_t k = 0; k < nx; ++k) for_code(G, node_code(G, N.xl[q + k]), emit);
    }
}

}  // namespace

// Exact (any-range) node contribution; WN_FIRST keeps ~index under atomicMax so the
// all-zero row means "no member" and the accumulators can self-clean to zero.
__device__ __forceinline__ void node_wide_add(const NodeDev& N, int64_t* __restrict__ wide,
                                              uint32_t f, int64_t i, uint32_t mb, int64_t cpu, int64_t m) {
    int64_t* r = wide + (int64_t)mg(mb) * WN_K;
    atomicMax(reinterpret_cast<unsigned long long*>(r + WN_FIRST), ~(unsigned long long)i);
    const int c = node_class(N, f, i, mb);
    if (c == 0) {
        g_add(r + WN_CPU_LO, (int64_t)((uint64_t)cpu & 0xFFFFFFFFull));
        g_add(r + WN_CPU_HI, cpu >> 32);
        g_add(r + WN_MEM_LO, (int64_t)((uint64_t)m & 0xFFFFFFFFull));
        g_add(r + WN_MEM_HI, m >> 32);
        g_add(r + WN_UNT, 1);
    } else {
        g_add(r + (c == 1 ? WN_TAINT : WN_CORD), 1);
    }
}

// grid (n_gtile, n_chunk): the group tiles of one node chunk are adjacent in dispatch
// order, so the chunk's repeat reads are served on-die.  LDS tile of gt groups: cc, mem,
// tc (u64), first (u32).  Each thread carries NODE_ILP nodes per iteration so their
// loads and pair-table gathers are in flight together.
constexpr int NODE_ILP = 4;

__global__ __launch_bounds__(BLOCK) void k_node_reduce(NodeDev N, GroupDev G, int32_t gt,
                                                       uint64_t* __restrict__ part,
                                                       int64_t* __restrict__ wide) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    uint64_t* cc = lds;
    uint64_t* mem = lds + gt;
    uint64_t* tc = lds + 2 * gt;
    uint32_t* first = reinterpret_cast<uint32_t*>(lds + 3 * gt);
    for (int32_t i = threadIdx.x; i < gt; i += BLOCK) { cc[i] = 0; mem[i] = 0; tc[i] = 0; first[i] = NONE; }
    __syncthreads();
    const uint32_t g_lo = blockIdx.x * (uint32_t)gt;
    const uint32_t g_n = (uint32_t)min(gt, G.G - (int32_t)g_lo);
    const int64_t n = N.hi - N.lo;
    const int64_t per = (n + gridDim.y - 1) / gridDim.y;
    const int64_t lo = N.lo + (int64_t)blockIdx.y * per;
    const int64_t hi = imin64(N.hi, lo + per);
    for (int64_t b = lo; b < hi; b += (int64_t)BLOCK * NODE_ILP) {
        // three dependent rounds for NODE_ILP nodes at once: node words (+ offset of the
        // extra label pairs), then pair codes and the first extra pair, then its code
        uint32_t f[NODE_ILP], l0[NODE_ILP], xo[NODE_ILP], x1[NODE_ILP], code[NODE_ILP], xcode[NODE_ILP];
        int64_t cpu[NODE_ILP], m[NODE_ILP];
#pragma unroll
        for (int k = 0; k < NODE_ILP; ++k) {
            const int64_t i = b + threadIdx.x + (int64_t)k * BLOCK;
            f[k] = 0; l0[k] = NONE; cpu[k] = 0; m[k] = 0; xo[k] = 0;
            if (i < hi) {
                f[k] = N.flags[i]; l0[k] = N.label0[i]; cpu[k] = N.cpu[i]; m[k] = N.mem[i]; xo[k] = N.xl_off[i];
            }
        }
#pragma unroll
        for (int k = 0; k < NODE_ILP; ++k) {
            code[k] = node_code(G, l0[k]);
            x1[k] = nf_xlbl(f[k]) ? N.xl[xo[k]] : NONE;
        }
#pragma unroll
        for (int k = 0; k < NODE_ILP; ++k) xcode[k] = node_code(G, x1[k]);
#pragma unroll
        for (int k = 0; k < NODE_ILP; ++k) {
            const int64_t i = b + threadIdx.x + (int64_t)k * BLOCK;
            if (i >= hi) continue;
            const uint32_t fk = f[k];
            const int64_t ck = cpu[k], mk = m[k];
            if ((uint64_t)ck >= (uint64_t)NODE_CPU_LIMIT || (uint64_t)mk >= (uint64_t)NODE_MEM_LIMIT) {
                node_groups(N, G, fk, i, [&](uint32_t mb) {
                    if (mg(mb) - g_lo < g_n) node_wide_add(N, wide, fk, i, mb, ck, mk);
                });
                continue;
            }
            auto visit = [&](uint32_t mb) {
                const uint32_t t = mg(mb) - g_lo;
                if (t >= g_n) return;
                atomicMin(first + t, (uint32_t)i);
                const int c = node_class(N, fk, i, mb);
                if (c == 0) { lds_add(cc + t, (uint64_t)ck | (1ull << CNT_SHIFT)); lds_add(mem + t, (uint64_t)mk); }
                else lds_add(tc + t, c == 1 ? 1ull : (1ull << 32));
            };
            for_code(G, code[k], visit);
            for_code(G, xcode[k], visit);
            const uint32_t nx = nf_xlbl(fk);
            for (uint32_t e = 1; e < nx; ++e) for_code(G, node_code(G, N.xl[xo[k] + e]), visit);
        }
    }
    __syncthreads();
    uint64_t* out = part + (int64_t)blockIdx.y * 4 * G.G + g_lo;
    for (uint32_t k = threadIdx.x; k < g_n; k += BLOCK) {
        out[k] = cc[k];
        out[G.G + k] = mem[k];
        out[2 * G.G + k] = tc[k];
        out[3 * G.G + k] = first[k];
    }
}

// Node pass without group tiles (ESC_K2 variant 1, for many groups): every node is
// read once and its memberships go straight to per-group global rows laid out like one
// k_node_reduce chunk (cc, mem, tc, first), which K3 reads and resets.  Exact while a
// node's cpu < 2^20 m and mem < 2^43 B and the rank streams <= 2^20 nodes (checked by the
// host): the packed row words cannot carry.  Other nodes take the wide words.
__global__ __launch_bounds__(256) void k_node_atomic(NodeDev N, GroupDev G, uint64_t* __restrict__ rows,
                                                     int64_t* __restrict__ wide) {
    const int64_t GG = G.G;
    for (int64_t i = N.lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N.hi;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t f = N.flags[i];
        const int64_t cpu = N.cpu[i], m = N.mem[i];
        if ((uint64_t)cpu >= (uint64_t)NODE_CPU_LIMIT || (uint64_t)m >= (uint64_t)NODE_MEM_LIMIT_ATOMIC) {
            node_groups(N, G, f, i, [&](uint32_t mb) { node_wide_add(N, wide, f, i, mb, cpu, m); });
            continue;
        }
        node_groups(N, G, f, i, [&](uint32_t mb) {
            const uint32_t g = mg(mb);
            atomicMin(reinterpret_cast<unsigned long long*>(rows + 3 * GG + g), (unsigned long long)i);
            const int c = node_class(N, f, i, mb);
            if (c == 0) {
                atomicAdd(reinterpret_cast<unsigned long long*>(rows + g), (unsigned long long)cpu | (1ull << CNT_SHIFT));
                atomicAdd(reinterpret_cast<unsigned long long*>(rows + GG + g), (unsigned long long)m);
            } else {
                atomicAdd(reinterpret_cast<unsigned long long*>(rows + 2 * GG + g), c == 1 ? 1ull : (1ull << 32));
            }
        });
    }
}

__global__ __launch_bounds__(256) void k_node_wide(NodeDev N, GroupDev G, int64_t* __restrict__ wide) {
    for (int64_t i = N.lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N.hi;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t f = N.flags[i];
        const int64_t cpu = N.cpu[i], m = N.mem[i];
        node_groups(N, G, f, i, [&](uint32_t mb) { node_wide_add(N, wide, f, i, mb, cpu, m); });
    }
}

// ===================================================================== K3 / K4
namespace {

constexpr int CB_WAVES = 8;

__device__ __forceinline__ void u128_add(uint64_t& lo, uint64_t& hi, uint64_t v) { lo += v; hi += (lo < v) ? 1 : 0; }

__device__ __forceinline__ void split_store(int64_t* w, int k, __int128 t) {
    w[k] = (int64_t)((unsigned __int128)t & 0xFFFFFFFFull);
    w[k + 1] = (int64_t)(t >> 32);
}

// Exact total from split words; false when it is outside int64 (Quantity -> inf.Dec).
__device__ __forceinline__ bool join_split(int64_t lo_sum, int64_t hi_sum, int64_t& out) {
    const __int128 t = ((__int128)hi_sum << 32) + (__int128)lo_sum;
    out = (int64_t)t;
    return t >= (__int128)INT64_MIN && t <= (__int128)INT64_MAX;
}

__device__ __forceinline__ void finalize(const GroupDev& G, const NodeDev& N, int32_t g,
                                         const int64_t* __restrict__ w, int64_t first,
                                         esc_group_decision* __restrict__ dec) {
    Totals t;
    int64_t flags = 0;
    if (!join_split(w[TW_POD_CPU_LO], w[TW_POD_CPU_HI], t.pod_cpu)) flags |= ESC_TF_POD_OVERFLOW;
    if (!join_split(w[TW_POD_MEM_LO], w[TW_POD_MEM_HI], t.pod_mem)) flags |= ESC_TF_POD_OVERFLOW;
    t.n_pods = w[TW_N_PODS];
    if (!join_split(w[TW_NODE_CPU_LO], w[TW_NODE_CPU_HI], t.node_cpu)) flags |= ESC_TF_NODE_OVERFLOW;
    if (!join_split(w[TW_NODE_MEM_LO], w[TW_NODE_MEM_HI], t.node_mem)) flags |= ESC_TF_NODE_OVERFLOW;
    t.n_unt = w[TW_N_UNT];
    t.n_taint = w[TW_N_TAINT];
    t.n_cord = w[TW_N_CORD];
    t.n_nodes = t.n_unt + t.n_taint + t.n_cord;
    t.first = first;
    t.first_cpu = first != INT64_MAX ? N.cpu[first] : 0;
    t.first_mem = first != INT64_MAX ? N.mem[first] : 0;
    t.flags = flags;
    decide_one(G.params[g], t, dec[g]);
}

}  // namespace

// Row-parallel reduction of the per-workgroup partials: a workgroup owns 64 groups (one
// per lane, coalesced 512-B row reads) and its 8 waves split the partial rows; the wide
// accumulators are merged and reset to zero (self-cleaning for the next decision).
__global__ __launch_bounds__(CB_WAVES * 64) void k_combine(GroupDev G, NodeDev N,
                                                           const uint64_t* __restrict__ pod_part, int nblk,
                                                           const uint64_t* __restrict__ node_part, int n_chunk,
                                                           int64_t* __restrict__ wide_pod,
                                                           int64_t* __restrict__ wide_node,
                                                           int64_t* __restrict__ words,
                                                           int64_t* __restrict__ firsts, int decide,
                                                           esc_group_decision* __restrict__ dec, int node_reset) {
    constexpr int NW = 12;
    __shared__ uint64_t red[CB_WAVES][NW][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int32_t g = blockIdx.x * 64 + lane;
    const bool ok = g < G.G;
    uint64_t a[NW] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // a: 0 pcpu 1 pcnt 2 pmem_lo 3 pmem_hi 4 ncpu 5 nunt 6 nmem_lo 7 nmem_hi 8 taint 9 cord 10 first
    a[10] = ~0ull;
    // The group's pod slot: its pair (NewPodAffinityFilterFunc) or the default filter's.
    const int64_t S = G.n_gp + 1;
    const int64_t slot = !ok ? 0 : ((uint32_t)g == G.default_group ? (int64_t)G.n_gp : (int64_t)G.gpair[g]);
    if (ok) {
        for (int b = wid; b < nblk; b += CB_WAVES) {
            const uint64_t c = pod_part[(int64_t)b * 2 * S + slot];
            a[0] += c & CPU_MASK;
            a[1] += c >> CNT_SHIFT;
            u128_add(a[2], a[3], pod_part[((int64_t)b * 2 + 1) * S + slot]);
        }
        for (int c = wid; c < n_chunk; c += CB_WAVES) {
            const uint64_t* r = node_part + (int64_t)c * 4 * G.G + g;
            const uint64_t x = r[0];
            a[4] += x & CPU_MASK;
            a[5] += x >> CNT_SHIFT;
            u128_add(a[6], a[7], r[G.G]);
            const uint64_t tc = r[2 * G.G];
            a[8] += tc & 0xFFFFFFFFull;
            a[9] += tc >> 32;
            const uint64_t fv = r[3 * G.G];
            a[10] = fv < a[10] ? fv : a[10];
            if (node_reset) {                             // k_node_atomic rows: ready for the next step
                uint64_t* w = const_cast<uint64_t*>(r);
                w[0] = 0; w[G.G] = 0; w[2 * G.G] = 0; w[3 * G.G] = NONE;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) red[wid][k][lane] = a[k];
    __syncthreads();
    if (wid != 0 || !ok) return;
    for (int w = 1; w < CB_WAVES; ++w) {
        a[0] += red[w][0][lane];
        a[1] += red[w][1][lane];
        u128_add(a[2], a[3], red[w][2][lane]); a[3] += red[w][3][lane];
        a[4] += red[w][4][lane];
        a[5] += red[w][5][lane];
        u128_add(a[6], a[7], red[w][6][lane]); a[7] += red[w][7][lane];
        a[8] += red[w][8][lane];
        a[9] += red[w][9][lane];
        a[10] = red[w][10][lane] < a[10] ? red[w][10][lane] : a[10];
    }
    const int64_t* wp = wide_pod + slot * WP_K;    // slots may be shared: zeroed per step by the host
    int64_t* wn = wide_node + (int64_t)g * WN_K;
    int64_t p[WP_K], q[WN_K];
#pragma unroll
    for (int k = 0; k < WP_K; ++k) p[k] = wp[k];
#pragma unroll
    for (int k = 0; k < WN_K; ++k) { q[k] = wn[k]; wn[k] = 0; }
    int64_t* w = words + (int64_t)g * TW_K;
    const __int128 pcpu = (__int128)a[0] + ((__int128)p[WP_CPU_HI] << 32) + (__int128)p[WP_CPU_LO];
    const __int128 pmem = (__int128)(((unsigned __int128)a[3] << 64) | a[2]) + ((__int128)p[WP_MEM_HI] << 32) +
                          (__int128)p[WP_MEM_LO];
    const __int128 ncpu = (__int128)a[4] + ((__int128)q[WN_CPU_HI] << 32) + (__int128)q[WN_CPU_LO];
    const __int128 nmem = (__int128)(((unsigned __int128)a[7] << 64) | a[6]) + ((__int128)q[WN_MEM_HI] << 32) +
                          (__int128)q[WN_MEM_LO];
    split_store(w, TW_POD_CPU_LO, pcpu);
    split_store(w, TW_POD_MEM_LO, pmem);
    w[TW_N_PODS] = (int64_t)a[1] + p[WP_CNT];
    split_store(w, TW_NODE_CPU_LO, ncpu);
    split_store(w, TW_NODE_MEM_LO, nmem);
    w[TW_N_UNT] = (int64_t)a[5] + q[WN_UNT];
    w[TW_N_TAINT] = (int64_t)a[8] + q[WN_TAINT];
    w[TW_N_CORD] = (int64_t)a[9] + q[WN_CORD];
    int64_t fst = a[10] >= (uint64_t)NONE ? INT64_MAX : (int64_t)a[10];
    if (q[WN_FIRST] != 0) {
        const int64_t fw = (int64_t)~(uint64_t)q[WN_FIRST];
        fst = fw < fst ? fw : fst;
    }
    firsts[g] = fst;
    if (decide) finalize(G, N, g, w, fst, dec);
}

__global__ __launch_bounds__(256) void k_decide(GroupDev G, NodeDev N, const int64_t* __restrict__ words,
                                                const int64_t* __restrict__ firsts,
                                                esc_group_decision* __restrict__ dec) {
    const int32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G.G) return;
    finalize(G, N, g, words + (int64_t)g * TW_K, firsts[g], dec);
}

// ===================================================================== K5 sort
// Key: [group | class(2) | creation offset (R bits)], value: node index.  Class 1
// (tainted) stores the complemented offset so ascending order is newest-first.
namespace {
constexpr int SORT_BLOCK = 1024;
constexpr int SORT_WAVES = SORT_BLOCK / 64;
}

// Membership count per node chunk (pass 1 of the deterministic expansion).
__global__ __launch_bounds__(SORT_BLOCK) void k_sort_count(NodeDev N, GroupDev G, uint32_t* __restrict__ hist) {
    __shared__ uint32_t tot;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    const int64_t n = N.hi - N.lo;
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = N.lo + (int64_t)blockIdx.x * per, hi = imin64(N.hi, lo + per);
    uint32_t c = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += SORT_BLOCK)
        node_groups(N, G, N.flags[i], i, [&](uint32_t) { ++c; });
    atomicAdd(&tot, c);
    __syncthreads();
    if (threadIdx.x == 0) hist[blockIdx.x] = tot;
}

// Exclusive scan of n u32 in place by one workgroup; total to *total.
__global__ __launch_bounds__(SORT_BLOCK) void k_scan_small(uint32_t* __restrict__ a, int n, uint32_t* __restrict__ total) {
    __shared__ uint32_t carry;
    __shared__ uint32_t wsum[SORT_WAVES];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int base = 0; base < n; base += SORT_BLOCK) {
        const int i = base + threadIdx.x;
        const uint32_t v = i < n ? a[i] : 0;
        uint32_t s = v;
        for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(s, d, 64); if (lane >= d) s += y; }
        if (lane == 63) wsum[wid] = s;
        __syncthreads();
        uint32_t wpre = 0;
        for (int k = 0; k < wid; ++k) wpre += wsum[k];
        uint32_t blk = 0;
        for (int k = 0; k < SORT_WAVES; ++k) blk += wsum[k];
        if (i < n) a[i] = carry + wpre + s - v;
        __syncthreads();
        if (threadIdx.x == 0) carry += blk;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

// Pass 2: write memberships in node order (stable => ties resolve by node index).
__global__ __launch_bounds__(SORT_BLOCK) void k_sort_expand(NodeDev N, GroupDev G, const uint32_t* __restrict__ base,
                                                            int64_t ts_min, uint64_t ts_div,
                                                            int R, uint64_t* __restrict__ keys,
                                                            uint32_t* __restrict__ vals) {
    __shared__ uint32_t wsum[SORT_WAVES];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = base[blockIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t n = N.hi - N.lo;
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = N.lo + (int64_t)blockIdx.x * per, hi = imin64(N.hi, lo + per);
    const uint64_t rmask = R >= 64 ? ~0ull : ((1ull << R) - 1);
    for (int64_t b = lo; b < hi; b += SORT_BLOCK) {
        const int64_t i = b + threadIdx.x;
        uint32_t c = 0;
        uint32_t f = 0;
        if (i < hi) { f = N.flags[i]; node_groups(N, G, f, i, [&](uint32_t) { ++c; }); }
        uint32_t s = c;
        for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(s, d, 64); if (lane >= d) s += y; }
        if (lane == 63) wsum[wid] = s;
        __syncthreads();
        uint32_t pos = carry + s - c;
        for (int k = 0; k < wid; ++k) pos += wsum[k];
        if (i < hi && c) {
            uint64_t off = (uint64_t)(N.created[i] - ts_min);
            off = ts_div > 1 ? off / ts_div : off;
            node_groups(N, G, f, i, [&](uint32_t mb) {
                const uint32_t g = mg(mb);
                const int cls = node_class(N, f, i, mb);
                const uint64_t ts = cls == 1 ? (~off & rmask) : off;
                keys[pos] = ((uint64_t)g << (R + 2)) | ((uint64_t)cls << R) | ts;
                vals[pos] = (uint32_t)i;
                ++pos;
            });
        }
        __syncthreads();
        if (threadIdx.x == 0) { uint32_t t = 0; for (int k = 0; k < SORT_WAVES; ++k) t += wsum[k]; carry += t; }
        __syncthreads();
    }
}

// One LSD pass, 8-bit digit at `shift`: per-block digit histogram.
__global__ __launch_bounds__(SORT_BLOCK) void k_radix_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                           uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    for (int i = threadIdx.x; i < 256; i += SORT_BLOCK) h[i] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(n, lo + per);
    for (int64_t i = lo + threadIdx.x; i < hi; i += SORT_BLOCK) atomicAdd(&h[(keys[i] >> shift) & 255], 1u);
    __syncthreads();
    for (int d = threadIdx.x; d < 256; d += SORT_BLOCK) hist[(int64_t)d * gridDim.x + blockIdx.x] = h[d];
}

// Stable scatter: rank = digit offset of the block + rank inside the block in input order.
__global__ __launch_bounds__(SORT_BLOCK) void k_radix_scatter(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                              uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                              int64_t n, int shift, const uint32_t* __restrict__ hist) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wh[SORT_WAVES][256];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int d = threadIdx.x; d < 256; d += SORT_BLOCK) run[d] = hist[(int64_t)d * gridDim.x + blockIdx.x];
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(n, lo + per);
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int64_t b = lo; b < hi; b += SORT_BLOCK) {
        for (int k = threadIdx.x; k < SORT_WAVES * 256; k += SORT_BLOCK) (&wh[0][0])[k] = 0;
        __syncthreads();
        const int64_t i = b + threadIdx.x;
        const bool ok = i < hi;
        uint64_t key = ok ? kin[i] : 0;
        uint32_t val = ok ? vin[i] : 0;
        const uint32_t d = (uint32_t)(key >> shift) & 255;
        unsigned long long m = __ballot(ok);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const unsigned long long bb = __ballot((d >> bit) & 1);
            m &= ((d >> bit) & 1) ? bb : ~bb;
        }
        const uint32_t r_in_wave = __popcll(m & lt);
        if (ok && r_in_wave == 0) wh[wid][d] = __popcll(m);
        __syncthreads();
        uint32_t pre = 0;
        for (int k = 0; k < wid; ++k) pre += wh[k][d];
        if (ok) {
            const uint32_t dst = run[d] + pre + r_in_wave;
            kout[dst] = key;
            vout[dst] = val;
        }
        __syncthreads();
        for (int dd = threadIdx.x; dd < 256; dd += SORT_BLOCK) {
            uint32_t t = 0;
            for (int k = 0; k < SORT_WAVES; ++k) t += wh[k][dd];
            run[dd] += t;
        }
        __syncthreads();
    }
}

// Lower bound of each (group, class) prefix in the sorted keys: seg[g*3+cls].
__global__ __launch_bounds__(256) void k_group_bounds(const uint64_t* __restrict__ keys, int64_t n, int key_shift,
                                                      int32_t nseg, int64_t* __restrict__ seg) {
    const int32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > nseg) return;
    const uint64_t target = (uint64_t)s;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((keys[mid] >> key_shift) < target) lo = mid + 1; else hi = mid;
    }
    seg[s] = lo;
}

// ===================================================================== launchers
hipError_t launch_pod_reduce(const PodDev& p, const GroupDev& g, int32_t g0, int32_t gw, int nblk, int variant,
                             uint64_t* part, int64_t* wide, hipStream_t st) {
    const size_t lds = (size_t)gw * 2 * sizeof(uint64_t);
#define ESC_K1(T, A) hipLaunchKernelGGL((k_pod_reduce<T, A>), dim3(nblk), dim3(T), lds, st, p, g, g0, (uint32_t)gw, part, wide)
    switch (variant) {
        case 2: ESC_K1(512, 0); break;
        // Timing-only ablations (wrong results; scripts/k1_variants.py), see k_pod_reduce.
        case 9: ESC_K1(1024, 1); break;
        case 10: ESC_K1(1024, 2); break;
        case 11: ESC_K1(1024, 4); break;
        case 12: ESC_K1(1024, 3); break;
        case 13: ESC_K1(1024, 5); break;
        default: ESC_K1(1024, 0); break;
    }
#undef ESC_K1
    return hipGetLastError();
}

hipError_t launch_node_atomic(const NodeDev& n, const GroupDev& g, uint64_t* rows, int64_t* wide, hipStream_t st) {
    const int64_t cnt = n.hi - n.lo;
    const int64_t nb = std::min<int64_t>((cnt + 255) / 256, 8192);
    if (nb > 0) hipLaunchKernelGGL(k_node_atomic, dim3((unsigned)nb), dim3(256), 0, st, n, g, rows, wide);
    return hipGetLastError();
}

hipError_t launch_fill(uint64_t* p, int64_t n, uint64_t v, hipStream_t st) {
    const int64_t nb = std::min<int64_t>((n + 255) / 256, 1024);
    if (nb > 0) hipLaunchKernelGGL(k_fill, dim3((unsigned)nb), dim3(256), 0, st, p, n, v);
    return hipGetLastError();
}

hipError_t launch_zero(int64_t* p, int64_t n, hipStream_t st) {
    const int64_t nb = std::min<int64_t>((n + 255) / 256, 1024);
    if (nb > 0) hipLaunchKernelGGL(k_zero, dim3((unsigned)nb), dim3(256), 0, st, p, n);
    return hipGetLastError();
}

hipError_t launch_pod_bigtiles(const PodDev& p, const GroupDev& g, const uint32_t* tiles, int64_t n_big,
                               int64_t* wide, hipStream_t st) {
    if (n_big <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pod_bigtiles, dim3((unsigned)n_big), dim3(64), 0, st, p, g, tiles, wide);
    return hipGetLastError();
}

hipError_t launch_node_reduce(const NodeDev& n, const GroupDev& g, int n_chunk, int gt,
                              uint64_t* part, int64_t* wide, hipStream_t st) {
    const int n_tiles = (g.G + gt - 1) / gt;
    const size_t lds = (size_t)gt * (3 * sizeof(uint64_t) + sizeof(uint32_t));
    hipLaunchKernelGGL(k_node_reduce, dim3(n_tiles, n_chunk), dim3(BLOCK), lds, st, n, g, gt, part, wide);
    return hipGetLastError();
}

hipError_t launch_combine(const GroupDev& g, const NodeDev& n, const uint64_t* pod_part, int nblk,
                          const uint64_t* node_part, int n_chunk, int64_t* wide_pod, int64_t* wide_node,
                          int64_t* words, int64_t* first, bool decide, esc_group_decision* dec, bool node_reset,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_combine, dim3((g.G + 63) / 64), dim3(CB_WAVES * 64), 0, st, g, n, pod_part, nblk,
                       node_part, n_chunk, wide_pod, wide_node, words, first, decide ? 1 : 0, dec,
                       node_reset ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_wide_pods(const PodDev& p, const GroupDev& g, int64_t* wide, hipStream_t st) {
    hipLaunchKernelGGL(k_pod_wide, dim3(1024), dim3(256), 0, st, p, g, wide);
    return hipGetLastError();
}

hipError_t launch_wide_nodes(const NodeDev& n, const GroupDev& g, int64_t* wide, hipStream_t st) {
    hipLaunchKernelGGL(k_node_wide, dim3(1024), dim3(256), 0, st, n, g, wide);
    return hipGetLastError();
}

hipError_t launch_decide(const GroupDev& g, const NodeDev& n, const int64_t* words,
                         const int64_t* first, esc_group_decision* dec, hipStream_t st) {
    hipLaunchKernelGGL(k_decide, dim3((g.G + 255) / 256), dim3(256), 0, st, g, n, words, first, dec);
    return hipGetLastError();
}

hipError_t launch_sort_count(const NodeDev& n, const GroupDev& g, int nblk, uint32_t* hist, hipStream_t st) {
    hipLaunchKernelGGL(k_sort_count, dim3(nblk), dim3(SORT_BLOCK), 0, st, n, g, hist);
    return hipGetLastError();
}

hipError_t launch_scan_small(uint32_t* a, int n, uint32_t* total, hipStream_t st) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(SORT_BLOCK), 0, st, a, n, total);
    return hipGetLastError();
}

hipError_t launch_sort_expand2(const NodeDev& n, const GroupDev& g, int nblk, const uint32_t* base,
                               int64_t ts_min, uint64_t ts_div, int R, uint64_t* keys, uint32_t* vals,
                               hipStream_t st) {
    hipLaunchKernelGGL(k_sort_expand, dim3(nblk), dim3(SORT_BLOCK), 0, st, n, g, base, ts_min, ts_div, R,
                       keys, vals);
    return hipGetLastError();
}

hipError_t launch_radix_pass(const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout,
                             int64_t n, int shift, int nblk, uint32_t* hist, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(SORT_BLOCK), 0, st, kin, n, shift, hist);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(SORT_BLOCK), 0, st, hist, nblk * 256, (uint32_t*)nullptr);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(SORT_BLOCK), 0, st, kin, vin, kout, vout, n, shift, hist);
    return hipGetLastError();
}

hipError_t launch_group_bounds(const uint64_t* keys, int64_t n, int key_shift, int32_t nseg, int64_t* seg,
                               hipStream_t st) {
    hipLaunchKernelGGL(k_group_bounds, dim3((nseg + 1 + 255) / 256), dim3(256), 0, st, keys, n, key_shift, nseg, seg);
    return hipGetLastError();
}

}  // namespace esc
