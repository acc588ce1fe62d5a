// esc_kernels.hip — gfx950 kernels of the scale-decision hot path.
//
//  K1 k_pod_reduce   : FilteredPodsLister.List (pod_listers.go:33) for EVERY group at once
//                      + ComputePodResourceRequest (scheduler/types.go:72) +
//                      CalculatePodsRequestsTotal (util.go:27).  One pass over the pod SoA,
//                      16-B-per-lane coalesced loads (4 pods per lane, 256 per wave), int64
//                      per-group partials privatised in LDS (ds_add_u64), flushed once per
//                      workgroup.  HBM-bound; no MFMA (nothing is a contraction).
//  K2 node pieces    : (k_step_tail) FilteredNodesLister.List + filterNodes (controller.go:120) +
//                      CalculateNodesCapacityTotal(untainted) (util.go:41) over the
//                      pair-major node entries: one wave per piece, register sums, one
//                      row per piece.  No LDS, no atomics, exact for any int64 input.
//  K3 fold           : (k_step_tail) the K1 partials of every pod slot summed into each
//                      group's pod words (int64 split lo32 / hi, exchanged when sharded);
//                      K2 and the packed K5 chunks run as other blocks of the same launch.
//  K2b+K4 k_node_groups: each group's node words from its pair's pieces (+ allNodes[0],
//                      controller.go:208, and the dry-mode tracker), then calcPercentUsage /
//                      switch / calcScaleUpDelta / scaleDownTaint clamp (util.go:13-81,
//                      controller.go:233-351, scale_down.go:138-158).
//  K5 ordering       : taintOldestN / untaintNewestN (scale_down.go:171, scale_up.go:118,
//                      sort.go:18,33): an age index (LSD radix sort of creation times,
//                      once per snapshot) + a per-decision stable partition by
//                      (group, class).
// Wide variants      : exact any-range pod fallback with global atomics.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "esc_kernels.h"

// Written for gfx950 only: K1's 10 240-slot LDS window (160 KB) and the age-index scatter's
// carried lines (~109 KB per 1024-thread block at 8-bit digits) need CDNA4's 160 KB of LDS
// per CU; a gfx942 (64 KB) build would fail to launch, so it is refused here.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "esc_kernels.hip targets gfx950 (160 KB LDS per CU); build with ARCH=gfx950"
#endif

#ifndef ESC_PART
#define ESC_PART 0
#endif
#ifndef K1_PK_DS
#define K1_PK_DS 6      // packed K tiles in flight per K1 wave (at most; the VGPR budget may allow fewer)
#endif
#ifndef K1_PK8_DS
#define K1_PK8_DS 8     // packed small K tiles in flight per K1 wave (at most)
#endif

namespace esc {

namespace {

// Streamed (read-once) snapshot loads are nontemporal: on this MI355X a 2.4 GB 16-B-per-
// lane sweep reads at 6.95 TB/s with nt loads vs 6.37 TB/s without (scripts/stream_probe.hip,
// profiles/r01_v4/stream_probe.json).
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint64_t v2u64 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld4(const uint32_t* p) {
    const v4u32 t = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ ulonglong2 ld2(const int64_t* p) {
    const v2u64 t = __builtin_nontemporal_load(reinterpret_cast<const v2u64*>(p));
    ulonglong2 r;
    r.x = t.x;
    r.y = t.y;
    return r;
}
template <class T>
__device__ __forceinline__ T ldnt(const T* p) { return __builtin_nontemporal_load(p); }

// Buffer loads through a wave-uniform descriptor (nontemporal: aux 2 = nt on gfx950).  An
// offset at or past the descriptor's size returns zeros without touching memory: K1's
// pipeline refills past the end of a run cost no traffic.
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rsrc(const void* base, int64_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bytes);
    void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)n, 0x00020000);
}
__device__ __forceinline__ uint4 ldb4(Rsrc rs, uint32_t off) {
    const v4u32 t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2);
    return make_uint4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ uint2 ldb8(Rsrc rs, uint32_t off) {     // 8 B per lane
    const auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 2);
    return make_uint2(t[0], t[1]);
}
__device__ __forceinline__ ulonglong2 ldb2(Rsrc rs, uint32_t off) {
    const v4u32 t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2);
    ulonglong2 r;
    r.x = ((uint64_t)t.y << 32) | t.x;
    r.y = ((uint64_t)t.w << 32) | t.z;
    return r;
}
constexpr uint32_t RUN_OOB = 0x7FFF0000u;     // a tile offset past every run (K1 runs are < 2 GB)

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

// Sum over the wave's 64 lanes of a 64-bit value with DPP (VALU only, no LDS round trips):
// the inclusive-scan pattern of wave_incl_scan32 on both halves, total read from lane 63.
// (The __shfl_xor butterfly is 12 dependent ds_bpermute per value; K2's 9-value piece
// reductions spent most of their time waiting on them.)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ unsigned long long dpp64(unsigned long long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW_MASK, 0xF, false);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_total32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(v), 63);
}
__device__ __forceinline__ unsigned long long wave_total64(unsigned long long v) {
    v += dpp64<0x111, 0xF>(v);
    v += dpp64<0x112, 0xF>(v);
    v += dpp64<0x114, 0xF>(v);
    v += dpp64<0x118, 0xF>(v);
    v += dpp64<0x142, 0xA>(v);
    v += dpp64<0x143, 0xC>(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
    return __shfl(v, src, 64);
}

// Sum over the wave's 64 lanes, result in every lane (butterfly).
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int64_t imin64(int64_t a, int64_t b) { return a < b ? a : b; }
__device__ __forceinline__ int64_t imax64(int64_t a, int64_t b) { return a > b ? a : b; }

// ------------------------------------------------------- selector-pair matching
// NewPodAffinityFilterFunc / NewNodeLabelFilterFunc (node_group.go:218, :278) for all
// groups at once: a pair id selects the groups whose (label_key, label_value) it is;
// ids >= n_gp are values no group selects.
//  - pods: K1 accumulates per pair (LDS slot = pair id, plus one slot for the default
//    filter) and K3 joins each group to its pair's slot — the per-pod test
//    "(K_g, V_g) in pod pairs" evaluated for every group without a per-pod lookup;
//  - nodes: K2 accumulates the pair-major entries per piece and K3 joins each group to
//    its pair's pieces; K5 resolves each label pair through the node code table (a group
//    id, NONE, or a list of the groups sharing the pair).
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
    uint32_t plim;       // pair slots of this window: pair q is slot q - g0 when that is < plim
    uint32_t dslot;      // the default filter's slot in this window, or NONE (none / another window)
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

// ------------------------------------------------------------------ K tiles
// Homogeneous 256-pod tiles: every pod of a class has the same record signature, so
// record k of a tile's pods is one 256-entry row and every array — the pods' own fields
// and each record / pair row — is one 16-B load per lane (4 pods per lane).  No per-pod
// offsets, no cross-lane moves, wave-uniform record semantics.
template <int R, int NXP, int PK>
struct KTile;
template <int R, int NXP>
struct KTile<R, NXP, 0> {            // plain block
    uint4 f, c, p;
    ulonglong2 m[2];
    ulonglong2 rc[R > 0 ? R : 1][2], rm[R > 0 ? R : 1][2];
    uint4 rq[NXP > 0 ? NXP : 1];
};
template <int R, int NXP>
struct KTile<R, NXP, 2> {            // packed small block (esc_kernels.h, kp8_*)
    ulonglong2 w[2];                 // cpu0 | mem0 << 14 | pair0 << 48 | flags << 62
    ulonglong2 r[R > 0 ? R : 1][2];  // records, cpu | mem << 20
    uint2 rq[NXP > 0 ? NXP : 1];     // u16 pairs, 4 per lane
};
template <int R, int NXP>
struct KTile<R, NXP, 1> {            // packed block (esc_kernels.h, kp_*)
    uint4 a;                         // pair0 | pod flags << 28
    ulonglong2 cm[2];                // cpu0 | mem0 << 20
    ulonglong2 r[R > 0 ? R : 1][2];  // records, cpu | mem << 20
    uint4 rq[NXP > 0 ? NXP : 1];
};

// pod j's u16 pair of a packed small block's 8-B lane load (0xFFFF: none -> above every slot)
__device__ __forceinline__ uint32_t kp8_xp(const uint2& v, int j) {
    return ((j < 2 ? v.x : v.y) >> (16 * (j & 1))) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t lane4(const uint4& v, int j) {
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}
__device__ __forceinline__ uint64_t lane4(const ulonglong2 (&v)[2], int j) {
    return (j & 1) ? v[j >> 1].y : v[j >> 1].x;
}

typedef __attribute__((address_space(4))) const PodClass cPodClass;   // scalar loads
__device__ __forceinline__ PodClass load_class(const PodClass* cls, int i) {
    const cPodClass* q = (const cPodClass*)cls + i;
    PodClass k;
    k.t0 = q->t0; k.t1 = q->t1; k.kb0 = q->kb0; k.rsv = 0;
    k.w0 = q->w0;
    k.xreg = q->xreg; k.xinit = q->xinit; k.ovh = q->ovh; k.nxp = q->nxp; k.kind = q->kind; k.wt = q->wt;
    return k;
}

// In-tile positions: pod j of lane l is element 4l + j of the 4-byte arrays and element
// (j / 2) * 128 + 2l + j % 2 of the 8-byte ones (pos64), so that every wave-load of either
// width reads one contiguous 1 KB (an 8-byte array read as lanes x 4 consecutive pods would
// stride 32 B and double the requests per byte).

// One tile = one contiguous block (esc_kernels.h, K blocks): every load below is lane l's
// 16 B at a compile-time offset from the block's first word, through the run's descriptor
// (`to` = the tile's byte offset in the run; RUN_OOB past its end: zeros, no traffic).
template <int R, int NXP>
__device__ __forceinline__ void k_load(Rsrc rs, uint32_t to, uint32_t lane, KTile<R, NXP, 2>& T, const PodClass&) {
    const uint32_t o = to + lane * 16;
    auto w = [&](int words) { return o + 4u * (uint32_t)words; };
    T.w[0] = ldb2(rs, o);
    T.w[1] = ldb2(rs, w(256));
#pragma unroll
    for (int k = 0; k < R; ++k) {
        T.r[k][0] = ldb2(rs, w(KP8_REC + 512 * k));
        T.r[k][1] = ldb2(rs, w(KP8_REC + 512 * k + 256));
    }
#pragma unroll
    for (int k = 0; k < NXP; ++k) T.rq[k] = ldb8(rs, to + lane * 8 + 4u * (KP8_REC + 512 * R + 128 * k));
}

// Packed (12-B) blocks: since the small blocks take most pods, one pipeline for every
// shape (R = NXP = 3 at most, the class's counts select the rows, as for plain blocks).
template <int R, int NXP>
__device__ __forceinline__ void k_load(Rsrc rs, uint32_t to, uint32_t lane, KTile<R, NXP, 1>& T, const PodClass& C) {
    const uint32_t o = to + lane * 16;
    const uint32_t nr = kb_nrec(C);
    auto w = [&](int words) { return o + 4u * (uint32_t)words; };
    T.a = ldb4(rs, o);
    T.cm[0] = ldb2(rs, w(KP_CM0));
    T.cm[1] = ldb2(rs, w(KP_CM0 + 256));
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const bool on = (uint32_t)k < nr;
        T.r[k][0] = ldb2(rs, on ? w(KP_REC + 512 * k) : RUN_OOB);
        T.r[k][1] = ldb2(rs, on ? w(KP_REC + 512 * k + 256) : RUN_OOB);
    }
#pragma unroll
    for (int k = 0; k < NXP; ++k)
        T.rq[k] = ldb4(rs, (uint32_t)k < C.nxp ? o + 4u * (KP_REC + 512u * nr + 256u * (uint32_t)k) : RUN_OOB);
}

// Plain blocks (pods outside the packed ranges: rare) go through ONE pipeline for every
// shape: R and NXP are the maxima (3, 3) and the class's own counts select the rows; the
// rows it lacks load through the descriptor's out-of-range offset (zeros, no traffic).
template <int R, int NXP>
__device__ __forceinline__ void k_load(Rsrc rs, uint32_t to, uint32_t lane, KTile<R, NXP, 0>& T, const PodClass& C) {
    const uint32_t o = to + lane * 16;
    const uint32_t nr = kb_nrec(C);
    auto w = [&](int words) { return o + 4u * (uint32_t)words; };
    T.f = ldb4(rs, o);
    T.c = ldb4(rs, w(KB_CPU0));
    T.m[0] = ldb2(rs, w(KB_MEM0));
    T.m[1] = ldb2(rs, w(KB_MEM0 + 256));
    T.p = ldb4(rs, w(KB_PAIR0));
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const bool on = (uint32_t)k < nr;
        T.rc[k][0] = ldb2(rs, on ? w(KB_REC + 1024 * k) : RUN_OOB);
        T.rc[k][1] = ldb2(rs, on ? w(KB_REC + 1024 * k + 256) : RUN_OOB);
        T.rm[k][0] = ldb2(rs, on ? w(KB_REC + 1024 * k + 512) : RUN_OOB);
        T.rm[k][1] = ldb2(rs, on ? w(KB_REC + 1024 * k + 768) : RUN_OOB);
    }
#pragma unroll
    for (int k = 0; k < NXP; ++k)
        T.rq[k] = ldb4(rs, (uint32_t)k < C.nxp ? o + 4u * (KB_REC + 1024u * nr + 256u * (uint32_t)k) : RUN_OOB);
}

// ComputePodResourceRequest (scheduler/types.go:72-89) for each of the lane's 4 pods:
// records [0, xreg) are regular containers (add), [xreg, xreg + xinit) init containers
// (max; an absent key is INT64_MIN), the last the overhead (add), with Go's wrapping
// int64 +=; then the pod's memberships (node_group.go:218-275).
// The same for a packed block: values unpacked in registers (an init record's absent key
// — its field's sentinel — takes no part in the max, as INT64_MIN would not).
template <int R, int NXP, int ABLATE>
__device__ __forceinline__ void k_process(const GroupDev& G, const PodSink<ABLATE>& K, const PodClass& C,
                                          const KTile<R, NXP, 1>& T) {
    const uint32_t init_end = C.xreg + C.xinit;
#pragma unroll
    for (int j = 0; j < PODS_PER_LANE; ++j) {
        const uint32_t a = lane4(T.a, j);
        if (a & (ESC_PF_DAEMONSET << KP_FLAG_SHIFT)) continue;      // node_group.go:221, :259
        const uint64_t cm = lane4(T.cm, j);
        uint64_t cpu = cm & KP_CPU_ABSENT, mem = cm >> KP_CPU_BITS;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint64_t v = lane4(T.r[k], j);
            const uint64_t c = v & KP_CPU_ABSENT, m = v >> KP_CPU_BITS;
            if ((uint32_t)k < C.xreg || (uint32_t)k >= init_end) {
                cpu += c;
                mem += m;
            } else {                                   // values and sums are >= 0 here
                cpu = (c == KP_CPU_ABSENT || cpu >= c) ? cpu : c;
                mem = (m == KP_MEM_ABSENT || mem >= m) ? mem : m;
            }
        }
        const bool in = in_range(cpu, mem);
        if ((a >> KP_FLAG_SHIFT) == 0 && G.default_group != NONE) K.add(G.n_gp, cpu, mem, in);   // pf_default_ok
        const uint32_t q0 = a & KP_PAIR_NONE;
        if (q0 < G.n_gp) K.add(q0, cpu, mem, in);
#pragma unroll
        for (int k = 0; k < NXP; ++k) {
            const uint32_t q = lane4(T.rq[k], j);
            if ((uint32_t)k < C.nxp && q < G.n_gp) K.add(q, cpu, mem, in);   // rows past the class's: zeros
        }
    }
}

// The packed small block: one u64 per pod (kp8_*), records as in the packed block.
template <int R, int NXP, int ABLATE>
__device__ __forceinline__ void k_process(const GroupDev& G, const PodSink<ABLATE>& K, const PodClass& C,
                                          const KTile<R, NXP, 2>& T) {
    const uint32_t init_end = C.xreg + C.xinit;
#pragma unroll
    for (int j = 0; j < PODS_PER_LANE; ++j) {
        // (a daemonset pod, node_group.go:221 / :259, is stored with no pairs and
        // blocks-default set: it is added nowhere, no test needed)
        const uint64_t w = lane4(T.w, j);
        uint64_t cpu = w & KP8_CPU_MASK, mem = (w >> KP8_CPU_BITS) & KP8_MEM_MASK;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint64_t v = lane4(T.r[k], j);
            const uint64_t c = v & KP_CPU_ABSENT, m = v >> KP_CPU_BITS;
            if ((uint32_t)k < C.xreg || (uint32_t)k >= init_end) {
                cpu += c;
                mem += m;
            } else {                                   // values and sums are >= 0 here
                cpu = (c == KP_CPU_ABSENT || cpu >= c) ? cpu : c;
                mem = (m == KP_MEM_ABSENT || mem >= m) ? mem : m;
            }
        }
        // without records the pod is inside the LDS range by construction (2^14, 2^34)
        const bool in = R == 0 ? true : in_range(cpu, mem);
        const uint32_t q0 = (uint32_t)(w >> KP8_PAIR_SHIFT) & KP8_PAIR_NONE;
        if (in) {
            if constexpr (ABLATE & 1) {
                asm volatile("" :: "v"(q0), "v"(cpu), "v"(mem));
            } else {
                // slot adds straight to LDS: pair q is slot q - g0 of this window when below
                // plim (NONE and pairs no group selects are above it), the default slot
                // when the pod passes the default filter (pf_default_ok)
                const uint64_t vcc = cpu | (1ull << CNT_SHIFT);
                if (K.acc.dslot != NONE && !(w & KP8_NODEF)) {
                    lds_add(K.acc.cc + K.acc.dslot, vcc);
                    lds_add(K.acc.mem + K.acc.dslot, mem);
                }
                const uint32_t i0 = q0 - (uint32_t)K.acc.g0;
                if (i0 < K.acc.plim) { lds_add(K.acc.cc + i0, vcc); lds_add(K.acc.mem + i0, mem); }
#pragma unroll
                for (int k = 0; k < NXP; ++k) {
                    const uint32_t i = kp8_xp(T.rq[k], j) - (uint32_t)K.acc.g0;
                    if (i < K.acc.plim) { lds_add(K.acc.cc + i, vcc); lds_add(K.acc.mem + i, mem); }
                }
            }
        } else {                                       // outside the LDS range: the exact words
            if (!(w & KP8_NODEF) && G.default_group != NONE) K.add(G.n_gp, cpu, mem, false);
            if (q0 < G.n_gp) K.add(q0, cpu, mem, false);
#pragma unroll
            for (int k = 0; k < NXP; ++k) {
                const uint32_t q = kp8_xp(T.rq[k], j);
                if (q < G.n_gp) K.add(q, cpu, mem, false);
            }
        }
    }
}

template <int R, int NXP, int ABLATE>
__device__ __forceinline__ void k_process(const GroupDev& G, const PodSink<ABLATE>& K, const PodClass& C,
                                          const KTile<R, NXP, 0>& T) {
    const uint32_t init_end = C.xreg + C.xinit;
#pragma unroll
    for (int j = 0; j < PODS_PER_LANE; ++j) {
        const uint32_t f = lane4(T.f, j);
        if (f & ESC_PF_DAEMONSET) continue;                          // node_group.go:221, :259
        uint64_t cpu = lane4(T.c, j), mem = lane4(T.m, j);
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const uint64_t c = lane4(T.rc[k], j), m = lane4(T.rm[k], j);
            if ((uint32_t)k < C.xreg || (uint32_t)k >= init_end) {
                cpu += c;
                mem += m;
            } else {
                cpu = ((int64_t)cpu >= (int64_t)c) ? cpu : c;
                mem = ((int64_t)mem >= (int64_t)m) ? mem : m;
            }
        }
        const bool in = in_range(cpu, mem);
        if (pf_default_ok(f) && G.default_group != NONE) K.add(G.n_gp, cpu, mem, in);
        const uint32_t q0 = lane4(T.p, j);
        if (q0 < G.n_gp) K.add(q0, cpu, mem, in);
#pragma unroll
        for (int k = 0; k < NXP; ++k) {
            const uint32_t q = lane4(T.rq[k], j);
            if ((uint32_t)k < C.nxp && q < G.n_gp) K.add(q, cpu, mem, in);   // rows past the class's: zeros
        }
    }
}

template <int R, int NXP>
__device__ __forceinline__ void k_sink(const KTile<R, NXP, 2>& T) {   // loads-only ablation
    uint64_t y = T.w[0].x ^ T.w[0].y ^ T.w[1].x ^ T.w[1].y;
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h) y ^= T.r[k][h].x ^ T.r[k][h].y;
#pragma unroll
    for (int k = 0; k < NXP; ++k) x ^= T.rq[k].x ^ T.rq[k].y;
    asm volatile("" :: "v"(x), "v"(y));
}

template <int R, int NXP>
__device__ __forceinline__ void k_sink(const KTile<R, NXP, 1>& T) {   // loads-only ablation
    uint32_t x = T.a.x ^ T.a.y ^ T.a.z ^ T.a.w;
    uint64_t y = T.cm[0].x ^ T.cm[0].y ^ T.cm[1].x ^ T.cm[1].y;
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h) y ^= T.r[k][h].x ^ T.r[k][h].y;
#pragma unroll
    for (int k = 0; k < NXP; ++k) x ^= T.rq[k].x ^ T.rq[k].y ^ T.rq[k].z ^ T.rq[k].w;
    asm volatile("" :: "v"(x), "v"(y));
}

template <int R, int NXP>
__device__ __forceinline__ void k_sink(const KTile<R, NXP, 0>& T) {   // loads-only ablation
    uint32_t x = T.f.x ^ T.f.y ^ T.f.z ^ T.f.w ^ T.c.x ^ T.c.y ^ T.c.z ^ T.c.w ^ T.p.x ^ T.p.y ^ T.p.z ^ T.p.w;
    uint64_t y = T.m[0].x ^ T.m[0].y ^ T.m[1].x ^ T.m[1].y;
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h) y ^= T.rc[k][h].x ^ T.rc[k][h].y ^ T.rm[k][h].x ^ T.rm[k][h].y;
#pragma unroll
    for (int k = 0; k < NXP; ++k) x ^= T.rq[k].x ^ T.rq[k].y ^ T.rq[k].z ^ T.rq[k].w;
    asm volatile("" :: "v"(x), "v"(y));
}

// Tiles a, a + NW, ... (< b) of one class for this wave: a rolling pipeline of DS tile
// slots (slot d is processed, then refilled with the tile DS rounds ahead).  DS follows
// the tile's register footprint.  Every load is unconditional, so the compiler's vmcnt
// accounting never waits early; the refills past the end go through the wave's run
// descriptor at an offset past its size, which returns zeros without a memory access (they
// used to re-read the slot's last tile: 1.2x K1's algorithmic fetch at 12.5 M pods).
template <int R, int NXP, int PK, int NW, int ABLATE, int ST>
__device__ __forceinline__ void k_run(const PodDev& P, const GroupDev& G, const PodSink<ABLATE>& K,
                                      const PodClass& C, int64_t a, int64_t b, uint32_t lane) {
    constexpr int W = (int)k_tile_weight(R, NXP, PK);    // block size, half-KB units (generic: at most)
    // VGPRs a tile slot holds: 4 per 16-B load, 2 per 8-B one (the packed small pair rows)
    constexpr int L = PK == 2 ? (4 + 4 * R + NXP) : W / 2;
    // block words: a compile-time constant for the specialised (packed small) shapes, the
    // class's own for the generic pipelines
    const int64_t BW = PK == 2 ? (int64_t)W * KB_UNIT : (int64_t)C.wt * KB_UNIT;
    // the wave's run: tiles [a, b) -> bytes [0, (b - a) * BW * 4) of its descriptor
    const Rsrc rs = rsrc(P.kb + C.kb0 + (a - C.t0) * BW, (b - a) * BW * 4);
    auto off = [&](int64_t u) { return u < b ? (uint32_t)((u - a) * BW * 4) : RUN_OOB; };
    // slots that fit the VGPR budget: 16 waves per CU leave 128 VGPRs a wave, 8 leave 256
    // (a packed tile is smaller, so more of them are in flight: up to K1_PK_DS)
    constexpr int DSM = PK == 2 ? K1_PK8_DS : (PK ? K1_PK_DS : 4);
    constexpr int VG = PK == 2 ? 2 * L : 4 * L;
    constexpr int DS0 = NW >= 16 ? (L <= 7 ? 3 : (L <= 10 ? 2 : 1))
                                 : (176 / VG >= DSM ? DSM : (176 / VG >= 1 ? 176 / VG : 1));
    // timing knobs (ABLATE bits 6/7): cap the slots in flight at 2 / 3
    constexpr int DS = (ABLATE & 64) ? (DS0 < 2 ? DS0 : 2) : ((ABLATE & 128) ? (DS0 < 3 ? DS0 : 3) : DS0);
    KTile<R, NXP, PK> T[DS];
#pragma unroll
    for (int d = 0; d < DS; ++d) {
        k_load(rs, off(a + (int64_t)d * ST), lane, T[d], C);
        __builtin_amdgcn_sched_barrier(0);            // slots issue in order (see below)
    }
    for (int64_t t = a; t < b; t += (int64_t)DS * ST) {
#pragma unroll
        for (int d = 0; d < DS; ++d) {
            const int64_t u = t + (int64_t)d * ST;
            if (u < b) {                                       // wave-uniform
                if constexpr (ABLATE & 32) k_sink(T[d]);
                else k_process<R, NXP, ABLATE>(G, K, C, T[d]);
            }
            // keep slot d's refill after its use: hoisting it would make the next slots'
            // waits count it (vmcnt is in order) and drain the pipeline
            __builtin_amdgcn_sched_barrier(0);
            k_load(rs, off(u + (int64_t)DS * ST), lane, T[d], C);
            __builtin_amdgcn_sched_barrier(0);
        }
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
    const int64_t i = t * CTILE + lane;                  // C arrays start at the C section
    T.b = b;
    T.f = ldnt(P.flags + i);
    T.c = ldnt(P.cpu0 + i);
    T.m = (uint64_t)ldnt(P.mem0 + i);
    T.p = ldnt(P.pair0 + i);
    const uint32_t lc = (b.xcn ? b.xcn : 1u) - 1u, lp = (b.xpn ? b.xpn : 1u) - 1u;
    const uint32_t c0 = b.xcb + min(lane, lc), c1 = b.xcb + min(lane + 64, lc);
    const uint32_t p0 = b.xpb + min(lane, lp), p1 = b.xpb + min(lane + 64, lp);
    T.xcc0 = (unsigned long long)ldnt(P.xc_cpu + c0);
    T.xcm0 = (unsigned long long)ldnt(P.xc_mem + c0);
    T.xcc1 = (unsigned long long)ldnt(P.xc_cpu + c1);
    T.xcm1 = (unsigned long long)ldnt(P.xc_mem + c1);
    T.xp0 = ldnt(P.xp + p0);
    T.xp1 = ldnt(P.xp + p1);
}

// Record k of every lane's run [o, o + n) of the tile's records (lane l holds records l
// and l + 64), fetched with ds_bpermute; `hi` = the tile has more than 64 records.
__device__ __forceinline__ void rec64(const unsigned long long (&r)[2], uint32_t rel, bool hi, unsigned long long& v) {
    v = shfl64(r[0], (int)(rel & 63));
    if (hi) {
        const unsigned long long v1 = shfl64(r[1], (int)(rel & 63));
        if (rel >= 64) v = v1;
    }
}
__device__ __forceinline__ uint32_t rec32(uint32_t r0, uint32_t r1, uint32_t rel, bool hi) {
    uint32_t v = __shfl(r0, (int)(rel & 63), 64);
    if (hi) {
        const uint32_t v1 = __shfl(r1, (int)(rel & 63), 64);
        if (rel >= 64) v = v1;
    }
    return v;
}

// ComputePodResourceRequest step for record k of a pod (types.go:72-89): regular extras
// add, init containers max, the overhead adds (Go's wrapping int64 +=).
__device__ __forceinline__ void apply_rec(uint32_t k, uint32_t nxc, uint32_t nreg, uint32_t add_from,
                                          unsigned long long c, unsigned long long m, uint64_t& cpu, uint64_t& mem) {
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

// One C tile: the per-pod record offsets come from a DPP wave prefix sum of the packed
// counts; each pod pulls its k-th record / pair with ds_bpermute in a wave-uniform loop.
// (Issuing the first rounds' bpermutes back to back measured slower: the C path is
// LDS-issue-bound, not latency-bound.)
template <int ABLATE>
__device__ __forceinline__ void c_process(const GroupDev& G, const PodSink<ABLATE>& K, const CTile& T) {
    const uint32_t f = T.f;
    const uint32_t nxc = pf_xctr(f), nxp = pf_xpair(f);
    const uint32_t v = nxc | (nxp << 16);                 // tile totals <= 128 each
    const uint32_t ex = wave_incl_scan32(v) - v;
    const uint32_t oc = ex & 0xFFFF, op = ex >> 16;
    const bool chi = T.b.xcn > 64, phi = T.b.xpn > 64;   // wave-uniform
    const unsigned long long xc[2] = {T.xcc0, T.xcc1}, xm[2] = {T.xcm0, T.xcm1};
    uint64_t cpu = T.c, mem = T.m;
    const uint32_t nreg = pf_xreg(f), add_from = nreg + pf_xinit(f);
    for (uint32_t k = 0; wave_any(k < nxc); ++k) {
        unsigned long long c, m;
        rec64(xc, oc + k, chi, c);
        rec64(xm, oc + k, chi, m);
        apply_rec(k, nxc, nreg, add_from, c, m, cpu, mem);
    }
    const bool live = !(f & ESC_PF_DAEMONSET);            // node_group.go:221, :259
    const bool in = in_range(cpu, mem);
    if (live) {
        if (pf_default_ok(f) && G.default_group != NONE) K.add(G.n_gp, cpu, mem, in);
        if (T.p < G.n_gp) K.add(T.p, cpu, mem, in);
    }
    for (uint32_t k = 0; wave_any(k < nxp); ++k) {
        const uint32_t q = rec32(T.xp0, T.xp1, op + k, phi);
        if (live && k < nxp && q < G.n_gp) K.add(q, cpu, mem, in);
    }
}

// Exact (any-range) evaluation of one C tile from memory, one pod per lane.
__device__ __forceinline__ void c_tile_exact(const PodDev& P, const GroupDev& G, int64_t t, uint32_t lane,
                                             int64_t* __restrict__ wide) {
    const int64_t i = t * CTILE + lane;
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

// ------------------------------------------------------------------ K2 spans
// (k_step_tail's piece role; inside K1's first window they cost K1 as much as they saved in
// the tail: +20 us, profiles/r02_v10)
namespace {
// Adds one entry to the piece accumulators: its wet class (filterNodes,
// controller.go:141-150: Spec.Unschedulable first, then the escalator taint) and the
// every-member sums used by dry-mode groups.
// A row's sums are exact as (LO, HI) with LO + HI * 2^32 = the int64 total (K2b joins them in
// 128 bits).  An entry whose cpu and memory are both in [0, 2^54) adds its whole value to LO
// (add_small: <= 1024 entries per piece keep LO below 2^64); otherwise its low 32 bits go to
// LO and its high part, signed, to HI (add_split), and the piece's HI words are reduced
// only when some wave-load of it took that path (`split`, wave-uniform) — allocatable
// values are always small in practice, so a flush reduces 5 words instead of 9.
struct PieceAcc {
    unsigned long long ucl = 0, uch = 0, uml = 0, umh = 0, acl = 0, ach = 0, aml = 0, amh = 0, cnt = 0;
    bool split = false;
    __device__ __forceinline__ void count(uint32_t f, bool& unt) {
        const int cls = (f & ESC_NF_UNSCHED) ? 2 : ((f & ESC_NF_TAINTED) ? 1 : 0);
        unt = cls == 0;
        cnt += 1ull << (NR_CNT_BITS * cls);
    }
    __device__ __forceinline__ void add_small(uint32_t f, int64_t c, int64_t m) {
        if (f & ESC_NF_ABSENT) return;               // spare entry or deleted node
        bool unt;
        count(f, unt);
        acl += (uint64_t)c; aml += (uint64_t)m;
        if (unt) { ucl += (uint64_t)c; uml += (uint64_t)m; }
    }
    __device__ __forceinline__ void add_split(uint32_t f, int64_t c, int64_t m) {
        if (f & ESC_NF_ABSENT) return;
        const unsigned long long cl = (uint64_t)c & 0xFFFFFFFFull, ml = (uint64_t)m & 0xFFFFFFFFull;
        const unsigned long long chh = (unsigned long long)(c >> 32), mhh = (unsigned long long)(m >> 32);
        bool unt;
        count(f, unt);
        acl += cl; ach += chh; aml += ml; amh += mhh;
        if (unt) { ucl += cl; uch += chh; uml += ml; umh += mhh; }
    }
};

// K2 span w (one wave; see node_piece_block).  The span's entry range comes from a scalar
// array (span_e), so the first round of entry loads is issued with the piece-bounds load
// instead of after it (one dependent round trip fewer).
__device__ __forceinline__ void node_span(const NodeDev& N, int64_t* __restrict__ rows, int64_t w, int lane) {
    if (w >= N.n_spans) return;
    typedef __attribute__((address_space(4))) const uint32_t cu32n;
    const uint32_t p0 = ((const cu32n*)N.span_off)[w], p1 = ((const cu32n*)N.span_off)[w + 1];
    const uint32_t e0 = ((const cu32n*)N.span_e)[w], z = ((const cu32n*)N.span_e)[w + 1];
    // the span's <= 64 piece bounds, one per lane (a span has <= 63 pieces), read with
    // readlane: no dependent load per piece
    const uint32_t np = p1 - p0;
    const uint32_t bound = N.piece_off[p0 + (lane < (int)np ? (uint32_t)lane : np)];
    constexpr int U = NODE_SPAN / 64;                // a NODE_SPAN span's loads in one round
    uint32_t f[U];
    int64_t c[U], m[U];
    auto load = [&](uint32_t base) {
#ifndef ESC_K2_ARRAYS                                // (timing builds: the three arrays only)
        if (N.e_pk) {                                // packed entries: one 16-B load each
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = base + u * 64 + lane, ii = i < z ? i : z - 1;
                const uint4 v = ld4(reinterpret_cast<const uint32_t*>(N.e_pk + ii));
                f[u] = v.x;
                c[u] = (int64_t)v.y;
                m[u] = (int64_t)((uint64_t)v.z | (uint64_t)v.w << 32);
            }
            return;
        }
#endif
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = base + u * 64 + lane, ii = i < z ? i : z - 1;
            f[u] = ldnt(N.e_flags + ii);
            c[u] = ldnt(N.e_cpu + ii);
            m[u] = ldnt(N.e_mem + ii);
        }
    };
    if (e0 < z) load(e0);
    auto off = [&](uint32_t k) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)bound, (int)k); };
    uint32_t p = p0, ps = e0, pe = off(1);
    PieceAcc acc;
    auto flush = [&]() {                             // piece p's row, then the next piece
        const bool sp = acc.split;                   // wave-uniform: HI words only if used
        const unsigned long long v[NR_K] = {wave_total64(acc.ucl), sp ? wave_total64(acc.uch) : 0ull,
                                            wave_total64(acc.uml), sp ? wave_total64(acc.umh) : 0ull,
                                            wave_total64(acc.acl), sp ? wave_total64(acc.ach) : 0ull,
                                            wave_total64(acc.aml), sp ? wave_total64(acc.amh) : 0ull,
                                            wave_total64(acc.cnt)};
        unsigned long long x = 0;
#pragma unroll
        for (int k = 0; k < NR_K; ++k) x = lane == k ? v[k] : x;
        if (rows && lane < NR_K) rows[(int64_t)lane * N.n_pieces + p] = (int64_t)x;
        acc = PieceAcc();
        ++p;
        ps = pe;
        if (p < p1) pe = off(p + 1 - p0);
    };
    for (uint32_t base = e0; base < z; base += 64 * U) {
        if (base != e0) load(base);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t lo = base + u * 64, i = lo + lane;
            if (lo >= z) break;
            constexpr uint64_t SMALL = 1ull << 54;
            const bool small = __ballot((uint64_t)c[u] >= SMALL || (uint64_t)m[u] >= SMALL) == 0;   // wave-uniform
            for (;;) {                                   // wave-uniform: p, ps, pe
                if (small) {
                    if (i >= ps && i < pe && i < z) acc.add_small(f[u], c[u], m[u]);
                } else {
                    acc.split = true;
                    if (i >= ps && i < pe && i < z) acc.add_split(f[u], c[u], m[u]);
                }
                if (p >= p1 || pe > lo + 63) break;      // piece p goes on in the next load
                flush();
            }
        }
    }
    while (p < p1) flush();                          // the span's last piece(s)
}

// Does node i carry label pair q (label0 or one of its ascending extra pairs)?
__device__ __forceinline__ bool node_has_pair(const NodeDev& N, int64_t i, uint32_t q) {
    const uint32_t l0 = N.label0[i];
    if (l0 == q) return true;
    if (l0 == NONE || l0 > q) return false;
    const uint32_t nx = nf_xlbl(N.flags[i]), o = N.xl_off[i];
    for (uint32_t k = 0; k < nx; ++k) {
        const uint32_t x = N.xl[o + k];
        if (x >= q) return x == q;
    }
    return false;
}

// Dry-mode tracker entry k (controller.go:128-133): a (node, dry group) entry whose node is
// a live member of the group, in this rank's share of the group's pieces, adds the node to
// the group's tracked sums (trk_acc, global atomics: a few thousand entries), which the node
// groups read and reset.  Membership comes from the node's own labels: a pair's entries are
// not node-sorted once relabels / adds have appended to them.
__device__ __forceinline__ void tracker_entry(const NodeDev& N, const GroupDev& G, int64_t* __restrict__ trk_acc,
                                              int64_t k) {
    if (k >= N.n_trk) return;
    const int32_t j = N.trk_node[k], g = N.trk_group[k];
    if (!G.dry[g]) return;                           // wet groups ignore the tracker
    const uint32_t q = G.gpair[g];
    const int64_t plo = imax64((int64_t)N.pp_off[q], N.pc_lo), phi = imin64((int64_t)N.pp_off[q + 1], N.pc_hi);
    if (phi <= plo) return;
    if ((N.flags[j] & ESC_NF_ABSENT) || !node_has_pair(N, j, q)) return;
    const int64_t c = N.cpu[j], m = N.mem[j];
    int64_t* r = trk_acc + (int64_t)g * TA_K;
    g_add(r + TA_CNT, 1);
    g_add(r + TA_CPU_LO, (int64_t)((uint64_t)c & 0xFFFFFFFFull));
    g_add(r + TA_CPU_HI, c >> 32);
    g_add(r + TA_MEM_LO, (int64_t)((uint64_t)m & 0xFFFFFFFFull));
    g_add(r + TA_MEM_HI, m >> 32);
}

}  // namespace

// =====================================================================  K1 (fast)
// Each workgroup takes an equal contiguous share of the K tiles' work weight (16-B loads)
// and of the C tiles.  K tiles: the share is walked class by class (the class table is sorted by tile), each
// class run by the pipeline instantiated for its record shape; waves interleave tiles
// (t = first + wave, + waves).  C tiles: a rolling pipeline of DC slots, as k_run.  The
// per-group partials stay in LDS and are flushed once.
// ABLATE (timing-only builds): bit 0 LDS sink, bit 1 skip K tiles, bit 2 skip C tiles,
// bit 5 loads only.
// DYN: the K tiles' weight is cut into gridDim.x * K1_CHUNKS chunks taken from a ticket
// counter (at most `cap` per workgroup), so workgroups that stream faster take more
// and the launch does not wait on the slowest static share; DYN 0: one static share each.
namespace {
// ---- K4 decision helpers (k_node_groups' decide)
// Exact total from split words; false when it is outside int64 (Quantity -> inf.Dec).
__device__ __forceinline__ bool join_split(int64_t lo_sum, int64_t hi_sum, int64_t& out) {
    const __int128 t = ((__int128)hi_sum << 32) + (__int128)lo_sum;
    out = (int64_t)t;
    return t >= (__int128)INT64_MIN && t <= (__int128)INT64_MAX;
}

__device__ __forceinline__ void finalize_p(const GroupParams& prm, const GroupNode& gn, int32_t g,
                                           const int64_t* __restrict__ pw, const int64_t* __restrict__ nw,
                                           esc_group_decision& dec, esc_group_metrics* __restrict__ met,
                                           esc_group_totals* __restrict__ htot) {
    Totals t;
    int64_t flags = nw[NW_FLAGS];
    if (!join_split(pw[PW_CPU_LO], pw[PW_CPU_HI], t.pod_cpu)) flags |= ESC_TF_POD_OVERFLOW;
    if (!join_split(pw[PW_MEM_LO], pw[PW_MEM_HI], t.pod_mem)) flags |= ESC_TF_POD_OVERFLOW;
    t.n_pods = pw[PW_N];
    t.node_cpu = nw[NW_CPU];
    t.node_mem = nw[NW_MEM];
    t.n_unt = nw[NW_N_UNT];
    t.n_taint = nw[NW_N_TAINT];
    t.n_cord = nw[NW_N_CORD];
    t.n_nodes = t.n_unt + t.n_taint + t.n_cord;
    t.first = gn.first;
    t.first_cpu = gn.first_cpu;
    t.first_mem = gn.first_mem;
    t.flags = flags;
    decide_one(prm, t, dec);
    if (met) {
        esc_group_metrics m;
        metrics_one(t, dec, m);
        met[g] = m;
    }
    if (htot) {                                          // esc_results' record, zero-copy
        static_assert(sizeof(esc_group_totals) == 13 * 8, "totals record is 13 words");
        const bool has = t.first != INT64_MAX;
        const int64_t w[13] = {t.pod_cpu, t.pod_mem, t.n_pods, t.node_cpu, t.node_mem, t.n_nodes, t.n_unt,
                               t.n_taint, t.n_cord, has ? t.first : -1, has ? t.first_cpu : 0,
                               has ? t.first_mem : 0, t.flags};
        int64_t* o = reinterpret_cast<int64_t*>(htot + g);
#pragma unroll
        for (int k = 0; k < 13; ++k) o[k] = w[k];
    }
}

__device__ __forceinline__ void finalize(const GroupDev& G, const GroupNode& gn, int32_t g,
                                         const int64_t* __restrict__ pw, const int64_t* __restrict__ nw,
                                         esc_group_decision& dec, esc_group_metrics* __restrict__ met) {
    finalize_p(G.params[g], gn, g, pw, nw, dec, met, G.htot);
}

__device__ __forceinline__ DecCompact compact_of(const esc_group_decision& d) {
    DecCompact c;
    c.cpu_pct = d.cpu_pct;
    c.mem_pct = d.mem_pct;
    const bool fits = d.delta == (int64_t)(int32_t)d.delta && d.n_to_taint == (int64_t)(int32_t)d.n_to_taint;
    c.delta = (int32_t)d.delta;
    c.n_to_taint = (int32_t)d.n_to_taint;
    c.status = (uint8_t)d.status;
    c.branch = (uint8_t)d.branch;
    c.taint_status = (uint8_t)d.taint_status;
    c.wide = fits ? 0 : 1;
    c.sel = SEL_NONE;
    return c;
}

__device__ __forceinline__ void store_full(esc_group_decision* dst, const esc_group_decision& d) {
    static_assert(sizeof(esc_group_decision) == 64, "decision record is 4 x 16 B");
    const uint4* s = reinterpret_cast<const uint4*>(&d);
    uint4* o = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = s[k];
}

// One group's decision from its pod / node words: the full record to device memory, the
// compact one to the decision buffer.
__device__ __forceinline__ void decide_store(const GroupDev& G, const GroupNode& gn, int32_t g, const int64_t* pw,
                                             const int64_t* nw, esc_group_decision* dec, DecCompact* cdec) {
    esc_group_decision d;
    finalize(G, gn, g, pw, nw, d, G.metrics);
    store_full(dec + g, d);
    const DecCompact cd = compact_of(d);
    const uint4* src = reinterpret_cast<const uint4*>(&cd);
    uint4* dst = reinterpret_cast<uint4*>(cdec + g);
    dst[0] = src[0];
    dst[1] = src[1];
}
}  // namespace

// Every K1 pipeline: (packed, records, extra pairs) of the K classes (PodClass::kind).
#define ESC_KRUN_SHAPES(PK)                                                     \
    ESC_KRUN(PK, 0, 0) ESC_KRUN(PK, 0, 1) ESC_KRUN(PK, 0, 2) ESC_KRUN(PK, 0, 3) \
    ESC_KRUN(PK, 1, 0) ESC_KRUN(PK, 1, 1) ESC_KRUN(PK, 1, 2) ESC_KRUN(PK, 1, 3) \
    ESC_KRUN(PK, 2, 0) ESC_KRUN(PK, 2, 1) ESC_KRUN(PK, 2, 2) ESC_KRUN(PK, 2, 3) \
    ESC_KRUN(PK, 3, 0) ESC_KRUN(PK, 3, 1) ESC_KRUN(PK, 3, 2) ESC_KRUN(PK, 3, 3)
// plain blocks: one generic pipeline (k_load above) for the 16 plain kinds
#define ESC_KRUN_PLAIN                                                                          \
    case 0: case 1: case 2: case 3: case 4: case 5: case 6: case 7:                            \
    case 8: case 9: case 10: case 11: case 12: case 13: case 14: ESC_KRUN(0, 3, 3)   /* = case 15 */
// packed (12-B) blocks: one generic pipeline for their 16 kinds too
#define ESC_KRUN_PK1                                                                            \
    case 16: case 17: case 18: case 19: case 20: case 21: case 22: case 23:                    \
    case 24: case 25: case 26: case 27: case 28: case 29: case 30: ESC_KRUN(1, 3, 3)   /* = case 31 */
#define ESC_KRUN_ALL ESC_KRUN_SHAPES(2) ESC_KRUN_PK1 ESC_KRUN_PLAIN
// LDS copies of the slot partials per K1 workgroup: K1_REPS when the window's slots are few
// (lane l adds to copy l % K1_REPS, so lanes of one wave that hit the same slot mostly hit
// different addresses — and, the copies 2 words apart mod the bank count, different banks;
// the copies are summed before the flush), else one.  With ~100 groups (configs 2 and 3) a
// wave's 64 ds_add_u64 met on the same few slots: K1 took 94 us for 99 MB at config 3,
// 25 us with the adds replaced by a sink (r06ab); one copy per wave changed nothing.
constexpr uint32_t K1_REPS = 8, K1_REP_LDS = 64 * 1024;
__host__ __device__ constexpr uint32_t k1_copy_words(uint32_t gw) { return (gw + FC_COL - 1) / FC_COL * FC_COL * 2 + 2; }
__host__ __device__ constexpr uint32_t k1_reps(uint32_t gw) {
    return (uint64_t)k1_copy_words(gw) * 8 * K1_REPS <= K1_REP_LDS ? K1_REPS : 1u;
}
template <int THREADS, int ABLATE = 0, int DC = 3, int DYN = 0, int WS = 0>
__global__ __launch_bounds__(THREADS) void k_pod_reduce(PodDev P, GroupDev G, int32_t g0, uint32_t gw,
                                                        uint64_t* __restrict__ part,
                                                        int64_t* __restrict__ wide,
                                                        uint32_t* __restrict__ ticket, int cap, K1Diag FF) {
    constexpr int NW = THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    __shared__ uint32_t s_chunk;
    uint64_t* const trace = FF.trace ? FF.trace + (int64_t)blockIdx.x * 8 : nullptr;
    if (trace && threadIdx.x == 0) {
        trace[0] = __builtin_amdgcn_s_memrealtime();
        trace[4] = (uint64_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
        trace[5] = (uint64_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
    }
    // cpu|count words [0, gwp), mem words [gwp, 2 gwp): whole FC_COL columns per half, so the
    // compact flush reads a column's 16 B per lane unconditionally (ds_read_b128, no conflicts)
    const uint32_t gwp = (gw + FC_COL - 1) / FC_COL * FC_COL;
    const uint32_t reps = k1_reps(gw), cw = k1_copy_words(gw);   // copies when the slots are few
    for (uint32_t i = threadIdx.x; i < (reps > 1 ? reps * cw : 2 * gwp); i += THREADS) lds[i] = 0;
    const uint32_t plim = (int64_t)G.n_gp <= (int64_t)g0 ? 0u : (uint32_t)imin64((int64_t)gw, (int64_t)G.n_gp - g0);
    const uint32_t dslot = (G.default_group != NONE && G.n_gp - (uint32_t)g0 < gw) ? G.n_gp - (uint32_t)g0 : NONE;
    uint64_t* const mine = lds + (reps > 1 ? (threadIdx.x & (reps - 1)) * cw : 0u);
    const PodSink<ABLATE> K{PodLds{mine, mine + gwp, g0, gw, plim, dslot}, PodWide{wide}};
    // compact flush: this workgroup's entry range and the descriptors of its first 32 rounds,
    // fetched now so the flush does not wait on them (see the flush)
    // (entries of workgroup b: wg_cols[b * n_col + i], i < wg_off[b]; fixed-stride, so the two
    // loads do not depend on each other and nothing waits on them before the flush)
    const int64_t n_col = G.sp / FC_COL;
    const uint2* fcols = P.wg_cols + (int64_t)blockIdx.x * n_col;
    uint32_t fe1 = 0;
    uint2 fdv = make_uint2(0xFFFFFFFFu, 0u);
    if (P.wg_off) {
        fe1 = P.wg_off[blockIdx.x];
        const uint32_t li = 2 * (threadIdx.x >> 6) + (threadIdx.x & 1) + ((threadIdx.x & 63) >> 1) * (THREADS / 32);
        if (li < n_col) fdv = fcols[li];
    }
    const uint32_t lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // WS: every wave takes its own contiguous share of the K weight (a wave's restarts at
    // class boundaries then idle only that wave, the WG's other waves keep streaming)
    const int64_t n_chunks = DYN ? (int64_t)gridDim.x * K1_CHUNKS : (WS ? (int64_t)gridDim.x * NW : gridDim.x);
    // every thread has read the previous ticket before thread 0 overwrites it
    auto grab = [&]() -> int64_t {
        __syncthreads();
        if (threadIdx.x == 0) s_chunk = atomicAdd(ticket, 1u);
        __syncthreads();
        return (int64_t)__builtin_amdgcn_readfirstlane(s_chunk);
    };
    int64_t chunk = WS ? (int64_t)blockIdx.x * NW + wid : blockIdx.x;
    if constexpr (DYN) chunk = grab();
    else __syncthreads();
    // the host's work plan: this workgroup's class runs, every wave interleaved over each
    typedef __attribute__((address_space(4))) const int64_t ci64;
    if (P.seg && !DYN && !WS && !(ABLATE & 2)) {
        const ci64* sg = (const ci64*)P.seg + (int64_t)blockIdx.x * (2 * K1_SEGS);
        uint64_t n_runs = 0, run_w = 0;                  // diagnostics (trace[6], trace[7])
#pragma unroll 1
        for (int k = 0; k < K1_SEGS; ++k) {
            const int64_t t0c = sg[2 * k], b = sg[2 * k + 1];
            if (b == 0) break;
            const PodClass C = load_class(P.cls, (int)(t0c >> 48));
            ++n_runs;
            run_w += (uint64_t)(b - (t0c & ((1ll << 48) - 1))) * C.wt;
            const int64_t a = (t0c & ((1ll << 48) - 1)) + wid;
            if (a >= b) continue;
            switch (C.kind) {
#define ESC_KRUN(PK, RR, XX) \
    case PK * 16 + RR * 4 + XX: k_run<RR, XX, PK, NW, ABLATE, NW>(P, G, K, C, a, b, lane); break;
                ESC_KRUN_ALL
#undef ESC_KRUN
                default: break;
            }
        }
        chunk = n_chunks;                                // skip the weight-range walk
        if (trace && threadIdx.x == 0) { trace[6] = n_runs; trace[7] = run_w; }
    }
    for (int taken = 1; !(ABLATE & 2) && chunk < n_chunks; ++taken) {
        // equal shares of work weight (bytes), not of tiles: a tile of a class with three
        // container records streams ~3.4x the bytes of a simple one
        const int64_t wl = P.k_weight * chunk / n_chunks, wh = P.k_weight * (chunk + 1) / n_chunks;
        for (int ci = 0; ci < P.n_cls; ++ci) {
            const PodClass C = load_class(P.cls, ci);
            if (C.w0 >= wh) break;
            // tiles of the class whose start weight lies in [wl, wh)
            const int64_t n = C.t1 - C.t0;
            const int64_t i0 = imin64(n, imax64(0, (wl - C.w0 + C.wt - 1) / C.wt));
            const int64_t i1 = imin64(n, imax64(0, (wh - C.w0 + C.wt - 1) / C.wt));
            const int64_t a = C.t0 + i0 + (WS ? 0 : wid), b = C.t0 + i1;
            if (a >= b) continue;
            switch (C.kind) {
#define ESC_KRUN(PK, RR, XX) \
    case PK * 16 + RR * 4 + XX: k_run<RR, XX, PK, NW, ABLATE, (WS ? 1 : NW)>(P, G, K, C, a, b, lane); break;
                ESC_KRUN_ALL
#undef ESC_KRUN
                default: break;
            }
        }
        if (!DYN || taken >= cap) break;
        chunk = grab();
    }
    if (trace) {
        __syncthreads();
        if (threadIdx.x == 0) trace[1] = __builtin_amdgcn_s_memrealtime();
    }
    if (!(ABLATE & 4)) {
        const int64_t per = (P.c_tiles + gridDim.x - 1) / gridDim.x;
        const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(lo + per, P.c_tiles);
        const int64_t t0 = lo + wid;
        if (t0 < hi) {
            // Record offsets of the tile a slot loads next are scalar loads, fetched one
            // round ahead (nb[d]).
            CTile T[DC];
            TileBases nb[DC];
            const TileBases b0 = tile_bases(P, t0);
#pragma unroll
            for (int d = 0; d < DC; ++d) {
                const int64_t u = t0 + (int64_t)d * NW;
                c_load(P, u < hi ? u : t0, lane, u < hi ? tile_bases(P, u) : b0, T[d]);
            }
#pragma unroll
            for (int d = 0; d < DC; ++d) {
                const int64_t nu = t0 + (int64_t)(d + DC) * NW;
                nb[d] = nu < hi ? tile_bases(P, nu) : T[d].b;
            }
            for (int64_t t = t0; t < hi; t += (int64_t)DC * NW) {
#pragma unroll
                for (int d = 0; d < DC; ++d) {
                    const int64_t u = t + (int64_t)d * NW;
                    if constexpr (ABLATE & 32) {
                        if (u < hi) asm volatile("" :: "v"(T[d].f ^ T[d].c ^ T[d].p ^ T[d].xp0 ^ T[d].xp1),
                                                 "v"(T[d].m ^ T[d].xcc0 ^ T[d].xcm0 ^ T[d].xcc1 ^ T[d].xcm1));
                    } else if (u < hi && T[d].b.xcn <= 128 && T[d].b.xpn <= 128) c_process<ABLATE>(G, K, T[d]);
                    const int64_t nu = u + (int64_t)DC * NW;
                    const int64_t ru = nu < hi ? nu : (u < hi ? u : t0);
                    c_load(P, ru, lane, nb[d], T[d]);
                    const int64_t nnu = nu + (int64_t)DC * NW;
                    nb[d] = nnu < hi ? tile_bases(P, nnu) : T[d].b;
                }
            }
        }
    }
    __syncthreads();
    if (reps > 1) {                                          // the waves' copies into copy 0
        for (uint32_t i = threadIdx.x; i < 2 * gwp; i += THREADS) {
            uint64_t s = lds[i];
            for (uint32_t r = 1; r < reps; ++r) s += lds[r * cw + i];
            lds[i] = s;
        }
        __syncthreads();
    }
    if (trace && threadIdx.x == 0) trace[2] = __builtin_amdgcn_s_memrealtime();
    const int64_t S = G.sp;                                  // row stride (K3 reads whole columns)
    uint64_t* out = part + (int64_t)blockIdx.x * 2 * S + g0;
    // 16-B nontemporal stores (rows and g0 are 16-B aligned: S is a multiple of FC_COL)
    typedef uint64_t v2u64s __attribute__((ext_vector_type(2)));
    if (P.wg_off) {
        // compact: the columns this share touches, 32 threads per column (16 write the
        // cpu|count words, 16 the mem words), each to its own 64-word entry
        // Wave w takes entries e0 + 2w + {0, 1} + (THREADS / 32) k; lane 2k + h holds the
        // descriptor of round k, half h (fetched at the start for rounds 0..31, by one load
        // per 32 rounds after that) and hands it out by readlane.
        const uint32_t e0 = 0, e1 = fe1;
        const uint32_t h = threadIdx.x & 31, j = 2 * (h & 15), half = h >> 4, eh = (threadIdx.x >> 5) & 1;
        constexpr uint32_t EPR = THREADS / 32;                         // entries per round
        const uint32_t wb = e0 + 2 * (uint32_t)wid;
        for (uint32_t r0 = 0; wb + r0 * EPR < e1; r0 += 32) {
            uint2 dv = fdv;
            if (r0) {
                const uint32_t li = wb + (lane & 1) + (r0 + (lane >> 1)) * EPR;
                dv = li < e1 ? fcols[li] : make_uint2(0xFFFFFFFFu, 0u);
            }
#pragma unroll 4
            for (uint32_t k = 0; k < 32; ++k) {
                if (wb + (r0 + k) * EPR >= e1) break;                  // wave-uniform
                const uint32_t x0 = __builtin_amdgcn_readlane(dv.x, 2 * k), x1 = __builtin_amdgcn_readlane(dv.x, 2 * k + 1);
                const uint32_t y0 = __builtin_amdgcn_readlane(dv.y, 2 * k), y1 = __builtin_amdgcn_readlane(dv.y, 2 * k + 1);
                const uint32_t col = eh ? x1 : x0, dst = eh ? y1 : y0;
                if (wb + (r0 + k) * EPR + eh >= e1) continue;          // past the list (second entry)
                const int64_t c0 = (int64_t)col * FC_COL - g0;         // column start in this window
                if (c0 < 0 || c0 >= (int64_t)gw) continue;             // the column is in another window
                const v2u64s v = *reinterpret_cast<const v2u64s*>(lds + half * gwp + c0 + j);
                __builtin_nontemporal_store(v, reinterpret_cast<v2u64s*>(part + (int64_t)dst * 2 * FC_COL +
                                                                         half * FC_COL + j));
            }
        }
    } else
    for (uint32_t i = 2 * threadIdx.x; i < gw; i += 2 * THREADS) {
        if (i + 1 < gw) {
            const v2u64s a = {lds[i], lds[i + 1]}, m = {lds[gwp + i], lds[gwp + i + 1]};
            __builtin_nontemporal_store(a, reinterpret_cast<v2u64s*>(out + i));
            __builtin_nontemporal_store(m, reinterpret_cast<v2u64s*>(out + S + i));
        } else {
            out[i] = lds[i];
            out[S + i] = lds[gwp + i];
        }
    }
    if (trace) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) trace[3] = __builtin_amdgcn_s_memrealtime();
    }
    if (DYN && threadIdx.x == 0) {
        // every workgroup's last grab precedes its increment here: the last one resets
        if (atomicAdd(ticket + 1, 1u) == gridDim.x - 1) {
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ticket + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ============================================================ K1 launchers by part
// The K1 template is instantiated once per (variant, 16 record shapes): the production
// variant in part 0 (with every other kernel) and the timing-only ablations in part 2, its
// own translation unit, linked only into the measurement library (Makefile ABLATIONS=1,
// libescalator_hip_measure.so).  The exact alternatives measured slower (1: two C tiles in
// flight, 2: 1024 threads, 5: dynamic shares, 6: per-wave shares) were
// removed from the product.
#define ESC_K1(T, A, DC) ESC_K1D(T, A, DC, 0)
#define ESC_K1D(T, A, DC, D) ESC_K1W(T, A, DC, D, 0)
#define ESC_K1W(T, A, DC, D, W)                                                                       \
    hipLaunchKernelGGL((k_pod_reduce<T, A, DC, D, W>), dim3(nblk), dim3(T), lds, st, p, g, g0, (uint32_t)gw, part, \
                       wide, ticket, cap, diag)
#define ESC_K1_ARGS const PodDev &p, const GroupDev &g, int32_t g0, int32_t gw, int nblk, int variant, uint64_t *part, \
                    int64_t *wide, uint32_t *ticket, int cap, const K1Diag &diag, hipStream_t st
hipError_t launch_pod_reduce_ablation(ESC_K1_ARGS) __attribute__((weak));

#if ESC_PART == 0
hipError_t launch_pod_reduce(ESC_K1_ARGS) {
    const size_t lds = k1_reps((uint32_t)gw) > 1 ? (size_t)k1_reps((uint32_t)gw) * k1_copy_words((uint32_t)gw) * 8
                                                 : (size_t)(gw + FC_COL - 1) / FC_COL * FC_COL * 2 * sizeof(uint64_t);
    switch (variant) {
        case 0: ESC_K1(512, 0, 3); break;
        default:                                  // timing-only ablations (measurement library only)
            if (!launch_pod_reduce_ablation) return hipErrorInvalidValue;
            return launch_pod_reduce_ablation(p, g, g0, gw, nblk, variant, part, wide, ticket, cap, diag,
                                              st);
    }
    return hipGetLastError();
}
#elif ESC_PART == 2
hipError_t launch_pod_reduce_ablation(ESC_K1_ARGS) {
    const size_t lds = k1_reps((uint32_t)gw) > 1 ? (size_t)k1_reps((uint32_t)gw) * k1_copy_words((uint32_t)gw) * 8
                                                 : (size_t)(gw + FC_COL - 1) / FC_COL * FC_COL * 2 * sizeof(uint64_t);
    switch (variant) {
        case 14: ESC_K1W(512, 4 | 32, 3, 0, 1); break;   // per-wave shares, K tiles, loads only
        case 3: ESC_K1(512, 64, 3); break;       // <= 2 K tiles in flight per wave
        case 4: ESC_K1(512, 128, 3); break;      // <= 3 K tiles in flight per wave
        // Timing-only ablations (wrong results; scripts/k1_variants.py), see k_pod_reduce.
        case 9: ESC_K1(512, 1, 3); break;        // LDS atomics replaced by a sink
        case 10: ESC_K1(512, 2, 3); break;       // C tiles only
        case 11: ESC_K1(512, 4, 3); break;       // K tiles only
        case 12: ESC_K1(512, 4 | 32, 3); break;  // K tiles, loads only
        case 13: ESC_K1(512, 2 | 32, 3); break;  // C tiles, loads only
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
#endif
#undef ESC_K1
#undef ESC_K1D
#undef ESC_K1W
#undef ESC_K1_ARGS

#if ESC_PART == 0
// C tiles with more than 128 extra records of a kind (listed by the host at load):
// one wave per tile, records read from memory, exact wide accumulation.
__global__ __launch_bounds__(64) void k_pod_bigtiles(PodDev P, GroupDev G, const uint32_t* __restrict__ tiles,
                                                     int64_t* __restrict__ wide) {
    c_tile_exact(P, G, tiles[blockIdx.x], threadIdx.x, wide);
}

// Touched pod-slot columns of every K1 workgroup's share (compact flush, launch_touch): the
// K1 plan's class runs and K1's C-tile share, walked pod by pod (once per plan, not per
// decision).  Daemonset pods of K tiles add nothing and are skipped (an upsert that later
// fills such a slot marks its columns on the host); C tiles are taken whole (a superset).
__global__ __launch_bounds__(256) void k_touch(PodDev P, GroupDev G, int tw, uint32_t* __restrict__ bits) {
    extern __shared__ uint32_t tb[];
    for (int i = threadIdx.x; i < tw; i += 256) tb[i] = 0;
    __syncthreads();
    auto mark = [&](uint32_t slot) {
        const uint32_t col = slot / FC_COL;
        atomicOr(&tb[col >> 5], 1u << (col & 31));
    };
    const int64_t* sg = P.seg + (int64_t)blockIdx.x * (2 * K1_SEGS);
    for (int k = 0; k < K1_SEGS; ++k) {
        const int64_t t0c = sg[2 * k], b = sg[2 * k + 1];
        if (b == 0) break;
        const PodClass C = P.cls[(int)(t0c >> 48)];
        const int64_t a = t0c & ((1ll << 48) - 1);
        for (int64_t i = threadIdx.x; i < (b - a) * TILE; i += 256) {
            const int64_t blk = kb_block(C, a + i / TILE), s = i % TILE;
            const KHead hd = kb_head(C, P.kb, blk, s);
            if (hd.flags & ESC_PF_DAEMONSET) continue;
            if (hd.pair0 < G.n_gp) mark(hd.pair0);
            for (uint32_t x = 0; x < C.nxp; ++x) {
                const uint32_t q = kb_pair(C, P.kb, blk, x, s);
                if (q < G.n_gp) mark(q);
            }
        }
    }
    const int64_t per = (P.c_tiles + gridDim.x - 1) / gridDim.x;       // K1's C-tile share
    const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(lo + per, P.c_tiles);
    if (lo < hi) {
        for (int64_t i = lo * CTILE + threadIdx.x; i < hi * CTILE; i += 256)
            if (P.pair0[i] < G.n_gp) mark(P.pair0[i]);
        for (int64_t i = P.xp_base[lo] + threadIdx.x; i < (int64_t)P.xp_base[hi]; i += 256)
            if (P.xp[i] < G.n_gp) mark(P.xp[i]);
    }
    if (threadIdx.x == 0 && G.default_group != NONE) mark(G.n_gp);
    __syncthreads();
    for (int i = threadIdx.x; i < tw; i += 256) bits[(int64_t)blockIdx.x * tw + i] = tb[i];
}

hipError_t launch_touch(const PodDev& p, const GroupDev& g, int nblk, int tw, uint32_t* bits, hipStream_t st) {
    if (nblk <= 0 || !p.seg) return hipSuccess;
    hipLaunchKernelGGL(k_touch, dim3(nblk), dim3(256), (size_t)tw * 4, st, p, g, tw, bits);
    return hipGetLastError();
}

// =====================================================================  K1 (wide)
namespace {
// Exact (any-range) evaluation of one K tile from memory, 4 pods per lane.
__device__ __forceinline__ void k_tile_exact(const PodDev& P, const GroupDev& G, const PodClass& C, int64_t t,
                                             uint32_t lane, int64_t* __restrict__ wide) {
    const PodWide acc{wide};
    const uint32_t R = kb_nrec(C);
    const int64_t blk = kb_block(C, t);
    for (int j = 0; j < PODS_PER_LANE; ++j) {
        const uint32_t s = lane * PODS_PER_LANE + j;
        const KHead h = kb_head(C, P.kb, blk, s);
        if (h.flags & ESC_PF_DAEMONSET) continue;
        uint64_t cpu = (uint64_t)h.cpu0, mem = (uint64_t)h.mem0;
        for (uint32_t k = 0; k < R; ++k) {
            int64_t rc, rm;
            kb_rec(C, P.kb, blk, k, s, rc, rm);
            apply_rec(k, R, C.xreg, C.xreg + C.xinit, (unsigned long long)rc, (unsigned long long)rm, cpu, mem);
        }
        if (pf_default_ok(h.flags) && G.default_group != NONE) acc.add(G.n_gp, (int64_t)cpu, (int64_t)mem);
        if (h.pair0 < G.n_gp) acc.add(h.pair0, (int64_t)cpu, (int64_t)mem);
        for (uint32_t k = 0; k < C.nxp; ++k) {
            const uint32_t q = kb_pair(C, P.kb, blk, k, s);
            if (q < G.n_gp) acc.add(q, (int64_t)cpu, (int64_t)mem);
        }
    }
}
}  // namespace

// The whole shard through the exact accumulators (esc_force_wide; fallback testing).
__global__ __launch_bounds__(256) void k_pod_wide(PodDev P, GroupDev G, int64_t* __restrict__ wide) {
    const uint32_t lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t t = wave; t < P.k_tiles; t += nwaves) {
        int ci = 0;
        while (ci + 1 < P.n_cls && t >= P.cls[ci].t1) ++ci;
        k_tile_exact(P, G, P.cls[ci], t, lane, wide);
    }
    for (int64_t t = wave; t < P.c_tiles; t += nwaves) c_tile_exact(P, G, t, lane, wide);
}

// =====================================================================  K2 nodes
namespace {

// Is (node, group) in the group's dry-mode taintTracker (controller.go:128-133)?
// Only called for nodes flagged ESC_NF_TRACKED; trk_start points at their first entry.
__device__ __forceinline__ bool tracked(const NodeDev& N, int32_t node, int32_t g) {
    for (int64_t k = N.trk_start[node]; k < N.n_trk && N.trk_node[k] == node; ++k)
        if (N.trk_group[k] == g) return true;
    return false;
}

// filterNodes classification (controller.go:125-150): 0 untainted, 1 tainted, 2 cordoned.
// Dry mode separates only tracker members; cordoned nodes are not split out there.
__device__ __forceinline__ int node_class(const NodeDev& N, uint32_t f, int64_t i, uint32_t m) {
    if (f & ESC_NF_ABSENT) return 3;                 // no node: in no class
    if (mdry(m)) return ((f & ESC_NF_TRACKED) && tracked(N, (int32_t)i, (int32_t)mg(m))) ? 1 : 0;
    if (f & ESC_NF_UNSCHED) return 2;
    return (f & ESC_NF_TAINTED) ? 1 : 0;
}

// Groups a node belongs to: NewNodeLabelFilterFunc (node_group.go:278) over its label
// pairs, resolved through the node pair table (K5).
// Only the groups of the pairs this rank owns (NodeDev q_lo / q_hi).
template <class F>
__device__ __forceinline__ void node_groups(const NodeDev& N, const GroupDev& G, uint32_t f, int64_t i,
                                            F&& emit) {
    if (f & ESC_NF_ABSENT) return;                   // a free / deleted slot is in no group
    auto pair = [&](uint32_t q) {
        if (q >= N.q_lo && q < N.q_hi) for_code(G, node_code(G, q), emit);
    };
    pair(N.label0[i]);
    const uint32_t nx = nf_xlbl(f);
    if (nx) {
        const uint32_t q = N.xl_off[i];
        for (uint32_t k = 0; k < nx; ++k) pair(N.xl[q + k]);
    }
}




}  // namespace

// K2: the pieces of this rank's group pairs (<= NODE_PIECE entries of one label pair each,
// 20 B per entry streamed coalesced) reduced to one NR_K-word row per piece, stored
// word-major (rows[k * n_pieces + p], so k_node_groups' lanes read consecutive pieces
// coalesced).  Pieces of pairs no group selects (ids >= n_gp) are in no span.
// Blocks past the pieces take the dry-mode tracker entries (controller.go:128-133): a
// (node, dry group) entry whose node is a member of the group and lies in this rank's
// share of the group's pieces adds the node to the group's tracked sums (trk_acc, global
// atomics: a few thousand entries), which K3 reads and resets.
namespace {

__device__ __forceinline__ void node_piece_block(const NodeDev& N, const GroupDev& G, int64_t nb_pieces,
                                                 int64_t* __restrict__ rows, int64_t* __restrict__ trk_acc, int64_t blk) {
    const int lane = threadIdx.x & 63;
    if (blk >= nb_pieces) {
        tracker_entry(N, G, trk_acc, (blk - nb_pieces) * (K2_WAVES * 64) + threadIdx.x);
        return;
    }
    // one wave per span of whole pieces (~NODE_SPAN entries): the span's entries stream
    // coalesced, U wave-loads in flight; a lane adds its entry to the piece whose range
    // holds it, and every piece that ends inside a wave-load is reduced (butterflies) and
    // stored there — small pieces share a wave instead of taking one each (a wave per
    // ~110-entry piece was latency-bound: 25 us for 26 MB at config 4)
    node_span(N, rows, blk * K2_WAVES + (threadIdx.x >> 6), lane);
}
}  // namespace

// ===================================================================== K3 / K4
namespace {

__device__ __forceinline__ void u128_add(uint64_t& lo, uint64_t& hi, uint64_t v) { lo += v; hi += (lo < v) ? 1 : 0; }

__device__ __forceinline__ void split_store(int64_t* w, int k, __int128 t) {
    w[k] = (int64_t)((unsigned __int128)t & 0xFFFFFFFFull);
    w[k + 1] = (int64_t)(t >> 32);
}


// (unsigned 128-bit sum of lo32 parts, int64 sum of hi parts) -> the exact total
__device__ __forceinline__ __int128 join_parts(uint64_t lo, uint64_t lo_carry, int64_t hi) {
    return (__int128)(((unsigned __int128)lo_carry << 64) | lo) + ((__int128)hi << 32);
}




// The compact decisions of n groups staged in LDS (sc), written as 16-B pieces: one
// contiguous run when the groups are consecutive ids (g0 ..), else per group (ids[k]).
// The destination is pinned host memory (zero-copy), where scattered narrow fields would
// each be a PCIe write.
__device__ __forceinline__ void store_compact(DecCompact* __restrict__ cdec, const DecCompact* sc, uint32_t n,
                                              bool seq, uint32_t g0, const uint32_t* ids, uint32_t tid,
                                              uint32_t nthreads) {
    const uint4* src = reinterpret_cast<const uint4*>(sc);
    for (uint32_t i = tid; i < n * 2; i += nthreads) {
        const uint32_t k = i >> 1;
        reinterpret_cast<uint4*>(cdec + (seq ? g0 + k : ids[k]))[i & 1] = src[i];
    }
}

__device__ __forceinline__ int64_t ld_agent(const int64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


}  // namespace

// K2b + K4 (k_node_groups, last kernel of the step): every group's node words from its
// pair's K2 piece rows — NewNodeLabelFilterFunc (node_group.go:278) + filterNodes
// (controller.go:120-154) + CalculateNodesCapacityTotal(untainted) (util.go:41-51): wet
// groups take the filterNodes classes, dry groups (controller.go:126-138) every member as
// untainted (cordoned ones included) except the tracked members (K2's tracker sums, read
// and reset here).  64 groups per block, the 4 waves split each group's pieces.  A rank
// reduces only the pieces of the pairs it owns and runs this over its own groups only.
// With a decision target (D.dec) the block then decides its groups (K4: at one rank on its
// fold, at several after the exchange) and writes the compact records to the decision
// buffer.
#ifndef ESC_NG_WAVES
#define ESC_NG_WAVES 4       // waves splitting a group's node pieces in k_node_groups (timing builds may override)
#endif
constexpr int NG_WAVES = ESC_NG_WAVES;


namespace {
// Entry q of a group's selection (SelOut): the untainted segment is stored oldest first
// (ties by ascending index, the age index's order), the tainted one newest first with equal
// creation times by DESCENDING index (it is written backward), so a tainted entry is taken
// from the mirror position inside its run of equal creation times — the runs are found by
// comparing neighbours (bounded by SEL_TIE_MAX each way; a longer run sets *cut and the host
// falls back to esc_group_order, which reads until the run ends).
__device__ __forceinline__ uint32_t sel_entry(const NodeDev& N, const uint32_t* __restrict__ sg, int64_t len,
                                              uint32_t q, bool newest, bool& cut) {
#ifdef ESC_SEL_NOTIE                                     // (timing builds: no tie resolution)
    newest = false;
#endif
    if (!newest) return sg[q];
    const int64_t t = N.created[sg[q]];
    int64_t a = q, b = (int64_t)q + 1;
    for (int k = 0; a > 0 && N.created[sg[a - 1]] == t; ++k) {
        if (k == SEL_TIE_MAX) { cut = true; break; }
        --a;
    }
    for (int k = 0; b < len && N.created[sg[b]] == t; ++k) {
        if (k == SEL_TIE_MAX) { cut = true; break; }
        ++b;
    }
    return sg[a + b - 1 - (int64_t)q];
}

// k_node_groups' work for up to 64 groups, group gid (NONE: no group) on lane l of every
// wave: the node words from the group pair's piece rows (the waves split the pieces), then
// the decision or the exchange words.  With `seq` the groups are g_first + l and their
// compact decisions go out as one contiguous run; else group by group.
__device__ __forceinline__ void node_groups_part(const GroupDev& G, const NodeDev& N,
                                                 const int64_t* __restrict__ node_rows,
                                                 int64_t* __restrict__ trk_acc, int64_t* __restrict__ nwords,
                                                 const NGDecide& D, uint32_t gid, bool seq, int32_t g_first,
                                                 uint32_t n_out) {
    __shared__ uint64_t red[NG_WAVES][6][64];
    __shared__ DecCompact sdec[64];
    __shared__ uint32_t sid[64];
    // selections: per lane's group its run's first word in the block's run (exclusive scan,
    // [64] = the block's words), which (0 none, 1 taint, 2 untaint), count, segment, cut
    __shared__ uint32_t s_ex[65], s_w[64], s_c[64], s_cut[64];
    __shared__ int64_t s_s[64], s_len[64];

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int32_t g = (int32_t)gid;
    const bool ok = gid != NONE && g < G.G;
    constexpr int NA = 15;   // 0-2 counts; node sums (lo, carry, hi): 3-5 unt cpu, 6-8 unt mem, 9-11 all cpu, 12-14 all mem
    uint64_t a[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) a[k] = 0;
    int64_t plo = 0, phi = 0;
    GroupNode gn{};
    GroupParams prm{};
    int64_t pwv[PW_K] = {};
    uint32_t sel_w = 0, sel_c = 0, sel_cut = 0, sel_tie = 0;   // this lane's group's selection (wave 0)
    int64_t sel_s = 0, sel_len = 0, segv[4] = {};
    if (ok) {
        gn = N.gnode[g];
        plo = gn.plo;
        phi = gn.phi;
        if (D.dec && wid == 0) {                     // K4's inputs (wave 0 decides), loaded beside the piece rows
            prm = G.params[g];
            const int64_t* pw = D.pwords + (int64_t)(G.xs ? G.xs[g] : (uint32_t)g) * PW_K;
#pragma unroll
            for (int k = 0; k < PW_K; ++k) pwv[k] = pw[k];
            if (D.sel.out) {                         // both orders' segment bounds, with them
                const int64_t* sg = D.sel.seg + 4 * (int64_t)g;
#pragma unroll
                for (int k = 0; k < 4; ++k) segv[k] = sg[k];
                sel_tie = D.sel.tie[g] ? 4u : 0u;
            }
        }
    }
    const int64_t np = N.n_pieces;
#pragma unroll 2
    for (int64_t pc = plo + wid; pc < phi; pc += NG_WAVES) {
        const int64_t* r = node_rows + pc;
        u128_add(a[3], a[4], (uint64_t)r[NR_UCPU_LO * np]); a[5] += (uint64_t)r[NR_UCPU_HI * np];
        u128_add(a[6], a[7], (uint64_t)r[NR_UMEM_LO * np]); a[8] += (uint64_t)r[NR_UMEM_HI * np];
        u128_add(a[9], a[10], (uint64_t)r[NR_ACPU_LO * np]); a[11] += (uint64_t)r[NR_ACPU_HI * np];
        u128_add(a[12], a[13], (uint64_t)r[NR_AMEM_LO * np]); a[14] += (uint64_t)r[NR_AMEM_HI * np];
        const uint64_t cn = (uint64_t)r[NR_COUNTS * np];
        a[0] += cn & NR_CNT_MASK;
        a[1] += (cn >> NR_CNT_BITS) & NR_CNT_MASK;
        a[2] += cn >> (2 * NR_CNT_BITS);
    }
    // merge the waves: counts, then the (lo, carry, hi) triples in two rounds
#pragma unroll
    for (int r0 = 0; r0 < NA; r0 += (r0 == 0 ? 3 : 6)) {
        const int nk = r0 == 0 ? 3 : 6;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (k < nk) red[wid][k][lane] = a[r0 + k];
        __syncthreads();
        if (wid == 0) {
            for (int w = 1; w < NG_WAVES; ++w) {
                if (r0 == 0) {
                    a[0] += red[w][0][lane]; a[1] += red[w][1][lane]; a[2] += red[w][2][lane];
                } else {
#pragma unroll
                    for (int k = 0; k < 6; k += 3) {
                        u128_add(a[r0 + k], a[r0 + k + 1], red[w][k][lane]);
                        a[r0 + k + 1] += red[w][k + 1][lane];
                        a[r0 + k + 2] += red[w][k + 2][lane];
                    }
                }
            }
        }
    }
    if (wid == 0 && ok) {
    __int128 ncpu, nmem;
    uint64_t n_unt = a[0], n_taint = a[1], n_cord = a[2];
    if (!G.dry[g]) {
        ncpu = join_parts(a[3], a[4], (int64_t)a[5]);
        nmem = join_parts(a[6], a[7], (int64_t)a[8]);
    } else {
        int64_t* t = trk_acc + (int64_t)g * TA_K;
        int64_t tr[TA_K];
#pragma unroll
        for (int k = 0; k < TA_K; ++k)
            tr[k] = __hip_atomic_exchange(t + k, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ncpu = join_parts(a[9], a[10], (int64_t)a[11]) - (((__int128)tr[TA_CPU_HI] << 32) + (__int128)tr[TA_CPU_LO]);
        nmem = join_parts(a[12], a[13], (int64_t)a[14]) - (((__int128)tr[TA_MEM_HI] << 32) + (__int128)tr[TA_MEM_LO]);
        const uint64_t n_all = n_unt + n_taint + n_cord;
        n_unt = n_all - (uint64_t)tr[TA_CNT];
        n_taint = (uint64_t)tr[TA_CNT];
        n_cord = 0;
    }
    const bool n_ok = ncpu >= (__int128)INT64_MIN && ncpu <= (__int128)INT64_MAX &&
                      nmem >= (__int128)INT64_MIN && nmem <= (__int128)INT64_MAX;
    const int64_t v[6] = {(int64_t)ncpu, (int64_t)nmem, (int64_t)n_unt, (int64_t)n_taint, (int64_t)n_cord,
                          n_ok ? 0 : ESC_TF_NODE_OVERFLOW};
    static_assert(NW_CPU == 0 && NW_MEM == 1 && NW_N_UNT == 2 && NW_N_TAINT == 3 && NW_N_CORD == 4 && NW_FLAGS == 5,
                  "node word order");
    {
        int64_t* nw = nwords + (int64_t)g * NW_K;
#pragma unroll
        for (int k = 0; k < 6; ++k) nw[k] = v[k];
    }
    if (D.dec) {
        esc_group_decision d;
        finalize_p(prm, gn, g, pwv, v, d, G.metrics, G.htot);
        store_full(D.dec + g, d);
        sdec[lane] = compact_of(d);
        sid[lane] = (uint32_t)g;
        if (D.sel.out) {                                 // which selection the decision asks for
            int64_t need = 0;
            if (d.delta > 0) { sel_w = 2 | sel_tie; need = d.delta; }             // ScaleUp: untaintNewestN
            else if (d.delta < 0 && d.taint_status == ESC_ST_OK) { sel_w = 1; need = d.n_to_taint; }   // taintOldestN
            if (sel_w) {
                sel_s = sel_w == 1 ? segv[0] : segv[2];
                sel_len = sel_w == 1 ? segv[1] - segv[0] : segv[3] - segv[2];   // (bit 2: ties, untaint only)
                const int64_t want = (need > 0 ? need : 0) + D.sel.slack;
                const int64_t c = want < sel_len ? want : sel_len;
                sel_c = (uint32_t)(c < D.sel.group_cap ? c : D.sel.group_cap);
                sel_cut = c > D.sel.group_cap ? SEL_CUT : 0u;
            }
        }
    }
    }
    if (D.dec && D.sel.out) {
        // the block's run starts at its own slot, blockIdx.x * 64 * (group_cap + 1) words (room
        // for 64 groups at their largest: no reservation across blocks); lane l's group takes
        // [base + ex, base + ex + 1 + count): its header, then its nodes
        const uint32_t base = blockIdx.x * 64u * (uint32_t)(D.sel.group_cap + 1);
        if (wid == 0) {
            const uint32_t words = sel_w ? sel_c + 1 : 0u;
            const uint32_t inc = wave_incl_scan32(words);
            const uint32_t tot = __builtin_amdgcn_readlane(inc, 63);
            const bool fits = (int64_t)base + tot <= D.sel.cap_words;
            s_ex[lane] = inc - words;
            if (lane == 63) s_ex[64] = fits ? tot : 0u;
            s_w[lane] = fits ? sel_w : 0u;
            s_c[lane] = sel_c;
            s_s[lane] = sel_s;
            s_len[lane] = sel_len;
            s_cut[lane] = sel_cut;
            if (ok) sdec[lane].sel = !sel_w ? SEL_NONE : (fits ? base + inc - words : SEL_OVERFLOW);
        }
        __syncthreads();
        const uint32_t total = s_ex[64];
        // SEL_U words per thread per round, their segment loads issued together (one memory
        // latency for the block's whole run in the common case); a group flagged with equal
        // creation times takes sel_entry's tie rule after
        constexpr int SEL_U = 4;
        constexpr uint32_t NT = NG_WAVES * 64;
        for (uint32_t f0 = threadIdx.x; f0 < total; f0 += SEL_U * NT) {
            uint32_t v[SEL_U], lu[SEL_U];
#pragma unroll
            for (int u = 0; u < SEL_U; ++u) {
                const uint32_t f = f0 + u * NT;
                lu[u] = 64;                              // none
                if (f >= total) continue;
                uint32_t l = 0;                          // the run holding word f: last l with s_ex[l] <= f
#pragma unroll
                for (uint32_t st = 32; st; st >>= 1)
                    if (s_ex[l + st] <= f) l += st;
                const uint32_t q = f - s_ex[l];
                if (q == 0) continue;                    // the header, once the cuts are known
                lu[u] = l;
                v[u] = D.sel.ord[s_s[l] + q - 1];
            }
#pragma unroll
            for (int u = 0; u < SEL_U; ++u) {
                if (lu[u] == 64) continue;
                const uint32_t l = lu[u], f = f0 + u * NT;
                if (s_w[l] & 4u) {                       // ties in the group: the mirror rule
                    bool cut = false;
                    v[u] = sel_entry(N, D.sel.ord + s_s[l], s_len[l], f - s_ex[l] - 1, true, cut);
                    if (cut) s_cut[l] |= SEL_TIE;
                }
                D.sel.out[base + f] = v[u];
            }
        }
        __syncthreads();
        if (wid == 0 && s_w[lane])
            D.sel.out[base + s_ex[lane]] = s_c[lane] | (s_w[lane] & 3u) << 28 | s_cut[lane];
    }
    if (D.dec) {                                         // 16-B pieces to pinned host memory (PCIe writes)
        __syncthreads();
        store_compact(D.cdec, sdec, n_out, seq, (uint32_t)g_first, sid, threadIdx.x, NG_WAVES * 64);
    }
}
}  // namespace

// K2b + K4 (k_node_groups, last kernel of the step): every group's node words from its
// pair's K2 piece rows — NewNodeLabelFilterFunc (node_group.go:278) + filterNodes
// (controller.go:120-154) + CalculateNodesCapacityTotal(untainted) (util.go:41-51): wet
// groups take the filterNodes classes, dry groups (controller.go:126-138) every member as
// untainted (cordoned ones included) except the tracked members (K2's tracker sums, read
// and reset here).  64 groups per block, the 4 waves split each group's pieces.  A rank
// reduces only the pieces of the pairs it owns, so a group's words are exact on its owner
// and zero elsewhere.  With a decision target (D.dec: one rank, no exchange) the block then
// decides its groups (K4) and writes the compact records to the decision buffer as one
// contiguous run; otherwise it writes only the node words.  With several ranks it runs
// after the exchange (esc_decide), over the rank's OWN groups (the list),
// their pod words at rows xs[g] of the reduce-scattered buffer.
// (Running this work inside k_step_tail's fold blocks measured slower)
__global__ __launch_bounds__(NG_WAVES * 64) void k_node_groups(GroupDev G, NodeDev N, GroupList L,
                                                               const int64_t* __restrict__ node_rows,
                                                               int64_t* __restrict__ trk_acc,
                                                               int64_t* __restrict__ nwords, NGDecide D) {
    const int32_t i0 = blockIdx.x * 64;
    const int32_t i = i0 + (int32_t)(threadIdx.x & 63);
    const uint32_t n = L.n - i0 < 64 ? (uint32_t)(L.n - i0) : 64u;
    const uint32_t g = i >= L.n ? NONE : L.ids ? L.ids[i] : (uint32_t)(L.first + i);
#if ESC_MEASURE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    node_groups_part(G, N, node_rows, trk_acc, nwords, D, g, !L.ids, L.first + i0, n);
#if ESC_MEASURE
    if (D.trace) {                                       // {start, end}
        __syncthreads();
        if (threadIdx.x == 0) {
            D.trace[2 * blockIdx.x] = t_start;
            D.trace[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
#endif
}

// K3 fold (fold_col, a role of k_step_tail): the K1 workgroups' slot partials folded and
// joined to the groups with no hand-off between workgroups: one 256-thread block per column
// of FC_COL pod slots reads every K1 row of its column (16-B loads; a wave-load covers
// FD_RPL rows of FC_COL slots, 4 waves x FD_U wave-loads in flight: every row of a
// 256-workgroup K1 grid in one round, read back from the Infinity Cache K1 just wrote it
// through), merges the lanes and waves in LDS, adds the slots' wide (exact-path) rows, and
// writes the pod words of every group whose pod slot lies in the column (col_off /
// col_groups).  Narrow columns give ~n_gp / 32 blocks (313 at 10 k groups).
//  - pods: the group's slot is its pair (NewPodAffinityFilterFunc, node_group.go:218) or,
//    for the group named "default", the default filter's slot (client.go:58-64);
//  - allNodes[0] (controller.go:208): the pair's first entry (GroupNode, set at load).
namespace {
constexpr int FD_WAVES = 4;
constexpr int FD_U = 4;                  // wave-loads per wave in flight (each array)
constexpr int FD_HL = FC_COL / 2;        // lanes per row (2 slots per 16-B lane load)
constexpr int FD_RPL = 64 / FD_HL;       // K1 rows per wave-load
static_assert(FD_RPL * FD_HL == 64 && FD_WAVES >= 2, "fold lane map");
}  // namespace

namespace {
// The fold's LDS (a member of k_step_tail's role union: the roles' LDS overlaid, so the
// tail's blocks are not limited by the sum of every role's arrays)
struct FoldLds {
    uint64_t red[FD_WAVES][8][64];                       // 16 KB
    uint64_t tot[4][FC_COL];                             // per slot: cpu, count, mem lo, mem carry
    int64_t wtot[WP_K][FC_COL];                          // per slot: its wide row
};
__device__ __forceinline__ void fold_col(const GroupDev& G, const FoldPlan& F, int64_t* __restrict__ wide_pod,
                                         int64_t* __restrict__ pwords, int col, FoldLds& S) {
    // F.ablate (timing-only, wrong results): 1 no group phase, 4 no fold loads
    const int ablate = F.ablate;
    auto& red = S.red;
    auto& tot = S.tot;
    auto& wtot = S.wtot;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int sub = lane / FD_HL, hl = lane % FD_HL;
    const int64_t s0 = (int64_t)col * FC_COL;
    const uint32_t ga = F.col_off[col], gb = F.col_off[col + 1];
    const uint32_t me = threadIdx.x;
    // loads that do not depend on the fold, issued before it so their latency overlaps the
    // fold's: the slots' wide rows (threads < FC_COL) and the first round of the column's
    // groups with their pod slots
    int64_t p[WP_K] = {0, 0, 0, 0, 0};
    const bool has_wide = me < FC_COL && s0 + me <= (int64_t)G.n_gp;
    int64_t* wp = wide_pod + (s0 + me) * WP_K;
    if (has_wide)
#pragma unroll
        for (int k = 0; k < WP_K; ++k) p[k] = ld_agent(wp + k);
    const bool g_ok0 = ga + me < gb;
    const int32_t g_0 = g_ok0 ? (int32_t)F.col_groups[ga + me] : 0;
    const uint32_t sl_0 = g_ok0 ? G.gslot[g_0] : 0;
    // ---- fold: every K1 row of the column; wave w's load u covers rows
    //      (w + FD_WAVES * u) * FD_RPL + sub
    uint64_t cp[2] = {0, 0}, cn[2] = {0, 0}, ml[2] = {0, 0}, mc[2] = {0, 0};
    // compact flush: the column's own entries (64 words each: cpu|count, then mem), else
    // column col of every K1 row
    const int64_t* pbase = reinterpret_cast<const int64_t*>(F.part);
    int64_t rstride = 2 * F.sp, mo = F.sp;
    int nrows = F.nblk;
    if (F.col_rows) {
        const uint32_t r0 = F.col_rows[col];
        nrows = (int)(F.col_rows[col + 1] - r0);
        pbase += (int64_t)r0 * 2 * FC_COL;
        rstride = 2 * FC_COL;
        mo = FC_COL;
    } else {
        pbase += s0;
    }
    if (ablate & 4) nrows = 0;
    constexpr int STEP = FD_WAVES * FD_U * FD_RPL;
    for (int b = wid * FD_RPL + sub; b - sub < nrows; b += STEP) {
        ulonglong2 c[FD_U], m[FD_U];
#pragma unroll
        for (int u = 0; u < FD_U; ++u) {
            const int r = b + FD_WAVES * FD_RPL * u;
            const int bb = r < nrows ? r : 0;
            const int64_t* row = pbase + (int64_t)bb * rstride + 2 * hl;
            c[u] = ld2(row);
            m[u] = ld2(row + mo);
        }
#pragma unroll
        for (int u = 0; u < FD_U; ++u) {
            if (b + FD_WAVES * FD_RPL * u >= nrows) continue;
            cp[0] += c[u].x & CPU_MASK; cn[0] += c[u].x >> CNT_SHIFT;
            cp[1] += c[u].y & CPU_MASK; cn[1] += c[u].y >> CNT_SHIFT;
            u128_add(ml[0], mc[0], m[u].x);
            u128_add(ml[1], mc[1], m[u].y);
        }
    }
    red[wid][0][lane] = cp[0]; red[wid][1][lane] = cp[1]; red[wid][2][lane] = cn[0]; red[wid][3][lane] = cn[1];
    red[wid][4][lane] = ml[0]; red[wid][5][lane] = ml[1]; red[wid][6][lane] = mc[0]; red[wid][7][lane] = mc[1];
    // the slots' wide rows (loaded above) are reset (every reader is in this block)
    if (has_wide && (p[0] | p[1] | p[2] | p[3] | p[4]) != 0)
#pragma unroll
        for (int k = 0; k < WP_K; ++k)
            __hip_atomic_store(wp + k, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (wid < 2 && lane < FD_HL) {                       // wave 0: slots 2l, 2l+1 words 0/1; wave 1: mem words
        const int j = lane;
        uint64_t x0 = 0, x1 = 0, y0 = 0, y1 = 0;
        for (int w = 0; w < FD_WAVES; ++w) {
#pragma unroll
            for (int q = 0; q < FD_RPL; ++q) {
                const int l = q * FD_HL + j;
                if (wid == 0) {
                    x0 += red[w][0][l]; x1 += red[w][1][l]; y0 += red[w][2][l]; y1 += red[w][3][l];
                } else {
                    u128_add(x0, y0, red[w][4][l]); y0 += red[w][6][l];
                    u128_add(x1, y1, red[w][5][l]); y1 += red[w][7][l];
                }
            }
        }
        if (wid == 0) { tot[0][2 * j] = x0; tot[0][2 * j + 1] = x1; tot[1][2 * j] = y0; tot[1][2 * j + 1] = y1; }
        else { tot[2][2 * j] = x0; tot[2][2 * j + 1] = x1; tot[3][2 * j] = y0; tot[3][2 * j + 1] = y1; }
    }
    if (me < FC_COL)
#pragma unroll
        for (int k = 0; k < WP_K; ++k) wtot[k][me] = p[k];
    __syncthreads();
    if (ablate & 1) return;
    // ---- the column's groups' pod words, one thread each (a column holds ~FC_COL groups)
    for (uint32_t base = ga; base < gb; base += FD_WAVES * 64) {
        const bool ok = base + me < gb;
        const bool first = base == ga;
        const int32_t g = first ? g_0 : (ok ? (int32_t)F.col_groups[base + me] : 0);
        if (ok) {
            const int sl = (int)((int64_t)(first ? sl_0 : G.gslot[g]) - s0);
            int64_t* pw = pwords + (int64_t)(G.xs ? G.xs[g] : (uint32_t)g) * PW_K;
            const __int128 pcpu = (__int128)tot[0][sl] + ((__int128)wtot[WP_CPU_HI][sl] << 32) + (__int128)wtot[WP_CPU_LO][sl];
            const __int128 pmem = (__int128)(((unsigned __int128)tot[3][sl] << 64) | tot[2][sl]) +
                                  ((__int128)wtot[WP_MEM_HI][sl] << 32) + (__int128)wtot[WP_MEM_LO][sl];
            split_store(pw, PW_CPU_LO, pcpu);
            split_store(pw, PW_MEM_LO, pmem);
            pw[PW_N] = (int64_t)tot[1][sl] + wtot[WP_CNT][sl];
        }
    }
}
}  // namespace


// ===================================================================== K5 ordering
// taintOldestN / untaintNewestN (scale_down.go:171, scale_up.go:118) order a group's
// untainted (tainted) nodes by CreationTimestamp (sort.go:6-39).  Creation times and
// label memberships are immutable, so the snapshot carries an AGE INDEX built once per
// load (esc_load_nodes): every group membership of this rank's nodes, with a copy of the
// node's flags, in (group, creation time, snapshot index) order — one LSD radix sort of
// 64-bit (group | creation offset) keys carrying (node | flags) as the value over the
// memberships listed in snapshot order, so no pass gathers at random.  Per decision
// only the class can change (taint / cordon / dry-mode tracker), so ordering = classify
// every membership and stable-partition by (group, class): LSD radix passes over the
// segment id alone.  A segment then lists its nodes oldest first; newest first is the
// segment read backwards (esc_group_order restores index order inside equal timestamps).
#ifndef ESC_SORT_BLOCK
#define ESC_SORT_BLOCK 1024   // sort workgroup size (timing builds may override)
#endif
#ifndef ESC_RS_MAXBLK
#define ESC_RS_MAXBLK 512     // the most workgroups per sort pass
#endif
namespace {
constexpr int SORT_BLOCK = ESC_SORT_BLOCK;
constexpr int SORT_WAVES = SORT_BLOCK / 64;
}

// Creation offset of node i (divided by div when exact): the low key bits of its memberships.
// x / d for the creation-time divisors the host picks (1, 10^3, 10^6, 10^9): divisions by
// constants (multiply-high) instead of the 64-bit division routine.
__device__ __forceinline__ uint64_t div_pow10(uint64_t x, uint64_t d) {
    switch (d) {
        case 1: return x;
        case 1000ull: return x / 1000ull;
        case 1000000ull: return x / 1000000ull;
        case 1000000000ull: return x / 1000000000ull;
        default: return x / d;
    }
}
// ---- LSD radix sort building blocks (stable), BITS-bit digits, KT = uint64_t or uint32_t.
// hist is digit-major: hist[d * nblk + b] = keys of block b with digit d.
template <class KT, int BITS>
__global__ __launch_bounds__(SORT_BLOCK) void k_rs_hist(const KT* __restrict__ keys, int64_t n, int shift,
                                                        uint32_t* __restrict__ hist) {
    // per wave: one LDS atomic add per key into the wave's own counters
    constexpr int NB = 1 << BITS;
    __shared__ uint32_t wh[SORT_WAVES][NB];
    for (int i = threadIdx.x; i < SORT_WAVES * NB; i += SORT_BLOCK) (&wh[0][0])[i] = 0;
    __syncthreads();
    const int wid = threadIdx.x >> 6;
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(n, lo + per);
    constexpr int U = 8;                                 // keys in flight per thread
    for (int64_t b = lo; b < hi; b += (int64_t)SORT_BLOCK * U) {
        KT k[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * SORT_BLOCK + threadIdx.x;
            k[u] = i < hi ? keys[i] : (KT)0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool ok = b + (int64_t)u * SORT_BLOCK + threadIdx.x < hi;
            const uint32_t d = (uint32_t)(k[u] >> shift) & (NB - 1);
            if (ok) atomicAdd(&wh[wid][d], 1u);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < NB; d += SORT_BLOCK) {
        uint32_t t = 0;
        for (int k = 0; k < SORT_WAVES; ++k) t += wh[k][d];
        hist[(int64_t)d * gridDim.x + blockIdx.x] = t;
    }
}

// Exclusive scan of each digit's row hist[d][0..nblk) in place (one wave per digit) and the
// digit totals into tot[d].
__global__ __launch_bounds__(256) void k_rs_scan_rows(uint32_t* __restrict__ hist, int nblk, int nb,
                                                      uint32_t* __restrict__ tot) {
    const int d = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (d >= nb) return;
    uint32_t* row = hist + (int64_t)d * nblk;
    uint32_t carry = 0;
    constexpr int RW = 8;                                // the row's loads in flight (rows <= 512 go in one round)
    for (int b0 = 0; b0 < nblk; b0 += 64 * RW) {
        uint32_t v[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int b = b0 + r * 64 + lane;
            v[r] = b < nblk ? row[b] : 0u;
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int b = b0 + r * 64 + lane;
            const uint32_t x = wave_incl_scan32(v[r]);   // DPP, no LDS round trips
            if (b < nblk) row[b] = carry + x - v[r];
            carry += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
        }
    }
    if (lane == 0) tot[d] = carry;
}


// Stable scatter of one pass, a chunk of RS_U * SORT_BLOCK keys at a time: ranks from
// ballot matching per wave and per-(round, wave) digit counts; the chunk is reordered by
// digit in LDS and written out in per-digit runs (stored straight from the ranking, a
// wave's 64 keys went to ~64 different buckets: 8-B scattered stores, 1.6x write traffic).
// A membership's sort value is its region word (esc_kernels.h MEMB_FLAG_SHIFT): 4 B instead
// of node | flags << 32, so every LSD pass moves 8 B less per membership.
// Sorted membership at position p (key = group << R | offset, value as above)
// into its group's region: pstart[g] + p - seg[g].  The sorted starts seg are the host's
// (live entries per pair); a position outside the group's [0, len) means the device listed a
// different count, and is flagged in *err instead of written.
// (value-less sorts carry the value in a packed element's low 32 bits, the key above it)
struct NoVal {};
template <class KT, class VT>
struct RsElem {
    static constexpr bool HASV = true;
};
template <class KT>
struct RsElem<KT, NoVal> {
    static constexpr bool HASV = false;
};
__device__ __forceinline__ void region_put(const RegionSink& S, uint32_t p, uint64_t key, uint32_t v) {
    const uint32_t g = (uint32_t)(key >> S.R);
    if (g >= (uint32_t)S.G) { *S.err = 1u; return; }   // (keys of a listing that gave up)
    const int64_t r = (int64_t)p - S.seg[g];
    if (r < 0 || r >= (int64_t)S.plen[g]) { *S.err = 1u; return; }
    S.g_memb[(int64_t)S.pstart[g] + r] = v;
}

// FINAL (the age index's last pass): a key's sorted position goes straight into its group's
// padded region (RegionSink) instead of the key / value arrays.
#ifndef ESC_RS_U
#define ESC_RS_U 3         // keys per thread per scatter chunk (r05w: 3 beat 2 and 4 by 4%)
#endif
#ifndef ESC_RS_CARRY
#define ESC_RS_CARRY 1     // whole-line digit runs (below); 0 = the plain scatter, for timing builds
#endif
constexpr int RS_U = ESC_RS_U;
#ifdef ESC_RS_WPE
#define RS_SCATTER_BOUNDS __launch_bounds__(SORT_BLOCK, ESC_RS_WPE)
#else
#define RS_SCATTER_BOUNDS __launch_bounds__(SORT_BLOCK)
#endif
template <class KT, class VT, int BITS, bool FINAL>
__global__ RS_SCATTER_BOUNDS void k_rs_scatter(const KT* __restrict__ kin, const VT* __restrict__ vin,
                                                           KT* __restrict__ kout, VT* __restrict__ vout,
                                                           int64_t n, int shift, const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ tot, RegionSink sink) {
    constexpr int NB = 1 << BITS, S = RS_U * SORT_WAVES, CH = RS_U * SORT_BLOCK;
    constexpr bool HASV = RsElem<KT, VT>::HASV;          // else: packed (key << 32 | value) elements
    static_assert(NB <= SORT_BLOCK, "one thread per digit");
    __shared__ uint32_t run[NB];                         // output position of the digit's next key
    __shared__ uint32_t lst[NB];                         // the digit's first slot in the chunk
    // (round, wave) digit counts -> offsets (< CH: 16 bits; the LDS then holds two workgroups
    // per CU instead of one)
    __shared__ uint16_t wh[S][NB];
    static_assert(CH <= 65535, "16-bit chunk offsets");
    __shared__ uint32_t ws[SORT_WAVES];
    __shared__ KT sk[CH];
    __shared__ VT sv[HASV ? CH : 1];
    // Whole lines per digit run (non-FINAL passes): a chunk writes each digit's keys only up
    // to the last 16-key boundary of its run (16 keys = one 128-B line of 8-B keys, half a
    // line of 4-B values) and carries the rest in LDS to the front of that digit's run in
    // the next chunk, where it continues; the block's last chunk flushes everything.  A
    // chunk's per-digit runs average ~16 keys, so writing each run whole left partial lines
    // at both ends (1.4x the bytes written).  (32-key alignment would double
    // the carry's LDS and halve the blocks per CU.)
    constexpr bool CARRY = !FINAL && ESC_RS_CARRY;
    constexpr int CW = 16, CD = CARRY ? NB : 1;
    __shared__ KT ck[CD][CW];
    __shared__ VT cv[HASV ? CD : 1][CW];
    __shared__ uint32_t c_n[CD], c_s[CD], c_e[CD];        // carry count, carry start, write end
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, t = threadIdx.x;
    {   // the digits' start: the exclusive scan of the digit totals (round 5: every block scans
        // the NB totals itself instead of a one-workgroup launch per pass), + this block's
        // prefix of its digit row (k_rs_scan_rows)
        const uint32_t dv = t < NB ? tot[t] : 0u;
        const uint32_t xi = wave_incl_scan32(dv);
        if (lane == 63) ws[wid] = xi;
        __syncthreads();
        uint32_t base = xi - dv;
        for (int k = 0; k < wid; ++k) base += ws[k];
        if (t < NB) run[t] = base + hist[(int64_t)t * gridDim.x + blockIdx.x];
    }
    if (CARRY && t < NB) c_n[t] = 0;
    for (int e = t; e < S * NB / 2; e += SORT_BLOCK) reinterpret_cast<uint32_t*>(&wh[0][0])[e] = 0;
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per, hi = imin64(n, lo + per);
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t dtot = 0;                                   // this thread's digit: keys in the last chunk
    KT key[RS_U];
    VT val[RS_U];
#pragma unroll
    for (int u = 0; u < RS_U; ++u) {
        const int64_t i = lo + u * SORT_BLOCK + t;
        key[u] = i < hi ? kin[i] : (KT)0;
        if constexpr (HASV) val[u] = i < hi ? vin[i] : (VT)0;
    }
    __syncthreads();
    for (int64_t b = lo; b < hi; b += CH) {
        uint32_t d[RS_U], r[RS_U];
        bool ok[RS_U];
#pragma unroll
        for (int u = 0; u < RS_U; ++u) {
            ok[u] = b + u * SORT_BLOCK + t < hi;
            d[u] = (uint32_t)(key[u] >> shift) & (NB - 1);
            unsigned long long m = __ballot(ok[u]);
#pragma unroll
            for (int bit = 0; bit < BITS; ++bit) {
                const unsigned long long bb = __ballot((d[u] >> bit) & 1);
                m &= ((d[u] >> bit) & 1) ? bb : ~bb;
            }
            r[u] = __popcll(m & lt);
            if (ok[u] && r[u] == 0) wh[u * SORT_WAVES + wid][d[u]] = (uint16_t)__popcll(m);
        }
        __syncthreads();
        // per digit: offsets of the (round, wave) segments, the digit's count; the previous
        // chunk's count moves run on (its write-out has finished)
        uint32_t c = 0;
        if (t < NB) {
            run[t] += dtot;
            uint32_t v[S];                               // every segment's count in flight at once
#pragma unroll
            for (int s = 0; s < S; ++s) v[s] = wh[s][t];
#pragma unroll
            for (int s = 0; s < S; ++s) { wh[s][t] = (uint16_t)c; c += v[s]; }
            dtot = c;
        }
        const uint32_t x = wave_incl_scan32(c);          // digits in thread order (0 past NB)
        if (lane == 63) ws[wid] = x;
        __syncthreads();
        if (t < NB) {
            uint32_t p = x - dtot;
            for (int k = 0; k < wid; ++k) p += ws[k];
            lst[t] = p;
            if constexpr (CARRY) {                      // this chunk writes [begin, E) of digit t
                const uint32_t begin = c_n[t] ? c_s[t] : run[t], endp = run[t] + dtot;
                c_e[t] = b + CH >= hi ? endp : imax64((int64_t)begin, (int64_t)(endp & ~(uint32_t)(CW - 1)));
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < RS_U; ++u)
            if (ok[u]) {
                const uint32_t s = lst[d[u]] + wh[u * SORT_WAVES + wid][d[u]] + r[u];
                sk[s] = key[u];
                if constexpr (HASV) sv[s] = val[u];
            }
        // the previous carry: written when below this chunk's write end, else kept (it moves
        // to the front of the new carry, after every thread has read the old one)
        constexpr int CN = CARRY ? (CD * CW + SORT_BLOCK - 1) / SORT_BLOCK : 1;
        KT okk[CN];
        VT ovv[CN];
        uint32_t opos[CN], odig[CN];
        bool keep[CN];
        if constexpr (CARRY) {
#pragma unroll
            for (int q = 0; q < CN; ++q) {
                const int idx = t + q * SORT_BLOCK, dg = idx / CW, j = idx % CW;
                keep[q] = false;
                if (dg < CD && j < (int)c_n[dg]) {
                    okk[q] = ck[dg][j];
                    if constexpr (HASV) ovv[q] = cv[dg][j];
                    opos[q] = c_s[dg] + (uint32_t)j;
                    odig[q] = (uint32_t)dg;
                    if (opos[q] < c_e[dg]) {
                        kout[opos[q]] = okk[q];
                        if constexpr (HASV) vout[opos[q]] = ovv[q];
                    } else {
                        keep[q] = true;
                    }
                }
            }
        }
        __syncthreads();
        if constexpr (CARRY) {
#pragma unroll
            for (int q = 0; q < CN; ++q)
                if (keep[q]) {
                    ck[odig[q]][opos[q] - c_e[odig[q]]] = okk[q];
                    if constexpr (HASV) cv[odig[q]][opos[q] - c_e[odig[q]]] = ovv[q];
                }
        }
        // the next chunk's keys in flight during the write-out
#pragma unroll
        for (int u = 0; u < RS_U; ++u) {
            const int64_t i = b + CH + u * SORT_BLOCK + t;
            key[u] = i < hi ? kin[i] : (KT)0;
            if constexpr (HASV) val[u] = i < hi ? vin[i] : (VT)0;
        }
        const int cn = (int)imin64(CH, hi - b);
        for (int e = t; e < cn; e += SORT_BLOCK) {
            const KT kk = sk[e];
            const uint32_t dd = (uint32_t)(kk >> shift) & (NB - 1);
            const uint32_t g = run[dd] + (uint32_t)e - lst[dd];
            if constexpr (FINAL) {
                if constexpr (HASV) {
                    region_put(sink, g, kk, sv[e]);
                    if (sink.fix) kout[g] = kk;                  // coarse keys: k_age_fix reads them
                } else {                                         // packed: key << 32 | value
                    region_put(sink, g, (uint64_t)kk >> 32, (uint32_t)kk);
                    if (sink.fix) reinterpret_cast<uint32_t*>(kout)[g] = (uint32_t)((uint64_t)kk >> 32);
                }
            }
            else if (!CARRY || g < c_e[dd]) {
                kout[g] = kk;
                if constexpr (HASV) vout[g] = sv[e];
            } else {                                     // the run's partial last line: carried
                ck[dd][g - c_e[dd]] = kk;
                if constexpr (HASV) cv[dd][g - c_e[dd]] = sv[e];
            }
        }
        for (int e = t; e < S * NB / 2; e += SORT_BLOCK) reinterpret_cast<uint32_t*>(&wh[0][0])[e] = 0;
        if constexpr (CARRY) {
            if (t < NB) {                                // the new carry: [E, run + count)
                c_n[t] = run[t] + dtot - c_e[t];
                c_s[t] = c_e[t];
            }
        }
        __syncthreads();
    }
}

// Coarse keys (launch_age_sort): the LSD sort orders the memberships by (group, creation
// offset >> shift), equal coarse keys in snapshot order.  Each run of equal coarse keys
// (k_rs_scatter's final pass also left the sorted keys in its key output) is put in exact order here:
// its region words re-sorted by (creation time, node) — the exact sort's order, as a group
// holds a node once and snapshot order is node order.  Runs are rare (config 5: a few per
// thousand memberships) and short; one longer than AF_RUN sets bit 2 of *S.err and the
// host rebuilds the index with the exact 64-bit keys.  A run holding equal creation times
// flags its group (S.tie; with exact keys (fix 2) every run does, and nothing is reordered).
constexpr int AF_RUN = 8;
// One run of equal coarse keys starting at sorted position i (len >= 2 members), put in
// exact (creation time, node) order in its group's region.
__device__ __forceinline__ void age_fix_run(const uint32_t* __restrict__ keys, int64_t n, const RegionSink& S,
                                            const int64_t* __restrict__ created, int64_t n_nodes, int64_t ts_min,
                                            int64_t i, uint32_t k) {
    const uint32_t g = k >> S.R;
    if (g >= (uint32_t)S.G) { atomicOr(S.err, 1u); return; }
    if (S.fix == 2) { S.tie[g] = 1u; return; }         // exact keys: equal keys are equal times
    int len = 2;                                       // the run's length: its next keys loaded together
    {
        uint32_t nk[AF_RUN - 1];
#pragma unroll
        for (int j = 0; j < AF_RUN - 1; ++j) nk[j] = i + 2 + j < n ? keys[i + 2 + j] : ~k;
        bool on = true;
#pragma unroll
        for (int j = 0; j < AF_RUN - 1; ++j) {
            on = on && nk[j] == k;
            len += on ? 1 : 0;
        }
    }
    if (len > AF_RUN) { atomicOr(S.err, 2u); return; }
    // the run lies inside its group's sorted range, and its words name table nodes — always,
    // unless the keys are not the listing's (bit 0: the build fails; nothing is touched)
    const int64_t r = i - S.seg[g];
    if (r < 0 || r + len > (int64_t)S.plen[g]) { atomicOr(S.err, 1u); return; }
    const int64_t d0 = (int64_t)S.pstart[g] + r;
    uint32_t w[AF_RUN];
    int64_t t[AF_RUN];
#pragma unroll
    for (int j = 0; j < AF_RUN; ++j) w[j] = j < len ? S.g_memb[d0 + j] : 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < AF_RUN; ++j)
        if (j < len && (int64_t)(w[j] & MEMB_NODE_MASK) >= n_nodes) { atomicOr(S.err, 1u); return; }
#pragma unroll
    for (int j = 0; j < AF_RUN; ++j) t[j] = j < len ? created[w[j] & MEMB_NODE_MASK] - ts_min : INT64_MAX;
#pragma unroll
    for (int a = 0; a < AF_RUN; ++a)                   // odd-even transposition: static indices only
#pragma unroll
        for (int j = a & 1; j + 1 < AF_RUN; j += 2) {
            const bool sw = t[j] > t[j + 1] ||
                            (t[j] == t[j + 1] && (w[j] & MEMB_NODE_MASK) > (w[j + 1] & MEMB_NODE_MASK));
            const uint32_t wa = sw ? w[j + 1] : w[j], wb = sw ? w[j] : w[j + 1];
            const int64_t ta = sw ? t[j + 1] : t[j], tb = sw ? t[j] : t[j + 1];
            w[j] = wa; w[j + 1] = wb; t[j] = ta; t[j + 1] = tb;
        }
#pragma unroll
    for (int j = 0; j < AF_RUN; ++j)
        if (j < len) S.g_memb[d0 + j] = w[j];
    bool tie = false;                                  // equal times side by side, now that they are sorted
#pragma unroll
    for (int j = 0; j + 1 < AF_RUN; ++j) tie |= j + 1 < len && t[j] == t[j + 1];
    if (tie) S.tie[g] = 1u;
}

// Two phases per block over its contiguous share of quads of the sorted coarse keys (one
// 16-B load + the neighbours at the quad's ends; a position starts a run when its key equals
// the next one and not the previous one): the run starts found are listed in LDS, then every
// listed run is fixed by its own thread, all of the block's runs in flight together.  Runs
// are rare (config 5: a few per 10^3 memberships) but each is a chain of dependent loads
// (region starts, region words, creation times): fixed where found, a grid-stride
// iteration that met one waited out its chain before its next quads (37 µs, round 6).
// (one call site: every inlined copy of age_fix_run is ~30 compare-exchanges and 16 loads)
constexpr int AF_QPT = 4;                                // quads per thread per round
constexpr int AF_CAP = 256 * AF_QPT * 2;                 // a round's run starts at most (one per two keys)
__global__ __launch_bounds__(256) void k_age_fix(const uint32_t* __restrict__ keys, int64_t n, RegionSink S,
                                                 const int64_t* __restrict__ created, int64_t n_nodes, int64_t ts_min) {
    __shared__ uint32_t s_n;
    __shared__ uint32_t s_i[AF_CAP];                     // run start - 4 * q0
    __shared__ uint32_t s_k[AF_CAP];
    if (*S.err & 1u) return;                             // the listing gave up: its keys are not memberships
    const int64_t nq = (n + 3) / 4;
    const int64_t per = (nq + gridDim.x - 1) / gridDim.x;
    const int64_t qa = (int64_t)blockIdx.x * per, qb = imin64(nq, qa + per);
    for (int64_t q0 = qa; q0 < qb; q0 += 256 * AF_QPT) {
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        uint32_t k[AF_QPT][6];                           // keys[i0 - 1 .. i0 + 4]; absent ends never match
#pragma unroll
        for (int u = 0; u < AF_QPT; ++u) {
            const int64_t q = q0 + u * 256 + threadIdx.x, i0 = 4 * q;
            if (q >= qb) { k[u][1] = 0; k[u][2] = 1; k[u][3] = 2; k[u][4] = 3; k[u][0] = k[u][5] = 4; continue; }
            if (i0 + 4 <= n) {
                const uint4 v = *reinterpret_cast<const uint4*>(keys + i0);
                k[u][1] = v.x; k[u][2] = v.y; k[u][3] = v.z; k[u][4] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) k[u][1 + j] = i0 + j < n ? keys[i0 + j] : ~keys[n - 1];
            }
            k[u][0] = i0 > 0 ? keys[i0 - 1] : ~k[u][1];
            k[u][5] = i0 + 4 < n ? keys[i0 + 4] : ~k[u][4];
        }
#pragma unroll
        for (int u = 0; u < AF_QPT; ++u) {
            const int64_t i0 = 4 * (q0 + u * 256 + threadIdx.x);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (i0 + j + 1 < n && k[u][1 + j] == k[u][2 + j] && k[u][j] != k[u][1 + j]) {
                    const uint32_t s = atomicAdd(&s_n, 1u);      // < AF_CAP: runs start >= 2 keys apart
                    s_i[s] = (uint32_t)(i0 + j - 4 * q0);
                    s_k[s] = k[u][1 + j];
                }
        }
        __syncthreads();
        const uint32_t m = s_n;
        for (uint32_t r = threadIdx.x; r < m; r += 256)
            age_fix_run(keys, n, S, created, n_nodes, ts_min, 4 * q0 + s_i[r], s_k[r]);
        __syncthreads();
    }
}

// ---- the age index (load time): memberships listed in snapshot order (streaming over
// the node table), then sorted by (group, creation offset) with (node | flags << 32)
// carried along, then written into the groups' padded regions (streaming).
// Memberships of the nodes of this block's share of [0, n) (snapshot order).
// (node_groups with the node's flags and the group code of its label0 already loaded,
// memb_codes)
template <class F>
__device__ __forceinline__ void node_groups_c0(const NodeDev& N, const GroupDev& G, uint32_t f, int64_t i, uint32_t c0,
                                               F&& emit) {
    if (f & ESC_NF_ABSENT) return;
    for_code(G, c0, emit);
    const uint32_t nx = nf_xlbl(f);
    if (nx) {
        const uint32_t q = N.xl_off[i];
        for (uint32_t k = 0; k < nx; ++k) {
            const uint32_t p = N.xl[q + k];
            if (p >= N.q_lo && p < N.q_hi) for_code(G, node_code(G, p), emit);
        }
    }
}
#ifndef ESC_MEMB_U
#define ESC_MEMB_U 4         // consecutive nodes per thread per tile (a multiple of 4; timing builds may override)
#endif
constexpr int MEMB_U = ESC_MEMB_U;
static_assert(MEMB_U % 4 == 0, "16-B loads of 4 nodes");
constexpr int MEMB_BLOCK = 512, MEMB_WAVES = MEMB_BLOCK / 64;
// LDS staging of one round's memberships (1.5 per node; a round with more stores directly)
constexpr int MEMB_CAP = MEMB_BLOCK * MEMB_U * 3 / 2;
// Flags, label0 (and creation times) of nodes [r0, r0 + MEMB_U) with 16-B loads when all are
// below hi (absent / NONE past it).
__device__ __forceinline__ void memb_load(const NodeDev& N, int64_t r0, int64_t hi, uint32_t (&f)[MEMB_U],
                                          uint32_t (&l0)[MEMB_U], int64_t* cr) {
    const int64_t i0 = N.lo + r0;
    if (r0 + MEMB_U <= hi && (i0 & 3) == 0) {
#pragma unroll
        for (int q = 0; q < MEMB_U; q += 4) {
            const uint4 a = *reinterpret_cast<const uint4*>(N.flags + i0 + q);
            const uint4 b = *reinterpret_cast<const uint4*>(N.label0 + i0 + q);
            f[q] = a.x; f[q + 1] = a.y; f[q + 2] = a.z; f[q + 3] = a.w;
            l0[q] = b.x; l0[q + 1] = b.y; l0[q + 2] = b.z; l0[q + 3] = b.w;
            if (cr) {
                const longlong2 c0 = *reinterpret_cast<const longlong2*>(N.created + i0 + q);
                const longlong2 c1 = *reinterpret_cast<const longlong2*>(N.created + i0 + q + 2);
                cr[q] = c0.x; cr[q + 1] = c0.y; cr[q + 2] = c1.x; cr[q + 3] = c1.y;
            }
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < MEMB_U; ++u) {
        const bool ok = r0 + u < hi;
        f[u] = ok ? N.flags[i0 + u] : ESC_NF_ABSENT;
        l0[u] = ok ? N.label0[i0 + u] : NONE;
        if (cr) cr[u] = ok ? N.created[i0 + u] : 0;
    }
}

// The group codes of the MEMB_U nodes' first labels, loaded together (unconditional loads
// at a clamped index: in branches they went out one after another).
__device__ __forceinline__ void memb_codes(const NodeDev& N, const GroupDev& G, const uint32_t (&f)[MEMB_U],
                                           const uint32_t (&l0)[MEMB_U], uint32_t (&c0)[MEMB_U]) {
#pragma unroll
    for (int u = 0; u < MEMB_U; ++u) {
        const uint32_t q = l0[u];
        const bool ok = !(f[u] & ESC_NF_ABSENT) && q >= N.q_lo && q < N.q_hi && q < G.n_gp;
        c0[u] = G.n_gp ? G.node_code[ok ? q : 0u] : NONE;
        if (!ok) c0[u] = NONE;
    }
}

// Lists the memberships in snapshot order (a tile's nodes in order, a node's groups in
// label order): key = group << R | (creation offset >> KS), value = node | membership
// flags << MEMB_FLAG_SHIFT — a dry group's membership carries "tracked by this group" in
// the tracker bit (controller.go:126-138), so the per-decision split needs no lookup.  KT =
// uint64_t with KS = 0 (the exact key); PACK: one 8-B element per membership, the 32-bit
// coarse key above the value (vals unused).
// Single pass (round 5; a counting pass + scan before it read the node table twice): one
// workgroup per tile of MEMB_BLOCK * MEMB_U nodes (tile = blockIdx.x); a tile publishes its
// membership count (LB_AGG) before it looks back, then its inclusive prefix (LB_INC) once
// one wave has summed its predecessors' words back to the nearest inclusive one.  No
// ticket: one shared ticket word serialises its grabs (≈ 88 per µs, the guide's dequeue
// price: 56 µs for config 5's 4 900 tiles).  HIP does not promise dispatch order, so the
// wait is bounded: a tile that waited `spins` probes gives up, publishes LB_ERR (its
// successors give up at once instead of waiting, and none publishes an inclusive prefix it
// could not compute), writes nothing and sets error bit 0 (the build then fails loudly)
// instead of hanging on a predecessor that was never dispatched.
constexpr uint64_t LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_ERR = 3ull << 62;
template <class KT, bool PACK = false>
__global__ __launch_bounds__(MEMB_BLOCK) void k_memb_keys(NodeDev N, GroupDev G, int64_t n, uint64_t* __restrict__ status,
                                                          uint32_t* __restrict__ total_out, uint32_t* __restrict__ err,
                                                          uint32_t spin_limit, int64_t cap, int64_t ts_min,
                                                          uint64_t div, int R, int KS, KT* __restrict__ keys,
                                                          uint32_t* __restrict__ vals) {
    // A tile's memberships are staged in LDS and written out as two contiguous streams:
    // stored straight from the walk, a wave's 8-B stores land ~4 entries apart per lane and
    // the listing took 5x its store-free time (measured, r03_mk).
    __shared__ uint32_t wsum[MEMB_WAVES];
    __shared__ KT sk[MEMB_CAP];
    __shared__ uint32_t sv[PACK ? 1 : MEMB_CAP];
    __shared__ uint32_t s_base, s_fail;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t n_tiles = (n + MEMB_BLOCK * MEMB_U - 1) / (MEMB_BLOCK * MEMB_U);
    const int64_t tile = blockIdx.x;
    if (tile >= n_tiles) return;                         // (the grid is exactly n_tiles)
    {
        const int64_t b = tile * (MEMB_BLOCK * MEMB_U), hi = imin64(n, b + MEMB_BLOCK * MEMB_U);
        // MEMB_U consecutive nodes per thread (snapshot order = thread order), loads first
        const int64_t r0 = b + (int64_t)threadIdx.x * MEMB_U;
        uint32_t f[MEMB_U], l0[MEMB_U];
        int64_t cr[MEMB_U];
        memb_load(N, r0, hi, f, l0, cr);
        uint32_t c0[MEMB_U];
        memb_codes(N, G, f, l0, c0);
        // a tracked node's first tracker entry, loaded with the codes (most tracked nodes are
        // tracked by one group: the per-membership lookup then needs nothing more)
        uint32_t tk[MEMB_U];
        int32_t tn[MEMB_U], tg[MEMB_U];
#pragma unroll
        for (int u = 0; u < MEMB_U; ++u) tk[u] = (f[u] & ESC_NF_TRACKED) ? N.trk_start[N.lo + r0 + u] : NONE;
#pragma unroll
        for (int u = 0; u < MEMB_U; ++u) {
            const bool v = tk[u] != NONE && (int64_t)tk[u] < N.n_trk;
            tn[u] = v ? N.trk_node[tk[u]] : -1;
            tg[u] = v ? N.trk_group[tk[u]] : -1;
        }
        uint32_t c = 0;
#pragma unroll
        for (int u = 0; u < MEMB_U; ++u) node_groups_c0(N, G, f[u], N.lo + r0 + u, c0[u], [&](uint32_t) { ++c; });
        const uint32_t x = wave_incl_scan32(c);
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
        uint32_t pos = x - c, total = 0;
#pragma unroll
        for (int k = 0; k < MEMB_WAVES; ++k) {
            const uint32_t s = wsum[k];
            pos += k < wid ? s : 0u;
            total += s;
        }
        const bool stage = total <= (uint32_t)MEMB_CAP;   // block-uniform
        if (threadIdx.x == 0)
            __hip_atomic_store(status + tile, (tile ? LB_AGG : LB_INC) | total, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        // look back (wave 0; lane l reads tile look - l) -> s_base, this tile's first position
        auto look_back = [&]() {
            uint32_t excl = 0;
            uint32_t spins = 0;                          // a bound on waiting (never reached when the
            bool failed = false;                         // status words were zeroed): err bit 0
            for (int64_t look = tile - 1; look >= 0;) {
                if (++spins > spin_limit) {
                    failed = true;
                    break;
                }
                const int64_t j = look - lane;
                // relaxed: a word carries its own value and nothing else is read through it (an
                // acquire invalidates the CU's vector L1 under the other workgroups' loads)
                const uint64_t w = j >= 0 ? __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                          : LB_INC;      // before tile 0: an inclusive 0
                // the nearest inclusive or failed word ends the look-back
                const unsigned long long inc = __ballot((w >> 62) >= 2), wait = __ballot((w >> 62) == 0);
                const int fi = inc ? __builtin_ctzll(inc) : 63;
                const unsigned long long need = ~0ull >> (63 - fi);      // lanes 0..fi
                if (wait & need) {                       // a predecessor has not counted yet
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                if (inc && (__builtin_amdgcn_readlane((uint32_t)(w >> 32), fi) >> 30) == 3) {   // it gave up
                    failed = true;
                    break;
                }
                excl += wave_total32(lane <= fi ? (uint32_t)w : 0u);
                if (inc) break;
                look -= 64;
            }
            if (lane == 0) {
                if (failed) atomicOr(err, 1u);
                if (tile) __hip_atomic_store(status + tile, failed ? LB_ERR : (LB_INC | (uint64_t)(uint32_t)(excl + total)),
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_base = excl;
                s_fail = failed ? 1u : 0u;
                if (tile == n_tiles - 1 && !failed) total_out[0] = excl + total;
            }
        };
        // staged tiles look back after their walk (the predecessors' counts are published by
        // then); a tile too large for the staging stores directly and needs its base first
        if (!stage) {
            if (wid == 0) look_back();
            __syncthreads();
            if (s_fail) return;                          // no base: write nothing (err is set)
        }
        const uint32_t carry = stage ? 0u : s_base;
#pragma unroll
        for (int u = 0; u < MEMB_U; ++u) {
            const int64_t i = N.lo + r0 + u;
            const uint64_t off = (uint64_t)(cr[u] - ts_min);
            const KT ak = (KT)(div_pow10(off, div) >> KS);
            const uint32_t fu = f[u];
            node_groups_c0(N, G, fu, i, c0[u], [&](uint32_t mb) {
                bool tr = false;
                if (mdry(mb) && (fu & ESC_NF_TRACKED))
                    tr = (tn[u] == (int32_t)i && tg[u] == (int32_t)mg(mb)) || tracked(N, (int32_t)i, (int32_t)mg(mb));
                const uint32_t mf = mdry(mb) ? ((fu & ~ESC_NF_TRACKED) | (tr ? ESC_NF_TRACKED : 0u)) : fu;
                const uint32_t vw = (uint32_t)i | ((mf & 0xFu) << MEMB_FLAG_SHIFT);
                const KT kw = PACK ? (KT)(((uint64_t)(((uint32_t)mg(mb) << R) | (uint32_t)ak) << 32) | vw)
                                   : (((KT)mg(mb) << R) | ak);
                if (stage) { sk[pos] = kw; if (!PACK) sv[pos] = vw; }
                else if (carry + pos < cap) { keys[carry + pos] = kw; if (!PACK) vals[carry + pos] = vw; }
                ++pos;
            });
        }
        if (stage) {
            if (wid == 0) look_back();
            __syncthreads();
            if (s_fail) return;
            const uint32_t base = s_base;
            for (uint32_t e = threadIdx.x; e < total && base + e < cap; e += MEMB_BLOCK) {
                keys[base + e] = sk[e];
                if (!PACK) vals[base + e] = sv[e];
            }
        }
    }
}

// ---- per decision: inside every group's run, a stable 3-way split by filterNodes class
// (controller.go:125-150; dry groups: tracker only).  Chunks never cross a group, so a
// chunk's untainted / tainted nodes go to two contiguous output streams; two passes:
//   A  classify (the 4-B region words) -> per-chunk class counts,
//   C  per chunk: its bases from the group's chunk counts, the words again (classes
//      recomputed: cheaper than writing and re-reading a class byte), DPP wave ranks, LDS
//      staging -> vals (<= 4 B written, coalesced), the group's segment bounds.
constexpr int ORD_BLOCK = 256, ORD_WAVES = ORD_BLOCK / 64;

// Membership flags: a dry group's membership has the tracker bit resolved for its group
// (k_memb_keys), so no per-decision lookup is needed.
__device__ __forceinline__ uint32_t ord_class(const NodeDev&, uint32_t, uint32_t grp, uint32_t f) {
    if ((grp & MEMB_PAD) || (f & ESC_NF_ABSENT)) return 3u;                      // padding, deleted node
    if (mdry(grp)) return (f & ESC_NF_TRACKED) ? 1u : 0u;
    if (f & ESC_NF_UNSCHED) return 2u;
    return (f & ESC_NF_TAINTED) ? 1u : 0u;
}

// Split groups (region > ORD_CHUNK memberships), ONE pass (round 5; it replaced a counting
// pass and a scatter pass that read every region word twice).  A split chunk holds one
// group's memberships, so the class is a function of the region word's flags alone: the
// group's dry mode comes with the chunk (OrdChunk::pad & ORD_CHUNK_DRY) and region padding
// is flagged ESC_NF_ABSENT (k_region_pad) like a deleted node.  Every chunk loads its
// region words (4 steps of 1 024, 4 per lane), classifies them, ranks them by packed DPP
// wave scans and publishes its two class counts; its group's earlier chunks' counts come
// from a decoupled look-back (one wave, 64 status words per probe, relaxed agent-scope
// atomics), so the bases need no second pass over the words.  Output layout (DESIGN.md §4
// K5): untainted forward from the region start, tainted BACKWARD from the region end — a
// chunk knows how many tainted nodes precede it in its group but not how many untainted
// nodes the whole group has — so the tainted segment is stored newest first.  Cordoned
// nodes (class 2) feed neither order and are not written.  The group's last chunk writes
// the segment bounds [start, start + untainted) and [end - tainted, end).
// Status words: flag << 62 | n1 << 28 | n0 (class counts < 2^28: nodes < 2^28) for chunk
// v = blockIdx.x in one of two arrays, ostat[par * n + v]; a decision uses array `par` and
// zeroes its chunk's word of the other, which the next decision (parity flipped by the
// host, a graph captured per parity) finds clear — no clearing launch (a memset before
// every decision cost ~6 µs of the 30).  The wait is bounded (OrdFail, esc_kernels.h): a
// chunk that gives up publishes OS_ERR — never an inclusive prefix it could not compute —
// so its group's later chunks give up at once, writes no output and sets the host-visible
// error word the runtime reports (ESC_E_ORDER) and clears.  A ticket for in-order chunk ids
// would serialise ~2 800 grabs on one word (≈ 32 µs: measured 49 µs per decision against
// 30 µs for the two-pass form).
constexpr uint64_t OS_AGG = 1ull << 62, OS_INC = 2ull << 62, OS_ERR = 3ull << 62;
constexpr uint32_t OS_M = (1u << 28) - 1;
__global__ __launch_bounds__(ORD_BLOCK) void k_ord_split(NodeDev N, const OrdChunk* __restrict__ chunks, int64_t n_chunks,
                                                         const uint32_t* __restrict__ g_memb,
                                                         const uint32_t* __restrict__ gch_off,
                                                         const uint32_t* __restrict__ grp_off,
                                                         uint64_t* __restrict__ ostat_all, int par,
                                                         uint32_t* __restrict__ vals, int64_t* __restrict__ seg,
                                                         OrdFail fail) {
    uint64_t* __restrict__ ostat = ostat_all + (par ? n_chunks : 0);
    uint64_t* __restrict__ onext = ostat_all + (par ? 0 : n_chunks);
    constexpr int STEPS = ORD_CHUNK / (4 * ORD_BLOCK);
    __shared__ uint32_t wt[STEPS][ORD_WAVES];
    __shared__ uint32_t stage[ORD_CHUNK];
    __shared__ uint32_t s_base[2], s_fail;
    const uint32_t v = blockIdx.x;
    const OrdChunk ch = chunks[v];
    if (threadIdx.x == 0) onext[v] = 0;                  // the next decision's word (last used two ago)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t gword = (ch.pad & ORD_CHUNK_DRY) ? NODE_DRY_BIT : 0u;   // ord_class's group word
    uint32_t packed[STEPS];
    uint4 nd[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        const uint32_t b = ch.start + st * 4 * ORD_BLOCK + 4 * threadIdx.x;
        nd[st] = ld4(g_memb + (b < ch.end ? b : ch.start));
    }
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {                 // one class byte per membership
        const uint32_t b = ch.start + st * 4 * ORD_BLOCK + 4 * threadIdx.x;
        packed[st] = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            packed[st] |= (b + j < ch.end ? ord_class(N, 0u, gword, lane4(nd[st], j) >> MEMB_FLAG_SHIFT) : 3u) << (8 * j);
    }
    uint32_t ex[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        uint32_t x = 0;                                  // class 0 | class 1 << 16
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = (packed[st] >> (8 * j)) & 0xFF;
            x += k == 0 ? 1u : (k == 1 ? 0x10000u : 0u);
        }
        const uint32_t inc = wave_incl_scan32(x);
        if (lane == 63) wt[st][wid] = inc;
        ex[st] = inc - x;
    }
    __syncthreads();
    uint32_t tot = 0;                                    // chunk totals (packed)
    uint32_t pre[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st)
#pragma unroll
        for (int w = 0; w < ORD_WAVES; ++w) {
            if (w == wid) pre[st] = tot;
            tot += wt[st][w];
        }
    const uint32_t n0 = tot & 0xFFFF, n1 = tot >> 16;
    const uint32_t g = ch.group, q0 = gch_off[g];
    if (threadIdx.x == 0)                                // the count first, then the look-back
        __hip_atomic_store(ostat + v, (v == q0 ? OS_INC : OS_AGG) | ((uint64_t)n1 << 28) | n0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // stage in chunk order: class 0 ascending at [0, n0), class 1 descending at [n0, n0 + n1)
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        const uint32_t x = pre[st] + ex[st];
        uint32_t r0 = x & 0xFFFF, r1 = n0 + n1 - 1 - (x >> 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = (packed[st] >> (8 * j)) & 0xFF;
            if (k == 0) stage[r0++] = lane4(nd[st], j) & MEMB_NODE_MASK;
            else if (k == 1) stage[r1--] = lane4(nd[st], j) & MEMB_NODE_MASK;
        }
    }
    if (wid == 0) {                                      // look back over the group's earlier chunks
        uint32_t e0 = 0, e1 = 0, spins = 0;
        bool failed = false;
        for (int64_t look = (int64_t)v - 1; look >= (int64_t)q0;) {
            if (++spins > fail.spins) {                  // never reached: every earlier chunk runs
                failed = true;
                break;
            }
            const int64_t jj = look - lane;
            const uint64_t w = jj >= (int64_t)q0 ? __hip_atomic_load(ostat + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                 : OS_INC;   // before the group: an inclusive 0
            const bool ready = (w >> 62) != 0;
            // the nearest inclusive (or failed) word ends the look-back
            const unsigned long long inc = __ballot((w >> 62) >= 2), wait = __ballot(!ready);
            const int fi = inc ? __builtin_ctzll(inc) : 63;
            const unsigned long long need = ~0ull >> (63 - fi);
            if (wait & need) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            if (inc && (__builtin_amdgcn_readlane((uint32_t)(w >> 32), fi) >> 30) == 3) {   // it gave up
                failed = true;
                break;
            }
            const bool mine = lane <= fi;
            e0 += wave_total32(mine ? (uint32_t)(w & OS_M) : 0u);
            e1 += wave_total32(mine ? (uint32_t)((w >> 28) & OS_M) : 0u);
            if (inc) break;
            look -= 64;
        }
        if (lane == 0) {
            const uint32_t t0 = e0 + n0, t1 = e1 + n1;
            s_fail = failed ? 1u : 0u;
            if (failed) {
                __hip_atomic_store(ostat + v, OS_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(fail.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                if (v != q0)
                    __hip_atomic_store(ostat + v, OS_INC | ((uint64_t)t1 << 28) | t0, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t s0 = grp_off[g], e = grp_off[g + 1];
                s_base[0] = s0 + e0;                     // class 0 output start
                s_base[1] = e - e1 - n1;                 // class 1 output start (stored descending)
                if (v + 1 == gch_off[g + 1]) {           // the group's last chunk: its bounds
                    seg[4 * (int64_t)g + 0] = s0;
                    seg[4 * (int64_t)g + 1] = (int64_t)s0 + t0;
                    seg[4 * (int64_t)g + 2] = (int64_t)e - t1;
                    seg[4 * (int64_t)g + 3] = e;
                }
            }
        }
    }
    __syncthreads();
    if (s_fail) return;                                  // no bases: nothing written
    const uint32_t b0 = s_base[0], b1 = s_base[1];
    for (uint32_t i = threadIdx.x; i < n0 + n1; i += ORD_BLOCK)
        __builtin_nontemporal_store(stage[i], vals + (i < n0 ? b0 + i : b1 + (i - n0)));   // read by the host only
}

// Small groups packed whole into one chunk (<= ORD_CHUNK memberships, regions start on
// quads): one pass, no cross-chunk prefix.  The chunk covers groups [ch.group, ch.group +
// ch.pad) (empty ones included); their region starts and dry flags are read once into LDS
// and every quad finds its group there by binary search (round 6: a group word per
// membership, 4 B read per membership and a dependent region-start load per quad, went).
// Classes are counted by one packed 64-bit block scan (class 0 | class 1 << 21 | class 2 <<
// 42) in membership order; a group's base is the scan value at its region's first quad (hp,
// indexed by quad), its class totals come from its region's last quad, and the output of
// group g lies in its own region: class 0 forward from its start, class 1 backward from its
// end (the split groups' layout, k_ord_split) — the chunk's own slots, so the nodes are
// staged in LDS and the chunk written back coalesced.  The last quad of each group writes its
// segment bounds.
// Inclusive 64-bit scan over the wave with DPP (see wave_total64).
__device__ __forceinline__ unsigned long long wave_incl_scan64(unsigned long long v) {
    v += dpp64<0x111, 0xF>(v);
    v += dpp64<0x112, 0xF>(v);
    v += dpp64<0x114, 0xF>(v);
    v += dpp64<0x118, 0xF>(v);
    v += dpp64<0x142, 0xA>(v);
    v += dpp64<0x143, 0xC>(v);
    return v;
}

// A packed ordering block's LDS (in k_step_tail, a member of the role union)
template <int STEPS>
struct OrdLds {
    static constexpr int CAP = STEPS * 4 * ORD_BLOCK;    // memberships per chunk
    unsigned long long wt[STEPS][ORD_WAVES];
    unsigned long long hp[CAP / 4];                      // scan value at each group's first quad
    uint32_t stage[CAP];
    uint32_t s_go[ORD_GCAP + 1];                         // the chunk's groups' region starts (+ the end)
    uint8_t s_dry[ORD_GCAP];
};
template <int STEPS>
__device__ __forceinline__ void ord_packed_block(const NodeDev& N, const OrdChunk* __restrict__ chunks,
                                                 const uint32_t* __restrict__ grp_off,
                                                 const uint8_t* __restrict__ dry,
                                                 const uint32_t* __restrict__ g_memb,
                                                 uint32_t* __restrict__ vals, int64_t* __restrict__ seg, int64_t blk,
                                                 OrdLds<STEPS>& S) {
    constexpr int C1 = 21, C2 = 42;
    constexpr unsigned long long M = (1ull << C1) - 1;
    auto& wt = S.wt;
    auto& hp = S.hp;
    auto& stage = S.stage;
    auto& s_go = S.s_go;
    auto& s_dry = S.s_dry;
    const OrdChunk ch = chunks[blk];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t g0 = ch.group, ng = ch.pad;           // ng <= ORD_GCAP (the host's chunking)
    uint4 nd[STEPS];                                     // region words
    bool ok[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        const uint32_t b = ch.start + st * 4 * ORD_BLOCK + 4 * threadIdx.x;
        ok[st] = b < ch.end;
        nd[st] = ld4(g_memb + (ok[st] ? b : ch.start));
    }
    for (uint32_t t = threadIdx.x; t <= ng; t += ORD_BLOCK) {
        s_go[t] = grp_off[g0 + t];
        if (t < ng) s_dry[t] = dry[g0 + t];
    }
    __syncthreads();
    // a quad lies in one group's region: the last table group starting at or before it (an
    // empty group shares its start with the next one, which is then the last)
    uint32_t gt[STEPS], grp[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        const uint32_t b = ch.start + st * 4 * ORD_BLOCK + 4 * threadIdx.x;
        uint32_t lo = 0, hi = ng - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_go[mid] <= b) lo = mid; else hi = mid - 1;
        }
        gt[st] = lo;
        grp[st] = (g0 + lo) | (s_dry[lo] ? NODE_DRY_BIT : 0u);
    }
    uint32_t cls[STEPS];
    unsigned long long ex[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        unsigned long long v = 0;
        cls[st] = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = ok[st] ? ord_class(N, 0u, grp[st], lane4(nd[st], j) >> MEMB_FLAG_SHIFT) : 3u;
            cls[st] |= k << (8 * j);
            v += k == 0 ? 1ull : (k == 1 ? (1ull << C1) : (k == 2 ? (1ull << C2) : 0ull));
        }
        const unsigned long long inc = wave_incl_scan64(v);
        if (lane == 63) wt[st][wid] = inc;
        ex[st] = inc - v;
    }
    __syncthreads();
    unsigned long long tot = 0, pre[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st)
#pragma unroll
        for (int w = 0; w < ORD_WAVES; ++w) {
            if (w == wid) pre[st] = tot;
            tot += wt[st][w];
        }
    // group heads publish their base; every quad then finds its group's head by address
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        ex[st] += pre[st];                               // exclusive scan value of this quad
        const uint32_t b = ch.start + st * 4 * ORD_BLOCK + 4 * threadIdx.x;
        if (ok[st] && b == s_go[gt[st]]) hp[(b - ch.start) >> 2] = ex[st];
    }
    __syncthreads();
    uint32_t hq[STEPS];
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        const uint32_t b = ch.start + st * 4 * ORD_BLOCK + 4 * threadIdx.x;
        if (!ok[st]) continue;
        const uint32_t g = mg(grp[st]);
        hq[st] = (s_go[gt[st]] - ch.start) >> 2;
        const uint32_t end = s_go[gt[st] + 1];
        if (b + 4 == end) {                              // the group's last quad: totals + bounds
            unsigned long long inc = ex[st];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = (cls[st] >> (8 * j)) & 0xFF;
                inc += k == 0 ? 1ull : (k == 1 ? (1ull << C1) : (k == 2 ? (1ull << C2) : 0ull));
            }
            const unsigned long long t = inc - hp[hq[st]];
            const int64_t s0 = s_go[gt[st]], t0 = (int64_t)(t & M), t1 = (int64_t)((t >> C1) & M);
            seg[4 * (int64_t)g + 0] = s0;                // untainted forward from the start,
            seg[4 * (int64_t)g + 1] = s0 + t0;           // tainted newest first at the end
            seg[4 * (int64_t)g + 2] = (int64_t)end - t1;
            seg[4 * (int64_t)g + 3] = end;
        }
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
        if (!ok[st]) continue;
        const unsigned long long base = hp[hq[st]];
        const uint32_t s0 = (hq[st] << 2);               // the group's first slot, chunk-relative
        const uint32_t e1 = s_go[gt[st] + 1] - ch.start - 1;           // its last slot
        uint32_t r0 = (uint32_t)((ex[st] - base) & M), r1 = (uint32_t)(((ex[st] - base) >> C1) & M);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = (cls[st] >> (8 * j)) & 0xFF;
            if (k == 0) stage[s0 + r0++] = lane4(nd[st], j) & MEMB_NODE_MASK;
            else if (k == 1) stage[e1 - r1++] = lane4(nd[st], j) & MEMB_NODE_MASK;   // newest first at the end
        }
    }
    __syncthreads();
    const uint32_t n = ch.end - ch.start;
    for (uint32_t i = 4 * threadIdx.x; i < n; i += 4 * ORD_BLOCK)
        __builtin_nontemporal_store(*reinterpret_cast<const v4u32*>(stage + i), reinterpret_cast<v4u32*>(vals + ch.start + i));
}

template <int STEPS>
__global__ __launch_bounds__(ORD_BLOCK) void k_ord_packed(NodeDev N, const OrdChunk* __restrict__ chunks,
                                                          const uint32_t* __restrict__ grp_off,
                                                          const uint8_t* __restrict__ dry,
                                                          const uint32_t* __restrict__ g_memb,
                                                          uint32_t* __restrict__ vals, int64_t* __restrict__ seg) {
    __shared__ OrdLds<STEPS> lds;
    ord_packed_block<STEPS>(N, chunks, grp_off, dry, g_memb, vals, seg, blockIdx.x, lds);
}

// The step's tail in ONE launch (horizontal fusion; every role is 256 threads and none
// waits on another): blocks [0, n_col) fold the K1 partials into the pod words (fold_col),
// the next ones reduce the node pieces and the dry-mode tracker entries (K2,
// node_piece_block), the last ones order the packed small groups (K5, ord_packed_block).
// Before, K2 and K5 ran on a side stream beside K1: K1 holds every CU's LDS and its loads
// starve K2's latency-bound waves, so the side chain ended after K1 and the cross-stream
// join cost ~10 us more (profiles/r02_v9 timeline): ~45 us after K1 at any pod count.


// The step's tail in ONE launch (horizontal fusion; every role is 256 threads): the K2
// node-piece blocks, the dry-mode tracker blocks, the K3 fold columns and the K5 packed
// small-group orderings, in that block order — the longest chains first (at config 4
// the grid is ~2.5 k blocks for ~1.3 k resident slots, and the short ordering blocks fill
// the second round).  (Before, K2 and K5
// ran on a side stream beside K1: K1 holds every CU's LDS and its loads starve K2's
// latency-bound waves, so the side chain ended after K1 and the cross-stream join cost
// ~10 us more (profiles/r02_v9 timeline): ~45 us after K1 at any pod count.)
// k_step_tail's blocks per CU the compiler must allow: 6 caps its VGPRs at 80 (84 unbounded:
// 5 blocks; 12 B spilled); with the roles' LDS overlaid (18.7 KB) 6 blocks fit.  r06o: the
// config-4 tail 20.8-21.5 -> 19.6-19.7 us (stage events); 8 (64 VGPRs) spilled 76 B and
// took 30 us.  0 = no bound (timing builds)
#ifndef ESC_TAIL_MINB
#define ESC_TAIL_MINB 6
#endif
#if ESC_TAIL_MINB > 0
#define TAIL_BOUNDS __launch_bounds__(256, ESC_TAIL_MINB)
#else
#define TAIL_BOUNDS __launch_bounds__(256)
#endif
__global__ TAIL_BOUNDS void k_step_tail(GroupDev G, NodeDev N, FoldPlan F, int64_t* __restrict__ wide_pod,
                                                   int64_t* __restrict__ pwords, int64_t nb_pieces, int64_t n_piece_blk,
                                                   int64_t* __restrict__ rows, int64_t* __restrict__ trk_acc,
                                                   const OrdChunk* __restrict__ chunks, int64_t n_small,
                                                   const uint32_t* __restrict__ grp_off,
                                                   const uint32_t* __restrict__ g_memb,
                                                   uint32_t* __restrict__ vals, int64_t* __restrict__ seg) {
    static_assert(FD_WAVES * 64 == 256 && K2_WAVES * 64 == 256 && ORD_BLOCK == 256, "one block size for every role");
    // the roles' LDS overlaid: a block takes one role, so its LDS is the largest role's (the
    // arrays of all roles side by side were 27.4 KB, which with 84 VGPRs held 5 blocks per CU)
#ifndef ESC_TAIL_NOUNION
    __shared__ union {
        FoldLds fold;
        OrdLds<ORD_PCHUNK / (4 * ORD_BLOCK)> ord;
    } lds;
#else                                                    // (timing builds: the roles' arrays side by side)
    __shared__ struct {
        FoldLds fold;
        OrdLds<ORD_PCHUNK / (4 * ORD_BLOCK)> ord;
    } lds;
#endif
    const int64_t b = blockIdx.x;
#if ESC_MEASURE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    // F.ablate (ESC_K3_ABLATE, timing-only, wrong results): 8 / 16 / 32 skip the fold /
    // node-piece / ordering role, 64 the dry-mode tracker blocks, 128 K2's row stores
    if (b < n_piece_blk) {
        const int64_t pb = b;
        if (!(F.ablate & 16) && !((F.ablate & 64) && pb >= nb_pieces))
            node_piece_block(N, G, nb_pieces, (F.ablate & 128) ? nullptr : rows, trk_acc, pb);
    } else if (b < n_piece_blk + F.n_col) {
        const uint32_t col = (uint32_t)(b - n_piece_blk);
        if (!(F.ablate & 8)) fold_col(G, F, wide_pod, pwords, (int)col, lds.fold);
    } else if (!(F.ablate & 32)) {
        ord_packed_block<ORD_PCHUNK / (4 * ORD_BLOCK)>(N, chunks, grp_off, G.dry, g_memb, vals, seg,
                                                       b - n_piece_blk - F.n_col, lds.ord);
    }
#if ESC_MEASURE
    if (F.trace) {                                       // {start, end, role: 0 pieces, 1 tracker, 2 fold, 3 ordering}
        __syncthreads();
        if (threadIdx.x == 0) {
            F.trace[3 * b] = t_start;
            F.trace[3 * b + 1] = __builtin_amdgcn_s_memrealtime();
            F.trace[3 * b + 2] = b < nb_pieces ? 0 : b < n_piece_blk ? 1 : b < n_piece_blk + F.n_col ? 2 : 3;
        }
    }
#endif
}

// Region padding: MEMB_PAD_WORD after each group's memberships (node 0, flagged absent:
// class 3 from the region word alone, k_ord_split and the packed orderings).
__global__ __launch_bounds__(256) void k_region_pad(const uint32_t* __restrict__ pstart,
                                                    const uint32_t* __restrict__ plen, int32_t G,
                                                    uint32_t* __restrict__ g_memb, int64_t* __restrict__ seg) {
    const int32_t g = blockIdx.x;
    if (g >= G) return;
    // the ordering's segment starts (the sort's last pass read seg as the unpadded starts):
    // all four of the group's at its region start
    if (threadIdx.x < 4) seg[4 * (int64_t)g + threadIdx.x] = pstart[g];
    if (g == 0 && threadIdx.x == 4) seg[4 * (int64_t)G] = pstart[G];
    for (uint32_t i = pstart[g] + plen[g] + threadIdx.x; i < pstart[g + 1]; i += blockDim.x) g_memb[i] = MEMB_PAD_WORD;
}

// Start of each (group, class) segment in the partitioned keys: seg[s] = first key >= s.

// ===================================================================== snapshot patches
// Incremental snapshot updates (esc_pods_upsert / esc_pods_delete / esc_nodes_update):
// element writes into the resident arrays; where[i] = target << 60 | index, targets 0-5
// are 4-byte arrays, 6-11 8-byte ones.  The host dedupes (target, index) first.
__global__ __launch_bounds__(256) void k_patch(PatchTargets T, const uint64_t* __restrict__ where,
                                               const uint64_t* __restrict__ what, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t w = where[i];
    const uint32_t t = (uint32_t)(w >> 60);
    const int64_t idx = (int64_t)(w & ((1ull << 60) - 1));
    if (t < 6) T.u32[t][idx] = (uint32_t)what[i];
    else if (t < 12) T.i64[t - 6][idx] = (int64_t)what[i];
    else T.u16[t - 12][idx] = (uint16_t)what[i];
}

// ===================================================================== scale-down reaping
// §8f rank 2: TryRemoveTaintedNodes (scale_down.go:51-136) for every group.
namespace {
// The pod behind device slot d, as a PodRef (pairs inline, or indirect for big C pods).
__device__ PodRef podref_of(const PodDev& P, uint32_t d) {
    PodRef r;
    r.p[0] = r.p[1] = r.p[2] = NONE;
    const int64_t kpods = P.k_tiles * TILE;
    if ((int64_t)d < kpods) {
        const int64_t t = d / TILE, sl = d % TILE;
        int lo = 0, hi = P.n_cls - 1;                      // class of tile t
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (P.cls[mid].t0 <= t) lo = mid; else hi = mid - 1;
        }
        const PodClass& C = P.cls[lo];
        const int64_t blk = kb_block(C, t);
        const KHead hd = kb_head(C, P.kb, blk, sl);
        r.flags = hd.flags;
        r.pair0 = hd.pair0;
        for (uint32_t k = 0; k < C.nxp && k < 3; ++k) r.p[k] = kb_pair(C, P.kb, blk, k, sl);
    } else {
        const int64_t c = (int64_t)d - kpods, t = c / CTILE, l = c % CTILE;
        r.flags = P.flags[c];
        r.pair0 = P.pair0[c];
        uint32_t off = P.xp_base[t];
        for (int64_t k = 0; k < l; ++k) off += pf_xpair(P.flags[t * CTILE + k]);
        const uint32_t nx = pf_xpair(r.flags);
        if (nx <= 3) {
            for (uint32_t k = 0; k < nx; ++k) r.p[k] = P.xp[off + k];
        } else {
            r.flags |= POD_REF_INDIRECT;
            r.p[0] = off;
            r.p[1] = nx;
        }
    }
    return r;
}

__device__ __forceinline__ bool podref_has(const PodRef& r, const uint32_t* xp, uint32_t q) {
    if (r.pair0 == q) return true;
    if (r.flags & POD_REF_INDIRECT) {
        for (uint32_t k = 0; k < r.p[1]; ++k) if (xp[r.p[0] + k] == q) return true;
        return false;
    }
    return r.p[0] == q || r.p[1] == q || r.p[2] == q;
}

// Go's time.Time.Sub saturates at the int64 Duration range.
__device__ __forceinline__ int64_t go_sub_ns(int64_t now_ns, int64_t t_s) {
    const __int128 d = (__int128)now_ns - (__int128)t_s * 1000000000;
    return d > (__int128)INT64_MAX ? INT64_MAX : (d < (__int128)INT64_MIN ? INT64_MIN : (int64_t)d);
}
}  // namespace

// PodRef of the pod in each listed slot, at position i (a whole placement) or run_pos[i]
// (pod events patching runs in place).
__global__ __launch_bounds__(256) void k_podref_fill(PodDev P, const uint32_t* __restrict__ run_slot, int64_t n,
                                                     const uint32_t* __restrict__ run_pos, PodRef* __restrict__ refs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) refs[run_pos ? (int64_t)run_pos[i] : i] = podref_of(P, run_slot[i]);
}

// K6: one wave per 64 pair-major entries; the entries whose node is escalator-tainted and
// not cordoned (the only nodes a wet group can reap) are taken in turn by the whole wave,
// which counts the node's pods that the entry's pair filter selects
// (NewPodAffinityFilterFunc: the pair among the pod's pairs) and that the default filter
// selects, daemonsets excluded — NodePodsRemaining over the group's NodeInfoMap, which
// only holds the group's own pods (controller.go:259, node_state.go:48-65).
__global__ __launch_bounds__(256) void k_occupancy(NodeDev N, GroupDev G, RemovalDev R) {
    const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
    const int lane = threadIdx.x & 63;
    const int64_t e = base + lane;
    bool want = false;
    uint32_t j = 0, q = 0;
    if (e < R.n_entries) {
        const uint32_t f = N.e_flags[e];
        q = R.e_pair[e];
        j = N.e_node[e];
        // every live entry: the words are kept current by events from here on, and any
        // node may become wet-tainted later
        want = q < G.n_gp && !(f & ESC_NF_ABSENT);
        if (!want) { R.occ_pair[e] = 0; R.occ_def[e] = 0; }
    }
    // the wave's entries two at a time: both nodes' PodRef runs are loaded
    // before either is reduced (DPP sums, no ds_bpermute chains)
    unsigned long long m = __ballot(want);
    while (m) {
        const int k0 = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int k1 = m ? __ffsll((long long)m) - 1 : -1;
        if (m) m &= m - 1;
        const uint32_t j0 = (uint32_t)__builtin_amdgcn_readlane((int)j, k0), q0 = (uint32_t)__builtin_amdgcn_readlane((int)q, k0);
        const uint32_t j1 = k1 >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)j, k1) : j0;
        const uint32_t q1 = k1 >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)q, k1) : q0;
        const uint32_t a0 = R.nrun_off[j0], n0 = R.nrun_len[j0];
        const uint32_t a1 = R.nrun_off[j1], n1 = k1 >= 0 ? R.nrun_len[j1] : 0u;
        uint32_t cp0 = 0, cd0 = 0, cp1 = 0, cd1 = 0;
        const uint32_t nmax = n0 > n1 ? n0 : n1;
        for (uint32_t i = lane; i < nmax; i += 64) {
            PodRef r0, r1;
            if (i < n0) r0 = R.refs[a0 + i];
            if (i < n1) r1 = R.refs[a1 + i];
            if (i < n0 && !(r0.flags & ESC_PF_DAEMONSET)) {
                cp0 += podref_has(r0, R.xp, q0) ? 1u : 0u;
                cd0 += pf_default_ok(r0.flags & ~POD_REF_INDIRECT) ? 1u : 0u;
            }
            if (i < n1 && !(r1.flags & ESC_PF_DAEMONSET)) {
                cp1 += podref_has(r1, R.xp, q1) ? 1u : 0u;
                cd1 += pf_default_ok(r1.flags & ~POD_REF_INDIRECT) ? 1u : 0u;
            }
        }
        cp0 = wave_total32(cp0); cd0 = wave_total32(cd0);
        if (lane == k0) { R.occ_pair[e] = cp0; R.occ_def[e] = cd0; }
        if (k1 >= 0) {
            cp1 = wave_total32(cp1); cd1 = wave_total32(cd1);
            if (lane == k1) { R.occ_pair[e] = cp1; R.occ_def[e] = cd1; }
        }
    }
}

// Occupancy deltas of pod events (launch_occ_delta): one thread per PodRef placement.
__global__ __launch_bounds__(256) void k_occ_delta(GroupDev G, RemovalDev R, const uint32_t* __restrict__ ne_off,
                                                   const uint32_t* __restrict__ ne_pos, const uint32_t* __restrict__ pos,
                                                   const uint32_t* __restrict__ node, int64_t n, int sign) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PodRef r = R.refs[pos[i]];
    if (r.flags & ESC_PF_DAEMONSET) return;                   // NodePodsRemaining skips daemonsets
    const bool dflt = pf_default_ok(r.flags & ~POD_REF_INDIRECT);
    const uint32_t j = node[i], d = (uint32_t)sign;
    for (uint32_t k = ne_off[j]; k < ne_off[j + 1]; ++k) {
        const uint32_t e = ne_pos[k];
        if (podref_has(r, R.xp, R.e_pair[e])) atomicAdd(R.occ_pair + e, d);
        if (dflt) atomicAdd(R.occ_def + e, d);
    }
}
// One wave per group over its pair's entries (pair-major, e_flags / e_node / the occupancy
// word contiguous), the next 64 entries' loads in flight while this chunk's nodes' taint
// times are read: one dependent load per chunk instead of two.  The record goes back
// compact (RmRec, 16 B; the host widens it to esc_removal).
__global__ __launch_bounds__(64) void k_try_remove(NodeDev N, GroupDev G, RemovalDev R) {
    const int32_t g = blockIdx.x;
    const int lane = threadIdx.x;
    const uint32_t q = G.gpair[g];
    const bool dry = G.dry[g] != 0, dflt = (uint32_t)g == G.default_group;
    const uint32_t* __restrict__ occw = dflt ? R.occ_def : R.occ_pair;
    const int64_t e0 = N.piece_off[N.pp_off[q]], e1 = N.piece_off[N.pp_off[q + 1]];
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t m = (uint32_t)g | (dry ? NODE_DRY_BIT : 0u);
    const int64_t soft = R.soft_ns[g], hard = R.hard_ns[g];
    uint32_t cand = 0, del = 0;
    int64_t pods = 0;
    uint32_t f = ESC_NF_ABSENT, j = 0, o = 0;
    if (e0 + lane < e1) { f = N.e_flags[e0 + lane]; j = N.e_node[e0 + lane]; o = occw[e0 + lane]; }
    for (int64_t b = e0; b < e1; b += 64) {
        const int64_t en = b + 64 + lane;
        uint32_t nf = ESC_NF_ABSENT, nj = 0, no = 0;
        if (en < e1) { nf = N.e_flags[en]; nj = N.e_node[en]; no = occw[en]; }
        const bool c = node_class(N, f, (int64_t)j, m) == 1;          // filterNodes: tainted (absent: 3)
        bool d = false;
        if (c && !dry) {
            const int64_t ts = R.taint_s[j];
            if (!R.no_delete[j] && ts != INT64_MIN) {
                const int64_t age = go_sub_ns(R.now_ns, ts);
                d = age > soft && (o == 0 || age > hard);
            }
        }
        const unsigned long long md = __ballot(d);
        if (d) R.rm_list[R.rm_off[g] + del + __popcll(md & lt)] = j;
        del += (uint32_t)__popcll(md);
        cand += (uint32_t)__popcll(__ballot(c));
        pods += (int64_t)wave_total64(d ? (unsigned long long)o : 0ull);
        f = nf; j = nj; o = no;
    }
    if (lane == 0) R.out[g] = RmRec{cand, del, pods};
}

// ===================================================================== launchers
hipError_t launch_pod_bigtiles(const PodDev& p, const GroupDev& g, const uint32_t* tiles, int64_t n_big,
                               int64_t* wide, hipStream_t st) {
    if (n_big <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pod_bigtiles, dim3((unsigned)n_big), dim3(64), 0, st, p, g, tiles, wide);
    return hipGetLastError();
}

hipError_t launch_node_groups(const GroupDev& g, const NodeDev& n, const GroupList& list, const int64_t* node_rows,
                              int64_t* trk_acc, int64_t* nwords, const NGDecide& nd, hipStream_t st) {
    if (list.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_node_groups, dim3((list.n + 63) / 64), dim3(NG_WAVES * 64), 0, st, g, n, list, node_rows,
                       trk_acc, nwords, nd);
    return hipGetLastError();
}

namespace {
constexpr int PEER_MAX = 16;
template <class T>
struct PeerSrc {
    const T* p[PEER_MAX];
};
// dst = the sum of every source buffer (the sources are other devices' memory, peer-mapped,
// or the same device's): 16-B loads where the words allow, one pass.
template <class T>
__global__ __launch_bounds__(256) void k_peer_sum(PeerSrc<T> S, int n_src, T* __restrict__ dst, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        T a = 0;
        for (int k = 0; k < n_src; ++k) a += S.p[k][i];
        dst[i] = a;
    }
}
template <class T>
hipError_t peer_sum(const T* const* src, int n_src, T* dst, int64_t n, hipStream_t st) {
    if (n_src < 1 || n_src > PEER_MAX) return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    PeerSrc<T> S{};
    for (int k = 0; k < n_src; ++k) S.p[k] = src[k];
    const unsigned blocks = (unsigned)std::min<int64_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_peer_sum<T>, dim3(blocks), dim3(256), 0, st, S, n_src, dst, n);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_peer_sum64(const int64_t* const* src, int n_src, int64_t* dst, int64_t n, hipStream_t st) {
    return peer_sum<int64_t>(src, n_src, dst, n, st);
}
hipError_t launch_peer_sum32(const uint32_t* const* src, int n_src, uint32_t* dst, int64_t n, hipStream_t st) {
    return peer_sum<uint32_t>(src, n_src, dst, n, st);
}

int64_t tail_span_blocks(const NodeDev& n) { return (n.n_spans + K2_WAVES - 1) / K2_WAVES; }
int64_t tail_trk_blocks(const NodeDev& n) { return (n.n_trk + K2_WAVES * 64 - 1) / (K2_WAVES * 64); }

hipError_t launch_step_tail(const GroupDev& g, const NodeDev& n, const FoldPlan& f, bool spans, int64_t* wide_pod,
                            int64_t* pwords, int64_t* rows, int64_t* trk_acc, const OrdChunk* chunks, int64_t n_small,
                            const uint32_t* grp_off, const uint32_t* g_memb,
                            uint32_t* vals, int64_t* seg, hipStream_t st) {
    const int64_t nb = spans ? tail_span_blocks(n) : 0;      // else K1 made the rows
    const int64_t nt = tail_trk_blocks(n);
    const int64_t grid = f.n_col + nb + nt + std::max<int64_t>(n_small, 0);
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_step_tail, dim3((unsigned)grid), dim3(256), 0, st, g, n, f, wide_pod, pwords, nb, nb + nt, rows,
                       trk_acc, chunks, std::max<int64_t>(n_small, 0), grp_off, g_memb, vals, seg);
    return hipGetLastError();
}

hipError_t launch_podref_fill(const PodDev& p, const uint32_t* run_slot, const uint32_t* run_pos, int64_t n, PodRef* refs,
                              hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_podref_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, run_slot, n, run_pos, refs);
    return hipGetLastError();
}

hipError_t launch_occ_delta(const GroupDev& g, const RemovalDev& r, const uint32_t* ne_off, const uint32_t* ne_pos,
                            const uint32_t* pos, const uint32_t* node, int64_t n, int sign, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_occ_delta, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, r, ne_off, ne_pos, pos, node, n,
                       sign);
    return hipGetLastError();
}

hipError_t launch_occupancy(const NodeDev& n, const GroupDev& g, const RemovalDev& r, hipStream_t st) {
    if (r.n_entries > 0)
        hipLaunchKernelGGL(k_occupancy, dim3((unsigned)((r.n_entries + 255) / 256)), dim3(256), 0, st, n, g, r);
    return hipGetLastError();
}

hipError_t launch_try_remove(const NodeDev& n, const GroupDev& g, const RemovalDev& r, hipStream_t st) {
    hipLaunchKernelGGL(k_try_remove, dim3(g.G), dim3(64), 0, st, n, g, r);
    return hipGetLastError();
}

hipError_t launch_patch(const PatchTargets& t, const uint64_t* where, const uint64_t* what, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_patch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, t, where, what, n);
    return hipGetLastError();
}

hipError_t launch_wide_pods(const PodDev& p, const GroupDev& g, int64_t* wide, hipStream_t st) {
    hipLaunchKernelGGL(k_pod_wide, dim3(1024), dim3(256), 0, st, p, g, wide);
    return hipGetLastError();
}


namespace {
int rs_blocks(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(ESC_RS_MAXBLK, (n + 8 * SORT_BLOCK - 1) / (8 * SORT_BLOCK)));
}

template <class KT, class VT, int BITS, bool FINAL = false>
hipError_t rs_pass(const KT* kin, const VT* vin, KT* kout, VT* vout, int64_t n, int shift, uint32_t* hist,
                   uint32_t* tot, const RegionSink& S, hipStream_t st) {
    const int nblk = rs_blocks(n), nb = 1 << BITS;
    hipLaunchKernelGGL((k_rs_hist<KT, BITS>), dim3(nblk), dim3(SORT_BLOCK), 0, st, kin, n, shift, hist);
    hipLaunchKernelGGL(k_rs_scan_rows, dim3((nb + 3) / 4), dim3(256), 0, st, hist, nblk, nb, tot);
    hipLaunchKernelGGL((k_rs_scatter<KT, VT, BITS, FINAL>), dim3(nblk), dim3(SORT_BLOCK), 0, st, kin, vin, kout, vout, n,
                       shift, hist, tot, S);
    return hipGetLastError();
}

// LSD passes over bits [0, bits) of keys[0] / vals[0] (ping-pong with [1]); returns the
// buffer index holding the result (the last pass writes the regions of S instead).
// The bits are split evenly over ceil(bits / 8) passes (9 bits -> 5 + 4, 41 -> 7 x 5 + 6):
// narrower digits cost the scatter fewer LDS histogram words per element at equal traffic.
template <class KT, class VT>
hipError_t rs_sort(KT* keys[2], VT* vals[2], int64_t n, int bits, uint32_t* hist, uint32_t* tot, int* src,
                   const RegionSink& S, hipStream_t st, int lo_bit = 0) {
    *src = 0;
    // digits of at most 8 bits (9-bit digits were measured: the scatter's per-chunk digit
    // bookkeeping grows with the bins, 5 passes of 8-9 bits took longer than 6 of 6-7);
    // the key is bits [lo_bit, lo_bit + bits) of the element
    const int passes = (bits + 7) / 8;
    for (int p = 0, shift = lo_bit; p < passes; ++p) {
        const int w = (lo_bit + bits - shift + (passes - p) - 1) / (passes - p);
        hipError_t e;
        KT *ki = keys[*src], *ko = keys[*src ^ 1];
        VT *vi = vals[*src], *vo = vals[*src ^ 1];
        if (p + 1 < passes) {
            switch (w) {
                case 1: case 2: case 3: case 4: e = rs_pass<KT, VT, 4>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                case 5: e = rs_pass<KT, VT, 5>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                case 6: e = rs_pass<KT, VT, 6>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                case 7: e = rs_pass<KT, VT, 7>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                default: e = rs_pass<KT, VT, 8>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
            }
        } else {
            switch (w) {
                case 1: case 2: case 3: case 4: e = rs_pass<KT, VT, 4, true>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                case 5: e = rs_pass<KT, VT, 5, true>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                case 6: e = rs_pass<KT, VT, 6, true>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                case 7: e = rs_pass<KT, VT, 7, true>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
                default: e = rs_pass<KT, VT, 8, true>(ki, vi, ko, vo, n, shift, hist, tot, S, st); break;
            }
        }
        if (e != hipSuccess) return e;
        *src ^= 1;
        shift += w;
    }
    return hipSuccess;
}
}  // namespace

size_t sort_hist_words(int64_t n) { return (size_t)256 * rs_blocks(n); }

size_t memb_status_words(int64_t n) { return (size_t)((n + MEMB_BLOCK * MEMB_U - 1) / (MEMB_BLOCK * MEMB_U)) + 1; }

hipError_t launch_age_sort(const NodeDev& nd, const GroupDev& g, uint64_t* status, uint32_t* total, int64_t n_memb,
                           int64_t cap, int64_t ts_min, uint64_t div, int R, int gbits, int coarse_shift,
                           uint64_t* keys[2], uint32_t* vals[2], uint32_t* hist, uint32_t* tot, const RegionSink& S,
                           hipStream_t st) {
    const int64_t n = nd.hi - nd.lo;
    const size_t nst = memb_status_words(n);
    const dim3 tiles((unsigned)(nst - 1));
    // (status: zeroed by the caller, with the index's other tables in one upload)
    if (coarse_shift < 0) {                          // exact 64-bit keys: group << R | offset
        if (n > 0)
            hipLaunchKernelGGL(k_memb_keys<uint64_t>, tiles, dim3(MEMB_BLOCK), 0, st, nd, g, n, status, total, S.err, S.spins, cap, ts_min,
                               div, R, 0, keys[0], vals[0]);
        if (n_memb > 0) {
            int src = 0;
            const hipError_t e = rs_sort<uint64_t, uint32_t>(keys, vals, n_memb, R + gbits, hist, tot, &src, S, st);
            if (e != hipSuccess) return e;
        }
        return hipGetLastError();
    }
    // coarse 32-bit keys: group << (32 - gbits) | (offset >> coarse_shift), packed with the
    // value into ONE 8-B element (key << 32 | value: one stream, whole 128-B lines per carried
    // digit run), sorted on the element's top 32 bits; then k_age_fix orders each run of
    // equal coarse keys by the exact creation time
    if (n > 0)
        hipLaunchKernelGGL((k_memb_keys<uint64_t, true>), tiles, dim3(MEMB_BLOCK), 0, st, nd, g, n, status, total, S.err, S.spins, cap,
                           ts_min, div, 32 - gbits, coarse_shift, keys[0], nullptr);
    if (n_memb > 0) {
        int src = 0;
        NoVal* nv[2] = {nullptr, nullptr};
        const hipError_t e = rs_sort<uint64_t, NoVal>(keys, nv, n_memb, 32, hist, tot, &src, S, st, 32);
        if (e != hipSuccess) return e;
        if (S.fix)                                   // the final pass's coarse keys (u32) in keys[src]
            hipLaunchKernelGGL(k_age_fix, dim3((unsigned)std::min<int64_t>(4096, (n_memb + 1023) / 1024)), dim3(256), 0, st,
                               reinterpret_cast<const uint32_t*>(keys[src]), n_memb, S, nd.created, nd.hi, ts_min);
    }
    return hipGetLastError();
}

hipError_t launch_order_packed(const NodeDev& nd, const OrdChunk* chunks, int64_t n_chunks, int64_t n_small,
                               const uint32_t* grp_off, const uint8_t* dry, const uint32_t* g_memb,
                               uint32_t* vals, int64_t* seg, hipStream_t st) {
    if (n_chunks <= 0) return hipSuccess;
    // chunks [0, n_small) hold <= ORD_PCHUNK memberships, the rest <= ORD_CHUNK
    if (n_small > 0)
        hipLaunchKernelGGL(k_ord_packed<ORD_PCHUNK / (4 * ORD_BLOCK)>, dim3((unsigned)n_small), dim3(ORD_BLOCK), 0, st,
                           nd, chunks, grp_off, dry, g_memb, vals, seg);
    if (n_chunks > n_small)
        hipLaunchKernelGGL(k_ord_packed<ORD_CHUNK / (4 * ORD_BLOCK)>, dim3((unsigned)(n_chunks - n_small)),
                           dim3(ORD_BLOCK), 0, st, nd, chunks + n_small, grp_off, dry, g_memb, vals, seg);
    return hipGetLastError();
}

hipError_t launch_region_pad(const uint32_t* pstart, const uint32_t* plen, int32_t G, uint32_t* g_memb, int64_t* seg,
                             hipStream_t st) {
    if (G <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_region_pad, dim3((unsigned)G), dim3(256), 0, st, pstart, plen, G, g_memb, seg);
    return hipGetLastError();
}

hipError_t launch_order(const NodeDev& nd, const OrdChunk* chunks, int64_t n_chunks, const uint32_t* gch_off,
                        const uint32_t* grp_off, const uint32_t* g_memb, uint64_t* ostat, int par, uint32_t* vals,
                        int64_t* seg, const OrdFail& fail, hipStream_t st) {
    if (n_chunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ord_split, dim3((unsigned)n_chunks), dim3(ORD_BLOCK), 0, st, nd, chunks, n_chunks, g_memb,
                       gch_off, grp_off, ostat, par, vals, seg, fail);
    return hipGetLastError();
}

#endif  // ESC_PART == 0

}  // namespace esc
