// esc_kernels.h — device-side argument blocks and launch wrappers (esc_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "esc_common.h"

namespace esc {

// A class of homogeneous pod tiles: every pod of the class has the same record
// signature (extra regular containers, init containers, overhead, extra pairs), so every
// field and record k of a tile's 256 pods is one contiguous 256-entry row.
struct PodClass {
    int64_t t0, t1;            // tiles [t0, t1) of the K section
    int64_t kb0, rsv;          // u32-word offset of tile t0's block in the K-block array
    int64_t w0;                // K1 work weight of the tiles before t0
    uint32_t xreg, xinit, ovh, nxp;
    uint32_t kind;             // packed * 16 + (xreg + xinit + ovh) * 4 + nxp: selects K1's pipeline
    uint32_t wt;               // work weight of one tile: its 16-B loads per lane (= block KB)
    uint32_t packed;           // 0 plain, 1 packed (12 B / pod), 2 packed small (8 B / pod): kp_*, kp8_* below
    uint32_t pad;
};
// weight of a K tile with R records and NXP extra pairs per pod: its block size in half-KB
// units (128 u32 words; the packed small block's u16 pair rows are half a KB each)
constexpr uint32_t k_tile_weight(uint32_t R, uint32_t NXP, uint32_t packed = 0) {
    return packed == 2 ? 4 + 4 * R + NXP : (packed ? 2 * (3 + 2 * R + NXP) : 2 * (5 + 4 * R + NXP));
}
constexpr uint32_t K_TILE_WEIGHT_MIN = 4;   // the lightest tile (packed small, no records or pairs)
constexpr int64_t KB_UNIT = 128;            // u32 words per weight unit
constexpr int POD_SIG_IDS = 128;     // signatures with <= 3 extra records and <= 3 extra pairs
constexpr int POD_CLASS_IDS = 384;   // class id = signature | packed << 7
constexpr int K1_SEGS = 4;           // class runs per K1 workgroup in the work plan (at most)

// K blocks (tile-major K section).  Tile t of a class is ONE contiguous block of wt KB
// (wt = 5 + 4R + NXP): a wave streams a tile as wt consecutive 1-KB wave-loads from one
// address range instead of wt loads from 4 + 2R + 1 separate arrays (the SoA streams cost
// 6.5 % at 100 M pods and 4 % at 12.5 M in scripts/k1_shape_probe.hip, profiles/r02_v8).
// Word offsets inside a block (u32 words; 8-byte rows are 512 words = 256 entries):
//   flags [0, 256)  cpu0 [256, 512)  mem0 [512, 1024)  pair0 [1024, 1280)
//   record k: cpu [1280 + 1024k, +512), mem [+512, +1024)   extra pair k: [1280 + 1024R + 256k, +256)
// 4-byte rows hold pod s at entry s; 8-byte rows at pos64(s) = (s%4/2)*128 + 2(s/4) + s%2,
// so that lane l's 16-B load of either width covers its pods 4l..4l+3 and every wave-load
// reads one contiguous 1 KB.
constexpr int KB_CPU0 = 256, KB_MEM0 = 512, KB_PAIR0 = 1024, KB_REC = 1280;
__host__ __device__ inline int64_t kb_pos64(int64_t s) { return ((s & 3) >> 1) * 128 + 2 * (s >> 2) + (s & 1); }
// first word of tile t's block (t a tile of class C)
__host__ __device__ inline int64_t kb_block(const PodClass& C, int64_t t) { return C.kb0 + (t - C.t0) * (int64_t)C.wt * KB_UNIT; }
__host__ __device__ inline uint32_t kb_nrec(const PodClass& C) { return C.xreg + C.xinit + C.ovh; }
// 8-byte element index (into the array viewed as int64) of record k's cpu (mem: +256) of pod s
__host__ __device__ inline int64_t kb_rec64(int64_t blk, uint32_t k, int64_t s) {
    return (blk + KB_REC + 1024 * (int64_t)k) / 2 + kb_pos64(s);
}
// Packed K blocks (PodClass::packed): the same tile-major block with every value of a pod
// that fits its range packed, 12 B per pod instead of 20 and 8 B per record instead of 16
// (DESIGN.md §3):
//   word  [0, 256)            pair0 (bits 0..27, KP_PAIR_NONE = no pair) | the pod's own flag
//                             bits DAEMONSET, STATIC, HAS_SEL, AFF_BLOCK at bits 28..31 (every
//                             other flag bit is the class signature's)
//   u64   [256, 768)          cpu0 | mem0 << 20 at kb_pos64(s)
//   u64   record k            [768 + 512k, +512): cpu | mem << 20 (an init container's absent
//                             key: cpu field KP_CPU_ABSENT / mem field KP_MEM_ABSENT = INT64_MIN)
//   u32   extra pair k        [768 + 512R + 256k, +256), as in the plain layout
// A pod is packed when cpu0 and every record cpu are in [0, 2^20 - 1), mem0 and every record
// mem in [0, 2^44 - 1) (an init record's key may instead be absent) and pair0 < 2^28 - 1:
// the range of K1's LDS fast path, so nothing that fits it is left unpacked; others keep
// the plain layout of their signature.
constexpr int KP_CM0 = 256, KP_REC = 768;
constexpr uint32_t KP_FLAG_SHIFT = 28;
constexpr uint32_t KP_PAIR_NONE = (1u << KP_FLAG_SHIFT) - 1;
constexpr uint32_t KP_POD_FLAGS = ESC_PF_DAEMONSET | ESC_PF_STATIC | ESC_PF_HAS_SEL | ESC_PF_AFF_BLOCK;
constexpr int KP_CPU_BITS = 20;
constexpr uint64_t KP_CPU_ABSENT = (uint64_t(1) << KP_CPU_BITS) - 1;
constexpr uint64_t KP_MEM_ABSENT = (uint64_t(1) << 44) - 1;
// Packed small K blocks (PodClass::packed == 2): a pod whose packed values also have
// cpu0 < 2^14 m and mem0 < 2^34 B (16 cores, 16 GiB in its first container: most pods), in
// a context with fewer than 2^14 - 1 group pairs, is ONE u64 (8 B):
//   u64   [0, 512)            cpu0 | mem0 << 14 | pair0 << 48 (14 bits; KP8_PAIR_NONE: no
//                             pair, or one no group selects) | daemonset << 62 |
//                             blocks-default << 63 (static, has-selector or affinity: the
//                             default filter's other conditions, node_group.go:263-273)
//                             A daemonset pod (and a free slot) is stored with no pairs and
//                             blocks-default set, so K1 adds it nowhere without a test.
//   u64   record k            [512 + 512k, +512): as in the packed block
//   u16   extra pair k        [512 + 512R + 128k, +128) words: pod s at u16 index s (0xFFFF:
//                             none, or one no group selects)
constexpr int KP8_REC = 512;
constexpr int KP8_CPU_BITS = 14, KP8_MEM_BITS = 34, KP8_PAIR_SHIFT = 48;
constexpr uint64_t KP8_CPU_MASK = (uint64_t(1) << KP8_CPU_BITS) - 1;
constexpr uint64_t KP8_MEM_MASK = (uint64_t(1) << KP8_MEM_BITS) - 1;
constexpr uint32_t KP8_PAIR_NONE = (1u << 14) - 1;
constexpr uint64_t KP8_DS = uint64_t(1) << 62, KP8_NODEF = uint64_t(1) << 63;
__host__ __device__ inline bool kp8_fits(uint32_t cpu0, int64_t mem0) {
    return (uint64_t)cpu0 <= KP8_CPU_MASK && mem0 >= 0 && (uint64_t)mem0 <= KP8_MEM_MASK;
}
__host__ __device__ inline uint64_t kp8_word(uint32_t f, uint32_t cpu0, int64_t mem0, uint32_t pair0) {
    const bool ds = (f & ESC_PF_DAEMONSET) != 0;
    const uint64_t q = pair0 < KP8_PAIR_NONE && !ds ? pair0 : KP8_PAIR_NONE;
    return (uint64_t)cpu0 | (uint64_t)mem0 << KP8_CPU_BITS | q << KP8_PAIR_SHIFT | (ds ? KP8_DS | KP8_NODEF : 0) |
           ((f & (ESC_PF_STATIC | ESC_PF_HAS_SEL | ESC_PF_AFF_BLOCK)) ? KP8_NODEF : 0);
}
// extra pair k of pod s: its u32-word index (plain and packed blocks) or, in a packed small
// block, its u16 index (kb_pair reads either)
constexpr uint32_t KP8_XP_NONE = 0xFFFFu;
__host__ __device__ inline int64_t kb_xp(const PodClass& C, int64_t blk, uint32_t k, int64_t s) {
    if (C.packed == 2) return (blk + KP8_REC + 512 * (int64_t)kb_nrec(C) + 128 * (int64_t)k) * 2 + s;
    if (C.packed) return blk + KP_REC + 512 * (int64_t)kb_nrec(C) + 256 * (int64_t)k + s;
    return blk + KB_REC + 1024 * (int64_t)kb_nrec(C) + 256 * (int64_t)k + s;
}
// the first u32 word of the extra-pair rows of the block at blk, and their size in words
__host__ __device__ inline int64_t kb_xp_row0(const PodClass& C, int64_t blk) {
    if (C.packed == 2) return blk + KP8_REC + 512 * (int64_t)kb_nrec(C);
    return kb_xp(C, blk, 0, 0);
}
__host__ __device__ inline int64_t kb_xp_words(const PodClass& C) { return (int64_t)C.nxp * (C.packed == 2 ? 128 : 256); }
__host__ __device__ inline uint32_t kb_pair(const PodClass& C, const uint32_t* kb, int64_t blk, uint32_t k, int64_t s) {
    if (C.packed == 2) {
        const uint32_t q = reinterpret_cast<const uint16_t*>(kb)[kb_xp(C, blk, k, s)];
        return q == KP8_XP_NONE ? NONE : q;
    }
    return kb[kb_xp(C, blk, k, s)];
}
// A freed / padding slot: daemonset-flagged, no pair (put as in kb_write_pod below).
// put(width, index, value): width 8 = int64 element index, 4 = u32 word, 2 = u16 element.
template <class Put>
__host__ __device__ inline void kb_write_free(const PodClass& C, int64_t blk, int64_t sl, Put&& put) {
    if (C.packed == 2) {
        put(8, blk / 2 + kb_pos64(sl), KP8_DS | KP8_NODEF | (uint64_t)KP8_PAIR_NONE << KP8_PAIR_SHIFT);
        for (uint32_t k = 0; k < C.nxp; ++k) put(2, kb_xp(C, blk, k, sl), KP8_XP_NONE);   // no pairs (see kp8_word)
    } else {
        put(4, blk + sl, C.packed ? (ESC_PF_DAEMONSET << KP_FLAG_SHIFT) | KP_PAIR_NONE : ESC_PF_DAEMONSET);
    }
}
// packed 8-byte value of a (cpu, mem) pair; init: an absent key becomes its field's sentinel
__host__ __device__ inline bool kp_val_fits(int64_t cpu, int64_t mem, bool init) {
    const bool c = (cpu >= 0 && (uint64_t)cpu < KP_CPU_ABSENT) || (init && cpu == INT64_MIN);
    const bool m = (mem >= 0 && (uint64_t)mem < KP_MEM_ABSENT) || (init && mem == INT64_MIN);
    return c && m;
}
__host__ __device__ inline uint64_t kp_val(int64_t cpu, int64_t mem) {
    const uint64_t c = cpu == INT64_MIN ? KP_CPU_ABSENT : (uint64_t)cpu;
    const uint64_t m = mem == INT64_MIN ? KP_MEM_ABSENT : (uint64_t)mem;
    return c | (m << KP_CPU_BITS);
}
__host__ __device__ inline int64_t kp_cpu(uint64_t v) {
    const uint64_t c = v & KP_CPU_ABSENT;
    return c == KP_CPU_ABSENT ? INT64_MIN : (int64_t)c;
}
__host__ __device__ inline int64_t kp_mem(uint64_t v) {
    const uint64_t m = v >> KP_CPU_BITS;
    return m == KP_MEM_ABSENT ? INT64_MIN : (int64_t)m;
}
__host__ __device__ inline uint32_t kp_word(uint32_t flags, uint32_t pair0) {
    return ((flags & KP_POD_FLAGS) << KP_FLAG_SHIFT) | (pair0 == NONE ? KP_PAIR_NONE : pair0);
}
__host__ __device__ inline uint32_t kp_pair0(uint32_t w) {
    const uint32_t q = w & KP_PAIR_NONE;
    return q == KP_PAIR_NONE ? NONE : q;
}
// full ESC_PF_* flags of a packed pod: its own bits + the class signature
__host__ __device__ inline uint32_t kp_flags(const PodClass& C, uint32_t w) {
    return (w >> KP_FLAG_SHIFT) | (C.ovh ? ESC_PF_HAS_OVH : 0u) | (C.xreg << ESC_PF_XREG_SHIFT) |
           (C.xinit << ESC_PF_XINIT_SHIFT) | (C.nxp << ESC_PF_XPAIR_SHIFT);
}
// Does the pod fit the packed layout?  (xc_cpu / xc_mem: its extra records, regular, then
// init, then overhead, as esc_pod_soa lists them.)
__host__ __device__ inline bool kp_fits(uint32_t f, uint32_t cpu0, int64_t mem0, uint32_t pair0, const int64_t* xc_cpu,
                                        const int64_t* xc_mem) {
    if (!(pair0 == NONE || pair0 < KP_PAIR_NONE) || !kp_val_fits((int64_t)cpu0, mem0, false)) return false;
    const uint32_t nreg = pf_xreg(f), ninit = pf_xinit(f), n = pf_xctr(f);
    for (uint32_t k = 0; k < n; ++k)
        if (!kp_val_fits(xc_cpu[k], xc_mem[k], k >= nreg && k < nreg + ninit)) return false;
    return true;
}
// The head of K pod s of the block at word blk, any layout: ESC_PF_* flags (the class
// signature's counts included; a packed small pod's static / has-selector / affinity bits
// read back as ESC_PF_HAS_SEL), pair0 (NONE: none, or no group's in a small block) and the
// first container's cpu / mem; kp_rec: record k's cpu / mem (an absent init key INT64_MIN).
struct KHead {
    uint32_t flags, pair0;
    int64_t cpu0, mem0;
};
__host__ __device__ inline KHead kb_head(const PodClass& C, const uint32_t* kb, int64_t blk, int64_t s) {
    KHead h;
    const int64_t* kb64 = reinterpret_cast<const int64_t*>(kb);
    if (C.packed == 2) {
        const uint64_t w = (uint64_t)kb64[blk / 2 + kb_pos64(s)];
        h.flags = kp_flags(C, 0) | ((w & KP8_DS) ? ESC_PF_DAEMONSET : 0u) | ((w & KP8_NODEF) ? ESC_PF_HAS_SEL : 0u);
        const uint32_t q = (uint32_t)(w >> KP8_PAIR_SHIFT) & KP8_PAIR_NONE;
        h.pair0 = q == KP8_PAIR_NONE ? NONE : q;
        h.cpu0 = (int64_t)(w & KP8_CPU_MASK);
        h.mem0 = (int64_t)((w >> KP8_CPU_BITS) & KP8_MEM_MASK);
    } else if (C.packed) {
        const uint32_t w0 = kb[blk + s];
        const uint64_t v = (uint64_t)kb64[(blk + KP_CM0) / 2 + kb_pos64(s)];
        h.flags = kp_flags(C, w0);
        h.pair0 = kp_pair0(w0);
        h.cpu0 = kp_cpu(v);
        h.mem0 = kp_mem(v);
    } else {
        h.flags = kb[blk + s];
        h.pair0 = kb[blk + KB_PAIR0 + s];
        h.cpu0 = kb[blk + KB_CPU0 + s];
        h.mem0 = kb64[(blk + KB_MEM0) / 2 + kb_pos64(s)];
    }
    return h;
}
__host__ __device__ inline void kb_rec(const PodClass& C, const uint32_t* kb, int64_t blk, uint32_t k, int64_t s,
                                       int64_t& cpu, int64_t& mem) {
    const int64_t* kb64 = reinterpret_cast<const int64_t*>(kb);
    if (C.packed) {
        const uint64_t v = (uint64_t)kb64[(blk + (C.packed == 2 ? KP8_REC : KP_REC) + 512 * (int64_t)k) / 2 + kb_pos64(s)];
        cpu = kp_cpu(v);
        mem = kp_mem(v);
    } else {
        const int64_t o = kb_rec64(blk, k, s);
        cpu = kb64[o];
        mem = kb64[o + 256];
    }
}

// Every word a K-class pod occupies in its tile (load and in-place upserts): put(width,
// index, value) as for kb_write_free.
template <class Put>
__host__ __device__ inline void kb_write_pod(const PodClass& C, int64_t blk, int64_t sl, uint32_t f, uint32_t cpu0,
                                             int64_t mem0, uint32_t pair0, const int64_t* xc_cpu,
                                             const int64_t* xc_mem, const uint32_t* xp, Put&& put) {
    const uint32_t R = kb_nrec(C);
    if (C.packed == 2) {
        put(8, blk / 2 + kb_pos64(sl), kp8_word(f, cpu0, mem0, pair0));
        for (uint32_t k = 0; k < R; ++k)
            put(8, (blk + KP8_REC + 512 * (int64_t)k) / 2 + kb_pos64(sl), kp_val(xc_cpu[k], xc_mem[k]));
    } else if (C.packed) {
        put(4, blk + sl, kp_word(f, pair0));
        put(8, (blk + KP_CM0) / 2 + kb_pos64(sl), kp_val((int64_t)cpu0, mem0));
        for (uint32_t k = 0; k < R; ++k)
            put(8, (blk + KP_REC + 512 * (int64_t)k) / 2 + kb_pos64(sl), kp_val(xc_cpu[k], xc_mem[k]));
    } else {
        put(4, blk + sl, f);
        put(4, blk + KB_CPU0 + sl, cpu0);
        put(8, (blk + KB_MEM0) / 2 + kb_pos64(sl), (uint64_t)mem0);
        put(4, blk + KB_PAIR0 + sl, pair0);
        for (uint32_t k = 0; k < R; ++k) {
            const int64_t o = kb_rec64(blk, k, sl);
            put(8, o, (uint64_t)xc_cpu[k]);
            put(8, o + 256, (uint64_t)xc_mem[k]);
        }
    }
    if (C.packed == 2) {                       // u16 pairs; a daemonset pod has none (kp8_word)
        for (uint32_t k = 0; k < C.nxp; ++k)
            put(2, kb_xp(C, blk, k, sl), (f & ESC_PF_DAEMONSET) || xp[k] >= KP8_XP_NONE ? KP8_XP_NONE : xp[k]);
    } else {
        for (uint32_t k = 0; k < C.nxp; ++k) put(4, kb_xp(C, blk, k, sl), xp[k]);
    }
}

// Device view of a pod shard.  Two sections, made at load (esc_load_pods; sums are
// order-independent):
//  - K: pods with at most 3 extra container records and at most 3 extra pairs, grouped by
//    record signature into 256-pod tiles, each tile one contiguous block (kb, above);
//  - C: the others, in 64-pod tiles (1 per lane) in their own SoA arrays (flags .. pair0
//    indexed from the C section's start), whose extra records are contiguous per tile
//    (xc_base / xp_base into xc_cpu / xc_mem / xp).
// Pod slot numbering (the host's and the reaping's): K pod s of tile t = t * 256 + s, C pod
// i = k_tiles * 256 + i.  Padding pods carry ESC_PF_DAEMONSET.
struct PodDev {
    const uint32_t* kb;        // K blocks
    const uint32_t* flags;     // C section
    const uint32_t* cpu0;
    const int64_t*  mem0;
    const uint32_t* pair0;
    const int64_t*  xc_cpu;
    const int64_t*  xc_mem;
    const uint32_t* xp;
    const PodClass* cls;       // [n_cls] K classes, in tile order
    const uint32_t* xc_base;   // [c_tiles + 1] extra-container offset of each C tile
    const uint32_t* xp_base;   // [c_tiles + 1] extra-pair offset
    // K1 work plan (ensure_work): per workgroup up to K1_SEGS runs of one
    // class, {t0 | class << 48, t1} (t1 == 0: unused), balanced in work weight, at most two
    // class boundaries per workgroup.  Null: the weight-range shares of variant 7.
    const int64_t* seg;
    // Compact K1 flush: workgroup b writes only the pod-slot columns its share
    // touches, wg_cols[b * n_col + i] = {column, destination} for i < wg_off[b] (n_col = the
    // columns of a partial row), each destination a 64-word partial (32 cpu|count words, 32
    // mem words) that K3 finds through FoldPlan::col_rows.  Null: every row flushed whole (no
    // static plan).
    const uint2* wg_cols;
    const uint32_t* wg_off;
    int32_t n_cls;
    int64_t k_tiles;           // K section: pods [0, k_tiles * 256)
    int64_t k_weight;          // total work weight of the K tiles (K1 splits it evenly)
    int64_t c_tiles;           // C section: pods [k_tiles * 256, + c_tiles * 64)
};

// Device view of the node snapshot.
//
// Two layouts of the same records, both resident on every rank:
//  - the node table in snapshot order: flags, label pairs, allocatable, creation time.
//    The K5 age index is listed from it (nodes [lo, hi) = the whole table), keeping the
//    memberships of this rank's groups; K3 reads allNodes[0]'s capacity.
//  - the pair-major entries: one entry per (label pair, node), sorted by (pair, node)
//    at load (e_flags / e_cpu / e_mem / e_node).  NewNodeLabelFilterFunc
//    (node_group.go:278) is "(K_g, V_g) in the node's label pairs", so a group's members
//    are exactly the entries of its pair, in snapshot order.  K2 reduces the entries per
//    piece (a run of entries of one pair that crosses no multiple of PIECE_ALIGN entries:
//    K2's spans of whole pieces come out full); this rank reduces the pieces
//    [pc_lo, pc_hi) of the pairs [q_lo, q_hi) it owns.  K3 joins each group to its pair's
//    pieces.
// Per-group node facts that are fixed for a loaded snapshot (esc_load_nodes): this rank's
// piece range of the group's pair (empty when another rank owns the pair) and allNodes[0]
// (controller.go:207-211, from the whole table on every rank) with its allocatable, so K3
// needs no dependent index chase.
struct GroupNode {
    int64_t first;             // lowest member node index (INT64_MAX: no member)
    int64_t first_cpu, first_mem;
    int64_t plo, phi;          // this rank's pieces of the group's pair
};

struct NodeDev {
    const GroupNode* gnode;    // [G]
    const uint32_t* flags;
    const uint32_t* label0;
    const int64_t*  cpu;
    const int64_t*  mem;
    const int64_t*  created;
    const uint32_t* xl;
    const uint32_t* xl_off;    // [n_nodes] offset of each node's extra labels
    const int32_t*  trk_node;  // dry-mode tracker, sorted by (node, group)
    const int32_t*  trk_group;
    const uint32_t* trk_start; // [n_nodes] first tracker entry of a tracked node
    int64_t n_trk;
    int64_t lo, hi;            // K5's node range
    // pair-major entries
    const uint32_t* e_flags;
    const int64_t*  e_cpu;
    const int64_t*  e_mem;
    // the same entries as one 16-B record each (flags, cpu as u32, mem lo, mem hi) when every
    // node's allocatable cpu is in [0, 2^32) (checked at load and by every node event; null
    // otherwise): K2 streams one load per entry instead of three, 16 B instead of 20
    const uint4*    e_pk;
    const uint32_t* e_node;    // snapshot index of the entry's node
    const uint32_t* piece_off; // [n_pieces + 1] entry offsets
    const uint32_t* piece_pair;// [n_pieces]
    const uint32_t* pp_off;    // [n_gp + 1]: pieces of group pair q are [pp_off[q], pp_off[q+1])
    // K2 work: span w = this rank's group-pair pieces [span_off[w], span_off[w + 1]), at
    // most NODE_SPAN entries of whole pieces, one wave per span
    const uint32_t* span_off;  // [n_spans + 1]
    const uint32_t* span_e;    // [n_spans + 1] the spans' entry bounds (piece_off[span_off[w]])
    int64_t n_pieces, pc_lo, pc_hi, n_spans;
    // the group pairs this rank owns: their pieces [pc_lo, pc_hi) are its K2
    // work, their groups' memberships its K5 age index; [0, n_gp) with one rank
    uint32_t q_lo, q_hi;
};

// K2 output row per piece (int64 words, stored word-major: rows[word * n_pieces + piece]).
// Sums travel split lo32 / hi (arithmetic) so they add without wrapping; counts are
// packed 21 bits each (a piece has <= NODE_PIECE entries).
enum NodeRow : int {
    NR_UCPU_LO = 0, NR_UCPU_HI, NR_UMEM_LO, NR_UMEM_HI,    // untainted members (wet classes)
    NR_ACPU_LO, NR_ACPU_HI, NR_AMEM_LO, NR_AMEM_HI,        // every member (dry mode)
    NR_COUNTS,                                             // unt | taint << 21 | cord << 42
    NR_K
};
constexpr int NODE_PIECE = 1024;
constexpr int PIECE_ALIGN = 256;           // no piece crosses a multiple of it (esc_load_nodes)
static_assert(NODE_PIECE % PIECE_ALIGN == 0, "the alignment bounds every piece");
#ifndef ESC_NODE_SPAN
#define ESC_NODE_SPAN 256                  // (timing builds may override; the runtime builds the spans too)
#endif
constexpr int NODE_SPAN = ESC_NODE_SPAN;   // entries per K2 wave (whole pieces, <= 63 of them)
constexpr int NR_CNT_BITS = 21;
constexpr uint64_t NR_CNT_MASK = (uint64_t(1) << NR_CNT_BITS) - 1;

struct GroupDev {
    const uint8_t*  dry;
    const GroupParams* params;
    const uint32_t* gpair;     // [G] group -> its pair id (K3 joins pod slots / node pieces to groups)
    const uint32_t* node_code; // [n_gp] pair id -> group code (K5)
    const uint32_t* code_list; // CODE_MULTI lists: [count, g...]
    const uint32_t* gslot;     // [G] the group's pod slot: its pair, or n_gp for the default group
    const uint32_t* xs;        // [G] the group's row of the exchanged pod words (owner-major)
    esc_group_metrics* metrics; // [G] gauges written by K4, or null (esc_set_metrics)
    esc_group_totals* htot;    // [G] totals written by K4 with the decision (pinned host memory,
                               // small contexts: esc_results then copies nothing), or null
    int64_t sp;                // K1 partial row stride: pod slots rounded up to FC_COL
    uint32_t n_gp;             // pod slots: pair ids [0, n_gp) + the default filter's slot n_gp
    int32_t G;
    uint32_t default_group;    // NONE when no group is named "default"
};

// Wide (exact, any-range) pod accumulators: global int64 atomics, one row per pod slot.
// K3 reads them and resets a non-zero row (every reader of a slot is in one K3 workgroup).
enum WidePod : int { WP_CPU_LO = 0, WP_CPU_HI, WP_MEM_LO, WP_MEM_HI, WP_CNT, WP_K };
// Per dry-mode group: the tracked members' count and split sums (K2 adds, K3 resets).
enum TrkAcc : int { TA_CNT = 0, TA_CPU_LO, TA_CPU_HI, TA_MEM_LO, TA_MEM_HI, TA_K };

// variant: 0 = the product K1 (512 threads: 8 waves per CU with up to 256 VGPRs, 3-4 K
// tiles in flight per wave, one static share per workgroup); 3, 4, 9-14 = timing-only
// ablations (wrong results), present in the measurement library only (ESC_K1_VARIANT,
// scripts/k1_variants.py).
// K1_CHUNKS: the unit of a static share's size bound (ensure_work); the K1 template's
// dynamic-share form (a ticket of nblk * K1_CHUNKS chunks) is instantiated only by the
// measurement library's ablations.
constexpr int K1_CHUNKS = 4;
struct DecCompact;
// K1 diagnostics.  trace: per workgroup 8 words (esc_k1_trace; the share calibration reads words
// 0-1): s_memrealtime (100 MHz) at start, after the K tiles, after the C tiles, after the
// flush; HW_ID, XCC_ID.
struct K1Diag {
    uint64_t* trace;
};
// Selections delivered with the decision (esc_set_selections; controller.go:367-383): K4
// also writes, for every group it decides with delta < 0 (and the taint clamp passed) the
// first min(n_to_taint + slack, group_cap) untainted nodes oldest first (taintOldestN's walk,
// scale_down.go:171-205), with delta > 0 the first min(delta + slack, group_cap) tainted
// nodes newest first (untaintNewestN, scale_up.go:118-163; equal creation times by ascending
// index, the ordering's tie rule), copied from the ordering of the same decision into the
// pinned buffer `out` — a block's groups as one contiguous run of [header, nodes...] words
// at the block's own slot (blockIdx.x * 64 * (group_cap + 1): no reservation across blocks)
// — and the run's offset into the compact record's `sel` field.  Header: count | which << 28
// (1 taint, 2 untaint) | SEL_CUT (more wanted than group_cap: the nodes are the walk's first
// ones) | SEL_TIE (a run of equal creation times longer than SEL_TIE_MAX: the nodes are not
// used; in both cases the host continues with esc_group_order).
struct SelOut {
    const uint32_t* ord;       // K5 output: every group's segments
    const int64_t* seg;        // [4G] segment bounds (K5)
    const uint32_t* tie;       // [G] RegionSink::tie: only these groups' untaint lists need the
                               // tie rule (the others copy their segment's prefix as it stands)
    uint32_t* out;             // device view of the pinned selection buffer; null: no selections
    int64_t cap_words;         // out's size (a block whose run does not fit gets SEL_OVERFLOW)
    int32_t slack, group_cap;
};
constexpr uint32_t SEL_NONE = 0xFFFFFFFFu, SEL_OVERFLOW = 0xFFFFFFFEu;   // DecCompact::sel without a run
constexpr uint32_t SEL_COUNT_MASK = (1u << 28) - 1, SEL_CUT = 1u << 30, SEL_TIE = 1u << 31;
constexpr int SEL_TIE_MAX = 64;
// k_node_groups' decision target: null dec = the node words only (a reduce that was never
// decided, esc_reduce).
struct NGDecide {
    const int64_t* pwords;
    esc_group_decision* dec;
    DecCompact* cdec;
    SelOut sel;
    uint64_t* trace = nullptr;         // measurement library: per block {start, end} (esc_debug_tail_trace)
};
// The groups a launch of k_node_groups covers: ids[i] for i < n, or, with null
// ids, the contiguous run first + i (a rank's owned groups).
struct GroupList {
    const uint32_t* ids;
    int32_t n;
    int32_t first;
};
hipError_t launch_pod_reduce(const PodDev& p, const GroupDev& g, int32_t g0, int32_t gw, int nblk, int variant,
                             uint64_t* part, int64_t* wide, uint32_t* ticket, int cap, const K1Diag& diag,
                             hipStream_t st);
hipError_t launch_pod_bigtiles(const PodDev& p, const GroupDev& g, const uint32_t* tiles, int64_t n_big,
                               int64_t* wide, hipStream_t st);
// Compact decision record (32 B) that K3 / K4 write to pinned host memory each decision
// instead of the ABI's 64-B esc_group_decision: esc_results rebuilds the full record on the
// host (the cached capacity from its node mirror: allNodes[0]'s allocatable when the group
// has nodes, else the state's, controller.go:207-211) and copies the full record, which
// the kernels also keep in device memory, for a group whose delta or n_to_taint leaves int32.
struct DecCompact {
    double cpu_pct, mem_pct;
    int32_t delta, n_to_taint;
    uint8_t status, branch, taint_status, wide;
    uint32_t sel;              // word offset of the group's selection run (SelOut), or SEL_NONE / SEL_OVERFLOW
};
static_assert(sizeof(DecCompact) == 32, "compact decision is 2 x 16 B");

// K2b + K4 (k_node_groups): the listed groups' final node words from K2's piece rows, then
// (nd.dec != null) their decisions (K4) from the pod words at rows xs[g] (or g).
// Peer exchange of a multi-device context (esc_ctx_create_multi): dst[i] = sum of src[k][i]
// over the n_src buffers (peer-mapped device memory), int64 or uint32 words.
hipError_t launch_peer_sum64(const int64_t* const* src, int n_src, int64_t* dst, int64_t n, hipStream_t st);
hipError_t launch_peer_sum32(const uint32_t* const* src, int n_src, uint32_t* dst, int64_t n, hipStream_t st);
hipError_t launch_node_groups(const GroupDev& g, const NodeDev& n, const GroupList& list, const int64_t* node_rows,
                              int64_t* trk_acc, int64_t* nwords, const NGDecide& nd, hipStream_t st);
// K3 fold (a role of k_step_tail): the K1 partials of FC_COL pod slots per block.
constexpr int FC_COL = 32;             // pod slots per K3 column (a 256-B piece of each K1 row)
struct FoldPlan {
    const uint64_t* part;              // K1 partials: row b = cc[sp], mem[sp] at part + 2 * sp * b
    int nblk;                          // K1 rows
    int64_t sp;                        // slots per partial row, a multiple of FC_COL
    int64_t n_col;                     // columns (grid)
    const uint32_t* col_off;           // [n_col + 1] the column's groups in col_groups
    const uint32_t* col_groups;        // group ids ordered by pod slot, then id
    const uint32_t* col_rows;          // compact flush: [n_col + 1] partial entries of each column (null: nblk rows)
    int ablate;                        // ESC_K3_ABLATE (timing-only knob)
    uint64_t* trace = nullptr;         // measurement library: per block {start, end, role} (esc_debug_tail_trace)
};
// The pod-slot columns each K1 workgroup's share touches (compact flush): bitmap words of
// tw u32 per workgroup, from the same work plan as K1 (daemonset pods skipped: they add
// nothing; the default filter's column always).
hipError_t launch_touch(const PodDev& p, const GroupDev& g, int nblk, int tw, uint32_t* bits, hipStream_t st);
struct OrdChunk;
// The step's tail in one launch (esc_kernels.hip k_step_tail): the K3 fold into the pod
// words, K2's dry-mode tracker entries (+ its piece rows when `spans`) and,
// with n_small > 0, the K5 ordering of the packed small-group chunks [0, n_small).
// the tail's K2 span blocks (K2_WAVES spans each) and dry-mode tracker blocks for this node view
constexpr int K2_WAVES = 4;
int64_t tail_span_blocks(const NodeDev& n);
int64_t tail_trk_blocks(const NodeDev& n);
hipError_t launch_step_tail(const GroupDev& g, const NodeDev& n, const FoldPlan& f, bool spans, int64_t* wide_pod,
                            int64_t* pwords, int64_t* rows, int64_t* trk_acc, const OrdChunk* chunks, int64_t n_small,
                            const uint32_t* grp_off, const uint32_t* g_memb,
                            uint32_t* vals, int64_t* seg, hipStream_t st);
hipError_t launch_wide_pods(const PodDev& p, const GroupDev& g, int64_t* wide, hipStream_t st);
// §8f rank 2: a loaded pod as seen by NodePodsRemaining, listed per node (runs in
// node order).  p[0..2]: the pod's extra pairs (NONE-padded); a C pod with more than 3
// has POD_REF_INDIRECT in flags and p[0] = offset, p[1] = count into xp.
struct PodRef {
    uint32_t flags, pair0, p[3];
};
constexpr uint32_t POD_REF_INDIRECT = 1u << 31;
// K7's per-group record on the device (esc_removal widened on the host)
struct RmRec {
    uint32_t n_candidates, n_delete;
    int64_t pods_remaining;
};
struct RemovalDev {
    const int64_t* taint_s;    // [n_nodes] escalator-taint time (INT64_MIN: none / unparsable)
    const uint8_t* no_delete;  // [n_nodes]
    const uint32_t* e_pair;    // [n_entries] pair of each pair-major entry
    int64_t n_entries;
    const uint32_t* nrun_off;  // [n_nodes + 1] runs of PodRef per node (capacity)
    const uint32_t* nrun_len;  // [n_nodes] PodRefs in each run
    const PodRef* refs;
    const uint32_t* xp;        // C-pod extra pairs (indirect refs)
    uint32_t* occ_pair;        // [entries] group pods on the node, by the entry's pair
    uint32_t* occ_def;         // [entries] default-filter pods on the node
    const int64_t* soft_ns;    // [G]
    const int64_t* hard_ns;    // [G]
    const uint32_t* rm_off;    // [G] offset of each group's deletable-node list
    uint32_t* rm_list;
    RmRec* out;                // [G]
    int64_t now_ns;
};
hipError_t launch_podref_fill(const PodDev& p, const uint32_t* run_slot, const uint32_t* run_pos, int64_t n, PodRef* refs,
                              hipStream_t st);
// K6: the occupancy words of every live pair-major entry (esc_load_placement; pod and node
// events then keep them current through launch_occ_delta instead of a recount per call).
hipError_t launch_occupancy(const NodeDev& n, const GroupDev& g, const RemovalDev& r, hipStream_t st);
// The occupancy change of n PodRef placements: the PodRef at run position pos[i], on node
// node[i], added (sign +1) to or removed (-1) from the words of the node's entries
// (ne_off / ne_pos: node -> its entry positions).
hipError_t launch_occ_delta(const GroupDev& g, const RemovalDev& r, const uint32_t* ne_off, const uint32_t* ne_pos,
                            const uint32_t* pos, const uint32_t* node, int64_t n, int sign, hipStream_t st);
hipError_t launch_try_remove(const NodeDev& n, const GroupDev& g, const RemovalDev& r, hipStream_t st);  // K7

struct PatchTargets {          // k_patch destinations: 4-byte arrays 0-5, 8-byte arrays 6-11, 2-byte 12-13
    uint32_t* u32[6];
    int64_t* i64[6];
    uint16_t* u16[2];
};
hipError_t launch_patch(const PatchTargets& t, const uint64_t* where, const uint64_t* what, int64_t n, hipStream_t st);


// Ordering (K5), see esc_kernels.hip: the age index (once per snapshot) and the per-decision
// (group, class) partition.
size_t sort_hist_words(int64_t n);   // digit-histogram words one LSD pass over n keys needs
struct OrdChunk {               // K5 per-decision chunk: memberships [start, end) of one group
    uint32_t start, end, group, pad;   // a packed chunk: its first group, and pad = how many
};                                     // groups [group, group + pad) it covers (<= ORD_GCAP)
constexpr uint32_t ORD_CHUNK_DRY = 2u;   // OrdChunk::pad bit of a split chunk: its group is in dry mode
constexpr uint32_t ORD_GCAP = 512;       // groups a packed chunk covers at most (empty ones included)
#ifndef ESC_ORD_CHUNK
#define ESC_ORD_CHUNK 4096         // (timing builds may override)
#endif
constexpr int ORD_CHUNK = ESC_ORD_CHUNK;   // memberships per K5 chunk (three-pass default)
// Every group owns a region of the group-order arrays: its memberships oldest first, then
// padding (the round-up to whole 16-B quads and the spare slots node additions take,
// DESIGN.md §4) — MEMB_PAD_WORD, class 3 from the word alone.  The packed orderings find a
// quad's group from the chunk's region starts (round 6: no group word per slot).
constexpr uint32_t MEMB_PAD = 0x80000000u;   // (a group word's padding bit: ord_class)
// A group region's membership word (g_memb, 4 B): node | the low four flag bits of the node
// as the per-decision split reads them (UNSCHED, TAINTED, TRACKED resolved for the group,
// ABSENT) << MEMB_FLAG_SHIFT — the age index's sort value, kept as is.  One 4-B word per
// membership is all the split reads besides the chunk (round 3 read node, flags and a class
// byte: 9 B).  Nodes < 2^28.  Padding: node 0, ABSENT.
constexpr uint32_t MEMB_FLAG_SHIFT = 28, MEMB_NODE_MASK = (1u << MEMB_FLAG_SHIFT) - 1;
constexpr uint32_t MEMB_PAD_WORD = ESC_NF_ABSENT << MEMB_FLAG_SHIFT;
inline uint32_t memb_word(uint32_t node, uint32_t flags) { return node | ((flags & 0xFu) << MEMB_FLAG_SHIFT); }
// Small groups (region <= ORD_CHUNK) are packed whole into chunks ordered in one pass:
// chunks [0, n_small) of groups with regions <= ORD_PCHUNK, packed up to ORD_PCHUNK
// memberships (more, shorter blocks), then chunks of up to ORD_CHUNK.
constexpr int ORD_PCHUNK = 1024;
hipError_t launch_order_packed(const NodeDev& nd, const OrdChunk* chunks, int64_t n_chunks, int64_t n_small,
                               const uint32_t* grp_off, const uint8_t* dry, const uint32_t* g_memb,
                               uint32_t* vals, int64_t* seg, hipStream_t st);
// Fills the padding of every group's region (after its `len` memberships) with MEMB_PAD_WORD
// and sets the ordering's segment starts (seg[4g + k] = pstart[g], seg[4G] = pstart[G]).
hipError_t launch_region_pad(const uint32_t* pstart, const uint32_t* plen, int32_t G, uint32_t* g_memb, int64_t* seg,
                             hipStream_t st);
// The age index (load time): memberships listed in one pass (per-tile counts, decoupled
// look-back: status = memb_status_words(n) u64 words, zeroed by the caller) with
// (group << R | creation offset) keys and (node | flags) values, LSD-sorted, then written
// into the groups' padded regions; *total = the listed count.
size_t memb_status_words(int64_t n);
// The age index's destination: every group's padded region (k_rs_scatter<FINAL>).
struct RegionSink {
    const int64_t* seg;        // sorted start of group g's memberships (host-computed)
    const uint32_t* pstart;    // region start of group g
    const uint32_t* plen;      // memberships of group g
    uint32_t* g_memb;          // region words (MEMB_FLAG_SHIFT)
    uint32_t* err;             // bit 0: a membership fell outside its group's count; bit 1: a
                               // coarse-key run too long for k_age_fix (rebuild exact)
    int32_t G;
    int R;                     // the group's shift in the key (key = group << R | time bits)
    int fix;                   // coarse keys: the final pass also writes the sorted keys and
                               // k_age_fix reads them — 1 (time bits were dropped): it orders each
                               // run of equal keys exactly and flags the groups with equal times;
                               // 2 (the keys are exact): it only flags the groups of equal-key runs
    uint32_t spins;            // the listing's look-back bound (LOOKBACK_SPINS; err bit 0 on a give-up)
    uint32_t* tie;             // [G] nonzero: two of the group's members share a creation time (the
                               // selections resolve such ties, SelOut); zeroed by the host first
};
// coarse_shift < 0: exact 64-bit keys (group << R | offset); >= 0: 32-bit coarse keys
// (group << (32 - gbits) | offset >> coarse_shift) + the run fix-up (S.R = 32 - gbits).
hipError_t launch_age_sort(const NodeDev& nd, const GroupDev& g, uint64_t* status, uint32_t* total, int64_t n_memb,
                           int64_t cap, int64_t ts_min, uint64_t div, int R, int gbits, int coarse_shift,
                           uint64_t* keys[2], uint32_t* vals[2], uint32_t* hist, uint32_t* tot, const RegionSink& S,
                           hipStream_t st);
// The bounded waits of the decoupled look-backs (k_ord_split, k_memb_keys): HIP does not
// promise dispatch order, so a chunk never waits unboundedly on one that was not dispatched.
// A chunk that waited `spins` probes gives up: it publishes a FAILED status word (never an
// inclusive prefix it could not compute; its successors fail in turn instead of waiting),
// writes none of its output and sets *err (k_ord_split: a pinned host word the runtime reads
// after its stream wait and reports as ESC_E_ORDER, then clears).
constexpr uint32_t LOOKBACK_SPINS = 1u << 22;
struct OrdFail {
    uint32_t* err;             // device view of a pinned host word: set to 1 by a give-up
    uint32_t spins;            // LOOKBACK_SPINS (smaller in measurement builds' tests)
};
// The split groups' ordering in one pass (k_ord_split): ostat = 2 * n_chunks + 1 u64 words,
// zeroed when the chunk table is made: two arrays of status words used by alternate
// decisions (par = 0, 1: a decision clears its chunks' words of the other).
// Output layout of every group (split and packed): untainted forward from the region start,
// tainted newest first backward from the region end; seg[4g..4g+3] = start, start +
// untainted, end - tainted, end.
hipError_t launch_order(const NodeDev& n, const OrdChunk* chunks, int64_t n_chunks, const uint32_t* gch_off,
                        const uint32_t* grp_off, const uint32_t* g_memb, uint64_t* ostat, int par, uint32_t* vals,
                        int64_t* seg, const OrdFail& fail, hipStream_t st);

}  // namespace esc
