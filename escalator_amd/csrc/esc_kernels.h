// esc_kernels.h — device-side argument blocks and launch wrappers (esc_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "esc_common.h"

namespace esc {

// Device view of a pod shard.  Two sections of the same arrays: pods without extra
// records ("simple": one container, at most one selector pair) in 256-pod S tiles
// (4 per lane), then the others in 64-pod C tiles (1 per lane) whose extra records are
// contiguous per tile.  The split is a stable partition made at load (esc_load_pods);
// sums are order-independent.  Padding pods carry ESC_PF_DAEMONSET.
struct PodDev {
    const uint32_t* flags;
    const uint32_t* cpu0;
    const int64_t*  mem0;
    const uint32_t* pair0;
    const int64_t*  xc_cpu;
    const int64_t*  xc_mem;
    const uint32_t* xp;
    const uint32_t* xc_base;   // [c_tiles + 1] extra-container offset of each C tile
    const uint32_t* xp_base;   // [c_tiles + 1] extra-pair offset
    int64_t s_tiles;           // S section: pods [0, s_tiles * 256)
    int64_t c_tiles;           // C section: pods [s_tiles * 256, + c_tiles * 64)
};

// Device view of the node table; this rank streams nodes [lo, hi).
struct NodeDev {
    const uint32_t* flags;
    const uint32_t* label0;
    const int64_t*  cpu;
    const int64_t*  mem;
    const int64_t*  created;
    const uint32_t* xl;
    const uint32_t* xl_off;    // [n_nodes] offset of each node's extra labels
    const int32_t*  trk_node;
    const int32_t*  trk_group;
    int64_t n_trk;
    int64_t lo, hi;
};

struct GroupDev {
    const uint8_t*  dry;
    const GroupParams* params;
    const uint32_t* gpair;     // [G] group -> its pair id (K3 joins pod slots to groups)
    const uint32_t* node_code; // [n_gp] pair id -> group code for nodes
    const uint32_t* code_list; // CODE_MULTI lists: [count, g...]
    uint32_t n_gp;             // pod slots: pair ids [0, n_gp) + the default filter's slot n_gp
    int32_t G;
    uint32_t default_group;    // NONE when no group is named "default"
};

// Wide (exact, any-range) accumulators: global int64 atomics, one row per group.
enum WidePod : int { WP_CPU_LO = 0, WP_CPU_HI, WP_MEM_LO, WP_MEM_HI, WP_CNT, WP_K };
enum WideNode : int { WN_CPU_LO = 0, WN_CPU_HI, WN_MEM_LO, WN_MEM_HI, WN_UNT, WN_TAINT, WN_CORD, WN_FIRST, WN_K };

// variant (ESC_K1_VARIANT, measurement knob): 0 = 1024 threads (default), 2 = 512 threads,
// 9.. = timing-only ablations (wrong results, scripts/k1_variants.py).
hipError_t launch_pod_reduce(const PodDev& p, const GroupDev& g, int32_t g0, int32_t gw, int nblk, int variant,
                             uint64_t* part, int64_t* wide, hipStream_t st);
hipError_t launch_zero(int64_t* p, int64_t n, hipStream_t st);
hipError_t launch_pod_bigtiles(const PodDev& p, const GroupDev& g, const uint32_t* tiles, int64_t n_big,
                               int64_t* wide, hipStream_t st);
hipError_t launch_node_reduce(const NodeDev& n, const GroupDev& g, int n_chunk, int gt,
                              uint64_t* part, int64_t* wide, hipStream_t st);
hipError_t launch_combine(const GroupDev& g, const NodeDev& n, const uint64_t* pod_part, int nblk,
                          const uint64_t* node_part, int n_chunk, int64_t* wide_pod, int64_t* wide_node,
                          int64_t* words, int64_t* first, bool decide, esc_group_decision* dec, bool node_reset,
                          hipStream_t st);
hipError_t launch_node_atomic(const NodeDev& n, const GroupDev& g, uint64_t* rows, int64_t* wide, hipStream_t st);
hipError_t launch_fill(uint64_t* p, int64_t n, uint64_t v, hipStream_t st);
hipError_t launch_wide_pods(const PodDev& p, const GroupDev& g, int64_t* wide, hipStream_t st);
hipError_t launch_wide_nodes(const NodeDev& n, const GroupDev& g, int64_t* wide, hipStream_t st);
hipError_t launch_decide(const GroupDev& g, const NodeDev& n, const int64_t* words,
                         const int64_t* first, esc_group_decision* dec, hipStream_t st);

// Ordering (K5): segmented LSD radix sort of (group, class, creation) keys.
hipError_t launch_sort_count(const NodeDev& n, const GroupDev& g, int nblk, uint32_t* hist, hipStream_t st);
hipError_t launch_scan_small(uint32_t* a, int n, uint32_t* total, hipStream_t st);
hipError_t launch_sort_expand2(const NodeDev& n, const GroupDev& g, int nblk, const uint32_t* base,
                               int64_t ts_min, uint64_t ts_div, int R, uint64_t* keys, uint32_t* vals,
                               hipStream_t st);
hipError_t launch_radix_pass(const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout,
                             int64_t n, int shift, int nblk, uint32_t* hist, hipStream_t st);
hipError_t launch_group_bounds(const uint64_t* keys, int64_t n, int key_shift, int32_t nseg, int64_t* seg,
                               hipStream_t st);

}  // namespace esc
