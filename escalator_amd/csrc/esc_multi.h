// esc_multi.h — RCCL entry points resolved at run time, and the single-process
// multi-device context (esc_ctx_create_multi, esc_multi.hip) behind the C ABI.
#pragma once

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "escalator_hip.h"

namespace esc {

// RCCL is resolved at first use: the copy already mapped into the process if there is one
// (PyTorch-ROCm ships its own librccl, and two RCCL instances in one process would each
// run their own proxy threads), else the system librccl.so.1.  Hosts that never exchange
// (world 1, the per-function drop-ins) need no RCCL at all.
struct RcclApi {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommCount) count = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
};
const RcclApi& rccl();

// Accessors the multi-device layer needs beyond the public ABI (esc_runtime.hip).
struct esc_multi_state;
esc_multi_state* ctx_multi(const esc_ctx* c);
void ctx_set_multi(esc_ctx* c, esc_multi_state* m);
hipStream_t ctx_stream(const esc_ctx* c);
int ctx_device(const esc_ctx* c);
// timing mode: one more stage boundary on the context's stream (the exchange's end)
int32_t ctx_stage_mark(esc_ctx* c);
int32_t fail_comm(const char* what, const char* why);
int32_t fail_hip(hipError_t e, const char* what);
// check phases of esc_pods_upsert / esc_pods_bind (nothing applied)
int32_t pods_upsert_check(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p);
int32_t pods_bind_check(esc_ctx* c, const int64_t* ids, const uint32_t* pod_node, int64_t n);
int32_t nodes_relabel_check(esc_ctx* c, const int64_t* ids, const esc_node_soa* s);

// ---- the multi-device context: every ABI call on it dispatches to these (esc_multi.hip)
void multi_destroy(esc_ctx* c);
int32_t multi_set_replicas(esc_ctx* c, int32_t n);
int32_t multi_load_pods(esc_ctx* c, const esc_pod_soa* p, int64_t global_offset);
int32_t multi_load_nodes(esc_ctx* c, const esc_node_soa* s, int64_t lo, int64_t hi);
int32_t multi_stream_bytes(const esc_ctx* c, int64_t* pod_bytes, int64_t* node_bytes);
int32_t multi_set_state(esc_ctx* c, const esc_group_state* st);
int32_t multi_step(esc_ctx* c);
int32_t multi_sync(esc_ctx* c);
int32_t multi_results(esc_ctx* c, esc_group_totals* t, esc_group_decision* d);
int32_t multi_metrics_results(esc_ctx* c, esc_group_metrics* out);
int32_t multi_each(esc_ctx* c, int32_t (*fn)(esc_ctx*, int32_t), int32_t arg);   // a setter on every device
esc_ctx* multi_sub(const esc_ctx* c, int i);                                     // device i's context
int32_t multi_k1_calibrate(esc_ctx* c, int32_t rounds);
int32_t multi_pods_upsert(esc_ctx* c, const int64_t* ids, const esc_pod_soa* p);
int32_t multi_pods_delete(esc_ctx* c, const int64_t* ids, int64_t n);
int32_t multi_pods_bind(esc_ctx* c, const int64_t* ids, const uint32_t* pod_node, int64_t n);
int32_t multi_nodes_update(esc_ctx* c, const int64_t* ids, int64_t n, const uint32_t* flags, const int64_t* cpu,
                           const int64_t* mem);
int32_t multi_nodes_add(esc_ctx* c, const esc_node_soa* s, int64_t* ids_out);
int32_t multi_nodes_delete(esc_ctx* c, const int64_t* ids, int64_t n);
int32_t multi_nodes_relabel(esc_ctx* c, const int64_t* ids, const esc_node_soa* s);
int32_t multi_tracker_update(esc_ctx* c, int32_t group, const int64_t* add, int64_t n_add, const int64_t* rm,
                             int64_t n_rm);
int32_t multi_load_placement(esc_ctx* c, const uint32_t* pod_node, const int64_t* taint_s, const uint8_t* no_delete);
int32_t multi_try_remove(esc_ctx* c, int64_t now_ns, const int64_t* soft, const int64_t* hard, esc_removal* out);
int32_t multi_order_info(const esc_ctx* c, int64_t* n_memb, int32_t* key_bits);
int32_t multi_group_order(esc_ctx* c, int32_t group, int32_t which, int64_t* idx, int64_t cap, int64_t* n_out);
int32_t multi_counts(const esc_ctx* c, int64_t* n_pod_ids, int64_t* n_nodes);
int32_t multi_size(const esc_ctx* c);

}  // namespace esc
