/*
 * escalator_hip.h — C ABI of the MI355X-native Escalator scale-decision hot path.
 *
 * The Go host (github.com/atlassian/escalator) keeps its pkg/k8s and pkg/controller
 * signatures and calls this library through a thin cgo shim.  Every
 * entry point below names the reference function it replaces (file:line, relative to
 * the reference repository root).
 *
 * Conventions
 *   - extern "C", plain pointers and sizes; no C++ or torch types cross this boundary.
 *   - Return value int32: ESC_OK (0) or a negative ESC_E_* code.  esc_strerror() gives
 *     the message.  Per-group outcomes that the reference reports as Go `error` values
 *     are carried as ESC_ST_* codes whose esc_status_string() is the reference's text
 *     verbatim.
 *   - Caller-owned input arrays are read during the call only and never retained (the
 *     cgo pointer-passing rule).  Outputs go to caller-allocated buffers.  Every array
 *     argument (and every array inside the object / SoA structs) may be NULL when its
 *     count is 0.
 *   - An esc_ctx is driven from one thread (the reference's RunOnce is a single
 *     goroutine, pkg/controller/controller.go:416).  Either one context per device and
 *     process (esc_ctx_create + esc_comm_init), or one context for several devices in one
 *     process (esc_ctx_create_multi: the fan-out and the exchange are internal).
 *
 * Hot path: group membership (a1-a7), per-pod effective requests (a8),
 * per-group int64 sums (a9, a10), node classification (a11), first-node capacity (a12),
 * gates + usage percentages + scale delta (a13-a17), and creation-time ordering (a18,
 * a19).  The HIP kernels run on gfx950; the decision arithmetic is bit-exact with the
 * Go code (int64 two's complement, IEEE float64 without contraction).
 */
#ifndef ESCALATOR_HIP_H
#define ESCALATOR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ESC_ABI_VERSION 6

/* ---------------------------------------------------------------- return codes */
#define ESC_OK          0
#define ESC_E_INVAL    -1   /* bad argument / shape                                  */
#define ESC_E_HIP      -2   /* HIP runtime error (no device, launch failure, fault)   */
#define ESC_E_NOMEM    -3   /* device or host allocation failed                      */
#define ESC_E_LIMIT    -4   /* input exceeds a documented encoding limit              */
#define ESC_E_STATE    -5   /* call order violated (e.g. decide before load)          */
#define ESC_E_NODEV    -6   /* library loaded without a usable gfx950 device          */
#define ESC_E_COMM     -7   /* RCCL not loadable, or an RCCL call failed               */
#define ESC_E_ORDER    -8   /* a K5 ordering's bounded look-back gave up: that ordering is
                               invalid (esc_sync reports it once, esc_group_order refuses it);
                               totals, decisions and the next ordering are unaffected      */

/* ------------------------------------------------------- per-group status codes
 * esc_status_string(code) returns the reference's error text verbatim.            */
#define ESC_ST_OK             0
#define ESC_ST_ERR_MIN_NODES  1  /* pkg/controller/controller.go:239 "node count less than the minimum"  */
#define ESC_ST_ERR_MAX_NODES  2  /* pkg/controller/controller.go:248 "node count larger than the maximum" */
#define ESC_ST_ERR_DIV_ZERO   3  /* pkg/controller/util.go:75 "cannot divide by zero in percent calculation" */
#define ESC_ST_ERR_NEG_DELTA  4  /* pkg/controller/util.go:43 "negative scale up delta"                   */
#define ESC_ST_ERR_OVERFLOW   5  /* a sum left int64: the reference switches Quantity to inf.Dec
                                    (apimachinery v0.22.5, not vendored) — reported, not emulated     */
#define ESC_ST_ERR_TAINT_MIN  6  /* pkg/controller/scale_down.go:150-154 (formatted; see esc_taint_error) */
#define ESC_ST_NOT_OWNED      7  /* world > 1: this group is decided on its owner rank (esc_group_owner);
                                    the record here is zero. Not a reference status.            */

/* ------------------------------------------------------------- decision branch
 * Which arm of scaleNodeGroup (pkg/controller/controller.go:192-397) produced delta. */
#define ESC_BR_EMPTY      0  /* no pods and no nodes -> 0, nil               controller.go:233 */
#define ESC_BR_GATE       1  /* min/max node-count gate error                controller.go:238-255 */
#define ESC_BR_BELOW_MIN  2  /* untainted < MinNodes -> ScaleUp(min-untainted) controller.go:281 */
#define ESC_BR_PCT_ERR    3  /* calcPercentUsage error                       controller.go:299 */
#define ESC_BR_LOCKED     4  /* scale-up lock held -> requestedNodes         controller.go:317 */
#define ESC_BR_FAST_DOWN  5  /* max% < TaintLower -> -FastNodeRemovalRate    controller.go:335 */
#define ESC_BR_SLOW_DOWN  6  /* max% < TaintUpper -> -SlowNodeRemovalRate    controller.go:338 */
#define ESC_BR_SCALE_UP   7  /* max% > ScaleUp   -> calcScaleUpDelta         controller.go:342 */
#define ESC_BR_NONE       8  /* no change                                    controller.go:377 */

/* ------------------------------------------------------------------ group spec
 * NodeGroupOptions fields the hot path reads (pkg/controller/node_group.go:20-52).
 * A group named "default" selects NewPodDefaultFilterFunc for pods
 * (pkg/controller/client.go:58-64, node_group.go:16); every group uses
 * NewNodeLabelFilterFunc(label_key, label_value) for nodes (node_group.go:278, :301). */
typedef struct esc_group_spec {
    const char* name;
    const char* label_key;
    const char* label_value;
    int32_t min_nodes;
    int32_t max_nodes;
    int32_t taint_upper_pct;     /* TaintUpperCapacityThresholdPercent */
    int32_t taint_lower_pct;     /* TaintLowerCapacityThresholdPercent */
    int32_t scale_up_pct;        /* ScaleUpThresholdPercent            */
    int32_t slow_removal_rate;   /* SlowNodeRemovalRate                */
    int32_t fast_removal_rate;   /* FastNodeRemovalRate                */
    int32_t dry_mode;            /* c.Opts.DryMode || group.DryMode (controller.go:115-117) */
} esc_group_spec;

/* Per-run host state of a group (NodeGroupState, pkg/controller/controller.go:28-44). */
typedef struct esc_group_state {
    int32_t locked;              /* nodeGroup.scaleUpLock.locked()              controller.go:317 */
    int32_t requested_nodes;     /* nodeGroup.scaleUpLock.requestedNodes        controller.go:322 */
    int64_t cached_cpu_m;        /* nodeGroup.cpuCapacity.MilliValue()          controller.go:209 */
    int64_t cached_mem_b;        /* nodeGroup.memCapacity.Value()               controller.go:210 */
} esc_group_state;

/* Per-group totals: the lister + filterNodes + Calculate*Total results. */
typedef struct esc_group_totals {
    int64_t pod_cpu_m;           /* CalculatePodsRequestsTotal cpu  pkg/k8s/util.go:27 */
    int64_t pod_mem_b;           /* CalculatePodsRequestsTotal mem                      */
    int64_t n_pods;              /* len(pods)                       controller.go:194  */
    int64_t node_cpu_m;          /* CalculateNodesCapacityTotal(untainted) cpu util.go:41, controller.go:268 */
    int64_t node_mem_b;
    int64_t n_nodes;             /* len(allNodes)                   controller.go:201  */
    int64_t n_untainted;         /* filterNodes                     controller.go:120  */
    int64_t n_tainted;
    int64_t n_cordoned;
    int64_t first_node;          /* snapshot index of allNodes[0], -1 if none  controller.go:208 */
    int64_t first_cpu_m;         /* allNodes[0].Status.Allocatable.Cpu().MilliValue() */
    int64_t first_mem_b;         /* allNodes[0].Status.Allocatable.Memory().Value()   */
    int64_t flags;               /* ESC_TF_* */
} esc_group_totals;

#define ESC_TF_POD_OVERFLOW   1  /* a pod sum left int64 (Quantity would switch to inf.Dec) */
#define ESC_TF_NODE_OVERFLOW  2  /* a node capacity sum left int64                          */
#define ESC_TF_NOT_OWNED      4  /* world > 1: totals held by the group's owner rank (zero here) */

/* Per-group scale decision. */
typedef struct esc_group_decision {
    double  cpu_pct;             /* calcPercentUsage  pkg/controller/util.go:58  */
    double  mem_pct;
    int64_t delta;               /* scaleNodeGroup's returned nodesDelta; BELOW_MIN: MinNodes-untainted;
                                    LOCKED: requestedNodes                                      */
    int64_t n_to_taint;          /* scaleDownTaint clamp (scale_down.go:138-158) when delta < 0 */
    int64_t cached_cpu_m;        /* updated cached capacity (controller.go:208-211)            */
    int64_t cached_mem_b;
    int32_t status;              /* ESC_ST_* of scaleNodeGroup                                  */
    int32_t branch;              /* ESC_BR_*                                                    */
    int32_t taint_status;        /* ESC_ST_OK or ESC_ST_ERR_TAINT_MIN                           */
    int32_t reserved;
} esc_group_decision;

/* Per-group gauges scaleNodeGroup sets on every run (pkg/metrics/metrics.go names;
 * set at controller.go:224-228, :275-278, :309-315).  `set_mask` bit ESC_M_* = the gauge
 * was Set this run; the others keep their previous value in the reference's registry
 * (a gate or early return skips them).                                              */
#define ESC_M_NODES          (1u << 0)   /* NodeGroupNodes            float64(len(allNodes))       */
#define ESC_M_NODES_CORDONED (1u << 1)   /* NodeGroupNodesCordoned                                   */
#define ESC_M_NODES_UNTAINTED (1u << 2)  /* NodeGroupNodesUntainted                                  */
#define ESC_M_NODES_TAINTED  (1u << 3)   /* NodeGroupNodesTainted                                    */
#define ESC_M_PODS           (1u << 4)   /* NodeGroupPods                                            */
#define ESC_M_CPU_REQUEST    (1u << 5)   /* NodeGroupCPURequest      float64(cpuRequest.MilliValue()) */
#define ESC_M_CPU_CAPACITY   (1u << 6)   /* NodeGroupCPUCapacity                                     */
#define ESC_M_MEM_CAPACITY   (1u << 7)   /* NodeGroupMemCapacity     float64(memCapacity.MilliValue() / 1000) */
#define ESC_M_MEM_REQUEST    (1u << 8)   /* NodeGroupMemRequest                                      */
#define ESC_M_CPU_PERCENT    (1u << 9)   /* NodeGroupsCPUPercent     0 when scaling up from 0        */
#define ESC_M_MEM_PERCENT    (1u << 10)  /* NodeGroupsMemPercent                                     */
typedef struct esc_group_metrics {
    double nodes, nodes_cordoned, nodes_untainted, nodes_tainted, pods;
    double cpu_request, cpu_capacity, mem_capacity, mem_request;
    double cpu_percent, mem_percent;
    uint32_t set_mask;
    uint32_t reserved;
} esc_group_metrics;

/* ---------------------------------------------------------- object-level input
 * What the cgo shim copies out of *v1.Pod / *v1.Node (no Go pointers retained).
 * Resource quantities arrive as Quantity.MilliValue() (cpu) and Quantity.Value()
 * (memory) with a presence flag — absent keys contribute nothing
 * (pkg/k8s/scheduler/types.go:14-43).                                              */
typedef struct esc_kv { const char* key; const char* value; } esc_kv;

typedef struct esc_request {
    int64_t cpu_m;
    int64_t mem_b;
    int32_t has_cpu;
    int32_t has_mem;
} esc_request;

typedef struct esc_selector_expr {       /* v1.NodeSelectorRequirement */
    const char*        key;
    const char*        op;               /* "In", "NotIn", "Exists", ...  only "In" matches */
    const char* const* values;
    int32_t            n_values;
    int32_t            term;             /* index of the NodeSelectorTerm it belongs to    */
} esc_selector_expr;

typedef struct esc_pod_obj {
    const char* const* owner_kinds;      /* ObjectMeta.OwnerReferences[*].Kind   util.go:11 */
    int32_t            n_owner_kinds;
    int32_t            has_config_source;/* Annotations["kubernetes.io/config.source"] present util.go:22 */
    const char*        config_source;
    const esc_kv*      node_selector;    /* Spec.NodeSelector                    node_group.go:226 */
    int32_t            n_node_selector;
    int32_t            has_affinity;     /* Spec.Affinity != nil                  node_group.go:271 */
    int32_t            has_node_affinity;
    int32_t            has_pod_affinity;
    int32_t            has_pod_anti_affinity;
    int32_t            has_required;     /* NodeAffinity.RequiredDuringScheduling... != nil node_group.go:211 */
    const esc_selector_expr* exprs;      /* flattened NodeSelectorTerms[*].MatchExpressions */
    int32_t            n_exprs;
    const esc_request* containers;       /* Spec.Containers[*].Resources.Requests  types.go:74 */
    int32_t            n_containers;
    const esc_request* init_containers;  /* Spec.InitContainers                    types.go:79 */
    int32_t            n_init_containers;
    int32_t            has_overhead;     /* Spec.Overhead != nil                   types.go:84 */
    esc_request        overhead;
} esc_pod_obj;

typedef struct esc_node_obj {
    const char*   name;
    const esc_kv* labels;                /* ObjectMeta.Labels                   node_group.go:280 */
    int32_t       n_labels;
    int32_t       unschedulable;         /* Spec.Unschedulable                   controller.go:141 */
    const char* const* taint_keys;       /* Spec.Taints[*].Key                   taint.go:80       */
    int32_t       n_taints;
    esc_request   allocatable;           /* Status.Allocatable cpu/memory        util.go:46        */
    int64_t       created_unix_ns;       /* CreationTimestamp (sec*1e9+nsec)     sort.go:19        */
} esc_node_obj;

/* ------------------------------------------------------------- packed snapshot
 * Struct-of-arrays layout streamed by the kernels.
 *
 * Selector pairs.  Every group filter is a (label_key, label_value) test
 * (NewPodAffinityFilterFunc node_group.go:218, NewNodeLabelFilterFunc :278), so pods and
 * nodes carry the (key, value) pairs they could be matched on, interned to u32 "pair
 * ids", and the kernels resolve pair -> groups on the device.  Numbering rule (shared by
 * every packer and checked by the oracle): ids 0 .. n_group_pairs-1 are the distinct
 * (label_key, label_value) of the context's groups in order of first appearance
 * (esc_ctx_pair_id); any other (key, value) whose key is some group's label_key gets an
 * id in [n_group_pairs, ESC_PAIR_LIMIT) that matches no group.  Keys no group uses are
 * never looked up by any filter and are not carried.
 *
 * Pods:
 *   flags  u32  ESC_PF_* bits + counts of extra records
 *   cpu0   u32  cpu (millicores) of the inline regular container
 *   mem0   i64  memory (bytes)   of the inline regular container
 *   pair0  u32  lowest pair id the pod selects through Spec.NodeSelector or an "In"
 *               expression of a required node-affinity term, ESC_NONE if none
 *   xc_cpu/xc_mem i64  extra containers per pod: [regular extras][init][overhead]
 *   xp_pair u32        the pod's other pair ids, ascending, de-duplicated (<= 63)
 * Nodes:
 *   nflags u32, label0 u32 (lowest label pair id), ncpu i64, nmem i64, created i64,
 *   xl_pair u32 (other label pair ids, ascending).                                  */
#define ESC_NONE 0xFFFFFFFFu
#define ESC_PAIR_LIMIT 0x7FFFFFFFu   /* pair ids are < this */

#define ESC_PF_DAEMONSET   (1u << 0)   /* PodIsDaemonSet  util.go:11   (also marks padding) */
#define ESC_PF_STATIC      (1u << 1)   /* PodIsStatic     util.go:21   */
#define ESC_PF_HAS_SEL     (1u << 2)   /* len(NodeSelector) > 0        node_group.go:271 */
#define ESC_PF_AFF_BLOCK   (1u << 3)   /* Affinity != nil && any sub-affinity != nil node_group.go:271-273 */
#define ESC_PF_HAS_OVH     (1u << 4)   /* overhead record present (Spec.Overhead != nil) */
#define ESC_PF_XREG_SHIFT  8           /* bits  8..15: regular containers beyond the inline one */
#define ESC_PF_XINIT_SHIFT 16          /* bits 16..23: init containers                         */
#define ESC_PF_XPAIR_SHIFT 24          /* bits 24..29: extra selector pairs (xp_pair)            */
#define ESC_PF_CNT_MASK    0xFFu
#define ESC_PF_PAIR_MASK   0x3Fu

#define ESC_NF_UNSCHED     (1u << 0)   /* Spec.Unschedulable           controller.go:141 */
#define ESC_NF_TAINTED     (1u << 1)   /* has atlassian.com/escalator  taint.go:31,80    */
#define ESC_NF_TRACKED     (1u << 2)   /* in some group's dry-mode taintTracker controller.go:128 */
#define ESC_NF_ABSENT      (1u << 3)   /* the slot holds no node (deleted, or a spare slot); owned by the context */
#define ESC_NF_XLBL_SHIFT  8           /* bits 8..15: extra label pairs (xl_pair)                */

typedef struct esc_pod_soa {
    int64_t         n_pods;
    const uint32_t* flags;
    const uint32_t* cpu0;
    const int64_t*  mem0;
    const uint32_t* pair0;
    const int64_t*  xc_cpu;
    const int64_t*  xc_mem;
    int64_t         n_xc;
    const uint32_t* xp_pair;
    int64_t         n_xp;
} esc_pod_soa;

typedef struct esc_node_soa {
    int64_t         n_nodes;
    const uint32_t* flags;
    const uint32_t* label0;
    const int64_t*  cpu;
    const int64_t*  mem;
    const int64_t*  created_ns;
    const uint32_t* xl_pair;
    int64_t         n_xl;
    const int32_t*  trk_node;    /* dry-mode taintTracker entries resolved to (node, group), */
    const int32_t*  trk_group;   /* sorted by (node, group); may be NULL when n_trk == 0     */
    int64_t         n_trk;
} esc_node_soa;

/* ------------------------------------------------------------------- library */
int32_t     esc_abi_version(void);
const char* esc_strerror(int32_t code);
const char* esc_status_string(int32_t status);
/* scale_down.go:150-154: "the number of nodes(%v) is less than specified minimum of %v. Taking no action" */
int32_t     esc_taint_error(int64_t n_untainted, int32_t min_nodes, char* buf, int32_t buf_len);

/* ------------------------------------------------------------------- context
 * Groups are fixed for the context's lifetime (the reference builds its listers once,
 * pkg/controller/client.go:55-64).  rank/world describe the sharding when one process
 * drives each GPU: rank r holds a contiguous shard of the pods and the whole node table,
 * of which it reduces and orders the node side of the group pairs it owns (a contiguous
 * pair range balanced by node entries, the same split on every rank: esc_group_owner,
 * DESIGN.md §7).  The pods' per-group words are reduce-scattered across ranks to each
 * group's owner inside the library (esc_comm_init + esc_step) or by the caller's collective
 * on esc_exchange_buffers; each rank then decides its OWN groups only.
 * device < 0 creates a host-only context (packer, scalar math, esc_node_owner_ranges). */
typedef struct esc_ctx esc_ctx;

int32_t esc_ctx_create(const esc_group_spec* groups, int32_t n_groups, int32_t device,
                       int32_t rank, int32_t world, esc_ctx** out);
/* One context driving n_dev devices from one thread: rank i of n_dev on
 * devices[i], one communicator set from ncclCommInitAll, and every call below fanned out
 * internally — esc_load_pods splits the pods into n_dev contiguous shards, esc_step /
 * esc_run enqueue every device's shard step, the ncclReduceScatter of the exchange words
 * inside ncclGroupStart / ncclGroupEnd and every device's decision of the groups it owns
 * (esc_results merges them: every group, as at one device); pod events are routed to the
 * shard holding the id, node events reach every device; esc_group_order answers from the
 * owner device.  The per-device calls esc_reduce, esc_exchange*, esc_decide, esc_comm_init,
 * esc_reap_* and esc_ctx_set_stream return ESC_E_STATE on it.  A device listed twice (or
 * ESC_EXCHANGE=peer) selects the peer exchange instead of RCCL: every device sums the others'
 * words over peer-mapped memory (a one-GPU machine runs several shards this way).
 * Replaces the sequential per-group loop of RunOnce, pkg/controller/controller.go:416-445. */
int32_t esc_ctx_create_multi(const esc_group_spec* groups, int32_t n_groups, const int32_t* devices,
                             int32_t n_dev, esc_ctx** out);
int32_t esc_ctx_destroy(esc_ctx* ctx);
int32_t esc_ctx_set_stream(esc_ctx* ctx, void* hip_stream);   /* NULL = ctx-owned stream */
int32_t esc_ctx_num_groups(const esc_ctx* ctx);
/* Pair id of (key,value) if some group selects it (the numbering rule above), else ESC_NONE. */
uint32_t esc_ctx_pair_id(const esc_ctx* ctx, const char* key, const char* value);
/* Number of distinct group pairs (ids 0 .. n-1). */
int32_t  esc_ctx_num_group_pairs(const esc_ctx* ctx);

/* ------------------------------------------------------------- K0 host packer
 * One pass over *v1.Pod / *v1.Node field copies: evaluates the object predicates
 * (util.go:11-24, node_group.go:208-215, :271-273, taint.go:80), interns the (key,value)
 * pairs whose key is a group label key, and packs the SoA above.  Which group a pair
 * selects is decided on the device (K1/K2), not here.                               */
typedef struct esc_packer esc_packer;
int32_t esc_packer_create(const esc_ctx* ctx, esc_packer** out);
int32_t esc_packer_destroy(esc_packer* pk);
int32_t esc_packer_add_pods(esc_packer* pk, const esc_pod_obj* pods, int64_t n);
int32_t esc_packer_add_nodes(esc_packer* pk, const esc_node_obj* nodes, int64_t n);
/* nodeGroup.taintTracker (controller.go:35) of `group`: node names, resolved at finish. */
int32_t esc_packer_set_tracker(esc_packer* pk, int32_t group, const char* const* names, int64_t n);
/* List mode, for the per-function drop-ins: every pod / node is a member of group 0,
 * no filter applied (CalculatePodsRequestsTotal / CalculateNodesCapacityTotal take an
 * already-filtered slice).                                                          */
int32_t esc_packer_set_list_mode(esc_packer* pk, int32_t list_mode);
int32_t esc_packer_view(esc_packer* pk, esc_pod_soa* pods, esc_node_soa* nodes);

/* -------------------------------------------------------------- device snapshot
 * esc_load_pods: copies this rank's pod shard (global pod indices [offset, offset+n)).
 * esc_load_nodes: copies the full node table (lo = 0, hi = n_nodes: every rank holds it)
 *   and builds its pair-major index (one entry per (label pair, node), sorted by pair then
 *   node — DESIGN.md §3); the decision reduces the pieces of the pairs this rank owns, and
 *   the age index (K5) lists the memberships of their groups.                        */
int32_t esc_load_pods(esc_ctx* ctx, const esc_pod_soa* pods, int64_t global_offset);
int32_t esc_load_nodes(esc_ctx* ctx, const esc_node_soa* nodes, int64_t lo, int64_t hi);
/* Number of device-resident copies of the pod shard to rotate through on successive
 * decisions (benchmarks use >1 so that timings are HBM-, not Infinity-Cache-, served). */
int32_t esc_set_replicas(esc_ctx* ctx, int32_t n_replicas);
/* Algorithmic HBM bytes one decision streams on this rank: K1 (pod shard) and K2
 * (this rank's node index share).  DESIGN.md §6; cross-checked by escalator_amd/layout.py. */
int32_t esc_stream_bytes(const esc_ctx* ctx, int64_t* pod_bytes, int64_t* node_bytes);
/* Sizes a host's per-pod and per-node arrays must match (esc_load_placement): pod ids
 * (esc_load_pods' count plus inserted ids) and node snapshot slots (loaded + added). */
int32_t esc_ctx_counts(const esc_ctx* ctx, int64_t* n_pod_ids, int64_t* n_nodes);
/* The rank that owns `group`'s node side: its totals' node words, its orderings
 * (esc_group_order answers on that rank; the others report 0 members). */
int32_t esc_group_owner(const esc_ctx* ctx, int32_t group, int32_t* rank);
/* The owner split as esc_load_nodes computes it, on the host only (no device needed):
 * q_bounds[r] = first group pair of rank r, q_bounds[world] = number of group pairs. */
int32_t esc_node_owner_ranges(const esc_ctx* ctx, const esc_node_soa* nodes, int32_t world, uint32_t* q_bounds);

/* ------------------------------------------------------------ scale decision
 * esc_reduce     : async. Per-shard group totals (K1 pods + K2 nodes + combine).
 * esc_exchange_buffers: device buffers to exchange between esc_reduce and esc_decide:
 *                  sum_buf  int64[sum_count]  with op SUM: the pods' per-group words
 *                  (5 per group: cpu and memory split lo32 / hi, count) in OWNER-MAJOR
 *                  rows, world x own_count / 5 rows; rank r needs only the SUM of its own
 *                  slice [r * own_count, (r + 1) * own_count) (esc_exchange_slice): a
 *                  reduce-scatter with recvcount own_count, or an all-reduce (a superset).
 *                  The node words never travel: each group's owner computes them whole.
 *                  min_buf  int64[min_count]  with op MIN (min_count 0 = nothing to
 *                  exchange: every rank holds the whole node table and resolves
 *                  allNodes[0] from it, so min_buf is NULL).
 * esc_decide     : async. K4 decide on the (exchanged) totals of the rank's own groups;
 *                  results land in the context's host buffers after esc_sync.
 * esc_run        : esc_reduce + esc_decide for world == 1, optionally graph-captured.
 * esc_sync       : waits for the queued work (records outside the fast path's packing
 *                  range are summed exactly in-kernel).               */
int32_t esc_set_state(esc_ctx* ctx, const esc_group_state* state);   /* NULL = zero state */
int32_t esc_reduce(esc_ctx* ctx);
int32_t esc_exchange_buffers(esc_ctx* ctx, void** sum_buf, int64_t* sum_count,
                             void** min_buf, int64_t* min_count);
/* This rank's slice of sum_buf (word offset, word count): the rows of the groups it owns,
 * whose SUM across ranks esc_decide reads.  At world 1: (0, sum_count). */
int32_t esc_exchange_slice(const esc_ctx* ctx, int64_t* offset, int64_t* count);
/* The owner-major row of every group (host only, like esc_node_owner_ranges): rows[g] =
 * owner * own_rows + its index among the owner's groups (ascending); *own_rows = the largest
 * owner's group count. */
int32_t esc_exchange_rows(const esc_ctx* ctx, const esc_node_soa* nodes, int32_t world, uint32_t* rows,
                          int32_t* own_rows);
/* Use caller-allocated device buffers (e.g. torch tensors handed to RCCL) as the
 * exchange buffers; sizes as reported by esc_exchange_buffers at the time of the bind
 * (a snapshot must be loaded).  NULL restores the context's own buffers (min_buf may be
 * NULL when min_count is 0).  sum_count follows the owner split, which every
 * esc_load_nodes recomputes: when a reload grows it past the bound buffer's size, every
 * call that would write the buffer returns ESC_E_STATE until a buffer of the new
 * sum_count (esc_exchange_buffers still reports it) is bound. */
int32_t esc_bind_exchange_buffers(esc_ctx* ctx, void* sum_buf, void* min_buf);
/* Host-staged exchange for hosts without a device collective (synchronous); the min
 * arrays are ignored (may be NULL) when min_count is 0. */
int32_t esc_exchange_download(esc_ctx* ctx, int64_t* sum_out, int64_t* min_out);
int32_t esc_exchange_upload(esc_ctx* ctx, const int64_t* sum_in, const int64_t* min_in);
int32_t esc_decide(esc_ctx* ctx);
int32_t esc_run(esc_ctx* ctx);
int32_t esc_sync(esc_ctx* ctx);
/* RCCL exchange inside the library (replaces the sequential per-group loop
 * of RunOnce, pkg/controller/controller.go:416-445, by one sharded decision).  One process
 * per GPU: rank 0 calls esc_comm_unique_id and ships the ESC_COMM_ID_BYTES bytes to the
 * other ranks over any host channel; every rank then calls esc_comm_init (collective,
 * blocking until all ranks joined; rank / world must equal the context's).  esc_exchange
 * enqueues ncclReduceScatter(int64, SUM) of the pod words (esc_exchange_buffers) in place
 * on the context's stream, every rank receiving its own slice (esc_exchange_slice);
 * esc_step = esc_reduce + esc_exchange + esc_decide (esc_run when
 * world == 1 and no communicator was set up).  The library resolves librccl at run time
 * (the copy already loaded in the process, else librccl.so.1).                         */
#define ESC_COMM_ID_BYTES 128
int32_t esc_comm_unique_id(void* id_out);
int32_t esc_comm_init(esc_ctx* ctx, const void* id, int32_t rank, int32_t world);
int32_t esc_exchange(esc_ctx* ctx);
int32_t esc_step(esc_ctx* ctx);
/* Ranks of the context's RCCL communicator (ncclCommCount; a multi-device context: of its
 * ncclCommInitAll communicators).  0 for a multi-device context on the peer exchange (no
 * communicator exists); ESC_E_STATE for a per-device context before esc_comm_init. */
int32_t esc_comm_size(const esc_ctx* ctx, int32_t* ranks);
/* Every group's totals and decision.  world > 1 (one process per GPU): the rank's own
 * groups; the others' records are zero, flagged ESC_TF_NOT_OWNED / ESC_ST_NOT_OWNED (their
 * owner's esc_results holds them).  A multi-device context returns every group. */
int32_t esc_results(esc_ctx* ctx, esc_group_totals* totals, esc_group_decision* decisions);
/* Metric gauges (§8f): computed by K4 beside the decisions when enabled (off by default;
 * they stay in device memory until esc_metrics_results copies them out, after esc_sync). */
int32_t esc_set_metrics(esc_ctx* ctx, int32_t enable);
int32_t esc_metrics_results(esc_ctx* ctx, esc_group_metrics* out);
int32_t esc_use_graph(esc_ctx* ctx, int32_t enable);
int32_t esc_force_wide(esc_ctx* ctx, int32_t enable);   /* testing: always take the wide path */
/* Device time in ms per stage of the last decision (timing mode), see DESIGN.md §6:
 * [0] K1, [1] the fused tail, [2] the remaining orderings, [3] node groups (+ K4 at world
 * 1), then at world > 1 [4] the exchange (esc_exchange) and [5] K4 (esc_decide);
 * ms_out[9] = the whole step (first to last event). */
int32_t esc_set_timing(esc_ctx* ctx, int32_t enable);
int32_t esc_stage_times(esc_ctx* ctx, double* ms_out, int32_t n);
/* K1 records per workgroup 8 words (s_memrealtime ticks at 100 MHz at start / after the K
 * tiles / after the C tiles / after the flush, HW_ID, XCC_ID, class runs of its work plan,
 * K weight of those runs in 16-B lane loads) of the last decision;
 * this copies them out (after esc_sync).  *n_out = workgroups; ESC_E_STATE before a run. */
int32_t esc_k1_trace(esc_ctx* ctx, uint64_t* out, int64_t cap_words, int64_t* n_out);
/* K1's device time (measurement): `reps` back-to-back K1 launches over the
 * current snapshot, rotating over its replicas as decisions do (esc_set_replicas: a replica
 * small enough for the Infinity Cache is not re-read from it), between two HIP events on
 * the context's stream; *ms_per_launch = elapsed / reps.  Synchronous; leaves every
 * decision result as it was. */
int32_t esc_k1_time(esc_ctx* ctx, int32_t reps, double* ms_per_launch);
/* Calibrates K1's work split on this device: `rounds` decisions, each moving
 * every workgroup's share of the pod bytes toward its measured streaming rate.  Results are
 * unchanged (integer sums are order-independent); call once after loading a snapshot. */
int32_t esc_k1_calibrate(esc_ctx* ctx, int32_t rounds);
/* K1's partial flush: *entries = 512-B column partials K1 writes (and K3 reads)
 * per decision, *full = entries of a whole-row flush (workgroups x pod-slot columns); equal
 * when the compact flush is off.  Multi-device: summed over the devices. */
int32_t esc_k1_flush_entries(const esc_ctx* ctx, int64_t* entries, int64_t* full);
/* The device's practical HBM read rate in K1's access shape (a contiguous share per
 * 512-thread workgroup, 16-B nontemporal loads, 8 in flight per lane) over a fresh buffer
 * of `bytes` (> the 256 MB Infinity Cache, so HBM-served): best of `reps` launches, GB/s.
 * The ceiling a roofline fraction of this box is read against (MI355X boards differ). */
int32_t esc_hbm_probe(esc_ctx* ctx, int64_t bytes, int32_t reps, double* read_gbps);

/* ------------------------------------------- incremental snapshot (§8f rank 1)
 * Informer-style events patch the resident snapshot in place instead of a reload
 * (the reference re-lists every pod and node per group per decision through its
 * informer caches, pkg/k8s/cache.go:16-56 -> pod_listers.go:33, node_listers.go:33).
 * Pod ids are the indices of esc_load_pods' input; new ids (< 2^31) insert.  A pod
 * lands in the spare slots of its record-signature class (esc_set_spare, before the
 * load, reserves them); a pod with > 3 container records or > 3 extra pairs (or whose
 * class is full) stays in its own C-section slot when that has room, else takes a spare
 * C slot (room for 4 extra regular and 2 init containers, an overhead and 6 extra pairs;
 * unused records stay neutral).  A batch that does not fit in place returns ESC_E_LIMIT
 * with nothing applied, and the caller reloads.  esc_nodes_update may change
 * Spec.Unschedulable, the escalator taint and allocatable; label or creation-time changes
 * go through esc_nodes_relabel (tracker changes: esc_tracker_update).  Every call
 * completes before returning.                                                       */
int32_t esc_set_spare(esc_ctx* ctx, double fraction);       /* spare room: per K pod class (esc_load_pods),
                                                                node slots / entries / K5 regions (esc_load_nodes) */
int32_t esc_pods_upsert(esc_ctx* ctx, const int64_t* ids, const esc_pod_soa* pods);
int32_t esc_pods_delete(esc_ctx* ctx, const int64_t* ids, int64_t n);
int32_t esc_nodes_update(esc_ctx* ctx, const int64_t* ids, int64_t n, const uint32_t* flags,
                         const int64_t* cpu_m, const int64_t* mem_b);
/* Node additions and deletions (the node informer's Add / Delete, pkg/k8s/cache.go:37-56)
 * in place.  esc_set_spare(f) before esc_load_nodes reserves room: table slots, spare
 * pair-major entries per group label pair and spare slots in every group's K5 region.
 * esc_nodes_add appends the nodes (packed like esc_load_nodes' input, n_trk = 0, no
 * ESC_NF_TRACKED) at the next snapshot indices, returned in ids_out: the lister order
 * lists them after every loaded node.  esc_nodes_delete removes nodes by index: the slot
 * becomes ESC_NF_ABSENT (no kernel counts it, allNodes[0] moves to the group's next
 * member) and its dry-mode tracker entries are dropped (a host that re-adds a tracked
 * name re-applies it with esc_tracker_update).  Both keep esc_load_placement's binding
 * (an added node starts with no pods, no taint time and no no-delete flag until
 * esc_pods_bind / a node-facts refresh); an add that does not fit returns ESC_E_LIMIT
 * with nothing applied (reload).  Every check
 * depends on the node table alone, which every rank holds, so all ranks of a sharded job
 * accept or refuse the same batch. */
int32_t esc_nodes_add(esc_ctx* ctx, const esc_node_soa* nodes, int64_t* ids_out);
int32_t esc_nodes_delete(esc_ctx* ctx, const int64_t* ids, int64_t n);
/* Node informer Update events that change any field of a node — its labels and creation
 * time included — in place (the reference re-reads the labels on every List:
 * NewNodeLabelFilterFunc pkg/controller/node_group.go:278-287 via FilteredNodesLister.List
 * pkg/k8s/node_listers.go:33-48, fed by pkg/k8s/cache.go:37-56).  `nodes` holds the new
 * packed records of the n = nodes->n_nodes nodes ids[0..n) (as esc_nodes_add's input:
 * n_trk = 0; a caller's ESC_NF_TRACKED bit is ignored, the tracker is the context's).  The
 * nodes keep their snapshot indices; they leave the groups whose pair they no longer carry
 * and join those whose pair they now carry (spare pair-major entries and K5 region slots,
 * esc_set_spare), allNodes[0] follows, a placement's occupancy follows.  A node that
 * returns to a pair it carried before reuses its own retired entry of that pair, so label
 * churn (A -> B -> A ...) takes spare room once per (node, pair), not per flip.  All or
 * nothing: ESC_E_LIMIT when the spare room is short (reload), ESC_E_INVAL for a bad or
 * absent id; a device failure after the first change marks the node side stale (decisions
 * and reaping return ESC_E_STATE until esc_load_nodes). */
int32_t esc_nodes_relabel(esc_ctx* ctx, const int64_t* ids, const esc_node_soa* nodes);

/* ------------------------------------------- dry-mode taintTracker (§8f rank 4)
 * nodeGroup.taintTracker (controller.go:35) as interned (node, group) pairs on the
 * device.  In dry mode taintOldestN appends the names it "taints" (scale_down.go:197-200)
 * and untaintNewestN deletes them (scale_up.go:146-158); filterNodes then splits a dry
 * group's nodes by tracker membership (controller.go:126-138).  esc_tracker_update applies
 * such a change for one group in place (no reload): `remove` first — nodes the group does
 * not track are ignored, like untaintNewestN's deleteIndex == -1 — then `add`; adding a
 * node the group already tracks (or twice) is ESC_E_INVAL with nothing applied (the
 * reference only appends untracked nodes, so its slice never holds a duplicate).  The
 * node's ESC_NF_TRACKED bit is maintained here: esc_nodes_update ignores the caller's.
 * esc_tracker_list returns the group's tracked node indices, ascending.              */
int32_t esc_tracker_update(esc_ctx* ctx, int32_t group, const int64_t* add, int64_t n_add,
                           const int64_t* remove, int64_t n_remove);
int32_t esc_tracker_list(const esc_ctx* ctx, int32_t group, int64_t* idx_out, int64_t cap, int64_t* n_out);

/* ------------------------------------------ scale-down reaping (§8f rank 2)
 * TryRemoveTaintedNodes (pkg/controller/scale_down.go:51-136) with NodeEmpty /
 * NodePodsRemaining over the group's NodeInfoMap (pkg/k8s/node_state.go:10-65), for every
 * group at once.  esc_load_placement binds the loaded pods to nodes (Spec.NodeName as a
 * snapshot node index, ESC_NONE when empty or not a known node — CreateNodeNameToInfoMap
 * drops those) and gives each node its escalator-taint time (GetToBeRemovedTime,
 * taint.go:91: Unix seconds, INT64_MIN when the taint is absent or its value does not
 * parse) and its atlassian.com/no-delete annotation (non-empty = safe from deletion).
 * Pod events keep the binding current: esc_pods_upsert rewrites a bound pod's reference,
 * esc_pods_delete drops it, esc_pods_bind moves pods between nodes (runs per node keep
 * esc_set_spare room; ESC_E_LIMIT when a run is full).  Node additions / deletions keep
 * it: every node-table slot (esc_set_spare's free slots included) has a run and facts, a
 * free slot's run sized for the mean pods per node plus the spare fraction; refresh the
 * facts (esc_load_placement with pod_node NULL, n_nodes entries: the table as it is now,
 * deleted slots included) when taints change.  esc_try_remove then evaluates, per
 * group, its tainted nodes in snapshot order: now - taintTime > soft grace and (NodeEmpty
 * or > hard grace) -> delete (never in dry mode).
 * Several ranks (each holding its pod shard): the per-node occupancy is this rank's pods
 * only, so esc_try_remove sums the occupancy words across ranks over the context's RCCL
 * communicator (esc_comm_init) between K6 and K7; hosts with their own collective use
 * esc_reap_occupancy, SUM-all-reduce esc_reap_buffer's uint32 words (or
 * esc_reap_download / esc_reap_upload), then esc_reap_finish.                        */
typedef struct esc_removal {
    int64_t n_candidates;        /* the group's tainted nodes (filterNodes)                    */
    int64_t n_delete;            /* len(toBeDeleted): TryRemoveTaintedNodes returns -n_delete  */
    int64_t pods_remaining;      /* sum of NodePodsRemaining over them (NodeGroupPodsEvicted)  */
    int64_t reserved;
} esc_removal;
int32_t esc_load_placement(esc_ctx* ctx, const uint32_t* pod_node, const int64_t* taint_unix_s,
                           const uint8_t* no_delete);
int32_t esc_try_remove(esc_ctx* ctx, int64_t now_unix_ns, const int64_t* soft_grace_ns,
                       const int64_t* hard_grace_ns, esc_removal* out);
int32_t esc_pods_bind(esc_ctx* ctx, const int64_t* ids, const uint32_t* pod_node, int64_t n);
int32_t esc_reap_occupancy(esc_ctx* ctx);
int32_t esc_reap_buffer(esc_ctx* ctx, void** buf, int64_t* n_words);
int32_t esc_reap_download(esc_ctx* ctx, uint32_t* out);
int32_t esc_reap_upload(esc_ctx* ctx, const uint32_t* in);
int32_t esc_reap_finish(esc_ctx* ctx, int64_t now_unix_ns, const int64_t* soft_grace_ns,
                        const int64_t* hard_grace_ns, esc_removal* out);
int32_t esc_removal_nodes(esc_ctx* ctx, int32_t group, int64_t* idx_out, int64_t cap, int64_t* n_out);

/* ----------------------------------------------------------------- ordering
 * K5: per-group creation-time order of the context's node shard (a18/a19):
 *   which 0: untainted members oldest-first (taintOldestN,   scale_down.go:171)
 *   which 1: tainted members newest-first   (untaintNewestN, scale_up.go:118)
 * Writes up to `cap` snapshot node indices; *n_out = number of members in that list.
 * Ties (equal timestamps) are broken by snapshot index (Go's sort.Sort is unstable,
 * so its tie order is not reproducible).                             */
/* esc_load_nodes builds the AGE INDEX once per snapshot: the group memberships listed in
 * one pass and sorted by (group, creation time) (LSD radix sort of coarse keys + an exact
 * fix-up of equal-key runs; exact 64-bit keys when a run is too long).
 * esc_sort_nodes (async, per decision) classifies every membership (filterNodes,
 * controller.go:120-154) and stable-partitions by (group, class) in one pass: a group's
 * untainted segment is stored oldest-first from its region's start, its tainted segment
 * newest-first from its region's end (esc_group_order reads both forward).
 * esc_build_age_index rebuilds the index (snapshot ingestion; exposed for measurement).
 * The index carries node indices in 28 bits: a node table of 2^28 slots or more returns
 * ESC_E_LIMIT.  Its group starts come from the host's live entry counts; the device's own
 * total is checked against them on a fresh build (every build with ESC_CHECK_INDEX=1),
 * a mismatch (or a listing chunk that gave up its bounded wait) returning ESC_E_HIP.       */
int32_t esc_sort_nodes(esc_ctx* ctx);
/* (esc_sort_nodes' look-backs are bounded waits: a chunk that gives up leaves that ordering
 * invalid and is reported as ESC_E_ORDER — once by esc_sync, and by esc_group_order and
 * esc_selections until the next ordering; the next ordering runs afresh.) */
/* Include the per-decision ordering in every decision (esc_run / esc_reduce / esc_step):
 * the packed small groups are ordered by blocks of the step's fused tail launch (after K1,
 * beside the fold and K2), the larger groups by the split kernel right after it, all on
 * the context's one stream (and in its graph when esc_use_graph); esc_group_order is then
 * valid after each decision without a separate esc_sort_nodes (one
 * decision = membership, sums, percentages, deltas and oldest-first ordering). */
int32_t esc_set_order_in_step(esc_ctx* ctx, int32_t enable);
int32_t esc_build_age_index(esc_ctx* ctx);
/* Size of the ordering problem: memberships of the node range and the bit width of the
 * creation-offset keys the index sorts on. */
int32_t esc_order_info(const esc_ctx* ctx, int64_t* n_memberships, int32_t* key_bits);
int32_t esc_group_order(esc_ctx* ctx, int32_t group, int32_t which,
                        int64_t* idx_out, int64_t cap, int64_t* n_out);

/* Selections delivered WITH the decision (controller.go:367-383: ScaleDown -> taintOldestN,
 * scale_down.go:171-205; ScaleUp -> untaintNewestN, scale_up.go:118-163), so a host walks
 * them without one esc_group_order round trip per group.  esc_set_selections(slack >= 0)
 * turns them on (the ordering must be in the step: esc_set_order_in_step), slack < 0 off;
 * group_cap <= 0 means 256.  Every decision then writes, for every group it decides:
 *   delta < 0 with taint_status ESC_ST_OK: the first min(n_to_taint + slack, untainted)
 *     untainted nodes, oldest first (ESC_SEL_TAINT);
 *   delta > 0 (scale-up and below-minimum branches): the first min(delta + slack, tainted)
 *     tainted nodes, newest first (ESC_SEL_UNTAINT);
 * at most group_cap nodes, ties by ascending snapshot index (as esc_group_order).  `slack`
 * covers the API writes that fail: the reference's walk skips a node whose taint / untaint
 * fails and goes on down the order.  The nodes go to pinned host memory inside the step
 * (zero-copy), so esc_selections copies nothing from the device. */
int32_t esc_set_selections(esc_ctx* ctx, int32_t slack, int32_t group_cap);
#define ESC_SEL_NONE    -1   /* the decision asks for no walk                          */
#define ESC_SEL_TAINT    0   /* untainted nodes, oldest first (taintOldestN)           */
#define ESC_SEL_UNTAINT  1   /* tainted nodes, newest first (untaintNewestN)            */
#define ESC_SEL_CUT      4   /* or'ed: the walk may need more than the list holds (group_cap,
                                or a tie run too long to resolve in-kernel: then the list is
                                empty): continue with esc_group_order                   */
/* After a decision: which[g] (ESC_SEL_*) and offsets[g] .. offsets[g + 1] (G + 1 entries)
 * of group g's nodes in idx (snapshot indices); idx == NULL (cap 0) fills which, offsets and
 * *n_total only (the size idx needs; ESC_E_LIMIT when cap is short).  world > 1: the rank's
 * own groups (the others ESC_SEL_NONE); a multi-device context: every group.  ESC_E_STATE
 * when selections are off; ESC_E_ORDER when the decision's ordering gave up (then use
 * esc_sort_nodes + esc_group_order). */
int32_t esc_selections(esc_ctx* ctx, int32_t* which, int64_t* offsets, int64_t* idx, int64_t cap, int64_t* n_total);

/* ----------------------------------------------- per-function drop-ins (GPU)
 * Same argument meaning as the Go functions; these pack the given slice in list mode
 * and run the batched kernels on it.                                                */
/* pkg/k8s/util.go:27 — returns (mem, cpu) like the Go function. */
int32_t esc_pods_requests_total(esc_ctx* ctx, const esc_pod_obj* pods, int64_t n,
                                int64_t* mem_b, int64_t* cpu_m);
/* pkg/k8s/util.go:41 */
int32_t esc_nodes_capacity_total(esc_ctx* ctx, const esc_node_obj* nodes, int64_t n,
                                 int64_t* mem_b, int64_t* cpu_m);
/* pkg/controller/scale_down.go:171 / scale_up.go:118 — indices into the given slice;
 * oldest != 0: oldest first, else newest first; returns min(n_take, n) indices.      */
int32_t esc_order_by_creation(esc_ctx* ctx, const int64_t* created_ns, int64_t n,
                              int32_t oldest, int64_t n_take, int64_t* idx_out);

/* --------------------------------------------- scalar decision math (host)
 * Bit-exact restatements used by the shim for single calls; the batched path runs
 * the same __host__ __device__ code inside the K4 kernel.                            */
/* pkg/controller/util.go:58 — returns ESC_ST_OK or ESC_ST_ERR_DIV_ZERO. */
int32_t esc_calc_percent_usage(int64_t cpu_req_m, int64_t mem_req_b, int64_t cpu_cap_m,
                               int64_t mem_cap_b, int64_t n_untainted,
                               double* cpu_pct, double* mem_pct);
/* pkg/controller/util.go:13 — returns ESC_ST_OK or ESC_ST_ERR_NEG_DELTA. */
int32_t esc_calc_scale_up_delta(int64_t n_untainted, double cpu_pct, double mem_pct,
                                int64_t cpu_req_m, int64_t mem_req_b,
                                int64_t cached_cpu_m, int64_t cached_mem_b,
                                int32_t scale_up_pct, int64_t* delta);

/* ------------------------------------------------- synthetic snapshots (bench)
 * Deterministic counter-hash generator of BASELINE.md's configs; fills the SoA of
 * pods [p_lo, p_hi) and nodes, plus the group specs.  Host memory is owned by the
 * returned handle.                                                                  */
typedef struct esc_synth esc_synth;
typedef struct esc_synth_params {
    int64_t  n_pods;
    int64_t  n_nodes;
    int32_t  n_groups;
    int32_t  config;             /* 1..5: BASELINE.md §3 row, selects distributions  */
    uint64_t seed;
    int32_t  with_default;       /* group 0 named "default"                          */
    int32_t  n_threads;          /* host threads for generation (0 = 1)              */
} esc_synth_params;
int32_t esc_synth_create(const esc_synth_params* p, int64_t p_lo, int64_t p_hi, esc_synth** out);
int32_t esc_synth_destroy(esc_synth* s);
int32_t esc_synth_groups(const esc_synth* s, const esc_group_spec** groups, int32_t* n);
int32_t esc_synth_states(const esc_synth* s, const esc_group_state** states);
int32_t esc_synth_view(const esc_synth* s, esc_pod_soa* pods, esc_node_soa* nodes);
/* The same snapshot as object structs (what the cgo shim fills from *v1.Pod / *v1.Node), for
 * timing the K0 packer and checking it against the generator; owned by the handle. */
int32_t esc_synth_objects(esc_synth* s, const esc_pod_obj** pods, int64_t* n_pods, const esc_node_obj** nodes,
                          int64_t* n_nodes);

#ifdef __cplusplus
}
#endif
#endif /* ESCALATOR_HIP_H */
