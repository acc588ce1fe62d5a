// Package escalatorhip binds Escalator's scale-decision hot path to the MI355X library
// libescalator_hip.so through its C ABI (include/escalator_hip.h).
//
// A maintainer adds this package to github.com/atlassian/escalator as pkg/escalatorhip
// (module path adjusted) and calls it from pkg/k8s and pkg/controller as INTEGRATION.md
// shows.  The exported functions keep the reference's signatures:
//
//	CalculatePodsRequestsTotal   pkg/k8s/util.go:27
//	CalculateNodesCapacityTotal  pkg/k8s/util.go:41
//	CalcPercentUsage             pkg/controller/util.go:58 (unexported there)
//	CalcScaleUpDelta             pkg/controller/util.go:13 (unexported there)
//
// and (*Context).RunOnce replaces the per-group loop of (*Controller).RunOnce
// (pkg/controller/controller.go:416-445 -> scaleNodeGroup :192-351) by one batched decision
// for every node group.
//
// No Go toolchain exists in the image this package was written in, so it has not been
// compiled there; go/escalatorhip/harness/esc_harness.c makes the same ABI calls in the
// same order from C and is run by the repository's tests (tests/test_harness.py).
package escalatorhip

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../escalator_amd -lescalator_hip -Wl,-rpath,${SRCDIR}/../../escalator_amd
#include <stdlib.h>
#include <string.h>
#include "escalator_hip.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/api/resource"
)

// ErrNoDevice is returned when the library finds no gfx950 device; the caller keeps the
// reference's Go path in that case.
var ErrNoDevice = errors.New(C.GoString(C.esc_strerror(C.ESC_E_NODEV)))

func rcErr(call string, rc C.int32_t) error {
	switch rc {
	case C.ESC_OK:
		return nil
	case C.ESC_E_NODEV:
		return ErrNoDevice
	}
	return fmt.Errorf("%s: %s", call, C.GoString(C.esc_strerror(rc)))
}

// statusErr is the reference's `error` value for a per-group status, text verbatim
// (controller.go:239, :248, util.go:43, :75).
func statusErr(st C.int32_t) error {
	if st == C.ESC_ST_OK {
		return nil
	}
	return errors.New(C.GoString(C.esc_status_string(st)))
}

// ------------------------------------------------------------------------ arena

// arena owns every C copy made for one call.  cgo forbids passing Go memory that holds
// Go pointers, so strings and object structs are built in C memory and freed after the
// call; the library never retains its inputs.
type arena struct{ ptrs []unsafe.Pointer }

func (a *arena) cstr(s string) *C.char {
	p := C.CString(s)
	a.ptrs = append(a.ptrs, unsafe.Pointer(p))
	return p
}

func (a *arena) alloc(n int, size uintptr) unsafe.Pointer {
	if n == 0 {
		n = 1
	}
	p := C.calloc(C.size_t(n), C.size_t(size))
	if p == nil {
		panic("escalatorhip: out of C memory")
	}
	a.ptrs = append(a.ptrs, p)
	return p
}

func (a *arena) free() {
	for _, p := range a.ptrs {
		C.free(p)
	}
	a.ptrs = nil
}

// ptr is &s[0], or nil for an empty slice: &s[0] of a zero-length slice panics, and the
// ABI takes NULL with a zero count for every array (include/escalator_hip.h conventions).
// Every slice handed to C goes through it.
func ptr[T any](s []T) *T {
	if len(s) == 0 {
		return nil
	}
	return &s[0]
}

// cslice is n zeroed elements of C memory owned by the arena, or nil when n == 0.
func cslice[T any](a *arena, n int) []T {
	if n == 0 {
		return nil
	}
	var z T
	return unsafe.Slice((*T)(a.alloc(n, unsafe.Sizeof(z))), n)
}

func (a *arena) cstrs(ss []string) **C.char {
	arr := cslice[*C.char](a, len(ss))
	for i, s := range ss {
		arr[i] = a.cstr(s)
	}
	return ptr(arr)
}

func (a *arena) kvs(m map[string]string) (*C.esc_kv, C.int32_t) {
	arr := cslice[C.esc_kv](a, len(m))
	i := 0
	for k, v := range m { // map order is irrelevant: pairs are interned and de-duplicated
		arr[i].key = a.cstr(k)
		arr[i].value = a.cstr(v)
		i++
	}
	return ptr(arr), C.int32_t(len(m))
}

// request copies one ResourceList: cpu as MilliValue, memory as Value, with presence flags
// (an absent key adds nothing, pkg/k8s/scheduler/types.go:14-43).
func request(rl v1.ResourceList) C.esc_request {
	var r C.esc_request
	if q, ok := rl[v1.ResourceCPU]; ok {
		r.cpu_m = C.int64_t(q.MilliValue())
		r.has_cpu = 1
	}
	if q, ok := rl[v1.ResourceMemory]; ok {
		r.mem_b = C.int64_t(q.Value())
		r.has_mem = 1
	}
	return r
}

func (a *arena) requests(cs []v1.Container) (*C.esc_request, C.int32_t) {
	arr := cslice[C.esc_request](a, len(cs))
	for i := range cs {
		arr[i] = request(cs[i].Resources.Requests) // types.go:74-83
	}
	return ptr(arr), C.int32_t(len(cs))
}

// podObj copies the fields the hot path reads from a pod (esc_pod_obj).
func (a *arena) podObj(p *v1.Pod, o *C.esc_pod_obj) {
	kinds := make([]string, 0, len(p.ObjectMeta.OwnerReferences))
	for _, ref := range p.ObjectMeta.OwnerReferences { // PodIsDaemonSet, util.go:11-18
		kinds = append(kinds, ref.Kind)
	}
	o.owner_kinds = a.cstrs(kinds)
	o.n_owner_kinds = C.int32_t(len(kinds))
	if src, ok := p.ObjectMeta.Annotations["kubernetes.io/config.source"]; ok { // PodIsStatic, util.go:21-24
		o.has_config_source = 1
		o.config_source = a.cstr(src)
	} else {
		o.config_source = a.cstr("")
	}
	o.node_selector, o.n_node_selector = a.kvs(p.Spec.NodeSelector) // node_group.go:226
	var exprs []C.esc_selector_expr
	if aff := p.Spec.Affinity; aff != nil { // node_group.go:208-215, :271-273
		o.has_affinity = 1
		if aff.PodAffinity != nil {
			o.has_pod_affinity = 1
		}
		if aff.PodAntiAffinity != nil {
			o.has_pod_anti_affinity = 1
		}
		if na := aff.NodeAffinity; na != nil {
			o.has_node_affinity = 1
			if req := na.RequiredDuringSchedulingIgnoredDuringExecution; req != nil {
				o.has_required = 1
				for t, term := range req.NodeSelectorTerms {
					for _, e := range term.MatchExpressions {
						exprs = append(exprs, C.esc_selector_expr{
							key:      a.cstr(e.Key),
							op:       a.cstr(string(e.Operator)),
							values:   a.cstrs(e.Values),
							n_values: C.int32_t(len(e.Values)),
							term:     C.int32_t(t),
						})
					}
				}
			}
		}
	}
	arr := cslice[C.esc_selector_expr](a, len(exprs))
	copy(arr, exprs)
	o.exprs = ptr(arr)
	o.n_exprs = C.int32_t(len(exprs))
	o.containers, o.n_containers = a.requests(p.Spec.Containers)
	o.init_containers, o.n_init_containers = a.requests(p.Spec.InitContainers)
	if p.Spec.Overhead != nil { // types.go:84-87
		o.has_overhead = 1
		o.overhead = request(p.Spec.Overhead)
	}
}

// nodeObj copies the fields the hot path reads from a node (esc_node_obj).
func (a *arena) nodeObj(n *v1.Node, o *C.esc_node_obj) {
	o.name = a.cstr(n.Name)
	o.labels, o.n_labels = a.kvs(n.Labels) // NewNodeLabelFilterFunc, node_group.go:278-287
	if n.Spec.Unschedulable {              // filterNodes, controller.go:141
		o.unschedulable = 1
	}
	keys := make([]string, len(n.Spec.Taints))
	for i, t := range n.Spec.Taints { // GetToBeRemovedTaint, taint.go:80-87
		keys[i] = t.Key
	}
	o.taint_keys = a.cstrs(keys)
	o.n_taints = C.int32_t(len(keys))
	o.allocatable = request(n.Status.Allocatable)                  // util.go:46-47
	o.created_unix_ns = C.int64_t(n.CreationTimestamp.UnixNano()) // sort.go:19
}

func (a *arena) pods(pods []*v1.Pod) (*C.esc_pod_obj, C.int64_t) {
	objs := cslice[C.esc_pod_obj](a, len(pods))
	for i, p := range pods {
		a.podObj(p, &objs[i])
	}
	return ptr(objs), C.int64_t(len(pods))
}

func (a *arena) nodes(nodes []*v1.Node) (*C.esc_node_obj, C.int64_t) {
	objs := cslice[C.esc_node_obj](a, len(nodes))
	for i, n := range nodes {
		a.nodeObj(n, &objs[i])
	}
	return ptr(objs), C.int64_t(len(nodes))
}

// ---------------------------------------------------------------------- context

// GroupSpec carries the NodeGroupOptions fields the hot path reads
// (pkg/controller/node_group.go:20-52); DryMode is c.Opts.DryMode || group.DryMode
// (controller.go:115-117).
type GroupSpec struct {
	Name, LabelKey, LabelValue                     string
	MinNodes, MaxNodes                             int
	TaintUpperPercent, TaintLowerPercent, ScaleUpPercent int
	SlowRemovalRate, FastRemovalRate               int
	DryMode                                        bool
}

// GroupState is the per-run host state of a group (NodeGroupState, controller.go:28-44).
type GroupState struct {
	Locked         bool  // nodeGroup.scaleUpLock.locked()            controller.go:317
	RequestedNodes int   // nodeGroup.scaleUpLock.requestedNodes      controller.go:322
	CachedCPUMilli int64 // nodeGroup.cpuCapacity.MilliValue()        controller.go:209
	CachedMemBytes int64 // nodeGroup.memCapacity.Value()             controller.go:210
}

// Decision is scaleNodeGroup's outcome for one group.
type Decision struct {
	PodCPUMilli, PodMemBytes   int64 // CalculatePodsRequestsTotal (controller.go:263)
	NodeCPUMilli, NodeMemBytes int64 // CalculateNodesCapacityTotal(untainted) (controller.go:268)
	Pods, Nodes                int64
	Untainted, Tainted, Cordoned int64
	CPUPercent, MemPercent     float64
	Delta                      int64 // nodesDelta
	NToTaint                   int64 // scaleDownTaint clamp (scale_down.go:138-158)
	CachedCPUMilli, CachedMemBytes int64
	Branch                     int32 // ESC_BR_*
	Err                        error // the reference's error, text verbatim
	TaintErr                   error // scaleDownTaint's formatted error
	// With SetSelections: the first nodes of the walk the decision asks for, delivered with
	// it — SelTaint: untainted oldest first (taintOldestN, scale_down.go:171-205), SelUntaint:
	// tainted newest first (untaintNewestN, scale_up.go:118-163), NToTaint / Delta + slack of
	// them.  The walk skips a node whose API write fails; when it runs past Selection (or
	// SelectionCut is set) it continues with Context.Order.
	SelectionKind int32 // SelNone, SelTaint, SelUntaint
	Selection     []int64
	SelectionCut  bool
}

// Selection kinds (ESC_SEL_*).
const (
	SelNone    = int32(C.ESC_SEL_NONE)
	SelTaint   = int32(C.ESC_SEL_TAINT)
	SelUntaint = int32(C.ESC_SEL_UNTAINT)
)

// PodsRequestsTotal is the group's CalculatePodsRequestsTotal(pods) (pkg/k8s/util.go:27-38,
// called at controller.go:262) answered from the batched decision: (mem, cpu) built with the
// constructors util.go:34-36 uses, no call into the library.  The controller wiring uses it
// (INTEGRATION.md §1); the per-call Context.CalculatePodsRequestsTotal stays for slices that
// are not a group's.
func (d *Decision) PodsRequestsTotal() (resource.Quantity, resource.Quantity) {
	return *resource.NewQuantity(d.PodMemBytes, resource.BinarySI),
		*resource.NewMilliQuantity(d.PodCPUMilli, resource.DecimalSI)
}

// NodesCapacityTotal is CalculateNodesCapacityTotal(untaintedNodes) (pkg/k8s/util.go:41-52,
// called at controller.go:268) from the batched decision, as PodsRequestsTotal.
func (d *Decision) NodesCapacityTotal() (resource.Quantity, resource.Quantity) {
	return *resource.NewQuantity(d.NodeMemBytes, resource.BinarySI),
		*resource.NewMilliQuantity(d.NodeCPUMilli, resource.DecimalSI)
}

// Context is one process's handle on one GPU (one esc_ctx, driven from one goroutine —
// the reference's RunOnce is single-threaded, controller.go:416).
type Context struct {
	c      *C.esc_ctx
	groups []GroupSpec
	cspecs unsafe.Pointer // C copy of the group specs, alive as long as the context
	names  arena
	sel    bool // SetSelections on: RunOnce returns the walks' first nodes
	selBuf []C.int64_t // RunOnce's selection buffer (grows once to the decisions' size)
}

// SetSelections puts the orderings into every decision and has RunOnce return each group's
// walk prefix (NToTaint or Delta, plus slack for failed API writes; at most groupCap nodes,
// 0 = 256) in its Decision, so the controller's taint / untaint loop needs no per-group
// Order call (controller.go:367-383).  slack < 0 turns them off.
func (x *Context) SetSelections(slack, groupCap int) error {
	if rc := C.esc_set_order_in_step(x.c, 1); rc != C.ESC_OK {
		return rcErr("esc_set_order_in_step", rc)
	}
	if rc := C.esc_set_selections(x.c, C.int32_t(slack), C.int32_t(groupCap)); rc != C.ESC_OK {
		return rcErr("esc_set_selections", rc)
	}
	x.sel = slack >= 0
	return nil
}

// NewContext creates the context for groups (fixed for its lifetime, client.go:55-64).
// rank/world describe the sharding when one process drives each GPU.
func NewContext(groups []GroupSpec, device, rank, world int) (*Context, error) {
	return newContext(groups, func(specs *C.esc_group_spec, n C.int32_t, out **C.esc_ctx) C.int32_t {
		return C.esc_ctx_create(specs, n, C.int32_t(device), C.int32_t(rank), C.int32_t(world), out)
	})
}

// NewContextMulti creates ONE context driving every listed GPU from this process
// (esc_ctx_create_multi): the pods are sharded over the devices, each owns the node side
// of a range of groups, and RunOnce's exchange is an in-place ncclReduceScatter per device
// (each receiving its own groups' rows) inside one RCCL group call — the reference stays one process with one informer set
// (cmd/main.go:187, controller.go:416-445).
func NewContextMulti(groups []GroupSpec, devices []int) (*Context, error) {
	if len(devices) == 0 {
		return nil, fmt.Errorf("escalatorhip: no devices")
	}
	dev := make([]C.int32_t, len(devices))
	for i, d := range devices {
		dev[i] = C.int32_t(d)
	}
	return newContext(groups, func(specs *C.esc_group_spec, n C.int32_t, out **C.esc_ctx) C.int32_t {
		return C.esc_ctx_create_multi(specs, n, ptr(dev), C.int32_t(len(dev)), out)
	})
}

func newContext(groups []GroupSpec, create func(*C.esc_group_spec, C.int32_t, **C.esc_ctx) C.int32_t) (*Context, error) {
	if len(groups) == 0 {
		return nil, fmt.Errorf("escalatorhip: no node groups")
	}
	x := &Context{groups: groups}
	specs := cslice[C.esc_group_spec](&x.names, len(groups))
	for i, g := range groups {
		s := &specs[i]
		s.name = x.names.cstr(g.Name)
		s.label_key = x.names.cstr(g.LabelKey)
		s.label_value = x.names.cstr(g.LabelValue)
		s.min_nodes = C.int32_t(g.MinNodes)
		s.max_nodes = C.int32_t(g.MaxNodes)
		s.taint_upper_pct = C.int32_t(g.TaintUpperPercent)
		s.taint_lower_pct = C.int32_t(g.TaintLowerPercent)
		s.scale_up_pct = C.int32_t(g.ScaleUpPercent)
		s.slow_removal_rate = C.int32_t(g.SlowRemovalRate)
		s.fast_removal_rate = C.int32_t(g.FastRemovalRate)
		if g.DryMode {
			s.dry_mode = 1
		}
	}
	x.cspecs = unsafe.Pointer(ptr(specs))
	rc := create(ptr(specs), C.int32_t(len(groups)), &x.c)
	if rc != C.ESC_OK {
		x.names.free()
		return nil, rcErr("esc_ctx_create", rc)
	}
	return x, nil
}

// Close releases the device snapshot, streams and communicator.
func (x *Context) Close() error {
	rc := C.esc_ctx_destroy(x.c)
	x.names.free()
	return rcErr("esc_ctx_destroy", rc)
}

// pack builds the SoA snapshot of pods and nodes (K0) and hands the packer to fn; the
// packer's arrays live until fn returns.
func (x *Context) pack(pods []*v1.Pod, nodes []*v1.Node, trackers map[int][]string, listMode bool,
	fn func(ps *C.esc_pod_soa, ns *C.esc_node_soa) error) error {
	var a arena
	defer a.free()
	var pk *C.esc_packer
	if rc := C.esc_packer_create(x.c, &pk); rc != C.ESC_OK {
		return rcErr("esc_packer_create", rc)
	}
	defer C.esc_packer_destroy(pk)
	if listMode {
		C.esc_packer_set_list_mode(pk, 1)
	}
	if len(pods) > 0 {
		po, n := a.pods(pods)
		if rc := C.esc_packer_add_pods(pk, po, n); rc != C.ESC_OK {
			return rcErr("esc_packer_add_pods", rc)
		}
	}
	if len(nodes) > 0 {
		no, n := a.nodes(nodes)
		if rc := C.esc_packer_add_nodes(pk, no, n); rc != C.ESC_OK {
			return rcErr("esc_packer_add_nodes", rc)
		}
	}
	for g, names := range trackers { // nodeGroup.taintTracker, controller.go:35
		if len(names) == 0 {
			continue
		}
		if rc := C.esc_packer_set_tracker(pk, C.int32_t(g), a.cstrs(names), C.int64_t(len(names))); rc != C.ESC_OK {
			return rcErr("esc_packer_set_tracker", rc)
		}
	}
	var ps C.esc_pod_soa
	var ns C.esc_node_soa
	if rc := C.esc_packer_view(pk, &ps, &ns); rc != C.ESC_OK {
		return rcErr("esc_packer_view", rc)
	}
	return fn(&ps, &ns)
}

// Load replaces the resident snapshot with the listers' current pods and nodes (this
// rank's pod shard starting at global index podOffset — every pod for a NewContextMulti
// context — and the full node list, which every rank holds).  trackers holds the dry-mode
// groups' taintTracker.
func (x *Context) Load(pods []*v1.Pod, podOffset int64, nodes []*v1.Node, trackers map[int][]string) error {
	return x.pack(pods, nodes, trackers, false, func(ps *C.esc_pod_soa, ns *C.esc_node_soa) error {
		if rc := C.esc_load_pods(x.c, ps, C.int64_t(podOffset)); rc != C.ESC_OK {
			return rcErr("esc_load_pods", rc)
		}
		return rcErr("esc_load_nodes", C.esc_load_nodes(x.c, ns, 0, ns.n_nodes))
	})
}

// SetSpare reserves room for informer events in the next Load (esc_set_spare): spare slots
// per pod class, node table slots, pair-major entries and K5 region slots, as a fraction of
// what the snapshot holds.  Events that do not fit return ErrReload.
func (x *Context) SetSpare(fraction float64) error {
	return rcErr("esc_set_spare", C.esc_set_spare(x.c, C.double(fraction)))
}

// Calibrate balances the pod pass's per-workgroup shares to this GPU's measured streaming
// rates (esc_k1_calibrate: `rounds` untimed decisions with the current state; results are
// unchanged).  Call it once after Load and the first RunOnce's state.
func (x *Context) Calibrate(rounds int) error {
	return rcErr("esc_k1_calibrate", C.esc_k1_calibrate(x.c, C.int32_t(rounds)))
}

// RunOnce evaluates scaleNodeGroup's decision for every group at once (controller.go:192-351):
// listers + filters + sums + filterNodes + cached capacity + gates + percentages + delta +
// the scale-down clamp.  With a communicator (CommInit) the per-group pod sums are
// reduce-scattered over RCCL inside esc_step, every rank receiving (and deciding) the
// groups it owns.
func (x *Context) RunOnce(states []GroupState) ([]Decision, error) {
	G := len(x.groups)
	if len(states) != G {
		return nil, fmt.Errorf("escalatorhip: %d states for %d groups", len(states), G)
	}
	cst := make([]C.esc_group_state, G) // plain integers: Go memory may be passed
	for g, s := range states {
		if s.Locked {
			cst[g].locked = 1
		}
		cst[g].requested_nodes = C.int32_t(s.RequestedNodes)
		cst[g].cached_cpu_m = C.int64_t(s.CachedCPUMilli)
		cst[g].cached_mem_b = C.int64_t(s.CachedMemBytes)
	}
	if rc := C.esc_set_state(x.c, ptr(cst)); rc != C.ESC_OK {
		return nil, rcErr("esc_set_state", rc)
	}
	if rc := C.esc_step(x.c); rc != C.ESC_OK {
		return nil, rcErr("esc_step", rc)
	}
	// ESC_E_ORDER: the step's ordering gave up a bounded wait; the totals and decisions
	// stand, and the walks order afresh through Order (esc_sort_nodes + esc_group_order)
	orderFailed := false
	if rc := C.esc_sync(x.c); rc == C.ESC_E_ORDER {
		orderFailed = true
	} else if rc != C.ESC_OK {
		return nil, rcErr("esc_sync", rc)
	}
	tot := make([]C.esc_group_totals, G)
	dec := make([]C.esc_group_decision, G)
	if rc := C.esc_results(x.c, ptr(tot), ptr(dec)); rc != C.ESC_OK {
		return nil, rcErr("esc_results", rc)
	}
	which := make([]C.int32_t, G)
	off := make([]C.int64_t, G+1)
	var sel []C.int64_t
	if x.sel && !orderFailed {
		// one call into the context's persistent buffer; a second only when it was short
		// (ESC_E_LIMIT reports the size: the buffer grows once and keeps that size)
		var n C.int64_t
		if len(x.selBuf) == 0 {
			x.selBuf = make([]C.int64_t, 4*G+1)
		}
		rc := C.esc_selections(x.c, ptr(which), ptr(off), ptr(x.selBuf), C.int64_t(len(x.selBuf)), &n)
		if rc == C.ESC_E_LIMIT {
			x.selBuf = make([]C.int64_t, 2*n+1)
			rc = C.esc_selections(x.c, ptr(which), ptr(off), ptr(x.selBuf), C.int64_t(len(x.selBuf)), &n)
		}
		if rc == C.ESC_OK {
			sel = x.selBuf[:n]
		}
		if rc == C.ESC_E_ORDER {
			orderFailed = true
		} else if rc != C.ESC_OK {
			return nil, rcErr("esc_selections", rc)
		}
	}
	if orderFailed {
		if err := x.SortNodes(); err != nil {
			return nil, err
		}
	}
	out := make([]Decision, G)
	for g := range out {
		t, d := &tot[g], &dec[g]
		out[g] = Decision{
			PodCPUMilli: int64(t.pod_cpu_m), PodMemBytes: int64(t.pod_mem_b),
			NodeCPUMilli: int64(t.node_cpu_m), NodeMemBytes: int64(t.node_mem_b),
			Pods: int64(t.n_pods), Nodes: int64(t.n_nodes),
			Untainted: int64(t.n_untainted), Tainted: int64(t.n_tainted), Cordoned: int64(t.n_cordoned),
			CPUPercent: float64(d.cpu_pct), MemPercent: float64(d.mem_pct),
			Delta: int64(d.delta), NToTaint: int64(d.n_to_taint),
			CachedCPUMilli: int64(d.cached_cpu_m), CachedMemBytes: int64(d.cached_mem_b),
			Branch: int32(d.branch), Err: statusErr(d.status),
			SelectionKind: SelNone,
		}
		if x.sel {
			if orderFailed {
				out[g].SelectionCut = true // no list: the walk reads Order
			} else if w := int32(which[g]); w != SelNone {
				out[g].SelectionKind = w & 3
				out[g].SelectionCut = w&int32(C.ESC_SEL_CUT) != 0
				out[g].Selection = make([]int64, off[g+1]-off[g])
				for i := range out[g].Selection {
					out[g].Selection[i] = int64(sel[int(off[g])+i])
				}
			}
		}
		if d.taint_status == C.ESC_ST_ERR_TAINT_MIN { // scale_down.go:150-154
			buf := make([]byte, 160)
			C.esc_taint_error(t.n_untainted, C.int32_t(x.groups[g].MinNodes), (*C.char)(unsafe.Pointer(ptr(buf))),
				C.int32_t(len(buf)))
			out[g].TaintErr = errors.New(C.GoString((*C.char)(unsafe.Pointer(ptr(buf)))))
		}
	}
	return out, nil
}

// SortNodes classifies and orders every group's nodes by creation time (K5); call once
// per decision before Order.
func (x *Context) SortNodes() error { return rcErr("esc_sort_nodes", C.esc_sort_nodes(x.c)) }

// Order returns up to n snapshot node indices of group g: untainted oldest-first
// (taintOldestN, scale_down.go:171) when oldest, else tainted newest-first
// (untaintNewestN, scale_up.go:118).
func (x *Context) Order(g int, oldest bool, n int) ([]int64, error) {
	which := C.int32_t(1)
	if oldest {
		which = 0
	}
	idx := make([]int64, n+1)
	var got C.int64_t
	rc := C.esc_group_order(x.c, C.int32_t(g), which, (*C.int64_t)(unsafe.Pointer(ptr(idx))), C.int64_t(n), &got)
	if rc == C.ESC_E_ORDER { // that ordering gave up its bounded wait: order afresh, once
		if err := x.SortNodes(); err != nil {
			return nil, err
		}
		rc = C.esc_group_order(x.c, C.int32_t(g), which, (*C.int64_t)(unsafe.Pointer(ptr(idx))), C.int64_t(n), &got)
	}
	if rc != C.ESC_OK {
		return nil, rcErr("esc_group_order", rc)
	}
	if int(got) < n {
		n = int(got)
	}
	return idx[:n], nil
}

// ------------------------------------------------------------------ drop-ins

// CalculatePodsRequestsTotal keeps the reference signature (pkg/k8s/util.go:27): the
// given, already-filtered pods, summed on the GPU; (mem, cpu) built with the same
// constructors as util.go:34-36.
func (x *Context) CalculatePodsRequestsTotal(pods []*v1.Pod) (resource.Quantity, resource.Quantity, error) {
	var a arena
	defer a.free()
	var mem, cpu C.int64_t
	po, n := a.pods(pods)
	if rc := C.esc_pods_requests_total(x.c, po, n, &mem, &cpu); rc != C.ESC_OK {
		return resource.Quantity{}, resource.Quantity{}, rcErr("esc_pods_requests_total", rc)
	}
	return *resource.NewQuantity(int64(mem), resource.BinarySI),
		*resource.NewMilliQuantity(int64(cpu), resource.DecimalSI), nil
}

// CalculateNodesCapacityTotal keeps the reference signature (pkg/k8s/util.go:41).
func (x *Context) CalculateNodesCapacityTotal(nodes []*v1.Node) (resource.Quantity, resource.Quantity, error) {
	var a arena
	defer a.free()
	var mem, cpu C.int64_t
	no, n := a.nodes(nodes)
	if rc := C.esc_nodes_capacity_total(x.c, no, n, &mem, &cpu); rc != C.ESC_OK {
		return resource.Quantity{}, resource.Quantity{}, rcErr("esc_nodes_capacity_total", rc)
	}
	return *resource.NewQuantity(int64(mem), resource.BinarySI),
		*resource.NewMilliQuantity(int64(cpu), resource.DecimalSI), nil
}

// CalcPercentUsage is calcPercentUsage (pkg/controller/util.go:58-81), bit-exact.
func CalcPercentUsage(cpuRequest, memRequest, cpuCapacity, memCapacity resource.Quantity, numberOfUntaintedNodes int64) (float64, float64, error) {
	var cpu, mem C.double
	st := C.esc_calc_percent_usage(C.int64_t(cpuRequest.MilliValue()), C.int64_t(memRequest.Value()),
		C.int64_t(cpuCapacity.MilliValue()), C.int64_t(memCapacity.Value()), C.int64_t(numberOfUntaintedNodes), &cpu, &mem)
	return float64(cpu), float64(mem), statusErr(st)
}

// CalcScaleUpDelta is calcScaleUpDelta (pkg/controller/util.go:13-46), bit-exact.
func CalcScaleUpDelta(untainted int, cpuPercent, memPercent float64, cpuRequest, memRequest, cpuCapacity, memCapacity resource.Quantity, scaleUpThreshold int) (int, error) {
	var d C.int64_t
	st := C.esc_calc_scale_up_delta(C.int64_t(untainted), C.double(cpuPercent), C.double(memPercent),
		C.int64_t(cpuRequest.MilliValue()), C.int64_t(memRequest.Value()),
		C.int64_t(cpuCapacity.MilliValue()), C.int64_t(memCapacity.Value()), C.int32_t(scaleUpThreshold), &d)
	return int(d), statusErr(st)
}

// ------------------------------------------------------------------ multi-GPU

// CommUniqueID is called on rank 0; its bytes go to every other rank over any host channel.
func CommUniqueID() ([]byte, error) {
	id := make([]byte, C.ESC_COMM_ID_BYTES)
	rc := C.esc_comm_unique_id(unsafe.Pointer(ptr(id)))
	return id, rcErr("esc_comm_unique_id", rc)
}

// CommInit joins the RCCL communicator (collective: blocks until every rank joined).
// RunOnce then reduce-scatters the owner-major pod words over xGMI inside esc_step.
func (x *Context) CommInit(id []byte, rank, world int) error {
	cid := C.CBytes(id)
	defer C.free(cid)
	return rcErr("esc_comm_init", C.esc_comm_init(x.c, cid, C.int32_t(rank), C.int32_t(world)))
}

// ------------------------------------------------------------ informer events

// PodsUpsert patches the resident snapshot with added / updated pods (ids = snapshot pod
// indices; new ids insert).  ErrReload means the batch did not fit in place (nothing was
// applied): call Load with the listers' state.
var ErrReload = errors.New(C.GoString(C.esc_strerror(C.ESC_E_LIMIT)))

func (x *Context) PodsUpsert(ids []int64, pods []*v1.Pod) error {
	if len(ids) != len(pods) {
		return fmt.Errorf("escalatorhip: %d ids for %d pods", len(ids), len(pods))
	}
	if len(ids) == 0 {
		return nil
	}
	return x.pack(pods, nil, nil, false, func(ps *C.esc_pod_soa, _ *C.esc_node_soa) error {
		rc := C.esc_pods_upsert(x.c, (*C.int64_t)(unsafe.Pointer(ptr(ids))), ps)
		if rc == C.ESC_E_LIMIT {
			return ErrReload
		}
		return rcErr("esc_pods_upsert", rc)
	})
}

// PodsDelete removes pods by snapshot index.
func (x *Context) PodsDelete(ids []int64) error {
	return rcErr("esc_pods_delete", C.esc_pods_delete(x.c, (*C.int64_t)(unsafe.Pointer(ptr(ids))), C.int64_t(len(ids))))
}

// NodesUpdate applies node watch events that change Spec.Unschedulable, the escalator
// taint or Status.Allocatable (flags are ESC_NF_* bits).
func (x *Context) NodesUpdate(ids []int64, flags []uint32, cpuMilli, memBytes []int64) error {
	if len(flags) != len(ids) || len(cpuMilli) != len(ids) || len(memBytes) != len(ids) {
		return fmt.Errorf("escalatorhip: NodesUpdate needs one flags / cpu / memory entry per id")
	}
	return rcErr("esc_nodes_update", C.esc_nodes_update(x.c, (*C.int64_t)(unsafe.Pointer(ptr(ids))), C.int64_t(len(ids)),
		(*C.uint32_t)(unsafe.Pointer(ptr(flags))), (*C.int64_t)(unsafe.Pointer(ptr(cpuMilli))),
		(*C.int64_t)(unsafe.Pointer(ptr(memBytes)))))
}

// NodesAdd applies node Add events (cache.go:37-56): the nodes are packed and appended at
// the next snapshot indices, returned in order.  ErrReload when the spare room is short.
func (x *Context) NodesAdd(nodes []*v1.Node) ([]int64, error) {
	ids := make([]int64, len(nodes)+1)
	if len(nodes) == 0 {
		return nil, nil
	}
	err := x.pack(nil, nodes, nil, false, func(_ *C.esc_pod_soa, ns *C.esc_node_soa) error {
		rc := C.esc_nodes_add(x.c, ns, (*C.int64_t)(unsafe.Pointer(ptr(ids))))
		if rc == C.ESC_E_LIMIT {
			return ErrReload
		}
		return rcErr("esc_nodes_add", rc)
	})
	return ids[:len(nodes)], err
}

// NodesRelabel applies node Update events that change labels or the creation time (any
// field): ids[i] takes nodes[i]'s record in place, moving between node groups as
// NewNodeLabelFilterFunc (node_group.go:278-287) would see it on the next List.  ErrReload
// when the spare room is short.
func (x *Context) NodesRelabel(ids []int64, nodes []*v1.Node) error {
	if len(ids) != len(nodes) {
		return fmt.Errorf("escalatorhip: %d ids for %d nodes", len(ids), len(nodes))
	}
	if len(nodes) == 0 {
		return nil
	}
	return x.pack(nil, nodes, nil, false, func(_ *C.esc_pod_soa, ns *C.esc_node_soa) error {
		rc := C.esc_nodes_relabel(x.c, (*C.int64_t)(unsafe.Pointer(ptr(ids))), ns)
		if rc == C.ESC_E_LIMIT {
			return ErrReload
		}
		return rcErr("esc_nodes_relabel", rc)
	})
}

// NodesDelete applies node Delete events by snapshot index.
func (x *Context) NodesDelete(ids []int64) error {
	return rcErr("esc_nodes_delete", C.esc_nodes_delete(x.c, (*C.int64_t)(unsafe.Pointer(ptr(ids))), C.int64_t(len(ids))))
}

// PodsBind records Spec.NodeName changes (the scheduler bound a pod, or it left its node):
// node snapshot indices, 0xFFFFFFFF for none.  ErrReload when a node's run is full
// (LoadPlacement again).
func (x *Context) PodsBind(ids []int64, nodeIdx []uint32) error {
	if len(ids) != len(nodeIdx) {
		return fmt.Errorf("escalatorhip: %d ids for %d node indices", len(ids), len(nodeIdx))
	}
	rc := C.esc_pods_bind(x.c, (*C.int64_t)(unsafe.Pointer(ptr(ids))), (*C.uint32_t)(unsafe.Pointer(ptr(nodeIdx))),
		C.int64_t(len(ids)))
	if rc == C.ESC_E_LIMIT {
		return ErrReload
	}
	return rcErr("esc_pods_bind", rc)
}

// TrackerUpdate applies one dry-mode group's taintTracker change in place: taintOldestN
// appends (scale_down.go:197-200), untaintNewestN deletes (scale_up.go:146-158).
func (x *Context) TrackerUpdate(g int, add, remove []int64) error {
	pa, pr := (*C.int64_t)(unsafe.Pointer(ptr(add))), (*C.int64_t)(unsafe.Pointer(ptr(remove)))
	return rcErr("esc_tracker_update", C.esc_tracker_update(x.c, C.int32_t(g), pa, C.int64_t(len(add)), pr,
		C.int64_t(len(remove))))
}

// ------------------------------------------------------------------- reaping

// Removal is TryRemoveTaintedNodes' outcome for one group (scale_down.go:51-136).
type Removal struct {
	Candidates, Delete, PodsRemaining int64
}

// LoadPlacement binds the loaded pods to nodes (Spec.NodeName as a snapshot node index,
// 0xFFFFFFFF when empty or unknown — CreateNodeNameToInfoMap drops those, node_state.go:27-36)
// and gives each node its escalator-taint time (GetToBeRemovedTime, taint.go:91) and its
// no-delete annotation (scale_down.go:39-46).
// podNode may be nil to refresh the per-node facts only (the binding is kept current by
// PodsUpsert / PodsDelete / PodsBind).  The library reads one entry per pod id and per node
// slot (esc_ctx_counts), so shorter slices are refused here instead of being over-read.
func (x *Context) LoadPlacement(podNode []uint32, taintUnixS []int64, noDelete []uint8) error {
	var nPods, nNodes C.int64_t
	if rc := C.esc_ctx_counts(x.c, &nPods, &nNodes); rc != C.ESC_OK {
		return rcErr("esc_ctx_counts", rc)
	}
	if podNode != nil && int64(len(podNode)) != int64(nPods) {
		return fmt.Errorf("escalatorhip: LoadPlacement: %d pod entries for %d pod ids", len(podNode), nPods)
	}
	if int64(len(taintUnixS)) != int64(nNodes) || int64(len(noDelete)) != int64(nNodes) {
		return fmt.Errorf("escalatorhip: LoadPlacement: %d taint times / %d no-delete flags for %d nodes",
			len(taintUnixS), len(noDelete), nNodes)
	}
	return rcErr("esc_load_placement", C.esc_load_placement(x.c, (*C.uint32_t)(unsafe.Pointer(ptr(podNode))),
		(*C.int64_t)(unsafe.Pointer(ptr(taintUnixS))), (*C.uint8_t)(unsafe.Pointer(ptr(noDelete)))))
}

// TryRemove evaluates TryRemoveTaintedNodes for every group at once; DeleteList(g) gives
// the group's toBeDeleted nodes in the reference's order.
func (x *Context) TryRemove(nowUnixNano int64, softGraceNs, hardGraceNs []int64) ([]Removal, error) {
	if len(softGraceNs) != len(x.groups) || len(hardGraceNs) != len(x.groups) {
		return nil, fmt.Errorf("escalatorhip: TryRemove needs one soft / hard grace period per group (%d)", len(x.groups))
	}
	out := make([]C.esc_removal, len(x.groups))
	rc := C.esc_try_remove(x.c, C.int64_t(nowUnixNano), (*C.int64_t)(unsafe.Pointer(ptr(softGraceNs))),
		(*C.int64_t)(unsafe.Pointer(ptr(hardGraceNs))), ptr(out))
	if rc != C.ESC_OK {
		return nil, rcErr("esc_try_remove", rc)
	}
	res := make([]Removal, len(out))
	for g, r := range out {
		res[g] = Removal{int64(r.n_candidates), int64(r.n_delete), int64(r.pods_remaining)}
	}
	return res, nil
}

// DeleteList returns group g's nodes chosen by the last TryRemove.
func (x *Context) DeleteList(g int, n int64) ([]int64, error) {
	idx := make([]int64, n+1)
	var got C.int64_t
	rc := C.esc_removal_nodes(x.c, C.int32_t(g), (*C.int64_t)(unsafe.Pointer(ptr(idx))), C.int64_t(n), &got)
	if rc != C.ESC_OK {
		return nil, rcErr("esc_removal_nodes", rc)
	}
	if got < C.int64_t(n) {
		n = int64(got)
	}
	return idx[:n], nil
}
