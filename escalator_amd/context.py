"""Python host of the batched scale decision (over the C ABI).

``Context`` is the MI355X-resident equivalent of the reference's per-scan loop
(``(*Controller).RunOnce`` pkg/controller/controller.go:400 -> ``scaleNodeGroup`` :192 per
group): it holds one device snapshot and computes every group's totals and decision in
one pass.  ``Synth`` wraps the deterministic snapshot generator used by tests and the
benchmark.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .objects import groups_from_c, groups_to_c, nodes_to_c, pods_to_c, states_to_c

TOTALS_DTYPE = np.dtype([(n, np.int64) for n, _ in L.GroupTotals._fields_])
METRICS_DTYPE = np.dtype([(n, np.float64) for n in L.METRIC_NAMES] + [("set_mask", np.uint32), ("reserved", np.uint32)])
REMOVAL_DTYPE = np.dtype([(n, np.int64) for n, _ in L.Removal._fields_])
DECISION_DTYPE = np.dtype({"names": [n for n, _ in L.GroupDecision._fields_],
                           "formats": [np.float64, np.float64, np.int64, np.int64, np.int64, np.int64,
                                       np.int32, np.int32, np.int32, np.int32]})
assert TOTALS_DTYPE.itemsize == C.sizeof(L.GroupTotals)
assert DECISION_DTYPE.itemsize == C.sizeof(L.GroupDecision)
assert METRICS_DTYPE.itemsize == C.sizeof(L.GroupMetrics)

_POD_FIELDS = [("flags", np.uint32, "n_pods"), ("cpu0", np.uint32, "n_pods"), ("mem0", np.int64, "n_pods"),
               ("pair0", np.uint32, "n_pods"), ("xc_cpu", np.int64, "n_xc"), ("xc_mem", np.int64, "n_xc"),
               ("xp_pair", np.uint32, "n_xp")]
_NODE_FIELDS = [("flags", np.uint32, "n_nodes"), ("label0", np.uint32, "n_nodes"), ("cpu", np.int64, "n_nodes"),
                ("mem", np.int64, "n_nodes"), ("created_ns", np.int64, "n_nodes"), ("xl_pair", np.uint32, "n_xl"),
                ("trk_node", np.int32, "n_trk"), ("trk_group", np.int32, "n_trk")]


def _view(struct, fields) -> dict:
    out = {}
    for name, dt, count in fields:
        n = int(getattr(struct, count))
        ptr = getattr(struct, name)
        out[name] = np.ctypeslib.as_array(ptr, shape=(n,)).view(dt) if n and ptr else np.zeros(0, dt)
    return out


def _soa_from(arrays: dict, fields, struct_t, count_names):
    """Build a SoA struct pointing at numpy arrays (kept alive by the caller)."""
    s = struct_t()
    keep = []
    for name, dt, count in fields:
        a = np.ascontiguousarray(arrays[name], dtype=dt)
        keep.append(a)
        setattr(s, name, a.ctypes.data_as(dict(s._fields_)[name]))
    for cname, val in count_names.items():
        setattr(s, cname, int(val))
    return s, keep


def pod_soa(arrays: dict):
    return _soa_from(arrays, _POD_FIELDS, L.PodSoA, {"n_pods": len(arrays["flags"]), "n_xc": len(arrays["xc_cpu"]),
                                                      "n_xp": len(arrays["xp_pair"])})


def node_soa(arrays: dict):
    return _soa_from(arrays, _NODE_FIELDS, L.NodeSoA, {"n_nodes": len(arrays["flags"]), "n_xl": len(arrays["xl_pair"]),
                                                        "n_trk": len(arrays["trk_node"])})


class Synth:
    """Deterministic synthetic snapshot."""

    def __init__(self, n_pods: int, n_nodes: int, n_groups: int, config: int = 2, seed: int = 0xE5CA1A7E00000002,
                 with_default: bool = True, p_lo: int = 0, p_hi: int | None = None, threads: int = 8):
        self.lib = L.load()
        p = L.SynthParams(n_pods, n_nodes, n_groups, config, seed & ((1 << 64) - 1), int(with_default), threads)
        self.handle = C.c_void_p()
        L.check(self.lib.esc_synth_create(C.byref(p), p_lo, n_pods if p_hi is None else p_hi, C.byref(self.handle)),
                "esc_synth_create")
        specs = C.POINTER(L.GroupSpec)()
        n = C.c_int32()
        L.check(self.lib.esc_synth_groups(self.handle, C.byref(specs), C.byref(n)))
        self.specs, self.n_groups = specs, n.value
        self.groups = groups_from_c(specs, n.value)
        st = C.POINTER(L.GroupState)()
        L.check(self.lib.esc_synth_states(self.handle, C.byref(st)))
        self.state_ptr = st
        self.states = [{"locked": st[i].locked, "requested_nodes": st[i].requested_nodes,
                        "cached_cpu_m": st[i].cached_cpu_m, "cached_mem_b": st[i].cached_mem_b}
                       for i in range(n.value)]
        self.pod_c = L.PodSoA()
        self.node_c = L.NodeSoA()
        L.check(self.lib.esc_synth_view(self.handle, C.byref(self.pod_c), C.byref(self.node_c)))

    def objects(self):
        """The snapshot as object structs (esc_synth_objects, built once, owned by the
        handle): (pod objects, n_pods, node objects, n_nodes) as ctypes pointers — the input
        of the K0 packer (esc_packer_add_pods / _add_nodes)."""
        po, no = C.POINTER(L.PodObj)(), C.POINTER(L.NodeObj)()
        npd, nnd = C.c_int64(), C.c_int64()
        L.check(self.lib.esc_synth_objects(self.handle, C.byref(po), C.byref(npd), C.byref(no), C.byref(nnd)),
                "esc_synth_objects")
        return po, npd.value, no, nnd.value

    def pods(self) -> dict:
        return _view(self.pod_c, _POD_FIELDS)

    def nodes(self) -> dict:
        return _view(self.node_c, _NODE_FIELDS)

    def close(self):
        if self.handle:
            self.lib.esc_synth_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One device snapshot + the batched decision over every group.

    ``devices=[d0, d1, ...]``: one context driving several devices from this process
    (esc_ctx_create_multi — pods sharded over the devices, the exchange internal); a device
    listed more than once selects the peer exchange (several shards on one GPU)."""

    def __init__(self, groups, device: int = 0, rank: int = 0, world: int = 1, devices=None):
        self.lib = L.load()
        if isinstance(groups, Synth):
            spec_ptr, self._gkeep, self.G = groups.specs, None, groups.n_groups
            self.groups = groups.groups
        else:
            spec_arr, self._gkeep = groups_to_c(groups)
            spec_ptr, self.G = spec_arr, len(groups)
            self.groups = list(groups)
        self.handle = C.c_void_p()
        if devices is not None:
            dv = (C.c_int32 * len(devices))(*devices)
            L.check(self.lib.esc_ctx_create_multi(spec_ptr, self.G, dv, len(devices), C.byref(self.handle)),
                    "esc_ctx_create_multi")
            self.devices = list(devices)
        else:
            L.check(self.lib.esc_ctx_create(spec_ptr, self.G, device, rank, world, C.byref(self.handle)),
                    "esc_ctx_create")
            self.devices = None
        self.world = world
        self._keep = []

    # ------------------------------------------------------------- loading
    def pack_objects(self, pod_objs, n_pods: int, node_objs, n_nodes: int, trackers: dict | None = None):
        """K0 packer over object structs already in C memory (Synth.objects): packed SoA
        (numpy copies).  trackers: {group: [node names]} (nodeGroup.taintTracker)."""
        pk = C.c_void_p()
        L.check(self.lib.esc_packer_create(self.handle, C.byref(pk)), "esc_packer_create")
        try:
            L.check(self.lib.esc_packer_add_pods(pk, pod_objs, n_pods), "esc_packer_add_pods")
            L.check(self.lib.esc_packer_add_nodes(pk, node_objs, n_nodes), "esc_packer_add_nodes")
            for g, names in (trackers or {}).items():
                arr = (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
                L.check(self.lib.esc_packer_set_tracker(pk, g, arr, len(names)), "esc_packer_set_tracker")
            ps, ns = L.PodSoA(), L.NodeSoA()
            L.check(self.lib.esc_packer_view(pk, C.byref(ps), C.byref(ns)), "esc_packer_view")
            return ({k: v.copy() for k, v in _view(ps, _POD_FIELDS).items()},
                    {k: v.copy() for k, v in _view(ns, _NODE_FIELDS).items()})
        finally:
            self.lib.esc_packer_destroy(pk)

    def pack(self, pods: list[dict], nodes: list[dict], trackers: dict | None = None, list_mode: bool = False):
        """K0 packer: objects -> packed SoA (numpy copies)."""
        pk = C.c_void_p()
        L.check(self.lib.esc_packer_create(self.handle, C.byref(pk)), "esc_packer_create")
        try:
            if list_mode:
                L.check(self.lib.esc_packer_set_list_mode(pk, 1))
            pc, npods, k1 = pods_to_c(pods)
            nc, nnodes, k2 = nodes_to_c(nodes)
            L.check(self.lib.esc_packer_add_pods(pk, pc, npods), "esc_packer_add_pods")
            L.check(self.lib.esc_packer_add_nodes(pk, nc, nnodes), "esc_packer_add_nodes")
            for g, names in (trackers or {}).items():
                arr = (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
                L.check(self.lib.esc_packer_set_tracker(pk, g, arr, len(names)), "esc_packer_set_tracker")
            ps, ns = L.PodSoA(), L.NodeSoA()
            L.check(self.lib.esc_packer_view(pk, C.byref(ps), C.byref(ns)), "esc_packer_view")
            pods_np = {k: v.copy() for k, v in _view(ps, _POD_FIELDS).items()}
            nodes_np = {k: v.copy() for k, v in _view(ns, _NODE_FIELDS).items()}
        finally:
            self.lib.esc_packer_destroy(pk)
        return pods_np, nodes_np

    def load(self, pods: dict, nodes: dict, pod_offset: int = 0, replicas: int = 1):
        """This rank's pod shard (global indices from pod_offset) and the whole node table
        (every rank holds it; its share of the node work is the pairs it owns)."""
        L.check(self.lib.esc_set_replicas(self.handle, replicas), "esc_set_replicas")
        ps, k1 = pod_soa(pods)
        ns, k2 = node_soa(nodes)
        L.check(self.lib.esc_load_pods(self.handle, C.byref(ps), pod_offset), "esc_load_pods")
        L.check(self.lib.esc_load_nodes(self.handle, C.byref(ns), 0, len(nodes["flags"])), "esc_load_nodes")

    def load_synth(self, s: Synth, pod_offset: int = 0, replicas: int = 1):
        L.check(self.lib.esc_set_replicas(self.handle, replicas), "esc_set_replicas")
        L.check(self.lib.esc_load_pods(self.handle, C.byref(s.pod_c), pod_offset), "esc_load_pods")
        L.check(self.lib.esc_load_nodes(self.handle, C.byref(s.node_c), 0, s.node_c.n_nodes), "esc_load_nodes")

    def counts(self) -> tuple[int, int]:
        """(pod ids, node slots): the sizes of load_placement's per-pod / per-node arrays."""
        a, b = C.c_int64(), C.c_int64()
        L.check(self.lib.esc_ctx_counts(self.handle, C.byref(a), C.byref(b)), "esc_ctx_counts")
        return a.value, b.value

    def group_owner(self, group: int) -> int:
        """The rank (device index of a multi-device context) owning the group's node side."""
        r = C.c_int32()
        L.check(self.lib.esc_group_owner(self.handle, group, C.byref(r)), "esc_group_owner")
        return r.value

    def comm_size(self) -> int:
        """Ranks of the context's communicator (ncclCommCount), or the devices of a
        multi-device context."""
        r = C.c_int32()
        L.check(self.lib.esc_comm_size(self.handle, C.byref(r)), "esc_comm_size")
        return r.value

    def exchange_rows(self, nodes: dict, world: int) -> tuple[np.ndarray, int]:
        """Host only: every group's owner-major row of the exchanged pod words and the rows
        per owner (esc_exchange_rows)."""
        ns, keep = node_soa(nodes)
        rows = np.zeros(self.G, np.uint32)
        cap = C.c_int32()
        L.check(self.lib.esc_exchange_rows(self.handle, C.byref(ns), world, rows.ctypes.data_as(C.POINTER(C.c_uint32)),
                                           C.byref(cap)), "esc_exchange_rows")
        del keep
        return rows, cap.value

    def exchange_slice(self) -> tuple[int, int]:
        """(word offset, word count) of this rank's own rows in the exchange buffer."""
        a, b = C.c_int64(), C.c_int64()
        L.check(self.lib.esc_exchange_slice(self.handle, C.byref(a), C.byref(b)), "esc_exchange_slice")
        return a.value, b.value

    def owner_ranges(self, nodes: dict, world: int) -> np.ndarray:
        """The owner split of the node side for `world` ranks (host only): rank r owns group
        pairs [q[r], q[r + 1])."""
        ns, keep = node_soa(nodes)
        out = np.zeros(world + 1, np.uint32)
        L.check(self.lib.esc_node_owner_ranges(self.handle, C.byref(ns), world,
                                               out.ctypes.data_as(C.POINTER(C.c_uint32))), "esc_node_owner_ranges")
        return out

    # ------------------------------------------------ incremental snapshot (§8f)
    def set_spare(self, fraction: float):
        """Spare slots per pod signature class at the next load (for pods_upsert)."""
        L.check(self.lib.esc_set_spare(self.handle, float(fraction)), "esc_set_spare")

    def pods_upsert(self, ids, pods: dict) -> int:
        """Patch / insert packed pods (a `pack` result) under the given ids.  Returns the
        ABI code: 0, or ESC_E_LIMIT when the batch does not fit in place (reload)."""
        ids = np.ascontiguousarray(ids, np.int64)
        ps, keep = pod_soa(pods)
        rc = self.lib.esc_pods_upsert(self.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(ps))
        if rc not in (0, L.ESC_E_LIMIT):
            L.check(rc, "esc_pods_upsert")
        return rc

    def pods_delete(self, ids):
        ids = np.ascontiguousarray(ids, np.int64)
        L.check(self.lib.esc_pods_delete(self.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)), len(ids)),
                "esc_pods_delete")

    def nodes_update(self, ids, flags, cpu, mem):
        ids = np.ascontiguousarray(ids, np.int64)
        f = np.ascontiguousarray(flags, np.uint32)
        c_ = np.ascontiguousarray(cpu, np.int64)
        m = np.ascontiguousarray(mem, np.int64)
        L.check(self.lib.esc_nodes_update(self.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)), len(ids),
                                          f.ctypes.data_as(C.POINTER(C.c_uint32)),
                                          c_.ctypes.data_as(C.POINTER(C.c_int64)),
                                          m.ctypes.data_as(C.POINTER(C.c_int64))), "esc_nodes_update")

    def nodes_add(self, nodes: dict) -> np.ndarray:
        """Node informer Add events (cache.go:37-56): packed nodes (n_trk = 0) appended in
        place; returns their snapshot indices.  EscError(ESC_E_LIMIT) when the spare room is short."""
        n = len(nodes["flags"])
        ns, keep = node_soa(nodes)
        out = np.zeros(max(n, 1), np.int64)
        L.check(self.lib.esc_nodes_add(self.handle, C.byref(ns), out.ctypes.data_as(C.POINTER(C.c_int64))),
                "esc_nodes_add")
        del keep
        return out[:n]

    def nodes_relabel(self, ids, nodes: dict):
        """Node informer Update events with any field changed, labels and creation time
        included (esc_nodes_relabel): `nodes` = the packed new records of the nodes `ids`
        (n_trk = 0).  EscError(ESC_E_LIMIT) when the spare room is short (reload)."""
        ids = np.ascontiguousarray(ids, np.int64)
        assert len(ids) == len(nodes["flags"])
        ns, keep = node_soa(nodes)
        L.check(self.lib.esc_nodes_relabel(self.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(ns)),
                "esc_nodes_relabel")
        del keep

    def nodes_delete(self, ids):
        """Node informer Delete events: the nodes' slots become absent."""
        ids = np.ascontiguousarray(ids, np.int64)
        L.check(self.lib.esc_nodes_delete(self.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)), len(ids)),
                "esc_nodes_delete")

    def tracker_update(self, group: int, add=(), remove=()):
        """Dry-mode taintTracker change of one group in place (esc_tracker_update): the
        nodes untaintNewestN deletes (scale_up.go:146-158), then the ones taintOldestN
        appends (scale_down.go:197-200), as snapshot node indices."""
        a = np.ascontiguousarray(add, np.int64)
        r = np.ascontiguousarray(remove, np.int64)
        L.check(self.lib.esc_tracker_update(self.handle, group, a.ctypes.data_as(C.POINTER(C.c_int64)), len(a),
                                            r.ctypes.data_as(C.POINTER(C.c_int64)), len(r)), "esc_tracker_update")

    def tracker_list(self, group: int) -> np.ndarray:
        """Snapshot indices of the nodes `group`'s tracker holds, ascending."""
        n = C.c_int64()
        L.check(self.lib.esc_tracker_list(self.handle, group, None, 0, C.byref(n)), "esc_tracker_list")
        out = np.zeros(n.value, np.int64)
        L.check(self.lib.esc_tracker_list(self.handle, group, out.ctypes.data_as(C.POINTER(C.c_int64)), len(out),
                                          C.byref(n)), "esc_tracker_list")
        return out

    def stream_bytes(self) -> tuple[int, int]:
        """Algorithmic HBM bytes one decision streams on this rank: (K1 pods, K2 nodes)."""
        a, b = C.c_int64(), C.c_int64()
        L.check(self.lib.esc_stream_bytes(self.handle, C.byref(a), C.byref(b)), "esc_stream_bytes")
        return a.value, b.value

    def set_state(self, states: list[dict] | None):
        self._state = states_to_c(states, self.G)
        L.check(self.lib.esc_set_state(self.handle, self._state), "esc_set_state")

    # ------------------------------------------------------------- decision
    def set_stream(self, stream_handle: int | None):
        L.check(self.lib.esc_ctx_set_stream(self.handle, C.c_void_p(stream_handle or 0)), "esc_ctx_set_stream")

    def use_graph(self, on: bool = True):
        L.check(self.lib.esc_use_graph(self.handle, int(on)))

    def force_wide(self, on: bool = True):
        L.check(self.lib.esc_force_wide(self.handle, int(on)))

    def set_timing(self, on: bool = True):
        L.check(self.lib.esc_set_timing(self.handle, int(on)))

    def stage_times(self) -> list[float]:
        """ms per stage of the last decision (timing mode): K1, tail, orderings, node groups
        (+ K4 at world 1), [exchange, K4 at world > 1]; [9] the whole step."""
        a = (C.c_double * 10)()
        L.check(self.lib.esc_stage_times(self.handle, a, 10))
        return list(a)

    def k1_calibrate(self, rounds: int = 4):
        """Balances K1's per-workgroup shares to this device's measured streaming rates
        (esc_k1_calibrate; results unchanged)."""
        L.check(self.lib.esc_k1_calibrate(self.handle, int(rounds)), "esc_k1_calibrate")

    def k1_flush_entries(self) -> tuple[int, int]:
        """(512-B column partials K1 flushes per decision, entries of a whole-row flush)."""
        a, b = C.c_int64(), C.c_int64()
        L.check(self.lib.esc_k1_flush_entries(self.handle, C.byref(a), C.byref(b)), "esc_k1_flush_entries")
        return a.value, b.value

    def hbm_probe(self, nbytes: int = 2 << 30, reps: int = 10) -> float:
        """The device's practical HBM read rate (GB/s) in K1's access shape (esc_hbm_probe)."""
        v = C.c_double()
        L.check(self.lib.esc_hbm_probe(self.handle, int(nbytes), int(reps), C.byref(v)), "esc_hbm_probe")
        return v.value

    def k1_time(self, reps=20):
        """K1's mean device time in ms over `reps` back-to-back launches (esc_k1_time)."""
        ms = C.c_double(0)
        L.check(self.lib.esc_k1_time(self.handle, int(reps), C.byref(ms)), "esc_k1_time")
        return ms.value

    def k1_trace(self):
        """Per-workgroup K1 timestamps of the last decision (diagnostics):
        uint64 [nblk, 8] = start, K tiles done, C tiles done, flushed (100 MHz ticks), HW_ID, XCC_ID."""
        n = C.c_int64(0)
        L.check(self.lib.esc_k1_trace(self.handle, None, 0, C.byref(n)))
        a = np.zeros((n.value, 8), dtype=np.uint64)
        L.check(self.lib.esc_k1_trace(self.handle, a.ctypes.data_as(C.POINTER(C.c_uint64)), a.size, C.byref(n)))
        return a

    def run(self):
        L.check(self.lib.esc_run(self.handle), "esc_run")

    def reduce(self):
        L.check(self.lib.esc_reduce(self.handle), "esc_reduce")

    def decide(self):
        L.check(self.lib.esc_decide(self.handle), "esc_decide")

    def sync(self):
        L.check(self.lib.esc_sync(self.handle), "esc_sync")

    # ------------------------------------------ RCCL exchange inside the library (§8e)
    @staticmethod
    def comm_unique_id() -> bytes:
        """ncclGetUniqueId (rank 0); ship the bytes to the other ranks, then comm_init."""
        buf = C.create_string_buffer(L.ESC_COMM_ID_BYTES)
        L.check(L.load().esc_comm_unique_id(buf), "esc_comm_unique_id")
        return buf.raw

    def comm_init(self, uid: bytes, rank: int, world: int):
        """ncclCommInitRank on the context's device (collective over the world's ranks)."""
        assert len(uid) == L.ESC_COMM_ID_BYTES
        buf = C.create_string_buffer(uid, L.ESC_COMM_ID_BYTES)
        L.check(self.lib.esc_comm_init(self.handle, buf, rank, world), "esc_comm_init")

    def exchange(self):
        """ncclReduceScatter(int64, SUM) of the owner-major pod words, in place, on the context's
        stream: this rank receives its own groups' rows (esc_exchange_slice)."""
        L.check(self.lib.esc_exchange(self.handle), "esc_exchange")

    def step(self):
        """esc_reduce + esc_exchange + esc_decide (esc_run without a communicator)."""
        L.check(self.lib.esc_step(self.handle), "esc_step")

    def exchange_buffers(self):
        sb, mb = C.c_void_p(), C.c_void_p()
        sc, mc = C.c_int64(), C.c_int64()
        L.check(self.lib.esc_exchange_buffers(self.handle, C.byref(sb), C.byref(sc), C.byref(mb), C.byref(mc)))
        return (sb.value, sc.value), (mb.value, mc.value)

    def bind_exchange(self, sum_ptr: int | None, min_ptr: int | None):
        L.check(self.lib.esc_bind_exchange_buffers(self.handle, C.c_void_p(sum_ptr or 0), C.c_void_p(min_ptr or 0)),
                "esc_bind_exchange_buffers")

    def exchange_download(self):
        """Host copies of the words to SUM-exchange and (if min_count > 0) to MIN-exchange."""
        (_, sc), (_, mc) = self.exchange_buffers()
        s = np.zeros(sc, np.int64)
        m = np.zeros(mc, np.int64)
        mp = m.ctypes.data_as(C.POINTER(C.c_int64)) if mc else None
        L.check(self.lib.esc_exchange_download(self.handle, s.ctypes.data_as(C.POINTER(C.c_int64)), mp),
                "esc_exchange_download")
        return s, m

    def exchange_upload(self, s: np.ndarray, m: np.ndarray):
        s = np.ascontiguousarray(s, np.int64)
        m = np.ascontiguousarray(m, np.int64)
        mp = m.ctypes.data_as(C.POINTER(C.c_int64)) if m.size else None
        L.check(self.lib.esc_exchange_upload(self.handle, s.ctypes.data_as(C.POINTER(C.c_int64)), mp),
                "esc_exchange_upload")

    def results(self):
        t = np.zeros(self.G, TOTALS_DTYPE)
        d = np.zeros(self.G, DECISION_DTYPE)
        L.check(self.lib.esc_results(self.handle, t.ctypes.data_as(C.POINTER(L.GroupTotals)),
                                     d.ctypes.data_as(C.POINTER(L.GroupDecision))), "esc_results")
        return t, d

    def set_metrics(self, on: bool = True):
        """K4 also computes the per-group gauges scaleNodeGroup sets (§8f)."""
        L.check(self.lib.esc_set_metrics(self.handle, int(on)), "esc_set_metrics")

    def metrics(self) -> np.ndarray:
        m = np.zeros(self.G, METRICS_DTYPE)
        L.check(self.lib.esc_metrics_results(self.handle, m.ctypes.data_as(C.POINTER(L.GroupMetrics))),
                "esc_metrics_results")
        return m

    def decide_all(self, states: list[dict] | None = None):
        """One full decision (world == 1): totals and decisions for every group."""
        self.set_state(states)
        self.run()
        return self.results()

    # ------------------------------------------------ scale-down reaping (§8f rank 2)
    def load_placement(self, pod_node, taint_s, no_delete):
        """Bind the loaded pods to nodes (node index per pod id, NONE = none) and load each
        node's escalator-taint time (Unix s, INT64_MIN = none) and no-delete flag
        (objects.placement builds them).  pod_node=None refreshes the node facts only."""
        t = np.ascontiguousarray(taint_s, np.int64)
        nd = np.ascontiguousarray(no_delete, np.uint8)
        pn = None if pod_node is None else np.ascontiguousarray(pod_node, np.uint32)
        L.check(self.lib.esc_load_placement(self.handle, None if pn is None else pn.ctypes.data_as(C.POINTER(C.c_uint32)),
                                            t.ctypes.data_as(C.POINTER(C.c_int64)),
                                            nd.ctypes.data_as(C.POINTER(C.c_uint8))), "esc_load_placement")

    def try_remove(self, now_ns: int, soft_ns, hard_ns) -> np.ndarray:
        """TryRemoveTaintedNodes for every group: (n_candidates, n_delete, pods_remaining)."""
        s_ = np.ascontiguousarray(np.broadcast_to(np.asarray(soft_ns, np.int64), (self.G,)))
        h_ = np.ascontiguousarray(np.broadcast_to(np.asarray(hard_ns, np.int64), (self.G,)))
        out = np.empty(self.G, REMOVAL_DTYPE)          # every record is written
        L.check(self.lib.esc_try_remove(self.handle, int(now_ns), s_.ctypes.data_as(C.POINTER(C.c_int64)),
                                        h_.ctypes.data_as(C.POINTER(C.c_int64)),
                                        out.ctypes.data_as(C.POINTER(L.Removal))), "esc_try_remove")
        return out

    def pods_bind(self, ids, pod_node):
        """Spec.NodeName changes of pods (node index, NONE = unbound): the placement follows."""
        ids = np.ascontiguousarray(ids, np.int64)
        pn = np.ascontiguousarray(pod_node, np.uint32)
        L.check(self.lib.esc_pods_bind(self.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)),
                                       pn.ctypes.data_as(C.POINTER(C.c_uint32)), len(ids)), "esc_pods_bind")

    # the sharded reaping steps (esc_try_remove does all three, with the RCCL sum)
    def reap_occupancy(self):
        L.check(self.lib.esc_reap_occupancy(self.handle), "esc_reap_occupancy")

    def reap_download(self) -> np.ndarray:
        buf, n = C.c_void_p(), C.c_int64()
        L.check(self.lib.esc_reap_buffer(self.handle, C.byref(buf), C.byref(n)), "esc_reap_buffer")
        out = np.zeros(max(n.value, 1), np.uint32)
        L.check(self.lib.esc_reap_download(self.handle, out.ctypes.data_as(C.POINTER(C.c_uint32))), "esc_reap_download")
        return out[:n.value]

    def reap_upload(self, words):
        w = np.ascontiguousarray(words, np.uint32)
        L.check(self.lib.esc_reap_upload(self.handle, w.ctypes.data_as(C.POINTER(C.c_uint32))), "esc_reap_upload")

    def reap_finish(self, now_ns: int, soft_ns, hard_ns) -> np.ndarray:
        s_ = np.ascontiguousarray(np.broadcast_to(np.asarray(soft_ns, np.int64), (self.G,)))
        h_ = np.ascontiguousarray(np.broadcast_to(np.asarray(hard_ns, np.int64), (self.G,)))
        out = np.zeros(self.G, REMOVAL_DTYPE)
        L.check(self.lib.esc_reap_finish(self.handle, int(now_ns), s_.ctypes.data_as(C.POINTER(C.c_int64)),
                                         h_.ctypes.data_as(C.POINTER(C.c_int64)),
                                         out.ctypes.data_as(C.POINTER(L.Removal))), "esc_reap_finish")
        return out

    def removal_nodes(self, group: int) -> np.ndarray:
        """Snapshot indices of the nodes the last try_remove deletes for `group`, in order."""
        n = C.c_int64()
        rc = self.lib.esc_removal_nodes(self.handle, group, None, 0, C.byref(n))
        if rc not in (0, L.ESC_E_LIMIT):
            L.check(rc, "esc_removal_nodes")
        out = np.zeros(max(n.value, 1), np.int64)
        L.check(self.lib.esc_removal_nodes(self.handle, group, out.ctypes.data_as(C.POINTER(C.c_int64)), len(out),
                                           C.byref(n)), "esc_removal_nodes")
        return out[:n.value]

    # ------------------------------------------------------------- ordering
    def sort_nodes(self):
        L.check(self.lib.esc_sort_nodes(self.handle), "esc_sort_nodes")

    def set_order_in_step(self, on: bool = True):
        """Run the K5 ordering inside every decision (beside K1, in the step's graph)."""
        L.check(self.lib.esc_set_order_in_step(self.handle, int(bool(on))), "esc_set_order_in_step")

    def order_info(self) -> tuple[int, int]:
        """(memberships of the node range, creation-key bits of the age index)."""
        n, b = C.c_int64(), C.c_int32()
        L.check(self.lib.esc_order_info(self.handle, C.byref(n), C.byref(b)), "esc_order_info")
        return n.value, b.value

    def build_age_index(self):
        """Re-run the snapshot's age index build (normally done by load)."""
        L.check(self.lib.esc_build_age_index(self.handle), "esc_build_age_index")

    def group_order(self, group: int, which: int, cap: int | None = None) -> np.ndarray:
        n = C.c_int64()
        L.check(self.lib.esc_group_order(self.handle, group, which, None, 0, C.byref(n)), "esc_group_order")
        m = n.value if cap is None else min(cap, n.value)
        out = np.zeros(max(m, 1), np.int64)
        L.check(self.lib.esc_group_order(self.handle, group, which, out.ctypes.data_as(C.POINTER(C.c_int64)), m,
                                         C.byref(n)), "esc_group_order")
        return out[:m]

    def set_selections(self, slack: int = 0, group_cap: int = 0):
        """Deliver every decided group's taint / untaint nodes with the decision
        (esc_set_selections; slack < 0 turns them off).  Needs the ordering in the step."""
        L.check(self.lib.esc_set_selections(self.handle, int(slack), int(group_cap)), "esc_set_selections")

    def selections(self):
        """The last decision's selections: (which[G] (ESC_SEL_*), offsets[G + 1], nodes) —
        group g's snapshot indices are nodes[offsets[g]:offsets[g + 1]] (esc_selections)."""
        which = np.zeros(self.G, np.int32)
        off = np.zeros(self.G + 1, np.int64)
        n = C.c_int64()
        wp, op = which.ctypes.data_as(C.POINTER(C.c_int32)), off.ctypes.data_as(C.POINTER(C.c_int64))
        L.check(self.lib.esc_selections(self.handle, wp, op, None, 0, C.byref(n)), "esc_selections")
        idx = np.zeros(max(n.value, 1), np.int64)
        L.check(self.lib.esc_selections(self.handle, wp, op, idx.ctypes.data_as(C.POINTER(C.c_int64)), len(idx),
                                        C.byref(n)), "esc_selections")
        return which, off, idx[:n.value]

    def close(self):
        if self.handle:
            self.lib.esc_ctx_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
