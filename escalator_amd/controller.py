"""Mirror of the reference's ``pkg/controller`` decision path over the GPU path.

* ``calc_percent_usage`` / ``calc_scale_up_delta`` — pkg/controller/util.go:58 / :13
  (the library's bit-exact scalar build of the K4 kernel's arithmetic).
* ``taint_oldest_n`` / ``untaint_newest_n`` — scale_down.go:171 / scale_up.go:118 orderings
  (GPU radix sort; every taint/untaint succeeds, i.e. the dry-mode walk).
* ``Controller`` — (*Controller).RunOnce (controller.go:400) over every group in ONE
  batched decision: listers -> K0 packer -> HIP reduce -> K4 decide.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

ERRORS = {L.ESC_ST_OK: None, L.ESC_ST_ERR_MIN_NODES: "node count less than the minimum",
          L.ESC_ST_ERR_MAX_NODES: "node count larger than the maximum",
          L.ESC_ST_ERR_DIV_ZERO: "cannot divide by zero in percent calculation",
          L.ESC_ST_ERR_NEG_DELTA: "negative scale up delta",
          L.ESC_ST_ERR_OVERFLOW: "int64 overflow (Quantity inf.Dec regime, not emulated)"}


def calc_percent_usage(cpu_request: int, mem_request: int, cpu_capacity: int, mem_capacity: int,
                       number_of_untainted_nodes: int):
    """calcPercentUsage — pkg/controller/util.go:58.  Returns (cpu%, mem%, error-or-None)."""
    a, b = C.c_double(), C.c_double()
    st = L.load().esc_calc_percent_usage(cpu_request, mem_request, cpu_capacity, mem_capacity,
                                         number_of_untainted_nodes, C.byref(a), C.byref(b))
    return a.value, b.value, ERRORS.get(st, "status %d" % st)


def calc_scale_up_delta(n_untainted: int, cpu_percent: float, mem_percent: float, cpu_request: int,
                        mem_request: int, cached_cpu_m: int, cached_mem_b: int, scale_up_threshold_percent: int):
    """calcScaleUpDelta — pkg/controller/util.go:13.  Returns (delta, error-or-None)."""
    d = C.c_int64()
    st = L.load().esc_calc_scale_up_delta(n_untainted, cpu_percent, mem_percent, cpu_request, mem_request,
                                          cached_cpu_m, cached_mem_b, scale_up_threshold_percent, C.byref(d))
    return d.value, ERRORS.get(st, "status %d" % st)


def _order(created_ns, n: int, oldest: bool, device: int) -> list[int]:
    from .k8s import _device_ctx
    ctx = _device_ctx(device)
    ts = np.ascontiguousarray(created_ns, np.int64)
    k = max(0, min(int(n), len(ts)))
    out = np.zeros(max(k, 1), np.int64)
    L.check(ctx.lib.esc_order_by_creation(ctx.handle, ts.ctypes.data_as(C.POINTER(C.c_int64)), len(ts),
                                          int(oldest), k, out.ctypes.data_as(C.POINTER(C.c_int64))),
            "esc_order_by_creation")
    return [int(x) for x in out[:k]]


def taint_oldest_n(created_ns, n: int, device: int = 0) -> list[int]:
    """taintOldestN — scale_down.go:171: indices (into the given list) of the n oldest."""
    return _order(created_ns, n, True, device)


def untaint_newest_n(created_ns, n: int, device: int = 0) -> list[int]:
    """untaintNewestN — scale_up.go:118: indices of the n newest (over the tainted list)."""
    return _order(created_ns, n, False, device)


# The methods Controller calls on its actuator (per node: taint / untaint return whether the
# API write succeeded; the cloud node group's TargetSize / MaxSize / IncreaseSize /
# DeleteNodes, cloudprovider/interface.go:45-80)
ACTUATOR_METHODS = ("taint", "untaint", "target_size", "max_size", "increase_size", "delete_nodes")


class SimulatedCloud:
    """The actuator used when none is given: every Kubernetes write succeeds, and the
    cloud node group behaves like the reference tests' mock (pkg/test/cloud_provider.go):
    TargetSize is the group's listed node count and MaxSize its ``max_nodes``;
    IncreaseSize and DeleteNodes succeed."""

    def __init__(self, groups):
        self.groups = groups
        self.size = [0] * len(groups)

    def observe(self, g: int, n_nodes: int):
        self.size[g] = int(n_nodes)

    def taint(self, g: int, node: int) -> bool:
        return True

    def untaint(self, g: int, node: int) -> bool:
        return True

    def target_size(self, g: int) -> int:
        return self.size[g]

    def max_size(self, g: int) -> int:
        return int(self.groups[g].get("max_nodes", 0))

    def increase_size(self, g: int, n: int):
        self.size[g] += n

    def delete_nodes(self, g: int, nodes: list[int]):
        self.size[g] -= len(nodes)


class Controller:
    """RunOnce over every node group as one GPU decision, plus the actuation bookkeeping
    the next run depends on.

    ``list_pods`` / ``list_nodes`` play the informer-backed listers
    (pkg/k8s/pod_listers.go:33, node_listers.go:33): callables returning the full
    cluster lists (plain-dict records, escalator_amd/objects.py) or raising.

    Host state kept across runs, as the reference's NodeGroupState (controller.go:28-44):
      * cached capacity of allNodes[0] (controller.go:207-211);
      * the scale-up lock (scale_lock.go): ScaleUp locks it with the nodes it added
        (scale_up.go:39); while ``clock() - lock_time < scale_up_cool_down_ns`` every run
        returns ``requestedNodes`` (controller.go:317-323), after that it unlocks;
      * the dry-mode taintTracker: taintOldestN appends the names it "taints"
        (scale_down.go:197-200), untaintNewestN deletes the newest tracked names
        (scale_up.go:146-158); filterNodes reads it on the next run (controller.go:126-138).

    Actuation follows the reference's walk: taintOldestN / untaintNewestN go down the GPU
    ordering one node at a time and skip a node whose API write fails until n writes
    succeeded (scale_down.go:179-202, scale_up.go:127-160); the cloud add is clamped to
    MaxSize - TargetSize (calculateNodesToAdd, scale_up.go:48-56) in wet and dry mode, and a
    clamp <= 0 is scaleUpCloudProviderNodeGroup's error without a lock (scale_up.go:66-74);
    TryRemoveTaintedNodes (scale_down.go:51-136) runs before tainting and in the no-change
    branch (controller.go:369-383) on the GPU's reaping pass.  The walks read the selections
    the decision delivers (esc_selections: each group's first n + ``selection_slack`` nodes of
    its order, written to pinned memory inside the step) and continue on esc_group_order only
    when failed writes use up the slack (``walk_fallback`` in the group's result).  The ``actuator`` provides
    ``taint(g, node) -> bool``, ``untaint(g, node) -> bool``, ``target_size(g)``,
    ``max_size(g)``, ``increase_size(g, n)`` and ``delete_nodes(g, nodes)`` (raising on an
    API error); without one a ``SimulatedCloud`` stands in (every write succeeds)."""

    def __init__(self, groups: list[dict], device: int = 0, dry_mode: bool = False, clock=None, actuator=None,
                 selection_slack: int = 4):
        import time
        from .context import Context
        self.groups = [dict(g, dry_mode=bool(g.get("dry_mode")) or dry_mode) for g in groups]
        self.ctx = Context(self.groups, device=device)
        self.ctx.set_order_in_step(True)                   # the orderings and the walks' prefixes
        self.ctx.set_selections(selection_slack)           # come with every decision
        self._sel = None
        self.state = [{"locked": False, "requested_nodes": 0, "cached_cpu_m": 0, "cached_mem_b": 0}
                      for _ in groups]
        self.lock_time = [None] * len(groups)          # scaleLock.lockTime (None: never locked)
        self.taint_tracker = {g: [] for g in range(len(groups))}
        self.clock = clock or time.time_ns
        self.actuator = actuator if actuator is not None else SimulatedCloud(self.groups)
        # the actuator protocol (per-node taint/untaint -> bool, the cloud group's sizes):
        # refused here rather than by an AttributeError after a decision
        missing = [m for m in ACTUATOR_METHODS if not callable(getattr(self.actuator, m, None))]
        if missing:
            raise TypeError("actuator %r lacks %s (the protocol: %s; see INTEGRATION.md §5)" %
                            (type(self.actuator).__name__, ", ".join(missing), ", ".join(ACTUATOR_METHODS)))

    def _lock_states(self, now: int):
        """scaleLock.locked() (scale_lock.go:22-29) for every group, before the decision."""
        for g, grp in enumerate(self.groups):
            t = self.lock_time[g]
            if t is not None and now - t < int(grp.get("scale_up_cool_down_ns", 0)):
                self.state[g]["locked"] = True
            else:                                          # unlock(): requestedNodes = 0
                self.state[g]["locked"] = False
                self.state[g]["requested_nodes"] = 0

    def _walk(self, g: int, which: int, n_avail: int, out: dict):
        """The order a taint / untaint walk goes down (0: untainted oldest first, 1: tainted
        newest first): the selection the decision delivered, then — only if the walk needs
        more (failed writes used up the slack, or the list was cut) — esc_group_order beyond it."""
        got = []
        if self._sel is not None:
            w, off, idx = self._sel
            if int(w[g]) >= 0 and int(w[g]) & 3 == which:
                got = [int(j) for j in idx[off[g]:off[g + 1]]]
        yield from got
        if len(got) >= n_avail:                             # the list is the whole order
            return
        out["walk_fallback"] = True
        yield from (int(j) for j in self.ctx.group_order(g, which)[len(got):])

    def _scale_up(self, g: int, n: int, n_tainted: int, names: list[str], out: dict):
        """ScaleUp (scale_up.go:14-46): untaintNewestN over the tainted nodes, the rest
        from the cloud node group (clamped to its MaxSize), then the lock.  Returns
        (nodes brought up, error-or-None)."""
        dry = self.groups[g]["dry_mode"]
        picked = []
        if n_tainted and n > 0:                            # scaleUpUntaint :98-116
            # the count is checked after each pick, so the walk never asks for a node past
            # the last one it needs (that would read on beyond the delivered selection)
            for j in self._walk(g, 1, n_tainted, out):     # newest first (sort.go:27-39), untaintNewestN :127-160
                if dry:                                    # delete the tracked name, if any
                    trk = self.taint_tracker[g]
                    if names[j] in trk:
                        trk.remove(names[j])
                        picked.append(j)
                elif self.actuator.untaint(g, j):          # a failed write moves on
                    picked.append(j)
                if len(picked) >= n:
                    break
        out["untainted_now"] = picked
        rest = n - len(picked)
        out["added"] = 0
        if rest <= 0:
            return len(picked), None
        # scaleUpCloudProviderNodeGroup :58-96 with calculateNodesToAdd :48-56
        target, mx = int(self.actuator.target_size(g)), int(self.actuator.max_size(g))
        add = mx - target if target + rest > mx else rest
        if add <= 0:
            return 0, ("refusing to scaleup up beyond the maximum size of the autoscaling group "
                       "(TargetSize: %d; MaxNodes: %d). Taking no action" % (target, int(self.groups[g].get("max_nodes", 0))))
        if not dry:
            try:
                self.actuator.increase_size(g, add)
            except Exception as e:                         # :84-87
                return 0, str(e)
        self.lock_time[g] = self.clock()                   # scaleLock.lock(added) :39
        self.state[g]["locked"] = True
        self.state[g]["requested_nodes"] = add
        out["added"] = add
        return len(picked) + add, None

    def _scale_down_taint(self, g: int, n: int, n_untainted: int, names: list[str], out: dict):
        """scaleDownTaint -> taintOldestN (scale_down.go:138-205) with the clamped n: the
        untainted nodes oldest first until n taints succeeded."""
        dry = self.groups[g]["dry_mode"]
        picked = []
        for j in (self._walk(g, 0, n_untainted, out) if n > 0 else ()):
            if dry:
                self.taint_tracker[g].append(names[j])
                picked.append(j)
            elif self.actuator.taint(g, j):
                picked.append(j)
            if len(picked) >= n:
                break
        out["tainted_now"] = picked

    def _reap(self, g: int, out: dict):
        """TryRemoveTaintedNodes (scale_down.go:51-136): the GPU pass's toBeDeleted list
        for the group, handed to the cloud node group (DeleteNodes) in wet mode."""
        n = int(self._removal[g]["n_delete"])
        nodes = [int(j) for j in self.ctx.removal_nodes(g)] if n else []
        out["removed"] = nodes
        out["pods_evicted"] = int(self._removal[g]["pods_remaining"]) if n else 0
        if nodes and not self.groups[g]["dry_mode"]:
            try:
                self.actuator.delete_nodes(g, nodes)
            except Exception as e:
                out["reap_err"] = str(e)

    def run_once(self, list_pods, list_nodes) -> list[dict]:
        try:
            pods = list_pods()
        except Exception as e:                   # controller.go:195-198
            return [{"delta": 0, "err": str(e)} for _ in self.groups]
        try:
            nodes = list_nodes()
        except Exception as e:                   # controller.go:202-205
            return [{"delta": 0, "err": str(e)} for _ in self.groups]
        from .objects import placement
        now = self.clock()
        self._lock_states(now)
        trackers = {g: list(t) for g, t in self.taint_tracker.items() if t}
        P, N = self.ctx.pack(pods, nodes, trackers)
        self.ctx.load(P, N)
        tot, dec = self.ctx.decide_all(self.state)       # the ordering is in the step
        try:
            self._sel = self.ctx.selections()
        except L.EscError as e:
            if e.code != L.ESC_E_ORDER:
                raise
            self._sel = None                               # that ordering gave up: order afresh,
            self.ctx.sort_nodes()                          # the walks read esc_group_order
        # CreateNodeNameToInfoMap (controller.go:259) + the reaping pass for every group
        self.ctx.load_placement(*placement(pods, nodes))
        soft = [int(grp.get("soft_delete_grace_ns", 0)) for grp in self.groups]
        hard = [int(grp.get("hard_delete_grace_ns", 0)) for grp in self.groups]
        self._removal = self.ctx.try_remove(now, soft, hard)
        names = [n.get("name", "") for n in nodes]
        out = []
        for g in range(len(self.groups)):
            d = dec[g]
            self.state[g]["cached_cpu_m"] = int(d["cached_cpu_m"])        # controller.go:208-211
            self.state[g]["cached_mem_b"] = int(d["cached_mem_b"])
            if hasattr(self.actuator, "observe"):
                self.actuator.observe(g, int(tot["n_nodes"][g]))
            branch = L.BRANCHES[int(d["branch"])]
            r = {"delta": int(d["delta"]), "err": ERRORS.get(int(d["status"])),
                 "branch": branch, "cpu_pct": float(d["cpu_pct"]),
                 "mem_pct": float(d["mem_pct"]), "n_to_taint": int(d["n_to_taint"]),
                 "totals": {k: int(tot[g][k]) for k in tot.dtype.names},
                 "tainted_now": [], "untainted_now": [], "added": 0, "removed": [], "pods_evicted": 0,
                 "walk_fallback": False}
            n_tainted, n_untainted = int(tot["n_tainted"][g]), int(tot["n_untainted"][g])
            if branch == "below_min":                                     # controller.go:281-295
                r["delta"], r["err"] = self._scale_up(g, r["delta"], n_tainted, names, r)
            elif r["err"] is None and branch in ("fast_down", "slow_down", "scale_up", "none"):
                # the action switch is on nodesDelta's sign, whichever branch computed it
                # (controller.go:367-383; a scale-up from zero can compute 0)
                if r["delta"] < 0:
                    self._reap(g, r)                                      # ScaleDown: reap first
                    if int(d["taint_status"]) == 0:
                        self._scale_down_taint(g, r["n_to_taint"], n_untainted, names, r)   # controller.go:368-371
                    else:
                        r["action_err"] = "taint clamp"                   # scale_down.go:150-154
                elif r["delta"] > 0:
                    _, r["action_err"] = self._scale_up(g, r["delta"], n_tainted, names, r)   # :372-375
                else:
                    self._reap(g, r)                                      # default: controller.go:377-383
            out.append(r)
        return out

    def scale_node_group(self, name: str, list_pods, list_nodes) -> tuple[int, str | None]:
        """(*Controller).scaleNodeGroup — controller.go:192, for one named group."""
        g = next(i for i, s in enumerate(self.groups) if s["name"] == name)
        r = self.run_once(list_pods, list_nodes)[g]
        return r["delta"], r["err"]
