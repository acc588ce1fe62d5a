"""Object builders mirroring the reference's test fixtures.

``build_test_pod`` / ``build_test_node`` follow ``pkg/test/builder.go:104-296``
(BuildTestNode, BuildTestNodes, BuildTestPod, BuildTestPods) field for field,
including their quirks:

* BuildTestNode always sets ``Labels{LabelKey: LabelValue}`` (the empty pair when the
  options leave them empty, builder.go:119-121) and copies Capacity into Allocatable;
  a negative CPU or Mem leaves that resource absent (:135-140).
* BuildTestPod always sets a non-nil (possibly empty) Overhead map (:239-245); a
  nodeSelector / affinity is created when key OR value is non-empty (:207, :214); the
  init-container loop tests ``opts.CPU[i]`` / ``opts.Mem[i]`` for presence but stores
  the init values (:276-283).

Objects are the plain-dict schema of ``escalator_amd/objects.py``.
"""
from __future__ import annotations

import datetime as _dt

EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


def unix_ns(year, month, day, hour=0, minute=0, sec=0, nsec=0) -> int:
    """time.Date(...).UnixNano() for a UTC date."""
    d = _dt.datetime(year, month, day, hour, minute, sec, tzinfo=_dt.timezone.utc)
    delta = d - EPOCH
    return (delta.days * 86400 + delta.seconds) * 1_000_000_000 + nsec


def build_test_node(opts: dict) -> dict:
    """BuildTestNode — pkg/test/builder.go:104-148."""
    cpu = opts.get("CPU", 0)
    mem = opts.get("Mem", 0)
    return {
        "name": opts.get("Name", ""),
        "labels": {opts.get("LabelKey", ""): opts.get("LabelValue", "")},
        "unschedulable": bool(opts.get("Unschedulable", False)),
        "taints": ["atlassian.com/escalator"] if opts.get("Tainted") else [],
        "cpu": cpu if cpu >= 0 else None,
        "mem": mem if mem >= 0 else None,
        "created_ns": opts.get("Creation", 0),
    }


def build_test_nodes(amount: int, opts: dict, name_prefix: str = "n") -> list[dict]:
    """BuildTestNodes — builder.go:151-158 (names are UUIDs there; unique names here)."""
    out = []
    for i in range(amount):
        o = dict(opts)
        o["Name"] = "%s-%d" % (name_prefix, i)
        out.append(build_test_node(o))
    return out


def build_test_pod(opts: dict) -> dict:
    """BuildTestPod — pkg/test/builder.go:180-286."""
    cpus = list(opts.get("CPU", []))
    mems = list(opts.get("Mem", []))
    icpus = list(opts.get("InitContainersCPU", []))
    imems = list(opts.get("InitContainersMem", []))
    sel_k = opts.get("NodeSelectorKey", "")
    sel_v = opts.get("NodeSelectorValue", "")
    aff_k = opts.get("NodeAffinityKey", "")
    aff_v = opts.get("NodeAffinityValue", "")
    node_selector = {sel_k: sel_v} if (sel_k or sel_v) else None
    affinity = None
    if aff_k or aff_v:
        affinity = {"node_affinity": {"required": [[{"key": aff_k, "op": opts.get("NodeAffinityOp") or "In",
                                                     "values": [aff_v]}]]},
                    "pod_affinity": False, "pod_anti_affinity": False}
    overhead = {"cpu": None, "mem": None}
    if opts.get("CPUOverhead", 0) > 0:
        overhead["cpu"] = opts["CPUOverhead"]
    if opts.get("MemOverhead", 0) > 0:
        overhead["mem"] = opts["MemOverhead"]
    containers = [{"cpu": cpus[i] if cpus[i] >= 0 else None,
                   "mem": mems[i] if mems[i] >= 0 else None} for i in range(len(cpus))]
    inits = [{"cpu": icpus[i] if cpus[i] >= 0 else None,        # quirk: tests opts.CPU[i]
              "mem": imems[i] if mems[i] >= 0 else None}        # quirk: tests opts.Mem[i]
             for i in range(len(icpus))]
    return {
        "name": opts.get("Name", ""),
        "owner_kinds": [opts["Owner"]] if opts.get("Owner") else [],
        "annotations": dict(opts.get("Annotations", {})),
        "node_selector": node_selector,
        "affinity": affinity,
        "containers": containers,
        "init_containers": inits,
        "overhead": overhead,
        "node_name": opts.get("NodeName", ""),
    }


def build_test_pods(amount: int, opts: dict) -> list[dict]:
    """BuildTestPods — builder.go:289-296."""
    out = []
    for i in range(amount):
        o = dict(opts)
        o["Name"] = "p%d" % i
        out.append(build_test_pod(o))
    return out
