"""Input writer and output reader for go/escalatorhip/harness/esc_harness (test
infrastructure): the harness makes the cgo shim's ABI calls on the object dicts of
escalator_amd/objects.py, serialised as whitespace-separated tokens."""
from __future__ import annotations

import os
import subprocess
from urllib.parse import quote

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS_DIR = os.path.join(ROOT, "go", "escalatorhip", "harness")
HARNESS = os.environ.get("ESC_HARNESS") or os.path.join(HARNESS_DIR, "esc_harness")


def build_harness() -> str:
    if not os.environ.get("ESC_HARNESS"):
        subprocess.run(["make", "-s", "-C", HARNESS_DIR], check=True)
    return HARNESS


def _s(x) -> str:
    return "s" + quote(x if x is not None else "", safe="")


def _req(r) -> list:
    if r is None:
        return [0, 0, 0, 0]
    cpu, mem = r.get("cpu"), r.get("mem")
    return [cpu or 0, mem or 0, int(cpu is not None), int(mem is not None)]


def _pod(p: dict) -> list:
    t = []
    kinds = list(p.get("owner_kinds") or [])
    t += [len(kinds)] + [_s(k) for k in kinds]
    ann = p.get("annotations") or {}
    has = "kubernetes.io/config.source" in ann
    t += [int(has), _s(ann.get("kubernetes.io/config.source", ""))]
    sel = p.get("node_selector") or {}
    t += [len(sel)]
    for k, v in sel.items():
        t += [_s(k), _s(v)]
    aff = p.get("affinity")
    exprs = []
    flags = [0, 0, 0, 0, 0]
    if aff is not None:
        na = aff.get("node_affinity")
        flags = [1, int(na is not None), int(bool(aff.get("pod_affinity"))),
                 int(bool(aff.get("pod_anti_affinity"))), 0]
        if na is not None and na.get("required") is not None:
            flags[4] = 1
            for ti, term in enumerate(na["required"]):
                for e in term:
                    vals = list(e.get("values") or [])
                    exprs.append([_s(e["key"]), _s(e["op"]), len(vals)] + [_s(v) for v in vals] + [ti])
    t += flags + [len(exprs)]
    for e in exprs:
        t += e
    cs = p.get("containers") or []
    t += [len(cs)]
    for c in cs:
        t += _req(c)
    ic = p.get("init_containers") or []
    t += [len(ic)]
    for c in ic:
        t += _req(c)
    ovh = p.get("overhead")
    t += [int(ovh is not None)] + _req(ovh)
    return t


def _node(n: dict) -> list:
    labels = n.get("labels") or {}
    t = [_s(n.get("name", "")), len(labels)]
    for k, v in labels.items():
        t += [_s(k), _s(v)]
    taints = list(n.get("taints") or [])
    t += [int(bool(n.get("unschedulable"))), len(taints)] + [_s(k) for k in taints]
    t += _req({"cpu": n.get("cpu"), "mem": n.get("mem")}) + [int(n.get("created_ns", 0))]
    return t


def write_input(path: str, groups, states, pods, nodes, trackers=None, device: int = 0):
    lines = ["ESCH1", "device %d" % device, "groups %d" % len(groups)]
    for g in groups:
        lines.append(" ".join(str(x) for x in [
            _s(g.get("name", "")), _s(g.get("label_key", "")), _s(g.get("label_value", "")),
            g.get("min_nodes", 0), g.get("max_nodes", 0), g.get("taint_upper_pct", 0), g.get("taint_lower_pct", 0),
            g.get("scale_up_pct", 0), g.get("slow_removal_rate", 0), g.get("fast_removal_rate", 0),
            int(bool(g.get("dry_mode", False)))]))
    lines.append("states")
    for i in range(len(groups)):
        st = (states[i] if states else None) or {}
        lines.append("%d %d %d %d" % (int(bool(st.get("locked", 0))), st.get("requested_nodes", 0),
                                      st.get("cached_cpu_m", 0), st.get("cached_mem_b", 0)))
    lines.append("pods %d" % len(pods))
    lines += [" ".join(str(x) for x in _pod(p)) for p in pods]
    lines.append("nodes %d" % len(nodes))
    lines += [" ".join(str(x) for x in _node(n)) for n in nodes]
    trackers = trackers or {}
    lines.append("trackers %d" % len(trackers))
    for g, names in sorted(trackers.items()):
        lines.append(" ".join(str(x) for x in [g, len(names)] + [_s(s) for s in names]))
    lines.append("end")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def run(path: str, timeout: int = 120, shards: int = 0) -> dict:
    """shards > 0: the NewContextMulti sequence (esc_ctx_create_multi over `shards` copies of
    the input's device)."""
    args = [HARNESS, path] + ([str(shards)] if shards else [])
    out = subprocess.run(args, check=True, capture_output=True, text=True, timeout=timeout).stdout
    res = {"totals": {}, "decision": {}, "status": {}, "order": {}, "nodev": None, "lines": out}
    for line in out.splitlines():
        w = line.split(" ")
        if w[0] == "totals":
            res["totals"][int(w[1])] = [int(x) for x in w[2:]]
        elif w[0] == "decision":
            g = int(w[1])
            res["decision"][g] = {"cpu_bits": int(w[2], 16), "mem_bits": int(w[3], 16), "delta": int(w[4]),
                                  "n_to_taint": int(w[5]), "cached_cpu_m": int(w[6]), "cached_mem_b": int(w[7]),
                                  "status": int(w[8]), "branch": int(w[9]), "taint_status": int(w[10])}
        elif w[0] == "status":
            res["status"][int(w[1])] = line.split(" ", 2)[2]
        elif w[0] == "order":
            res["order"][(int(w[1]), int(w[2]))] = [int(x) for x in w[4:4 + int(w[3])]]
        elif w[0] == "select":
            res.setdefault("select", {})[int(w[1])] = (int(w[2]), [int(x) for x in w[4:4 + int(w[3])]])
        elif w[0] == "nodev":
            res["nodev"] = w[1]
        elif w[0] in ("list_pods", "list_nodes"):
            res[w[0]] = None if w[1] == "overflow" else (int(w[1]), int(w[2]))
        elif w[0] in ("pct", "delta", "packed", "abi"):
            res[w[0]] = w[1:]
    return res
