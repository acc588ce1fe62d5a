"""Random object-level clusters (pods, nodes, groups) exercising every hot-path branch:
daemonset/static pods, nodeSelector and affinity routes (In / NotIn / several values /
several terms), default-group pods, PodAffinity-only pods, absent / zero / negative /
huge requests, init containers, empty and non-empty overhead, groups sharing one label
pair, a "default" group, dry-mode groups with taint trackers, cordoned and tainted
nodes, nodes in several groups and equal creation timestamps."""
from __future__ import annotations

import random

KEYS = ["customer", "pool", "team", ""]


def make_groups(rng: random.Random, G: int, with_default: bool = True) -> list[dict]:
    groups = []
    for g in range(G):
        if with_default and g == 0:
            name, k, v = "default", rng.choice(["customer", ""]), rng.choice(["default", ""])
        else:
            name = "ng-%d" % g
            k = rng.choice(KEYS[:3]) if rng.random() > 0.03 else ""
            v = "v%d" % rng.randrange(max(2, G))
            if g > 1 and rng.random() < 0.1:           # share the pair of an earlier group
                j = rng.randrange(1, g)
                k, v = groups[j]["label_key"], groups[j]["label_value"]
        lower = rng.randrange(0, 50)
        upper = lower + rng.randrange(0, 40)
        up = upper + rng.randrange(0, 60)
        if rng.random() < 0.05:
            up = 0                                      # validation bypassed (as reference tests do)
        slow = rng.randrange(0, 4)
        groups.append({"name": name, "label_key": k, "label_value": v,
                       "min_nodes": rng.choice([0, 0, 1, 2, 3, 5, 30]),
                       "max_nodes": rng.choice([0, 5, 1000, 1000, 1000, 1000]),
                       "taint_lower_pct": lower, "taint_upper_pct": upper, "scale_up_pct": up,
                       "slow_removal_rate": slow, "fast_removal_rate": slow + rng.randrange(0, 4),
                       "dry_mode": rng.random() < 0.15})
    return groups


def _req(rng, big=False):
    r = {}
    x = rng.random()
    r["cpu"] = None if x < 0.05 else (0 if x < 0.1 else rng.randrange(1, 4000))
    y = rng.random()
    r["mem"] = None if y < 0.05 else (0 if y < 0.1 else rng.randrange(1, 1 << 34))
    if big and rng.random() < 0.5:
        r["cpu"] = rng.choice([(1 << 20) + rng.randrange(100), (1 << 33), -rng.randrange(1, 1000)])
    if big and rng.random() < 0.5:
        r["mem"] = rng.choice([(1 << 44) + 7, (1 << 50), -rng.randrange(1, 1 << 20)])
    if big and rng.random() < 0.3:           # the packed K blocks' edges (kp_fits, kp8_fits): just in / out
        r["cpu"] = rng.choice([(1 << 14) - 1, 1 << 14, (1 << 20) - 2, (1 << 20) - 1])
        r["mem"] = rng.choice([(1 << 34) - 1, 1 << 34, (1 << 44) - 2, (1 << 44) - 1])
    return r


def make_pods(rng: random.Random, n: int, groups: list[dict], big_frac: float = 0.01) -> list[dict]:
    pairs = [(g["label_key"], g["label_value"]) for g in groups]
    pods = []
    for i in range(n):
        big = rng.random() < big_frac
        p = {"name": "p%d" % i, "owner_kinds": [], "annotations": {}, "node_selector": None, "affinity": None,
             "containers": [_req(rng, big) for _ in range(rng.choice([0, 1, 1, 1, 1, 2, 3]))],
             "init_containers": [_req(rng, big) for _ in range(rng.choice([0, 0, 0, 0, 1, 2]))],
             "overhead": None, "node_name": ""}
        if rng.random() < 0.05:
            p["owner_kinds"] = rng.choice([["DaemonSet"], ["ReplicaSet", "DaemonSet"], ["Job"]])
        if rng.random() < 0.03:
            p["annotations"]["kubernetes.io/config.source"] = rng.choice(["file", "api"])
        if rng.random() < 0.3:
            p["overhead"] = rng.choice([{"cpu": None, "mem": None}, _req(rng, big)])
        r = rng.random()
        if r < 0.2:
            pass                                          # default-group candidate
        elif r < 0.25:
            p["affinity"] = {"node_affinity": None, "pod_affinity": True, "pod_anti_affinity": False}
        else:
            if rng.random() < 0.7:
                sel = {}
                for _ in range(rng.choice([1, 1, 2])):
                    k, v = rng.choice(pairs) if rng.random() < 0.85 else ("zone", "z1")
                    sel[k] = v
                p["node_selector"] = sel
            if rng.random() < 0.4:
                terms = []
                for _ in range(rng.choice([1, 1, 2])):
                    term = []
                    for _ in range(rng.choice([1, 2])):
                        k, v = rng.choice(pairs)
                        vals = [v] + [rng.choice(pairs)[1] for _ in range(rng.randrange(0, 3))]
                        op = "In" if rng.random() < 0.85 else rng.choice(["NotIn", "Exists"])
                        term.append({"key": k, "op": op, "values": vals})
                    terms.append(term)
                req = terms if rng.random() < 0.9 else None
                p["affinity"] = {"node_affinity": {"required": req}, "pod_affinity": rng.random() < 0.1,
                                 "pod_anti_affinity": False}
        pods.append(p)
    return pods


def make_nodes(rng: random.Random, n: int, groups: list[dict], big_frac: float = 0.01) -> list[dict]:
    pairs = [(g["label_key"], g["label_value"]) for g in groups]
    base = 1_700_000_000_000_000_000
    nodes = []
    for i in range(n):
        labels = {}
        for _ in range(rng.choice([0, 1, 1, 1, 2, 3])):
            k, v = rng.choice(pairs) if rng.random() < 0.9 else ("os", "linux")
            labels[k] = v
        cpu = rng.choice([None, 0, 2000, 4000, 16000, 64000])
        mem = rng.choice([None, 0, 8 << 30, 64 << 30, (256 << 30) - 12345])
        if rng.random() < big_frac:
            cpu = rng.choice([(1 << 20) + 5, -5, 1 << 40])
            mem = rng.choice([(1 << 46) + 1, -7])
        taints = []
        if rng.random() < 0.2:
            taints = rng.choice([["atlassian.com/escalator"], ["other"], ["other", "atlassian.com/escalator"]])
        nodes.append({"name": "node-%d" % i, "labels": labels, "unschedulable": rng.random() < 0.08,
                      "taints": taints, "cpu": cpu, "mem": mem,
                      "created_ns": base + rng.randrange(0, max(2, n // 2)) * 1_000})
    return nodes


def make_trackers(rng: random.Random, groups: list[dict], nodes: list[dict]) -> dict:
    out = {}
    for g, spec in enumerate(groups):
        if spec.get("dry_mode"):
            names = [nd["name"] for nd in nodes if rng.random() < 0.2] + ["ghost-node"]
            out[g] = names
    return out


def make_states(rng: random.Random, G: int) -> list[dict]:
    return [{"locked": rng.random() < 0.1, "requested_nodes": rng.randrange(0, 5),
             "cached_cpu_m": rng.choice([0, 4000]), "cached_mem_b": rng.choice([0, 8 << 30])} for _ in range(G)]


def make_reaping_cluster(rng: random.Random, G: int, n_pods: int, n_nodes: int):
    """A cluster for TryRemoveTaintedNodes: escalator taints with valid / unparsable
    values, no-delete annotations, pods bound to listed, unknown and no nodes."""
    groups = make_groups(rng, G, with_default=rng.random() < 0.7)
    pods = make_pods(rng, n_pods, groups, big_frac=0.0)
    nodes = make_nodes(rng, n_nodes, groups, big_frac=0.0)
    now_s = 1_700_000_000
    for nd in nodes:
        if rng.random() < 0.4 and "atlassian.com/escalator" not in nd["taints"]:
            nd["taints"] = nd["taints"] + ["atlassian.com/escalator"]
        nd["taint_value"] = rng.choice([str(now_s - rng.randrange(0, 900)), str(now_s - rng.randrange(0, 900)),
                                        "+%d" % (now_s - 400), "bad", "", "-5", "99999999999999999999", None])
        if rng.random() < 0.1:
            nd["annotations"] = {"atlassian.com/no-delete": rng.choice(["true", ""])}
    for p in pods:
        r = rng.random()
        p["node_name"] = "" if r < 0.1 else ("ghost" if r < 0.15 else rng.choice(nodes)["name"])
    return groups, pods, nodes, now_s * 1_000_000_000
