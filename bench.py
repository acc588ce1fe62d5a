"""Benchmark: pod+node records evaluated per second per scale decision (BASELINE.json).

One "step" = one complete scale decision over a device-resident synthetic snapshot:
K1 (pods) + K2 (nodes) + K3 combine (+ RCCL exchange when N > 1) + K4 decide + the copy
of every group's decision to pinned host memory.  Default workload: BASELINE config #4
(100M pods / 1M nodes / 10k node groups), sharded over the N GPUs (strong scaling: the
snapshot is fixed, each GPU streams 1/N of it).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4|2|3|5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # BASELINE.md §3 rows
    2: dict(P=1_000_000, N=10_000, G=100, name="config2: 1M pods / 10k nodes / 100 node groups (BASELINE.json configs[1])"),
    3: dict(P=10_000_000, N=100_000, G=100, name="config3: 10M pods / 100k nodes / 100 multi-instance-type groups (configs[2])"),
    4: dict(P=100_000_000, N=1_000_000, G=10_000,
            name="config4: 100M pods / 1M nodes / 10k node groups (BASELINE.json configs[3]), sharded over N GPUs"),
}
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
# rocprofv3 kernel-trace + PMC passes of this same command (scripts/gpu.sh prof:NAME), reduced to
# the timed launches by scripts/prof_summary.py: HBM bytes per K1 launch, by workload
PROF_DIR = os.path.join(ROOT, "profiles", "r06_prof")
PMC_SUMMARY = {(4, 1): os.path.join(PROF_DIR, "summary_full.json"),       # (config, shard-of)
               (4, 8): os.path.join(PROF_DIR, "summary_shard8.json")}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stream_bytes(ctx, s, rank, world) -> tuple[int, int]:
    """Algorithmic bytes K1 / K2 stream per decision on this rank (esc_stream_bytes),
    cross-checked against the independent restatement in escalator_amd/layout.py."""
    from escalator_amd import layout
    from oracle import soa
    pb, nb = ctx.stream_bytes()
    n_gp = len(soa.group_tables(s.groups)["pair_ids"])
    assert pb == layout.pod_bytes(s.pods(), n_gp), "K1 bytes"
    assert nb == layout.node_bytes(s.nodes(), n_gp, rank, world), "K2 bytes"
    return pb, nb


def pmc_traffic(kernel: str, key):
    """HBM bytes per launch of `kernel` over the timed launches, from the committed PMC
    summary of this workload (or None), and that summary's path."""
    path = PMC_SUMMARY.get(key)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError, TypeError):
        return None, None
    return d.get("kernels", {}).get(kernel, {}).get("hbm_bytes"), os.path.relpath(path, ROOT)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """The host cores this process may use: its affinity mask, capped by OMP_NUM_THREADS
    (the GPU box sets 16, its CPU share per GPU)."""
    n = len(os.sched_getaffinity(0))
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def cpu_baseline(cfg, G, full=None, seconds=12.0):
    """CPU baselines on the GPU box's host cores (reported, never the target):
    - B-opt (``value``): the oracle's single-pass SoA totals (orc_totals_par, OpenMP) over
      the whole snapshot ``full`` on every host core this process may use — the honest
      "best CPU" comparator of BASELINE.md §4 (decision math excluded: O(G));
    - reference-shaped: one full rescan per group, single thread like the reference's
      RunOnce (controller.go:416): over the whole snapshot for a spread of groups,
      extrapolated to all groups (round 3 used a 2 M-pod sample and extrapolated twice;
      that remains the fallback when the rank holds no full snapshot)."""
    import numpy as np
    from escalator_amd.context import Synth
    from oracle import soa
    threads = host_threads()
    out = {"unit": "records/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    if full is not None:
        pods, nodes = full.pods(), full.nodes()
        n_rec = len(pods["flags"]) + len(nodes["flags"])
        soa.totals(pods, nodes, full.groups, threads=threads)          # warm the pages
        ts, t0 = [], time.perf_counter()
        while len(ts) < 30 or time.perf_counter() - t0 < 6.0:
            t1 = time.perf_counter()
            soa.totals(pods, nodes, full.groups, threads=threads)
            ts.append(time.perf_counter() - t1)
        dt = float(np.median(ts))
        q1, q3 = np.percentile(ts, [25, 75])
        out["value"] = n_rec / dt
        out["spread"] = [n_rec / max(ts), n_rec / min(ts)]
        out["iqr"] = [float(n_rec / q3), float(n_rec / q1)]
        out["sample"] = ("B-opt: oracle/esc_oracle.c orc_totals_par (single pass over the SoA snapshot, per-thread "
                         "group accumulators, OpenMP) over the full %d-record snapshot on %d threads, median of %d "
                         "passes (iqr: their middle half), %.3f s per decision" % (n_rec, threads, len(ts), dt))
    if full is not None:
        # the whole snapshot, rescanned once per group for a spread of groups (every
        # (G / k)-th), k sized to ~`seconds`: only the group count is extrapolated — the
        # scan's per-record cost depends on the records streamed from DRAM, which a small
        # pod sample (cache-resident on this host) would understate
        pods, nodes, groups = full.pods(), full.nodes(), full.groups
        P_s, N_s = len(pods["flags"]), len(nodes["flags"])
        t0 = time.perf_counter()
        soa.totals(pods, nodes, groups, reference_shaped=True, g_range=(G // 2, G // 2 + 1))
        t1 = time.perf_counter() - t0
        k = int(max(1, min(G, seconds / max(t1, 1e-6))))
        picks = sorted(set(int(i * G // k) for i in range(k)))
        t0 = time.perf_counter()
        for g in picks:
            soa.totals(pods, nodes, groups, reference_shaped=True, g_range=(g, g + 1))
        t_scan = time.perf_counter() - t0
        how = "the full %d-pod / %d-node snapshot, %d of %d groups (every %d-th) timed (%.1f s), extrapolated " \
              "linearly to all groups" % (P_s, N_s, len(picks), G, max(1, G // k), t_scan)
    else:
        P_s, N_s = 2_000_000, 20_000
        s = Synth(P_s, N_s, G, config=cfg["cfg"], seed=0xE5CA1A7E00000000 + cfg["cfg"], threads=16)
        pods, nodes, groups = s.pods(), s.nodes(), s.groups
        t0 = time.perf_counter()
        soa.totals(pods, nodes, groups, reference_shaped=True, g_range=(1, 2))
        t1 = time.perf_counter() - t0
        picks = list(range(1, 1 + int(max(1, min(G - 1, seconds / max(t1, 1e-6))))))
        t0 = time.perf_counter()
        soa.totals(pods, nodes, groups, reference_shaped=True, g_range=(picks[0], picks[-1] + 1))
        t_scan = time.perf_counter() - t0
        how = "a %d-pod / %d-node sample of the same config, %d of %d groups timed (%.1f s), extrapolated linearly " \
              "to the snapshot and to all groups" % (P_s, N_s, len(picks), G, t_scan)
    per_group = t_scan / len(picks)
    t0 = time.perf_counter()
    soa.totals(pods, nodes, groups)
    t_single = time.perf_counter() - t0
    ref = {
        "value": (P_s + N_s) / (per_group * G),
        "cores": 1,
        "sample": ("oracle/esc_oracle.c orc_ref_scan (reference-shaped: every group rescans all pods and nodes, "
                   "controller.go:416 + pod_listers.go:33) over " + how),
        "single_pass_1thread_records_per_s": (P_s + N_s) / t_single,
    }
    out["reference_shaped"] = ref
    if "value" not in out:                  # no full snapshot on this rank: report the scan
        out.update(value=ref["value"], cores=1, sample=ref["sample"])
    return out


PARITY_EXIT = 3                 # exit status of a run whose results differ from the oracle's


def report(out: dict, parity_ok: bool) -> int:
    """Print the bench line; a parity mismatch still prints it (the numbers are evidence)
    but makes the run fail: a wrong decision must never pass as a measurement."""
    print(json.dumps(out), flush=True)
    if not parity_ok:
        log("bench: PARITY MISMATCH against the C oracle: %s" % out.get("parity"))
        return PARITY_EXIT
    return 0


def stage_layout(world: int, shard_world: int, multi, backend: str) -> list[str]:
    """Names of the timing-mode stages enqueue_step / esc_exchange / esc_decide record."""
    names = ["k_pod_reduce", "k_step_tail", "k_order_split", "k_node_groups"]
    if os.environ.get("ESC_NO_ZEROCOPY", "0") not in ("", "0"):
        names.append("d2h")
    if world == 1 and shard_world == 1 and not multi:
        return names                              # K4 inside k_node_groups
    names = names[:3] + names[4:]                 # node groups run with K4, after the exchange
    if multi:                                     # device 0's events; the exchange marks its end
        names.append("exchange")
    elif world > 1:
        names.append("exchange" if backend == "nccl" else "exchange_host_staged")
    return names + ["k_node_groups+decide"]


def rccl_ranks_field(comm_size, multi, world: int, backend: str):
    """The bench line's `rccl_ranks`: ncclCommCount of the live communicators (esc_comm_size),
    None where no RCCL communicator exists — one rank, a gloo run, or a multi-device context on
    its peer exchange (esc_comm_size reports 0 there)."""
    if not (multi or (world > 1 and backend == "nccl")):
        return None
    return comm_size() or None


SEL_SLACK, SEL_CAP = 4, 256     # selections delivered with each decision (esc_set_selections)


def selections_ok(sel, dec, want, owned, slack=SEL_SLACK, cap=SEL_CAP):
    """Every owned group's delivered selection (esc_selections) is the prefix of the oracle's
    order its decision walks: delta < 0 (taint clamp passed) the untainted oldest first,
    n_to_taint + slack of them; delta > 0 the tainted newest first, delta + slack; at most cap
    (then flagged cut).  Returns (ok, groups with a list, nodes delivered)."""
    import numpy as np
    which, off, idx = sel
    ok, n_lists = True, 0
    for g in range(len(which)):
        if not owned[g]:
            continue
        delta, ts = int(dec["delta"][g]), int(dec["taint_status"][g])
        w, need = (1, delta) if delta > 0 else ((0, int(dec["n_to_taint"][g])) if delta < 0 and ts == 0 else (-1, 0))
        got = idx[off[g]:off[g + 1]]
        if w < 0:
            ok &= bool(which[g] == -1 and len(got) == 0)
            continue
        order = want[(g, w)]
        c = min(max(need, 0) + slack, len(order))
        ok &= bool(which[g] & 3 == w and bool(which[g] & 4) == (c > cap) and np.array_equal(got, order[:min(c, cap)]))
        n_lists += 1
    return ok, n_lists, len(idx)


def resident_run_once(ctx, select: bool, reps: int = 30) -> dict:
    """The Go shim's RunOnce on the resident snapshot (go/escalatorhip: esc_set_state +
    esc_step + esc_sync + esc_results of every group + ONE esc_selections into the context's
    persistent buffer, allocated once at its largest here): the wall time a controller scan
    waits for before it walks the selections, median of `reps`."""
    import ctypes as C
    import numpy as np
    from escalator_amd import _lib as L
    from escalator_amd.context import DECISION_DTYPE, TOTALS_DTYPE
    lib, h, G = ctx.lib, ctx.handle, ctx.G
    tot, dec = np.zeros(G, TOTALS_DTYPE), np.zeros(G, DECISION_DTYPE)
    which, off = np.zeros(G, np.int32), np.zeros(G + 1, np.int64)
    idx = np.zeros(G * (SEL_CAP + 1), np.int64)
    tp, dp = tot.ctypes.data_as(C.POINTER(L.GroupTotals)), dec.ctypes.data_as(C.POINTER(L.GroupDecision))
    wp, op, ip = (which.ctypes.data_as(C.POINTER(C.c_int32)), off.ctypes.data_as(C.POINTER(C.c_int64)),
                  idx.ctypes.data_as(C.POINTER(C.c_int64)))
    n = C.c_int64()
    ms = []
    for _ in range(reps):
        t0 = time.perf_counter()
        L.check(lib.esc_set_state(h, ctx._state))
        L.check(lib.esc_step(h))
        L.check(lib.esc_sync(h))
        L.check(lib.esc_results(h, tp, dp))
        if select:
            L.check(lib.esc_selections(h, wp, op, ip, len(idx), C.byref(n)))
        ms.append((time.perf_counter() - t0) * 1e3)
    return {"ms": float(np.median(ms)), "p90_ms": float(np.percentile(ms, 90)), "selections": select,
            "groups_walking": int((which >= 0).sum()) if select else None, "nodes_delivered": int(n.value),
            "how": "esc_set_state + esc_step + esc_sync + esc_results (every group) + one esc_selections into "
                   "a persistent buffer, on the resident snapshot: the Go shim's RunOnce; median of %d" % reps}


def check_parity(args, ctx, s, multi, rank, world, backend, dist, P, N, G, n_gpus):
    """Every group's totals and decision against the C oracle over the whole snapshot (at
    N > 1 the owners' records gathered to every rank, and a second, unsharded generation of
    the config on rank 0), and every group's two orderings on the rank that orders it, against
    the oracle's over the node table every rank holds.  Returns (text, ok) on every rank."""
    import numpy as np
    import torch
    from oracle import soa
    if multi or world == 1:
        tot, dec = ctx.results()
    else:
        from escalator_amd.dist import gather_results
        tot, dec = gather_results(ctx)              # collective: every rank
    ord_ok, n_ord, n_sel = True, 0, 0
    if not args.no_order:
        want = soa.order_all(s.nodes(), s.groups)
        owned = [bool(multi or world == 1 or ctx.group_owner(g) == rank) for g in range(G)]
        for g in range(G):
            if owned[g]:
                n_ord += 1
                for w in (0, 1):
                    ord_ok &= bool(np.array_equal(ctx.group_order(g, w), want[(g, w)]))
        if not args.no_select:                      # the walks' prefixes delivered with the decision
            sok, n_sel, _ = selections_ok(ctx.selections(), dec, want, owned)
            ord_ok &= sok
    tot_ok = True
    if rank == 0:
        from escalator_amd import Synth
        full = s if world == 1 else Synth(P, N, G, config=args.config, seed=0xE5CA1A7E00000000 + args.config,
                                          threads=16)
        otot = soa.totals(full.pods(), full.nodes(), full.groups, threads=16)
        odf, odi = soa.decide(full.groups, full.states, otot)
        tot_ok = all(np.array_equal(tot[n], otot[:, k]) for k, n in enumerate(soa.TOT_FIELDS[:12]))
        tot_ok &= np.array_equal(dec["cpu_pct"].view(np.uint64), odf[:, 0].view(np.uint64))
        tot_ok &= np.array_equal(dec["mem_pct"].view(np.uint64), odf[:, 1].view(np.uint64))
        for k, n in enumerate(["delta", "n_to_taint", "cached_cpu_m", "cached_mem_b", "status", "branch",
                               "taint_status"]):
            tot_ok &= np.array_equal(dec[n].astype(np.int64), odi[:, k])
    if dist is not None:                            # the verdict of every rank's checks
        v = torch.tensor([int(ord_ok and tot_ok), n_ord, n_sel], dtype=torch.int64,
                         device="cuda" if backend == "nccl" else "cpu")
        ok_t = v[:1].clone()
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        dist.all_reduce(v[1:], op=dist.ReduceOp.SUM)
        ok, n_ord, n_sel = bool(ok_t.item()), int(v[1].item()), int(v[2].item())
    else:
        ok = bool(ord_ok and tot_ok)
    text = ("bit-exact vs C oracle: all %d groups' totals and decisions%s%s%s" % (
            G, "" if args.no_order else ", all %d groups' two orderings" % n_ord,
            "" if args.no_order or args.no_select else ", the %d taint / untaint selections delivered with the "
                                                       "decision" % n_sel,
            "" if n_gpus == 1 else " (the owners' records over %d ranks gathered; oracle over the unsharded "
                                   "snapshot)" % n_gpus)
            if ok else "MISMATCH vs C oracle")
    return text, ok


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker_command(argv: list[str], n: int, port: int) -> list[str]:
    """The launch of `n` ranks of this script (one process per GPU, RANK / WORLD_SIZE /
    LOCAL_RANK / MASTER_* in their env), the shape the driver uses for its N > 1 runs."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def needs_launch(gpus: int, single_process: bool, env=None) -> bool:
    """`--gpus N` (N > 1) run without a launcher: this process must start the N ranks itself
    (the one-process-per-GPU shape), unless --single-process drives the devices from here."""
    env = os.environ if env is None else env
    return gpus > 1 and not single_process and "WORLD_SIZE" not in env


def launch_workers(argv: list[str], n: int) -> int:
    """Start the N ranks as child processes (nothing in this process has touched the GPU:
    torch is not imported yet) and return their launcher's exit code."""
    import subprocess
    cmd = worker_command(argv, n, _free_port())
    log("bench: --gpus %d without a launcher: starting %d ranks (%s)" % (n, n, " ".join(cmd[1:8])))
    return subprocess.call(cmd)


def check_world(gpus: int, world: int, single_process: bool) -> None:
    """Fail loudly when the ranks running do not match --gpus (a run would otherwise print
    another N's numbers under this N)."""
    if single_process:
        return
    if world != gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d ranks are running" % (gpus, world))


def init_dist(gpus: int = 1):
    """RANK / WORLD_SIZE / LOCAL_RANK from the launcher; one process per GPU over RCCL.
    ESC_BENCH_BACKEND / ESC_BENCH_DEVICE: rehearsal knobs (gloo, every rank on one device)
    for exercising the N > 1 path on a one-GPU box; the driver's runs use the defaults."""
    import torch
    rank, world, local = (int(os.environ.get(k, d)) for k, d in (("RANK", 0), ("WORLD_SIZE", 1), ("LOCAL_RANK", 0)))
    check_world(gpus, world, False)
    backend = os.environ.get("ESC_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("ESC_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local, dist, backend


def bench_order(args):
    """BASELINE config #5: the scale-down / scale-up orderings over 10M nodes (taintOldestN
    scale_down.go:171, untaintNewestN scale_up.go:118).  Times (a) the per-decision ordering
    (esc_sort_nodes: classify every membership, stable 3-way split by class inside each
    group's run) and (b) the age-index build it relies on (esc_build_age_index: LSD radix
    sort of the creation times + the memberships in age order, once per snapshot).  On N
    GPUs every rank orders its contiguous 1/N of the nodes (strong scaling); the taint /
    untaint selections are the k-way merge of the ranks' per-group prefixes
    (escalator_amd.dist.gather_orders, one all_gather), parity-checked against the
    whole-snapshot order."""
    import numpy as np
    import torch
    import escalator_amd as esc
    from escalator_amd.dist import gather_orders, shard_range
    from oracle import soa
    rank, world, local, dist, backend = init_dist(args.gpus)
    N, G, P = 10_000_000, 100, 100_000
    lo, hi = shard_range(P, rank, world)
    s = esc.Synth(P, N, G, config=5, seed=0xE5CA1A7E00000005, p_lo=lo, p_hi=hi, threads=16)
    ctx = esc.Context(s, device=local, rank=rank, world=world)
    ctx.load_synth(s, pod_offset=lo)          # every rank orders the groups whose pairs it owns

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(fn, k):
        for _ in range(args.warmup):
            fn()
        ctx.sync()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        ctx.sync()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if dist is not None:                      # max over ranks
            e = torch.tensor([el], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el / k * 1e3

    def cold(fn, k):
        """Per-decision device time with the Infinity Cache flushed before each one: the
        ordering's working set (~130 MB of region words and orders) fits the 256 MB MALL, so
        back-to-back decisions would be MALL-served.  A 1 GiB write on the context's stream
        evicts it, then HIP events bracket the ordering kernels alone; mean over k."""
        ctx.sync()
        stream = torch.cuda.Stream()                  # a real stream (the default one's handle is 0)
        ctx.set_stream(stream.cuda_stream)
        scrub = torch.empty(1 << 28, dtype=torch.int32, device="cuda")
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        with torch.cuda.stream(stream):
            for a, b in ev:
                scrub.fill_(1)
                a.record(stream)
                fn()
                b.record(stream)
        stream.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        del scrub
        ctx.set_stream(None)
        if dist is not None:                      # max over ranks
            e = torch.tensor([ms], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            ms = float(e.item())
        return ms

    warm_ms = timed(ctx.sort_nodes, args.steps)
    order_ms = cold(ctx.sort_nodes, args.steps)
    index_ms = timed(ctx.build_age_index, max(3, args.steps // 4))
    ctx.sort_nodes()
    n_memb, R = ctx.order_info()
    nodes = s.nodes()
    if world == 1:
        want = soa.order_all(nodes, s.groups)
        counts = [len(ctx.group_order(g, w)) for g in range(G) for w in (0, 1)]
        parity = all(np.array_equal(ctx.group_order(g, w), want[(g, w)]) for g in range(G) for w in (0, 1))
        how = "bit-exact vs C oracle: all %d groups, both orders" % G
        sel_ms = None
    else:
        dev = torch.device("cuda", local) if backend == "nccl" else None
        tot = torch.tensor([n_memb], dtype=torch.int64, device=dev if dev is not None else "cpu")
        dist.all_reduce(tot)
        n_memb = int(tot.item())
        n_sel = 64
        t0 = time.perf_counter()
        merged = {w: gather_orders(ctx, w, n_sel, nodes["created_ns"], device=dev) for w in (0, 1)}
        sel_ms = (time.perf_counter() - t0) * 1e3
        counts = [len(merged[w][g]) for g in range(G) for w in (0, 1)]
        parity = all(np.array_equal(merged[w][g], soa.order(nodes, s.groups, g, w, cap=n_sel)) for g in range(G)
                     for w in (0, 1))
        how = ("merged first %d per group (all_gather of the ranks' prefixes) bit-exact vs the C oracle's "
               "whole-snapshot order: all %d groups, both orders" % (n_sel, G))
    if rank != 0:
        dist.destroy_process_group()
        return 0 if parity else PARITY_EXIT
    if world != args.gpus:
        raise SystemExit("bench: n_gpus %d != --gpus %d" % (world, args.gpus))
    # bytes per membership: SURVEY.md §8(d) prices an ordering at the 8-B key and the 4-B node
    # index, 12 B.  The resident layout moves 8 B: one 4-B region word (node | flags << 28:
    # the key's order is the region's, the group implied by the region) read once by the
    # one-pass split (k_ord_split / k_ord_packed), and the node written (cordoned nodes feed
    # neither order, so 8 B is an upper bound).  The roofline's frac is on the 8 B moved (a
    # physical fraction of the HBM peak); frac_8d on §8(d)'s 12 B.
    order_bytes = n_memb * 12
    moved_bytes = n_memb * 8
    # the index build: node table read twice (count: flags, label 8 B; list: flags, label,
    # created 16 B), each membership written once (12 B: 8-B key, 4-B node | flags value),
    # LSD passes of <= 8 bits over the (group << R | creation offset) keys (hist: 8 B read;
    # scatter: 12 B read + 12 B written), the last pass writing the regions instead (12 B)
    gbits = max(1, (G - 1).bit_length())
    coarse = gbits <= 16                          # build_age_index: 32-bit coarse keys
    if coarse:
        # 8-B (key, value) pairs, four 8-bit passes (hist 4 B read; scatter 8 B read + 8 B
        # written; the last pass 8 B read + 8 B region words + 4 B sorted keys), the run
        # fix-up reading the keys once
        idx_passes = 4
        index_bytes = N * 24 + n_memb * (8 + 3 * 20 + (4 + 20) + 4)
    else:
        idx_passes = -(-(R + gbits) // 8)
        index_bytes = N * 24 + n_memb * (12 + idx_passes * 32)
    out = {
        "metric": "config5 node orderings: memberships ordered/sec per decision (taint/untaint selection)",
        "value": n_memb / (order_ms * 1e-3),
        "unit": "memberships/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": order_ms,
        "higher_is_better": True,
        "scaling": "strong",
        "dtype": "int64 keys",
        "data": "synthetic (esc_synth.cpp config 5: 10M nodes, 100 groups, unique ns creation times)",
        "config": {"workload": "config5: 10M nodes oldest-first / newest-first orderings, 100 node groups",
                   "nodes": N, "node_groups": G, "memberships": n_memb, "parallelism": "shard%d" % world},
        "roofline": {"bound": "hbm", "kernel": "per-decision ordering (k_ord_split + k_ord_packed)",
                     "bytes_moved_per_decision": moved_bytes,
                     "achieved": moved_bytes / (order_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                     "frac": moved_bytes / (order_ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                     "frac_8d": order_bytes / (order_ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                     "bytes_per_decision": moved_bytes,
                     "bytes_8d_per_decision": order_bytes,
                     "bytes_note": "the kernels move 8 B per membership (4-B region word read once, <= 4-B node "
                                   "written); SURVEY.md §8(d) prices 12 B (8-B key + 4-B index): frac_8d",
                     "timing": "cold: the Infinity Cache flushed (1 GiB write) before every decision, HIP events "
                               "around the ordering kernels alone",
                     "warm_ms": warm_ms, "frac_warm": moved_bytes / (warm_ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                     "warm_note": "back-to-back decisions; the ~130 MB working set may be served from the MALL"},
        "age_index_build": {"ms": index_ms, "nodes_per_s": N / (index_ms * 1e-3), "creation_offset_bits": R,
                            "keys": ("32-bit coarse (group | top time bits) + exact fix-up of equal-key runs"
                                     if coarse else "64-bit exact (group << R | offset)"),
                            "lsd_passes": idx_passes, "GBps_moved": index_bytes / (index_ms * 1e-3) / 1e9},
        "selection_merge_ms": sel_ms,
        "segments_nonempty": int(sum(1 for c in counts if c)),
        "parity": how if parity else "MISMATCH vs C oracle",
    }
    if dist is not None:
        dist.destroy_process_group()
    return report(out, parity)


def host_side(esc, ctx_dev, device: int):
    """BASELINE.md §2's host-side figures: the K0 packer over object structs (esc_synth_objects:
    what the cgo shim fills from *v1.Pod / *v1.Node) of BASELINE config #2, in objects/s on
    one host thread; and the per-call drop-in esc_pods_requests_total (pkg/k8s/util.go:27:
    the slice's records into reused pinned buffers, one kernel reading them zero-copy, the
    exact sums back) over config #1's 1000 pod objects, beside the single-thread C oracle
    (orc_totals) over the same pods' SoA."""
    import ctypes as C
    import numpy as np
    from escalator_amd import _lib as L
    from oracle import soa
    from escalator_amd.context import TOTALS_DTYPE
    s = esc.Synth(1_000_000, 10_000, 100, config=2, seed=0xE5CA1A7E00000002, threads=16)
    po, n, no, nn = s.objects()
    host = esc.Context(s.groups, device=-1)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        host.pack_objects(po, n, no, nn)
        times.append(time.perf_counter() - t0)
    t_pack = float(np.median(times))
    c1 = esc.Synth(1000, 50, 1, config=1, seed=0xE5CA1A7E00000001)
    pa, na, o1, m1 = c1.objects()
    # what scaleNodeGroup hands CalculatePodsRequestsTotal: the group's filtered pods
    # (controller.go:194, :262): not a daemonset, and the group's pair among the pod's pairs
    sp = c1.pods()
    f = sp["flags"].astype(np.int64)
    nxp = (f >> 24) & 0x3F
    xo = np.concatenate([[0], np.cumsum(nxp)])
    sel = [i for i in range(na) if not (f[i] & 1) and (sp["pair0"][i] == 0 or
                                                       0 in sp["xp_pair"][xo[i]:xo[i + 1]])]
    p1 = (L.PodObj * max(len(sel), 1))()
    for j, i in enumerate(sel):
        p1[j] = pa[i]
    n1 = len(sel)
    mem, cpu = C.c_int64(), C.c_int64()
    lib = ctx_dev.lib
    L.check(lib.esc_pods_requests_total(ctx_dev.handle, p1, n1, C.byref(mem), C.byref(cpu)))   # warm
    calls = []
    for _ in range(200):
        t0 = time.perf_counter()
        L.check(lib.esc_pods_requests_total(ctx_dev.handle, p1, n1, C.byref(mem), C.byref(cpu)))
        calls.append(time.perf_counter() - t0)
    ncalls = []
    for _ in range(200):
        t0 = time.perf_counter()
        L.check(lib.esc_nodes_capacity_total(ctx_dev.handle, o1, m1, C.byref(mem), C.byref(cpu)))
        ncalls.append(time.perf_counter() - t0)
    fn = soa.totals_fn(c1.pods(), c1.nodes(), c1.groups)
    fn()
    reps, t0 = 2000, time.perf_counter()
    for _ in range(reps):
        fn()
    t_orc = (time.perf_counter() - t0) / reps
    want = fn()[0]
    L.check(lib.esc_pods_requests_total(ctx_dev.handle, p1, n1, C.byref(mem), C.byref(cpu)))
    assert int(want[2]) == n1, "config #1 filter restatement"
    # the controller wiring's answer: config #1 resident on the device, one
    # batched decision (RunOnce: esc_set_state + esc_step + esc_sync + esc_results), then the
    # group's CalculatePodsRequestsTotal read from esc_results' totals
    r1 = esc.Context(c1, device=device)
    r1.load_synth(c1)
    r1.set_state(c1.states)
    r1.step()
    r1.sync()
    tot = np.zeros(1, TOTALS_DTYPE)
    tptr = tot.ctypes.data_as(C.POINTER(L.GroupTotals))
    runs, answers = [], []
    for _ in range(200):
        t0 = time.perf_counter()
        L.check(lib.esc_set_state(r1.handle, r1._state))
        L.check(lib.esc_step(r1.handle))
        L.check(lib.esc_sync(r1.handle))
        L.check(lib.esc_results(r1.handle, tptr, None))
        runs.append(time.perf_counter() - t0)
    for _ in range(200):
        t0 = time.perf_counter()
        L.check(lib.esc_results(r1.handle, tptr, None))
        answers.append(time.perf_counter() - t0)
    resident_ok = bool(int(tot["pod_cpu_m"][0]) == int(want[0]) and int(tot["pod_mem_b"][0]) == int(want[1]))
    return {"packer_objects_per_s": (n + nn) / t_pack,
            "packer_sample": "esc_packer_add_pods + _add_nodes + _view over config #2's %d pod and %d node "
                             "objects (esc_synth_objects), one host thread, median of 3: %.3f s" % (n, nn, t_pack),
            "dropin_pods_requests_total_ms": float(np.median(calls)) * 1e3,
            "dropin_pods_requests_total_p90_ms": float(np.percentile(calls, 90)) * 1e3,
            "dropin_nodes_capacity_total_ms": float(np.median(ncalls)) * 1e3,
            "dropin_oracle_1thread_ms": t_orc * 1e3,
            "dropin_parity": bool(cpu.value == want[0] and mem.value == want[1]),
            "resident_pods_requests_total_ms": float(np.median(answers)) * 1e3,
            "resident_run_once_ms": float(np.median(runs)) * 1e3,
            "resident_parity": resident_ok,
            "resident_sample": "config #1 resident (1000 pods, 50 nodes, 1 group): the controller wiring answers "
                               "CalculatePodsRequestsTotal from the batched decision's totals (Decision."
                               "PodsRequestsTotal in the Go shim); resident_pods_requests_total_ms = one "
                               "esc_results(totals) after the decision (the pod and node words to pinned memory, "
                               "one wait), resident_run_once_ms = the whole RunOnce (esc_set_state + esc_step + "
                               "esc_sync + esc_results), medians of 200",
            "dropin_sample": "config #1 (1000 pods, 50 nodes, 1 group): esc_pods_requests_total over the group's "
                             "%d filtered pod objects (what scaleNodeGroup passes, controller.go:262) / "
                             "esc_nodes_capacity_total over the 50 nodes per call (records into reused "
                             "pinned buffers, one k_list_sum launch reading them zero-copy, sums back), median of "
                             "200 calls; oracle: orc_totals over the same pods' SoA on one thread (every group's "
                             "totals, arguments marshalled once), mean of %d calls" % (n1, reps)}


def upload_ms(s, device):
    """Host -> device copy of the snapshot's SoA arrays (pageable numpy memory, the form a
    host packs into), through torch on the device: what one decision would add if the
    snapshot were not resident ('including H2D upload')."""
    import numpy as np
    import torch
    arrs = [a for d in (s.pods(), s.nodes()) for a in d.values() if a.size]
    total = sum(a.nbytes for a in arrs)
    buf = torch.empty(total, dtype=torch.uint8, device=device)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        off = 0
        for a in arrs:
            buf[off:off + a.nbytes].copy_(torch.from_numpy(a.view(np.uint8)), non_blocking=False)
            off += a.nbytes
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    del buf
    return float(np.median(ts)) * 1e3, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=4, choices=sorted(CONFIGS) + [5])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-side packer / upload figures")
    ap.add_argument("--pods", type=int, default=None, help="override the config's pod count (experiments)")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step from a captured hipGraph (default: enqueue its three kernels directly; "
                         "a graph launch left ~8 us idle between back-to-back decisions, profiles/r02_v10)")
    ap.add_argument("--shard-of", type=int, default=1, metavar="W",
                    help="at N=1: run rank 0's shard of a W-GPU job (1/W of the pods, the node side of the pairs "
                         "rank 0 owns) with no exchange -- the per-rank device time of an N=W run (no parity check)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives --gpus devices through ONE multi-device context (esc_ctx_create_multi: "
                         "the Go host's drop-in shape; ESC_BENCH_DEVICES=0,0 rehearses it on one GPU)")
    ap.add_argument("--no-order", action="store_true",
                    help="leave the K5 ordering out of the decision (ablation; BASELINE.md §2 includes it)")
    ap.add_argument("--no-select", action="store_true",
                    help="do not deliver the taint / untaint selections with the decision (ablation)")
    ap.add_argument("--launch-check", action="store_true",
                    help="print this rank's RANK / WORLD_SIZE and exit before any GPU call (tests the launch)")
    args = ap.parse_args()

    if needs_launch(args.gpus, args.single_process):
        return launch_workers(sys.argv[1:], args.gpus)
    if args.launch_check:
        rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
        check_world(args.gpus, world, args.single_process)
        print(json.dumps({"rank": rank, "world": world, "local_rank": int(os.environ.get("LOCAL_RANK", 0))}),
              flush=True)
        return 0
    if args.config == 5:
        return bench_order(args)
    cfg = dict(CONFIGS[args.config], cfg=args.config)
    if args.pods:
        cfg["P"] = args.pods
        cfg["name"] += " [pods overridden: %d]" % args.pods
    P, N, G = cfg["P"], cfg["N"], cfg["G"]

    import numpy as np
    import torch
    import escalator_amd as esc
    from escalator_amd.dist import Exchange, shard_range

    multi = None
    if args.single_process and args.gpus > 1:
        env = os.environ.get("ESC_BENCH_DEVICES")
        multi = [int(x) for x in env.split(",")] if env else list(range(args.gpus))
        rank, world, local, dist, backend = 0, 1, multi[0], None, "multi"
        torch.cuda.set_device(local)
    else:
        rank, world, local, dist, backend = init_dist(args.gpus)
    n_gpus = len(multi) if multi else world

    lo, hi = shard_range(P, rank, world)
    shard_rank, shard_world = rank, world
    if world == 1 and args.shard_of > 1 and not multi:
        lo, hi = shard_range(P, 0, args.shard_of)
        shard_rank, shard_world = 0, args.shard_of
        cfg["name"] += " [rank 0 of %d, no exchange]" % args.shard_of
        args.no_parity = True
    t0 = time.time()
    s = esc.Synth(P, N, G, config=args.config, seed=0xE5CA1A7E00000000 + args.config, p_lo=lo, p_hi=hi, threads=16)
    from escalator_amd import layout
    from oracle import soa as _soa
    shard_bytes = layout.pod_bytes(s.pods(), len(_soa.group_tables(s.groups)["pair_ids"])) // (len(multi) if multi else 1)
    replicas = int(max(1, min(8, -(-1_000_000_000 // max(shard_bytes, 1)))))   # >= 1 GB resident: HBM-served
    if multi:
        ctx = esc.Context(s, devices=multi)
    else:
        ctx = esc.Context(s, device=local, rank=shard_rank, world=shard_world)
    t_load = time.perf_counter()
    ctx.load_synth(s, pod_offset=lo, replicas=replicas)
    load_ms = (time.perf_counter() - t_load) * 1e3
    ctx.set_state(s.states)
    ctx.set_order_in_step(not args.no_order)          # oldest-first ordering is part of a decision
    args.no_select = args.no_select or args.no_order
    if not args.no_select:                            # and the walks' first nodes go out with it
        ctx.set_selections(SEL_SLACK, SEL_CAP)
    n_memb = ctx.order_info()[0]
    if multi:
        pod_b, node_b = ctx.stream_bytes()            # every device's shard
    else:
        pod_b, node_b = stream_bytes(ctx, s, shard_rank, shard_world)
    log("rank %d: shard pods [%d,%d), %.1f MB x %d replicas, setup %.1fs" %
        (rank, lo, hi, shard_bytes / 1e6, replicas, time.time() - t0))

    exchange = None
    if multi:
        step = ctx.step
        exchange = "rccl (esc_ctx_create_multi: ncclCommInitAll, one in-place ncclReduceScatter per device in a group call)" \
            if len(set(multi)) == len(multi) and os.environ.get("ESC_EXCHANGE") != "peer" else \
            "peer (esc_ctx_create_multi: every device sums the others' words over peer-mapped memory)"
    elif world == 1 and shard_world > 1:
        def step():                        # rank 0's device work of an N-GPU step, without the SUM
            ctx.reduce()
            ctx.decide()
    elif world == 1:
        step = ctx.run
    else:
        ex = Exchange(ctx, device_collective=backend == "nccl")
        step = ex.step
        exchange = ("rccl (esc_comm_init + esc_step: in-place ncclReduceScatter on the context's stream)" if backend == "nccl"
                    else "host-staged over torch.distributed %s" % backend)
    ctx.use_graph(args.graph)
    rccl_ranks = rccl_ranks_field(ctx.comm_size, multi, world, backend)
    ctx.k1_calibrate(16)                          # K1 shares to this device's rates (untimed, once per load)
    fe, ff = ctx.k1_flush_entries()
    k1_partials = {"entries": fe, "whole_row_entries": ff, "bytes": fe * 512,
                   "note": "512-B pod-slot column partials K1 writes and K3 reads per decision (compact flush: "
                           "only the columns a workgroup's share touches, DESIGN.md §4)"}

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    ms_per_step = elapsed / args.steps * 1e3

    # Per-kernel device time of K1 (the dominant kernel), HIP events on the context's stream
    # (a multi-device context: device 0's).
    kp = min(args.steps, 10)
    ctx.set_timing(True)
    k1 = []
    stages = []
    for _ in range(kp):
        step()
        ctx.sync()
        st = ctx.stage_times()
        k1.append(st[0])
        stages.append(st)
    ctx.set_timing(False)
    k1_stage_ms = float(np.mean(k1))
    # the roofline's K1 time: back-to-back K1 launches between two HIP events on the
    # context's stream (esc_k1_time) -- the stage events above add their own gap to a short
    # kernel (0.83x rocprof's duration at a rank's shard with them)
    k1_ms = ctx.k1_time(50)
    # stages in timing mode: K1, the fused tail (fold + node pieces + packed small-group
    # orderings), the remaining ordering kernels, node groups (+ K4 at one rank), then at
    # world > 1 the exchange (ncclReduceScatter of the pod words, esc_exchange) and K4 over
    # the rank's own groups (esc_decide); [9] = the whole step
    stage_names = stage_layout(world, shard_world, multi, backend)
    stage_mean = np.mean(np.array(stages), axis=0)
    stage_ms = {k: float(v) for k, v in zip(stage_names, stage_mean) if v > 0}
    stage_ms["step_events"] = float(stage_mean[9])

    # BASELINE.md §2 logical bytes: this rank's pods (every pod for a multi-device context),
    # its ordered memberships (the groups it owns) -- summed over the ranks -- and the node
    # table once
    from escalator_amd import layout as _layout
    md = np.array([_layout.baseline_md_pod_bytes(s.pods()), 0 if args.no_order else n_memb], np.int64)
    if dist is not None:
        tmd = torch.from_numpy(md).to("cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(tmd)
        md = tmd.cpu().numpy()

    parity, parity_ok = None, True
    if not args.no_parity:
        parity, parity_ok = check_parity(args, ctx, s, multi, rank, world, backend, dist, P, N, G, n_gpus)

    run_once = resident_run_once(ctx, not args.no_select) if world == 1 and shard_world == 1 and not multi else None

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return 0 if parity_ok else PARITY_EXIT

    # K1's algorithmic bytes per launch on device 0 (its share of the pods)
    algo = pod_b // (len(multi) if multi else 1)
    achieved = algo / (k1_ms * 1e-3) / 1e9
    records = P + N
    value = records * args.steps / elapsed
    # shards are near-equal: rank 0's bytes x N (pods, the node index, the orderings); a
    # multi-device context reports every device's bytes already
    decision_bytes = (pod_b + node_b + (0 if args.no_order else n_memb * 16)) * (1 if multi else world)
    # PMC passes are taken on the single-GPU config-4 run (scripts/pmc_job.sh); a shard's
    # K1 launch moves other bytes, so the committed figure applies to N = 1 only
    traffic, traffic_src = (pmc_traffic("k_pod_reduce", (args.config, shard_world))
                            if n_gpus == 1 and not args.pods else (None, None))
    # BASELINE.md §2's definition of the metric's bytes (the uncompressed reference-shaped
    # SoA; the north star's "% of aggregate HBM" is quoted on it), beside the physical frac
    nmd = _layout.baseline_md_node_bytes(s.nodes())
    bmd = {"pods": int(md[0]), "nodes": nmd, "orderings": 12 * int(md[1]), "total": int(md[0]) + nmd + 12 * int(md[1])}
    frac_md = bmd["total"] / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9 * n_gpus)
    probe = ctx.hbm_probe() if n_gpus == 1 else None
    out = {
        "metric": "pod+node records evaluated/sec per scale decision & % HBM peak, 1/2/4/8 GPUs",
        "value": value,
        "unit": "records/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (deterministic counter-hash generator, escalator_amd/csrc/esc_synth.cpp)",
        "config": {"workload": cfg["name"], "pods": P, "nodes": N, "node_groups": G,
                   "parallelism": ("single-process x%d" % n_gpus) if multi else "shard%d" % world,
                   "replicas_rotated": replicas},
        "hbm_frac_decision": decision_bytes / (ms_per_step * 1e-3) / (HBM_PEAK_GBS * 1e9 * n_gpus),
        "roofline": {"bound": "hbm", "kernel": "k_pod_reduce", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src if traffic else None,
                     "algorithmic_bytes_per_launch": algo, "launch_ms": k1_ms,
                     "launch_ms_how": "esc_k1_time: 50 back-to-back K1 launches between two HIP events",
                     "launch_ms_stage_events": k1_stage_ms,
                     "box_read_ceiling_GBps": probe,
                     "frac_of_box_ceiling": achieved / probe if probe else None},
        "frac_baseline_md": frac_md,
        "baseline_md_bytes": dict(bmd, note="BASELINE.md §2 logical bytes (uncompressed reference-shaped SoA: 33 B/pod "
                                            "at C=S=1, 24 + 4 L B/node, 12 B per ordered membership) over the generated "
                                            "arrays, all ranks; frac_baseline_md = total / ms_per_step / (n_gpus x 8 TB/s) "
                                            "(> 1 possible: the resident format is packed, see roofline for the physical "
                                            "bytes)"),
        "k1_partials": k1_partials,
        # this rank's (device 0's) algorithmic bytes per step: K1's pod blocks, K2's node
        # entries, 12 B per ordered membership (the region and group words read, the node
        # written) -- what scripts/prof_summary.py sets the step's PMC traffic against
        "step_bytes": {"pods": int(algo), "nodes": int(node_b // (len(multi) if multi else 1)),
                       "orderings": 0 if args.no_order else int(12 * n_memb // (len(multi) if multi else 1)),
                       "total": int(algo + node_b // (len(multi) if multi else 1) +
                                    (0 if args.no_order else 12 * n_memb // (len(multi) if multi else 1)))},
        "node_bytes_per_decision": node_b,
        "exchange": exchange,
        "rccl_ranks": rccl_ranks,
        # stages timed in order on the context's stream (timing mode, rank 0 / device 0)
        "stage_ms": stage_ms,
        "exchange_ms": (stage_ms.get("exchange", stage_ms.get("exchange_host_staged")) if stage_ms else None),
        "stage_note": ("HIP events between the step's launches, timing mode (each event pair adds a few us); "
                       "k_order_split launches nothing when every group is packed into the tail (config 4); "
                       "exchange = the in-place ncclReduceScatter of the owner-major pod words (DESIGN.md §7), "
                       "k_node_groups+decide = the rank's own groups' node words and K4, after the exchange"),
        "ordering": None if args.no_order else {
            "kernels": "groups of <= 1024 memberships packed as blocks of k_step_tail (one pass); mid-size groups by k_ord_packed, larger ones by k_ord_split (one pass, look-back over the group's chunks) after it; all on the context's one stream (esc_set_order_in_step)",
            "memberships": n_memb, "algorithmic_bytes": n_memb * 16},
        "selections": None if args.no_select else {
            "slack": SEL_SLACK, "group_cap": SEL_CAP,
            "note": "every decided group's taint / untaint walk prefix (n_to_taint or delta + slack nodes of its "
                    "order) written by K4 to pinned host memory inside the step (esc_set_selections)"},
        "run_once": run_once,
        "parity": parity,
    }
    if not args.no_host and n_gpus == 1 and shard_world == 1:
        up_ms, up_bytes = upload_ms(s, torch.device("cuda", local))
        out["snapshot_load"] = {"esc_load_ms": load_ms, "h2d_ms": up_ms, "h2d_bytes": up_bytes,
                                "ms_per_step_with_h2d": ms_per_step + up_ms,
                                "note": "esc_load_ms: esc_load_pods + esc_load_nodes (host layout, the H2D copies of "
                                        "every replica, the age index), once per snapshot; h2d_ms: the SoA's "
                                        "pageable host -> HBM copy alone, what a non-resident decision would add"}
        out["host_side"] = host_side(esc, ctx, local)
    if world == 1 and shard_world == 1 and not multi and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, G, full=s)
    if n_gpus != args.gpus or (rccl_ranks is not None and rccl_ranks != args.gpus):
        raise SystemExit("bench: n_gpus %d / rccl_ranks %s != --gpus %d" % (n_gpus, rccl_ranks, args.gpus))
    if dist is not None:
        dist.destroy_process_group()
    return report(out, parity_ok)


if __name__ == "__main__":
    sys.exit(main())
