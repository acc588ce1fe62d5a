"""Algorithmic HBM bytes of the streamed snapshot — an independent
restatement of what ``esc_stream_bytes`` reports, used to cross-check it.

K1 reads the pod shard once per decision: per pod flags 4 + cpu0 4 + mem0 8 + pair0 4 B,
16 B per extra container record, 4 B per extra selector pair, and 8 B of record offsets
per 64-pod C tile (pods with more than 3 extra container records or more than 3 extra
pairs; all other pods sit in homogeneous 256-pod K tiles that need no offsets).  A K pod
whose values fit the packed block (``packed_mask``) takes 12 B (pair0 | flags 4, cpu0 | mem0
8) and 8 B per record; one that also fits the packed small block (``small_mask``) 8 B
(cpu0 | mem0 | pair0 | flags in one u64), 8 B per record and 2 B per extra pair.
K2 reads the node index once per decision: per (label pair, node) entry of a pair some group
selects 16 B when every node's allocatable cpu is in [0, 2^32) (one packed record: flags 4 +
cpu 4 + mem 8), else 20 B (flags 4 + cpu 8 + mem 8), and 8 B per piece (offset + pair).
With several ranks each reads the pieces of the group pairs it owns (``owner_ranges``:
contiguous pair ranges balanced by entry count).
"""
import numpy as np

NODE_PIECE = 1024
PIECE_ALIGN = 256          # esc_kernels.h: no piece crosses a multiple of it (K2's spans come out full)
NONE = 0xFFFFFFFF


def complex_pods(flags: np.ndarray) -> int:
    """Pods outside the homogeneous K classes (more than 3 extra container records or
    more than 3 extra pairs): they go to the 64-pod C tiles."""
    f = np.asarray(flags, np.uint64)
    recs = ((f >> 8) & 0xFF) + ((f >> 16) & 0xFF) + ((f >> 4) & 1)
    return int(np.count_nonzero((recs > 3) | (((f >> 24) & 0x3F) > 3)))


KP_CPU_ABSENT = (1 << 20) - 1      # packed K blocks (esc_kernels.h kp_*): field ranges / sentinels
KP_MEM_ABSENT = (1 << 44) - 1
KP_PAIR_NONE = (1 << 28) - 1
INT64_MIN = -(1 << 63)


def packed_mask(pods: dict) -> np.ndarray:
    """Pods of a K class whose values fit the packed block: cpu0 and every record cpu in
    [0, 2^20 - 1), mem0 and every record mem in [0, 2^44 - 1) (an init container's key may be
    absent, INT64_MIN, instead) and pair0 NONE or < 2^28 - 1."""
    f = np.asarray(pods["flags"], np.uint64)
    nreg, ninit = (f >> 8) & 0xFF, (f >> 16) & 0xFF
    nrec = (nreg + ninit + ((f >> 4) & 1)).astype(np.int64)
    kcls = (nrec <= 3) & (((f >> 24) & 0x3F) <= 3)
    cpu0 = np.asarray(pods["cpu0"], np.int64)
    mem0 = np.asarray(pods["mem0"], np.int64)
    pair0 = np.asarray(pods["pair0"], np.uint32)
    ok = kcls & (cpu0 < KP_CPU_ABSENT) & (mem0 >= 0) & (mem0 < KP_MEM_ABSENT)
    ok &= (pair0 == NONE) | (pair0 < KP_PAIR_NONE)
    n_rec = int(nrec.sum())
    if n_rec:
        xc = np.asarray(pods["xc_cpu"], np.int64)[:n_rec]
        xm = np.asarray(pods["xc_mem"], np.int64)[:n_rec]
        owner = np.repeat(np.arange(len(f), dtype=np.int64), nrec)
        k = np.arange(n_rec, dtype=np.int64) - np.repeat(np.cumsum(nrec) - nrec, nrec)
        init = (k >= nreg.astype(np.int64)[owner]) & (k < (nreg + ninit).astype(np.int64)[owner])
        rc = ((xc >= 0) & (xc < KP_CPU_ABSENT)) | (init & (xc == INT64_MIN))
        rm = ((xm >= 0) & (xm < KP_MEM_ABSENT)) | (init & (xm == INT64_MIN))
        bad = np.bincount(owner[~(rc & rm)], minlength=len(f)) > 0
        ok &= ~bad
    return ok


KP8_CPU_MAX = (1 << 14) - 1       # packed small block (kp8_*): cpu0, mem0 ranges, pair-id field
KP8_MEM_MAX = (1 << 34) - 1
KP8_PAIR_NONE = (1 << 14) - 1


def small_mask(pods: dict, n_gp: int) -> np.ndarray:
    """Packed pods that also fit the packed small block: cpu0 < 2^14, mem0 < 2^34, in a
    context with fewer than 2^14 - 1 group pairs."""
    if n_gp >= KP8_PAIR_NONE:
        return np.zeros(len(pods["flags"]), bool)
    cpu0 = np.asarray(pods["cpu0"], np.int64)
    mem0 = np.asarray(pods["mem0"], np.int64)
    return packed_mask(pods) & (cpu0 <= KP8_CPU_MAX) & (mem0 >= 0) & (mem0 <= KP8_MEM_MAX)


def pod_bytes(pods: dict, n_gp: int, lo: int = 0, hi: int | None = None) -> int:
    """K1's algorithmic bytes for pods [lo, hi) of a snapshot (one shard) in a context with
    n_gp group pairs."""
    f = np.asarray(pods["flags"], np.uint64)
    hi = len(f) if hi is None else hi
    nrec = (((f >> 8) & 0xFF) + ((f >> 16) & 0xFF) + ((f >> 4) & 1)).astype(np.int64)[lo:hi]
    nxp = ((f >> 24) & 0x3F).astype(np.int64)[lo:hi]
    pk = packed_mask(pods)[lo:hi]
    sm = small_mask(pods, n_gp)[lo:hi]
    c_tiles = (complex_pods(f[lo:hi]) + 63) // 64
    plain = (20 + 16 * nrec + 4 * nxp)[~pk].sum()
    packed = (12 + 8 * nrec + 4 * nxp)[pk & ~sm].sum()
    small = (8 + 8 * nrec + 2 * nxp)[sm].sum()
    return int(plain + packed + small + c_tiles * 8)


def node_entries(nodes: dict) -> np.ndarray:
    """Label pair of every (pair, node) entry, in entry (pair-sorted) order."""
    label0 = np.asarray(nodes["label0"], np.uint32)
    pairs = np.concatenate([label0[label0 != NONE], np.asarray(nodes["xl_pair"], np.uint32)])
    return np.sort(pairs, kind="stable")


OWN_PAD = 64          # per-pair weight beside its entries (esc_runtime.hip owned_pairs)


def pair_counts(nodes: dict, n_gp: int) -> np.ndarray:
    """Node entries of every group pair (ids < n_gp)."""
    q = node_entries(nodes)
    return np.bincount(q[q < n_gp].astype(np.int64), minlength=n_gp)[:n_gp]


def owner_ranges(nodes: dict, n_gp: int, world: int) -> list[int]:
    """The owner split of the node side: pair q, weighted by its entries +
    OWN_PAD, goes to rank floor(S_q * world / W) with S_q the weight before q and W the
    total; returns q_bounds (rank r owns pairs [q_bounds[r], q_bounds[r + 1]))."""
    if world <= 1:
        return [0, n_gp]
    w = [int(x) + OWN_PAD for x in pair_counts(nodes, n_gp)]
    W = sum(w)
    owner, S = [], 0
    for x in w:
        owner.append(S * world // W)
        S += x
    bounds = []
    for r in range(world):
        bounds.append(next((q for q, o in enumerate(owner) if o >= r), n_gp))
    return bounds + [n_gp]


def exchange_rows(gpair, bounds: list[int]) -> tuple[np.ndarray, int]:
    """Owner-major rows of the exchanged pod words: the owner of group g is
    the rank whose pair range [bounds[r], bounds[r + 1]) holds gpair[g]; its row is
    owner * cap + its index among the owner's groups (ascending), cap the largest owner's
    group count.  A reduce-scatter of cap * 5 words per rank then hands every owner exactly
    its own groups' sums."""
    gpair = np.asarray(gpair, np.int64)
    world = len(bounds) - 1
    owner = np.searchsorted(np.asarray(bounds[:-1], np.int64), gpair, side="right") - 1 if world > 1 \
        else np.zeros(len(gpair), np.int64)
    counts = np.bincount(owner, minlength=world)
    cap = max(1, int(counts.max()) if len(counts) else 1)
    rows = np.zeros(len(gpair), np.uint32)
    seen = np.zeros(world, np.int64)
    for g, r in enumerate(owner):
        rows[g] = r * cap + seen[r]
        seen[r] += 1
    return rows, cap


def node_bytes(nodes: dict, n_gp: int, rank: int = 0, world: int = 1) -> int:
    q = node_entries(nodes)
    E = len(q)
    if E == 0:
        return 0
    # pieces: runs of one pair's entries cut at every multiple of PIECE_ALIGN entries too
    # (K2's spans come out full, esc_runtime.hip esc_load_nodes), so <= NODE_PIECE long
    assert NODE_PIECE % PIECE_ALIGN == 0
    starts = np.flatnonzero(np.r_[True, q[1:] != q[:-1]])
    p_start = np.union1d(starts, np.arange(0, E, PIECE_ALIGN))
    p_len = np.diff(np.r_[p_start, E])
    p_pair = q[p_start]
    b = owner_ranges(nodes, n_gp, world)
    mine = (p_pair >= b[rank]) & (p_pair < b[rank + 1])
    # K2 reads 16 B per entry when every node's cpu fits the packed record (flags, cpu as u32,
    # memory), else the three arrays' 20 B (esc_runtime.hip esc_load_nodes)
    cpu = np.asarray(nodes["cpu"], np.int64)
    per_entry = 16 if bool(((cpu >= 0) & (cpu <= 0xFFFFFFFF)).all()) else 20
    return int(8 * int(mine.sum()) + per_entry * int(p_len[mine].sum()))


def baseline_md_pod_bytes(pods: dict) -> int:
    """BASELINE.md §2's logical bytes of the pods (see ``baseline_md_bytes``)."""
    f = np.asarray(pods["flags"], np.uint64)
    ctr = 1 + (((f >> 8) & 0xFF) + ((f >> 16) & 0xFF) + ((f >> 4) & 1)).astype(np.int64)
    pairs = (np.asarray(pods["pair0"], np.uint32) != NONE).astype(np.int64) + ((f >> 24) & 0x3F).astype(np.int64)
    return int((12 + 17 * ctr + 4 * pairs).sum())


def baseline_md_node_bytes(nodes: dict) -> int:
    """BASELINE.md §2's logical bytes of the nodes (see ``baseline_md_bytes``)."""
    nf = np.asarray(nodes["flags"], np.uint64)
    labels = (np.asarray(nodes["label0"], np.uint32) != NONE).astype(np.int64) + ((nf >> 8) & 0xFF).astype(np.int64)
    return int((24 + 4 * labels).sum())


def baseline_md_bytes(pods: dict, nodes: dict, n_memb: int = 0) -> dict:
    """The logical bytes of BASELINE.md §2's metric definition over the generated arrays —
    the reference-shaped, uncompressed SoA the north star's "% of HBM" is quoted on:
    per pod 4 (flags) + 4 (ctr_off) + 17 per container (cpu 8, mem 8, kind 1; regular, init
    and the overhead pseudo-container) + 4 (pair_off) + 4 per selector pair; per node 4
    (flags) + 8 + 8 (allocatable) + 4 (label_off) + 4 per carried label pair; 12 B per
    ordered membership (8-B key + 4-B permutation).  The resident format streams fewer bytes
    (``pod_bytes``: packed tiles), so this figure, divided by the decision time, can exceed
    the HBM peak; the physical roofline is ``pod_bytes`` over K1's launch time."""
    pb, nb = baseline_md_pod_bytes(pods), baseline_md_node_bytes(nodes)
    return {"pods": pb, "nodes": nb, "orderings": 12 * int(n_memb), "total": pb + nb + 12 * int(n_memb)}
