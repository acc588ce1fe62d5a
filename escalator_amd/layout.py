"""Algorithmic HBM bytes of the streamed snapshot.

K1 reads the pod shard once per decision: per pod flags 4 + cpu0 4 + mem0 8 + pair0 4 B,
16 B per extra container record, 4 B per extra selector pair, and 8 B of record offsets
per 64-pod C tile (the pods that own extra records, placed in their own section at load).
K2 streams per node flags 4 + label0 4 + cpu 8 + mem 8 B, plus 4 B per extra label pair
and 4 B of offset for each node that has extra label pairs.
"""
import numpy as np

XTRA_MASK = 0x3FFFFF10      # ESC_PF_HAS_OVH | extra container counts | extra pair count


def complex_pods(flags: np.ndarray) -> int:
    return int(np.count_nonzero(np.asarray(flags) & XTRA_MASK))


def pod_bytes(flags: np.ndarray, n_xc: int, n_xp: int) -> int:
    n = len(flags)
    c_tiles = (complex_pods(flags) + 63) // 64
    return n * 20 + int(n_xc) * 16 + int(n_xp) * 4 + c_tiles * 8


def node_bytes(n_streamed: int, n_xl: int) -> int:
    return n_streamed * 28 + int(n_xl) * 4
