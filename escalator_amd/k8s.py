"""Mirror of the reference's ``pkg/k8s`` resource arithmetic over the GPU path.

Same names, argument meaning and return order as the Go functions; each call packs the
given slice (list mode: no filter, as the Go functions take an already-filtered slice)
and runs the batched HIP kernels on it.
"""
from __future__ import annotations

import ctypes as C

from . import _lib as L
from .objects import nodes_to_c, pods_to_c

_ctx = {}


def _device_ctx(device: int = 0):
    """A one-group context per device that owns the drop-ins' list contexts."""
    if device not in _ctx:
        from .context import Context
        _ctx[device] = Context([{"name": "drop-in", "label_key": "\x01", "label_value": "\x01"}], device=device)
    return _ctx[device]


def calculate_pods_requests_total(pods: list[dict], device: int = 0) -> tuple[int, int]:
    """CalculatePodsRequestsTotal — pkg/k8s/util.go:27.  Returns (memory bytes, cpu millicores).

    Raises OverflowError where the reference's Quantity would leave int64 (inf.Dec)."""
    ctx = _device_ctx(device)
    arr, n, keep = pods_to_c(pods)
    mem, cpu = C.c_int64(), C.c_int64()
    rc = ctx.lib.esc_pods_requests_total(ctx.handle, arr, n, C.byref(mem), C.byref(cpu))
    if rc == L.ESC_E_LIMIT:
        raise OverflowError("pod requests total left int64")
    L.check(rc, "esc_pods_requests_total")
    del keep
    return mem.value, cpu.value


def calculate_nodes_capacity_total(nodes: list[dict], device: int = 0) -> tuple[int, int]:
    """CalculateNodesCapacityTotal — pkg/k8s/util.go:41.  Returns (memory bytes, cpu millicores)."""
    ctx = _device_ctx(device)
    arr, n, keep = nodes_to_c(nodes)
    mem, cpu = C.c_int64(), C.c_int64()
    rc = ctx.lib.esc_nodes_capacity_total(ctx.handle, arr, n, C.byref(mem), C.byref(cpu))
    if rc == L.ESC_E_LIMIT:
        raise OverflowError("node capacity total left int64")
    L.check(rc, "esc_nodes_capacity_total")
    del keep
    return mem.value, cpu.value
