"""escalator_amd — MI355X-native scale-decision hot path of the Escalator autoscaler.

The compute runs in hand-written HIP kernels for gfx950 behind a C ABI
(include/escalator_hip.h, built in-tree as libescalator_hip.so).  This package is the
Python host over that ABI, mirroring the reference's interfaces:

* ``escalator_amd.k8s``        — pkg/k8s (CalculatePodsRequestsTotal, CalculateNodesCapacityTotal)
* ``escalator_amd.controller`` — pkg/controller (calcPercentUsage, calcScaleUpDelta,
  taintOldestN, untaintNewestN, scaleNodeGroup over every group at once)
* ``escalator_amd.context``    — the device snapshot + batched decision
* ``escalator_amd.dist``       — one process per GPU, sharded snapshot, RCCL exchange

Importing the package loads the library and raises if it has not been built.
"""
from . import _lib

_lib.load()

from .context import Context, Synth  # noqa: E402

__all__ = ["Context", "Synth"]
