"""pygrid_amd -- MI355X-native aggregation engine for PyGrid Node's model-centric cycle close.

The product is ``libpygrid_hip.so`` (C ABI: ``include/pgh_api.h``; gfx950 HIP kernels in
``csrc/``).  This package is the host side a PyGrid node imports:

* ``engine.Engine``       -- one GPU context (ingest, fedavg, secagg, stats)
* ``cycle``               -- mirror of ``CycleManager._average_plan_diffs`` / readiness / dispatch
* ``state``               -- syft State codec (replaces model_manager.py:79-103 serde)
* ``sharding``            -- parameter-axis shards + RCCL all-gather across GPUs

Nothing here computes on the CPU: without the built library and a GPU the engine raises.
Importing the package raises HIP's hardware-queue count (``hipenv``) when HIP is not yet up and
keeps big host buffers on glibc's heap (``hostmem``; ``PGH_MALLOC_TUNE=0`` opts out).
"""
from . import hipenv, hostmem

hipenv.prepare()
hostmem.tune()

from .exceptions import (AggregationError, EngineUnavailableError, ModelNotAcceleratedError, PlanNotAcceleratedError,
                         PyGridError, StateParseError)
from .engine import F32, I64, ITERATIVE_MEAN, MEAN, STREAM_SECAGG, WEIGHTED_MEAN, Engine, PinnedBuffer, device_count

__all__ = [
    "AggregationError", "EngineUnavailableError", "ModelNotAcceleratedError", "PlanNotAcceleratedError", "PyGridError",
    "StateParseError",
    "Engine", "PinnedBuffer", "device_count", "STREAM_SECAGG", "MEAN", "ITERATIVE_MEAN", "WEIGHTED_MEAN", "F32", "I64",
]
__version__ = "0.1.0"
