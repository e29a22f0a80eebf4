"""pygrid_amd -- MI355X-native aggregation engine for PyGrid Node's model-centric cycle close.

The product is ``libpygrid_hip.so`` (C ABI: ``include/pgh_api.h``; gfx950 HIP kernels in
``csrc/``).  This package is the host side a PyGrid node imports:

* ``engine.Engine``       -- one GPU context (ingest, fedavg, secagg, stats)
* ``cycle``               -- mirror of ``CycleManager._average_plan_diffs`` / readiness / dispatch
* ``incremental``         -- report-time folding (``submit_worker_diff`` -> HBM slots)
* ``node``                -- ``install(...)``: one opt-in patch wiring the engine into a node
* ``state``               -- syft State codec (replaces model_manager.py:79-103 serde)
* ``sharding``            -- parameter-axis shards + RCCL all-gather across GPUs

Nothing here computes on the CPU: without the built library and a GPU the engine raises.
Importing the package changes nothing in the host process; ``tune_process()`` is the explicit
opt-in for the process-wide settings the engine benefits from (HIP hardware queues, glibc
thresholds for 47 MB buffers).
"""
from .exceptions import (AggregationError, EngineUnavailableError, ModelNotAcceleratedError, PlanNotAcceleratedError,
                         PyGridError, StateParseError)
from .engine import F32, I64, ITERATIVE_MEAN, MEAN, STREAM_SECAGG, WEIGHTED_MEAN, Engine, PinnedBuffer, device_count


def tune_process(hw_queues: bool = True, malloc: bool = True) -> dict:
    """Process-wide settings, applied only when the host application asks for them:

    * ``hw_queues``: ``GPU_MAX_HW_QUEUES`` (``hipenv.prepare``; only if unset or ``PGH_HW_QUEUES``
      is given; must run before the first HIP call of the process);
    * ``malloc``: glibc mmap / trim thresholds (``hostmem.tune``) so 47 MB diffs and checkpoints
      are reused from the heap.

    Returns what was applied: ``{"hw_queues": int | None, "malloc": bool}``."""
    from . import hipenv, hostmem

    return {"hw_queues": hipenv.prepare() if hw_queues else None,
            "malloc": hostmem.tune() if malloc else False}


__all__ = [
    "AggregationError", "EngineUnavailableError", "ModelNotAcceleratedError", "PlanNotAcceleratedError", "PyGridError",
    "StateParseError",
    "Engine", "PinnedBuffer", "device_count", "STREAM_SECAGG", "MEAN", "ITERATIVE_MEAN", "WEIGHTED_MEAN", "F32", "I64",
    "tune_process",
]
__version__ = "0.3.0"
