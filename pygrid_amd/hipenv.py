"""HIP runtime settings the engine needs, applied before HIP initialises in this process.

HIP maps every stream of a process onto ``GPU_MAX_HW_QUEUES`` hardware queues (4 by default) and
streams that share a queue run in order.  A process that drives the engine beside torch has many
streams: the library's own (kernel, copy, aux), torch's current stream, its pool streams (a side
stream, ProcessGroupNCCL's collective stream).  With 4 queues the N > 1 step's RCCL all-gather
landed on the queue of the next range's fold and the two serialised: the ranged fold + all-gather
took 7.59 ms against 6.86 ms for one whole fold at 4 queues, 7.38 at 8 and 6.96 at 16
(``tools/ab_overlap_world1.py`` 8:3 under ``tools/ab_env.py``, ``profiles/r02u/``).

``prepare()`` raises the queue count to at least ``PGH_HW_QUEUES`` (default 16; the pool's limit
is 32) unless the environment already asks for more.  The runtime reads the variable once, at its
initialisation, so this only takes effect when called before the first HIP call of the process
(``bench.py`` does so first thing; importing ``pygrid_amd`` does too, which covers a node that
imports the engine before torch touches the GPU).  Returns the value in effect for this process
if it was set in time, else None.
"""
from __future__ import annotations

import os

DEFAULT_HW_QUEUES = 16
_MAX_HW_QUEUES = 32


def prepare() -> int | None:
    try:
        want = int(os.environ.get("PGH_HW_QUEUES", DEFAULT_HW_QUEUES))
    except ValueError:
        want = DEFAULT_HW_QUEUES
    want = max(1, min(want, _MAX_HW_QUEUES))
    try:
        have = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        have = 0
    if "PGH_HW_QUEUES" in os.environ or have < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    if _hip_initialised():
        return None
    return int(os.environ["GPU_MAX_HW_QUEUES"])


def _hip_initialised() -> bool:
    """True when torch (the only other HIP user in a node process) already initialised HIP here."""
    import sys

    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:  # noqa: BLE001
        return False
