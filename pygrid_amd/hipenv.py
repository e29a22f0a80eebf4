"""HIP runtime settings the engine benefits from, applied before HIP initialises in this process.

HIP maps every stream of a process onto ``GPU_MAX_HW_QUEUES`` hardware queues (4 by default) and
streams that share a queue run in order.  A process that drives the engine beside torch has many
streams: the library's own (kernel, copy, aux), torch's current stream, its pool streams (a side
stream, ProcessGroupNCCL's collective stream).  With 4 queues the N > 1 step's RCCL all-gather
landed on the queue of the next range's fold and the two serialised: the ranged fold + all-gather
took 7.59 ms against 6.86 ms for one whole fold at 4 queues, 7.38 at 8 and 6.96 at 16
(``tools/ab_overlap_world1.py`` 8:3 under ``tools/ab_env.py``, ``profiles/r02u/``).

``prepare()`` is NOT run on import: it is part of ``pygrid_amd.tune_process()``, which a host
application calls explicitly (a drop-in must not retune its host process by being imported).  It
sets ``GPU_MAX_HW_QUEUES`` only

* when the variable is unset (to ``PGH_HW_QUEUES``, default 16), or
* when ``PGH_HW_QUEUES`` is given explicitly (the operator asked for that count; clamped to the
  pool's limit of 32).

An operator's own ``GPU_MAX_HW_QUEUES`` is never changed otherwise, and every change is logged.
The runtime reads the variable once, at its initialisation, so this only takes effect before the
first HIP call of the process.  Returns the value in effect for this process if it was set in
time, else None.
"""
from __future__ import annotations

import logging
import os

DEFAULT_HW_QUEUES = 16
_MAX_HW_QUEUES = 32

log = logging.getLogger(__name__)


def prepare() -> int | None:
    explicit = "PGH_HW_QUEUES" in os.environ
    try:
        want = int(os.environ.get("PGH_HW_QUEUES", DEFAULT_HW_QUEUES))
    except ValueError:
        want = DEFAULT_HW_QUEUES
    want = max(1, min(want, _MAX_HW_QUEUES))
    have = os.environ.get("GPU_MAX_HW_QUEUES")
    if have is None or explicit:
        if have != str(want):
            os.environ["GPU_MAX_HW_QUEUES"] = str(want)
            log.info("GPU_MAX_HW_QUEUES %s -> %d (%s)", have if have is not None else "unset", want,
                     "PGH_HW_QUEUES" if explicit else "default")
    if _hip_initialised():
        return None
    try:
        return int(os.environ["GPU_MAX_HW_QUEUES"])
    except ValueError:
        return None


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
