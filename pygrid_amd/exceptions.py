"""Error types, mirroring the reference's ``PyGridError`` hierarchy
(``apps/node/src/app/main/core/exceptions.py:4``).

The reference's cycle-close task catches every exception and logs it
(``apps/node/src/app/main/model_centric/tasks/cycle.py:28-37``); raising a ``PyGridError``
subclass from the engine keeps that contract.
"""


class PyGridError(Exception):
    def __init__(self, message):
        super().__init__(message)


class AggregationError(PyGridError):
    """A libpygrid_hip call returned a negative status."""

    def __init__(self, message, status=None):
        super().__init__(message)
        self.status = status


class EngineUnavailableError(PyGridError):
    """The HIP library is not built or no GPU is visible.  The product path never falls back
    to a CPU implementation: it raises this instead."""


class StateParseError(AggregationError):
    """Malformed syft State protobuf bytes."""


class PlanNotAcceleratedError(PyGridError):
    """The hosted avg plan is not one the engine implements (user-defined non-iterative plan,
    or an iterative plan that does not match ``(avg * num + item) / (num + 1)``).  The caller
    keeps running the reference's own CPU path for it."""


class ModelNotAcceleratedError(PlanNotAcceleratedError):
    """The checkpoint or a diff holds well-formed tensors that are not float32 (another dtype, or a
    serializer other than syft's "all").  The reference averages them with torch's type promotion;
    the engine is fp32-only, so the caller runs the reference path for this cycle, as for an
    unaccelerated plan (malformed bytes still raise ``StateParseError``)."""
