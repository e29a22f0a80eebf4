"""In-memory checkpoint store: the consumer side of the cycle-close path.

Mirrors ``ModelManager.save`` / ``load`` (``apps/node/src/app/main/model_centric/models/
model_manager.py:30-60``) and the checkpoint selection of ``/retrieve-model``
(``routes/model_centric/routes.py:471-516``): a new checkpoint gets ``number = count + 1`` and the
``latest`` alias, which is removed from the previous one; ``load`` returns the newest matching
checkpoint (``Warehouse.last``: highest id) or raises ``ModelNotFoundError``.

The node keeps writing checkpoints to its DB; this store serves ``/get-model`` and
``/retrieve-model`` from memory and hands the very bytes object the engine produced back to the
next cycle, so ``CycleAggregator`` recognises it (identity) and reuses the copy already resident
in HBM instead of uploading the checkpoint again.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Dict, List, Optional

from .exceptions import PyGridError


class ModelNotFoundError(PyGridError):
    """Mirrors ``core/exceptions.py`` ModelNotFoundError."""

    def __init__(self):
        super().__init__("Model not found!")


@dataclass
class Checkpoint:
    id: int
    model_id: int
    number: int
    alias: str
    value: bytes


class CheckpointStore:
    def __init__(self):
        self._rows: List[Checkpoint] = []
        self._by_model: Dict[int, List[Checkpoint]] = {}
        self._lock = threading.Lock()
        self._next_id = 1

    def create(self, model_id: int, value: bytes) -> Checkpoint:
        """``ModelManager.create``: checkpoint #1 with alias ``latest`` (model_manager.py:19-28)."""
        return self.save(model_id, value)

    def save(self, model_id: int, value: bytes) -> Checkpoint:
        """``ModelManager.save`` (model_manager.py:30-51)."""
        with self._lock:
            rows = self._by_model.setdefault(model_id, [])
            for r in rows:
                if r.alias == "latest":
                    r.alias = ""
            cp = Checkpoint(self._next_id, model_id, len(rows) + 1, "latest", value)
            self._next_id += 1
            rows.append(cp)
            self._rows.append(cp)
            return cp

    def load(self, **kwargs) -> Checkpoint:
        """``ModelManager.load``: the last (highest id) checkpoint matching every given field."""
        with self._lock:
            for cp in reversed(self._rows):
                if all(getattr(cp, k) == v for k, v in kwargs.items()):
                    return cp
        raise ModelNotFoundError()

    def retrieve(self, model_id: int, checkpoint: Optional[str] = None) -> bytes:
        """Checkpoint selection of ``/retrieve-model`` (routes.py:488-498)."""
        query = {"model_id": model_id}
        if checkpoint:
            if checkpoint.isnumeric():
                query["number"] = int(checkpoint)
            else:
                query["alias"] = checkpoint
        else:
            query["alias"] = "latest"
        return self.load(**query).value

    def latest(self, model_id: int) -> bytes:
        """What ``/get-model`` sends (routes.py:183-187)."""
        return self.load(model_id=model_id).value
