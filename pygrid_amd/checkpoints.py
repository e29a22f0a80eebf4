"""Bounded checkpoint cache: the consumer side of the cycle-close path.

Mirrors ``ModelManager.save`` / ``load`` (``apps/node/src/app/main/model_centric/models/
model_manager.py:30-60``) and the checkpoint selection of ``/get-model`` and ``/retrieve-model``
(``routes/model_centric/routes.py:183, 488-498``): a new checkpoint gets ``number = count + 1``
and the ``latest`` alias, which is removed from the previous one; ``load`` returns the newest
matching checkpoint (``Warehouse.last``: highest id) or raises ``ModelNotFoundError``.

It keeps only the newest ``keep`` checkpoints of at most ``max_models`` models (least recently
used model dropped first), so memory is bounded (``keep`` x 47 MB for ResNet-18).  In a node it
is a write-through cache in front of the DB (``pygrid_amd.node``): every save still goes to the DB
and is then cached; ``lookup`` answers a query only when the answer is certain -- the cache holds a
contiguous newest run of the model's checkpoints, so the newest cached match IS the DB's newest
match -- and returns None otherwise (an older checkpoint, a query on other columns), so the caller
asks the DB.  It hands the very bytes object the engine produced back to the next cycle, so
``CycleAggregator`` / ``IncrementalCycle`` recognise it (identity) and reuse the copy already
resident in HBM instead of uploading the checkpoint again.  Standalone (no DB), ``save`` numbers
checkpoints itself and ``load`` raises ``ModelNotFoundError`` for anything not cached.
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional

from .exceptions import PyGridError


class ModelNotFoundError(PyGridError):
    """Mirrors ``core/exceptions.py`` ModelNotFoundError."""

    def __init__(self):
        super().__init__("Model not found!")


@dataclass
class Checkpoint:
    """The columns of ``ModelCheckPoint`` (``ai_model.py``) the node's readers use."""
    id: int
    model_id: int
    number: int
    alias: str
    value: bytes

    def __str__(self):
        return f"<CheckPoint id: {self.id}, number: {self.number}, alias: {self.alias}, model_id: {self.model_id}>"


_KEYS = ("model_id", "number", "alias", "id")


class CheckpointStore:
    def __init__(self, keep: int = 4, max_models: int = 8):
        if keep < 1 or max_models < 1:
            raise ValueError("keep and max_models must be >= 1")
        self.keep = int(keep)
        self.max_models = int(max_models)
        self._by_model: "OrderedDict[int, List[Checkpoint]]" = OrderedDict()  # oldest..newest, LRU order
        self._count: Dict[int, int] = {}  # standalone numbering
        self._lock = threading.Lock()
        self._next_id = 1
        self.hits = self.misses = 0

    # ---- write-through cache (pygrid_amd.node) ---------------------------------------------------
    def put(self, cp: Checkpoint) -> Checkpoint:
        """``cp`` was just saved to the DB (so it is that model's newest checkpoint): cache it as such,
        demote the previous ``latest``, drop the oldest beyond ``keep``."""
        with self._lock:
            rows = self._rows(cp.model_id)
            if rows and cp.id <= rows[-1].id:  # not newer than what we hold: the cache is not a clean suffix
                rows.clear()
            for r in rows:
                if r.alias == cp.alias:
                    r.alias = ""
            rows.append(cp)
            del rows[:-self.keep]
            self._count[cp.model_id] = max(self._count.get(cp.model_id, 0), cp.number)
            return cp

    def seed(self, cp: Checkpoint):
        """``cp`` is the model's newest checkpoint as the DB returned it (``load(model_id=...)``):
        start (or restart) the model's cached run with it unless it is already the newest cached."""
        with self._lock:
            rows = self._rows(cp.model_id)
            if rows and rows[-1].id == cp.id:
                return
            rows[:] = [cp]
            self._count[cp.model_id] = max(self._count.get(cp.model_id, 0), cp.number)

    def lookup(self, **kwargs) -> Optional[Checkpoint]:
        """The checkpoint ``ModelManager.load(**kwargs)`` would return, when the cache can tell;
        None when the DB must answer."""
        if "model_id" not in kwargs or any(k not in _KEYS for k in kwargs):
            self.misses += 1
            return None
        with self._lock:
            rows = self._by_model.get(kwargs["model_id"])
            if rows:
                self._by_model.move_to_end(kwargs["model_id"])
                for cp in reversed(rows):
                    if all(getattr(cp, k) == v for k, v in kwargs.items()):
                        self.hits += 1
                        return cp
        self.misses += 1
        return None

    def invalidate(self, model_id: Optional[int] = None):
        with self._lock:
            if model_id is None:
                self._by_model.clear()
            else:
                self._by_model.pop(model_id, None)

    def _rows(self, model_id: int) -> List[Checkpoint]:
        rows = self._by_model.get(model_id)
        if rows is None:
            rows = self._by_model[model_id] = []
            while len(self._by_model) > self.max_models:
                self._by_model.popitem(last=False)
        self._by_model.move_to_end(model_id)
        return rows

    @property
    def cached_bytes(self) -> int:
        with self._lock:
            return sum(len(cp.value) for rows in self._by_model.values() for cp in rows)

    # ---- standalone (no DB) -------------------------------------------------------------------
    def create(self, model_id: int, value: bytes) -> Checkpoint:
        """``ModelManager.create``: checkpoint #1 with alias ``latest`` (model_manager.py:19-28)."""
        return self.save(model_id, value)

    def save(self, model_id: int, value: bytes) -> Checkpoint:
        """``ModelManager.save`` (model_manager.py:30-51)."""
        with self._lock:
            number = self._count.get(model_id, 0) + 1
            cp = Checkpoint(self._next_id, model_id, number, "latest", value)
            self._next_id += 1
        return self.put(cp)

    def load(self, **kwargs) -> Checkpoint:
        """``ModelManager.load``: the last (highest id) cached checkpoint matching every field."""
        cp = self.lookup(**kwargs)
        if cp is None:
            raise ModelNotFoundError()
        return cp

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
