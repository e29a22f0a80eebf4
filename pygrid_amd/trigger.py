"""When the cycle-close hot path runs.

Reference behaviour (``apps/node/src/app/main/model_centric/tasks/cycle.py:9-25``,
``cycle_manager.py:176-178, :202``):

* ``run_task_once("complete_cycle", ...)`` is called from every ``submit_worker_diff``; if a
  previous ``complete_cycle`` is still running the new request is dropped ("Skipping ...
  because previous one is not finished").  A report that lands while an average is in flight
  therefore never triggers the readiness check it needed; if it was the last report, the cycle
  stays open until some later report arrives.
* ``cycle.end`` is only compared with ``now`` inside ``complete_cycle`` (``:202``), i.e. only
  when a report arrives: a time-limited cycle with no further reports never closes.

``CycleCloseTrigger`` keeps the single-flight guarantee (one close at a time, as the reference
wants: the GPU context is single-owner) and fixes both: a request that arrives during a run
marks the run dirty and is replayed as soon as it finishes, and ``schedule_deadline`` arms a
timer that runs the same readiness check at ``cycle.end``.
"""
from __future__ import annotations

import logging
import threading
import traceback
from datetime import datetime
from typing import Callable, Dict, Optional


class CycleCloseTrigger:
    def __init__(self, complete_cycle: Callable[[int], object], name: str = "complete_cycle"):
        """``complete_cycle(cycle_id)`` is the node's readiness check + close
        (``CycleManager.complete_cycle``, ``cycle_manager.py:180-217``)."""
        self._fn = complete_cycle
        self._name = name
        self._lock = threading.Lock()
        self._running = False
        self._pending: Dict[int, None] = {}  # cycle ids requested while a run was in flight (ordered)
        self._timers: Dict[int, threading.Timer] = {}
        self._idle = threading.Event()
        self._idle.set()
        self.runs = 0
        self.errors = 0

    # -- the run_task_once replacement ----------------------------------------------------------
    def request(self, cycle_id: int):
        """Called where the reference calls ``run_task_once`` (``cycle_manager.py:178``)."""
        with self._lock:
            self._pending[cycle_id] = None
            if self._running:
                return  # replayed by the running worker when it finishes (the reference drops it)
            self._running = True
            self._idle.clear()
        threading.Thread(target=self._drain, name=f"{self._name}-worker", daemon=True).start()

    def _drain(self):
        while True:
            with self._lock:
                if not self._pending:
                    self._running = False
                    self._idle.set()
                    return
                cycle_id = next(iter(self._pending))
                del self._pending[cycle_id]
            try:
                self._fn(cycle_id)
            except Exception as e:  # the reference's task wrapper logs and swallows (tasks/cycle.py:33-37)
                self.errors += 1
                logging.error("Error in %s task: %s %s", self._name, e, traceback.format_exc())
            self.runs += 1

    # -- deadline ------------------------------------------------------------------------------
    def schedule_deadline(self, cycle_id: int, end: Optional[datetime], now: Optional[datetime] = None):
        """Arm a timer that requests the readiness check at ``end`` (``cycle.end``, set from
        ``cycle_length`` when the cycle is created, ``cycle_manager.py:28-54``)."""
        if end is None:
            return
        now = now or datetime.now()
        delay = max(0.0, (end - now).total_seconds())
        t = threading.Timer(delay, self.request, args=(cycle_id,))
        t.daemon = True
        with self._lock:
            old = self._timers.pop(cycle_id, None)
            self._timers[cycle_id] = t
        if old:
            old.cancel()
        t.start()

    def cancel_deadline(self, cycle_id: int):
        with self._lock:
            t = self._timers.pop(cycle_id, None)
        if t:
            t.cancel()

    def wait_idle(self, timeout: Optional[float] = None) -> bool:
        return self._idle.wait(timeout)

    def shutdown(self):
        with self._lock:
            timers = list(self._timers.values())
            self._timers.clear()
        for t in timers:
            t.cancel()
