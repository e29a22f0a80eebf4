#!/usr/bin/env python3
"""What a PyGrid node sees per cycle with the engine installed, through
the reference's own storage types and report handler code:

* the node's tables in SQLAlchemy on SQLite (tests/sql_node.py: ``WorkerCycle.diff`` a
  ``LargeBinary``, the reference's ``Warehouse``), in memory by default (``--db=PATH``: a file);
* each client's report through the reference's handler restated (tests/ref_fl_events.py:
  ``base64.b64decode(data.get(CYCLE.DIFF).encode())``, fl_events.py:257 -- the ``.encode()`` copy
  of the 62 MB text included) -> ``submit_worker_diff`` (the DB write + commit) -> the engine's
  ``on_report`` (the diff into an HBM slot, folded);
* the close requested the reference's way: the report that reaches ``max_diffs`` calls
  ``run_task_once("complete_cycle", ...)`` (cycle_manager.py:176-178), run on an executor thread
  (tasks/cycle.py:9-25).

ResNet-18, 100 workers assigned per cycle, 80 report (worker 0 and 19 others never do,
routes.py:314; ``max_diffs`` = 80), shuffled arrival.  Arms: reports ``paced`` ``--gap-ms`` apart
(default 5) or back to back (``b2b``), x the product default (``default``: report-time
aggregation) / the close-time path only (``closetime``: ``install(report_time=False)``, every diff
read from the DB and folded at the close).  (The speculative arms of r04 went with the speculative
close in r05.)

    python tools/node_sim.py [cycles] [--gap-ms=5] [--no-pinned] [--db=PATH] [--arms=paced_default,b2b_closetime,...] [--cpu]
                             [--devices=0,0]   (a one-process group, as install(devices=[...]))

Prints one JSON line: per arm the report handler latency (p50 / p99 / max) and its phases (the
handler's base64 decode including ``.encode()``, the DB write + commit, the engine's ingest), and
``close_ms``: from the last report's handler returning to the new checkpoint committed in the DB
and the next cycle open (the executor's ``complete_cycle``), with the engine's share
(``IncrementalCycle.finish``).  Dev tool: imports tests/ infrastructure; never a product path.
"""
import base64
import functools
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import ref_fl_events  # noqa: E402
from fake_node import assign, host_process  # noqa: E402
from pygrid_amd import Engine, incremental  # noqa: E402
from pygrid_amd import node as pnode  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import RESNET18_SHAPES  # noqa: E402
from sql_node import make_sql_node  # noqa: E402

ASSIGNED, REPORTERS = 100, 80


def pct(xs, q):
    return round(float(np.percentile(xs, q)), 3) if xs else None


class Executor:
    """``run_task_once`` (tasks/cycle.py:9-25): one named future on a worker thread."""

    def __init__(self):
        self.pool = ThreadPoolExecutor(1, thread_name_prefix="executor")
        self.futures = {}

    def run_task_once(self, name, func, *args):
        f = self.futures.get(name)
        if f is None or f.done():
            self.futures[name] = self.pool.submit(func, *args)


class Timer:
    """Wraps callables to add their wall time (ms) to a per-thread bucket."""

    def __init__(self):
        self.local = threading.local()

    def bucket(self):
        b = getattr(self.local, "b", None)
        if b is None:
            b = self.local.b = {}
        return b

    def wrap(self, owner, name, key):
        f = getattr(owner, name)

        @functools.wraps(f)
        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                b = self.bucket()
                b[key] = b.get(key, 0.0) + (time.perf_counter() - t0) * 1e3
        setattr(owner, name, g)
        return f


def run_arm(eng, cycles, gap_ms, opts, pinned, db, rng, ckpt, texts, framing="fresh"):
    if db != "sqlite://":  # a file: a fresh one per arm (each arm hosts its own FL process)
        path = db[len("sqlite:///"):]
        for suffix in ("", "-journal", "-wal", "-shm"):
            if os.path.exists(path + suffix):
                os.remove(path + suffix)
    mod, store = make_sql_node(db)
    ex = Executor()
    mod.run_task_once = ex.run_task_once
    node = pnode.install(mod, engine=eng, report_module=ref_fl_events, pinned_reports=16 if pinned else 0,
                         framing=framing, **opts)
    ref_fl_events.processes = type("P", (), {"submit_diff": staticmethod(
        lambda *a: mod.cycle_manager.submit_worker_diff(*a))})
    timer = Timer()
    timer.wrap(ref_fl_events.base64, "b64decode", "decode")
    timer.wrap(node, "on_report", "ingest")
    # the close's phases on the executor thread (its own bucket): the whole _average_plan_diffs,
    # the checkpoint save (the node's DB write), preparing the next cycle's report-time state
    timer.wrap(node, "average_plan_diffs", "close_average_plan_diffs")
    timer.wrap(mod.model_manager, "save", "close_save")
    timer.wrap(node, "on_cycle_created", "close_next_cycle_prepare")
    timer.wrap(mod.cycle_manager, "complete_cycle", "close_complete_cycle")
    finish = incremental.IncrementalCycle.finish
    engine_close = []

    close_info = []

    def timed_finish(self, *a, **k):
        t0 = time.perf_counter()
        try:
            return finish(self, *a, **k)
        finally:
            engine_close.append((time.perf_counter() - t0) * 1e3)
            close_info.append({k_: self.last_close.get(k_) for k_ in ("early", "n", "from_db", "refold")})
    incremental.IncrementalCycle.finish = timed_finish
    try:
        cfg = {"min_diffs": REPORTERS, "max_diffs": REPORTERS, "num_cycles": 0}
        proc, _, _ = host_process(mod, cfg, ckpt)
        handler, encode, decode, write, ingest, closes, engine_share = [], [], [], [], [], [], []
        phases = []
        for cyc in range(cycles + 1):  # cycle 0 warms up
            keys = {w: assign(mod, f"w{w}", proc) for w in range(ASSIGNED)}
            reporters = [w for w in rng.permutation(ASSIGNED) if w != 0][:REPORTERS]
            engine_close.clear()
            for i, w in enumerate(reporters):
                if i and gap_ms:
                    time.sleep(gap_ms / 1e3)
                text = texts[w % len(texts)]
                msg = {"data": {"worker_id": f"w{w}", "request_key": keys[w], "diff": text}}
                e0 = time.perf_counter()
                text.encode()  # the handler's .encode() copy, timed apart (it runs before b64decode)
                enc = (time.perf_counter() - e0) * 1e3
                timer.bucket().clear()
                t0 = time.perf_counter()
                resp = ref_fl_events.report(msg)
                t1 = time.perf_counter()
                if resp["data"] != {"status": "success"}:
                    raise SystemExit(f"report failed: {resp}")
                if cyc:
                    b = timer.bucket()
                    total = (t1 - t0) * 1e3
                    handler.append(total)
                    encode.append(enc)
                    decode.append(b.get("decode", 0.0))
                    ingest.append(b.get("ingest", 0.0))
                    write.append(total - enc - b.get("decode", 0.0) - b.get("ingest", 0.0))
            fut = ex.futures["complete_cycle"]
            fut.result(120)
            if cyc:
                phases.append(ex.pool.submit(lambda: dict(timer.bucket())).result())
            ex.pool.submit(lambda: timer.bucket().clear()).result()
            if mod.cycle_manager.task_errors:
                raise SystemExit(f"close failed: {mod.cycle_manager.task_errors!r}")
            t2 = time.perf_counter()
            if cyc:
                closes.append((t2 - t1) * 1e3)
                engine_share.append(engine_close[-1] if engine_close else None)
            # untimed: the closed cycle's blobs are not needed again (bounds the DB's size)
            cid = store.session.query(store.Cycle.id).filter_by(is_completed=True).order_by(store.Cycle.id.desc()).first()[0]
            store.session.query(store.WorkerCycle).filter_by(cycle_id=cid).update({"diff": None})
            store.session.commit()
        stats = dict(node.stats)
        pools = {"hits": node.pinned.hits, "misses": node.pinned.misses} if node.pinned else None
    finally:
        incremental.IncrementalCycle.finish = finish
        node.uninstall()
        ex.pool.shutdown()
        store.close()
    return {"report_handler_ms": {"p50": pct(handler, 50), "p99": pct(handler, 99), "max": round(max(handler), 3)},
            "handler_phases_p50_ms": {"str_encode": pct(encode, 50), "b64decode": pct(decode, 50),
                                      "submit_worker_diff_db_write_commit": pct(write, 50),
                                      "engine_on_report_ingest": pct(ingest, 50)},
            "close_ms": pct(closes, 50), "closes_ms": [round(c, 3) for c in closes],
            "engine_close_ms": pct([e for e in engine_share if e is not None], 50),
            "engine_closes": close_info[1:],
            "close_phases_ms": [{k: round(v, 3) for k, v in p.items()} for p in phases],
            "node_stats": stats, "pinned_pool": pools}


class _nullctx:
    def __init__(self, x):
        self.x = x

    def __enter__(self):
        return self.x

    def __exit__(self, *a):
        return False


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    opt = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    cycles = int(args[0]) if args else 3
    gap = float(opt.get("gap-ms", 5.0))
    pinned = "--no-pinned" not in sys.argv
    db = f"sqlite:///{opt['db']}" if "db" in opt else "sqlite://"
    want = opt.get("arms", "paced_default,b2b_default").split(",")
    rng = np.random.default_rng(2024)
    ckpt = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    texts = [base64.b64encode(build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                                for s in RESNET18_SHAPES])).decode("ascii") for _ in range(4)]
    arms = {}
    if "--cpu" in sys.argv:  # dev check of this tool on a GPU-less box: the tests' numpy engine
        from fake_engine import NumpyEngine
    kinds = {"default": {}, "closetime": {"report_time": False}}
    framing = "template" if "--cpu" in sys.argv else "fresh"
    devices = [int(d) for d in opt["devices"].split(",")] if "devices" in opt else None
    with (_nullctx(NumpyEngine()) if "--cpu" in sys.argv else Engine(devices=devices) if devices else Engine(0)) as eng:
        # An untimed pass of the first arm: the process's first arm ran its report handlers at
        # 74-81 ms p50 against 29-37 for every later arm, whatever the arm (the .encode() copy 12-14 ms
        # instead of 2, the DB write 60 instead of 25: first-touch host memory, profiles/r04d, r04i,
        # r04p), so each arm is measured in the same warm process.
        pace, kind = want[0].split("_")
        run_arm(eng, 1, gap if pace == "paced" else 0.0, kinds[kind], pinned, db, rng, ckpt, texts, framing=framing)
        for name in want:
            pace, kind = name.split("_")
            arms[name] = run_arm(eng, cycles, gap if pace == "paced" else 0.0, kinds[kind],
                                 pinned, db, rng, ckpt, texts, framing=framing)
            print(f"# {name}: close {arms[name]['close_ms']} ms, handler p50 {arms[name]['report_handler_ms']['p50']} ms",
                  file=sys.stderr, flush=True)
    print(json.dumps({
        "workload": f"ResNet-18 (62 tensors), {ASSIGNED} assigned per cycle, {REPORTERS} report (max_diffs) in "
                    "shuffled order; JSON base64 text -> restated fl_events.report (.encode() + b64decode) -> "
                    "submit_worker_diff (SQLAlchemy LargeBinary write + commit) -> engine ingest; close by "
                    "run_task_once on an executor thread",
        "db": db, "pinned_reports": pinned, "cycles": cycles, "gap_ms": gap, "devices": devices,
        "warmup": f"one untimed cycle of {want[0]} first, then every arm's own untimed cycle 0",
        "close_definition": "last report handler returned -> new checkpoint committed + next cycle open "
                            "(complete_cycle on the executor thread)",
        "arms": arms}))


if __name__ == "__main__":
    main()
