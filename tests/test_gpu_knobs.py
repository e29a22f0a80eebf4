"""GPU: every environment knob the library still reads (environment knobs), at a
non-default value, closes bit-exact against the oracle.  PGH_BLOCK_BYTES,
PGH_FINAL_RANGES and PGH_PINNED_GATHER have their own tests (test_gpu_parity.py,
test_gpu_pipelined_close.py, test_gpu_pinned_report.py).  The library reads the environment when
a context is created, so each case creates its own."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32
SHAPES = [(1100, 1000), (1000,), (10, 1000), (10,)]  # > 1 M params: the split FINAL pass applies


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _case(seed, n=5):
    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng(seed)
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for _ in range(n)]
    return ckpt, diffs, build_state_fast(ckpt), [build_state_fast(d) for d in diffs]


def _check(new_pb, want):
    from pygrid_amd.state_schema import parse_state

    for g, w in zip(parse_state(new_pb), want):
        assert np.array_equal(bits(g), bits(w))


@pytest.mark.parametrize("env", [{"PGH_COPY_THREADS": "1"}, {"PGH_NUMA": "0"}, {"PGH_WARMUP": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_close_time_knobs(monkeypatch, env):
    from pygrid_amd import Engine
    from pygrid_amd.cycle import CycleAggregator

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ckpt, diffs, ck_pb, d_pbs = _case(900)
    with Engine(0) as eng:
        for _ in range(2):  # the first close after create (no warm-up) and a second one
            _check(CycleAggregator(eng).average_plan_diffs({}, ck_pb, d_pbs), O.fedavg_mean(ckpt, diffs))


D2H_MODES = ["1", "0"]
D2H_IDS = ["d2h-default (own stream and cells, SDMA)", "PGH_D2H_STREAM=0 (copy stream, staging slots)"]


@pytest.mark.parametrize("own", D2H_MODES, ids=D2H_IDS)
@pytest.mark.parametrize("pinned", [0, 2 << 20, 2 * 81_920], ids=["ring-default", "ring-2MiB", "ring-160KiB"])
def test_d2h_pieces_wrap_a_small_pinned_ring(monkeypatch, pinned, own):
    """stage_d2h_pieces queues every D2H piece that fits the pinned ring at once and refills a cell
    as soon as its piece is copied out: a 4.4 MB checkpoint through a ring of 2 x 1 MiB (5 pieces
    over 2 cells) or 2 x 80 KiB (55 pieces), after a close-time fold and -- with PGH_D2H_STREAM=0,
    where the report-time close's pieces also use the staging slots -- after a report-time close
    (its pieces wait on the FINAL ranges' marks), bit-exact.  By default the report-time close's
    pieces run on the D2H stream's own cells whatever the staging ring's size."""
    from pygrid_amd import Engine
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.incremental import IncrementalCycle

    monkeypatch.setenv("PGH_D2H_STREAM", own)
    ckpt, diffs, ck_pb, d_pbs = _case(915, n=4)
    want = O.fedavg_mean(ckpt, diffs)
    with Engine(0, pinned_bytes=pinned) as eng:
        inc = IncrementalCycle(eng, [int(np.prod(s)) for s in SHAPES], slots=6, checkpoint=ck_pb)
        for w in range(5):
            inc.assigned(w)
        for w in (3, 1, 2, 4):  # worker 0 never reports: every row folds at close, in ranges
            inc.reported(w, d_pbs[w - 1])
        _check(inc.close(ck_pb), want)
        _check(CycleAggregator(eng).average_plan_diffs({}, ck_pb, d_pbs), want)


@pytest.mark.parametrize("own", D2H_MODES, ids=D2H_IDS)
def test_report_time_close_in_output_ranges(monkeypatch, own):
    """The report-time close's FINAL pass runs as ranges of 4 MiB of output on one stream, the D2H
    pieces behind them (no knob since r04): a 1.1 M-param shard (two ranges, the second short)
    closes bit-exact -- its pieces on the D2H stream's own cells (default) or on the copy stream
    through the staging slots (0), every one an SDMA copy.  The stats count the result's bytes."""
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle

    monkeypatch.setenv("PGH_D2H_STREAM", own)
    ckpt, diffs, ck_pb, d_pbs = _case(911, n=6)
    with Engine(0) as eng:
        inc = IncrementalCycle(eng, [int(np.prod(s)) for s in SHAPES], slots=8, checkpoint=ck_pb)
        for w in range(7):
            inc.assigned(w)
        for w in (5, 1, 3, 0, 2, 4):  # worker 6 never reports
            inc.reported(w, d_pbs[w])
        eng.reset_stats()
        _check(inc.close(ck_pb), O.fedavg_mean(ckpt, diffs))
        st = eng.stats()
        P = sum(int(np.prod(s)) for s in SHAPES)
        assert st["d2h_bytes_total"] == 4 * P
        assert st["d2h_kernel_bytes_total"] == 0  # no kernel copies since r06s


@pytest.mark.parametrize("mode", ["1", "0"], ids=["d2h-default", "PGH_D2H_STREAM=0"])
def test_report_time_close_wraps_the_d2h_cells(monkeypatch, mode):
    """A shard of 20 M params (80 MB: 10 D2H pieces) has more pieces than the D2H stream's 8 cells:
    pieces 9-10 go out into cells the host has copied out, behind the FINAL ranges that wrote
    them; three chained report-time closes (the cells reused across closes), each right behind its
    last report, bit-exact."""
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast

    monkeypatch.setenv("PGH_D2H_STREAM", mode)
    shapes = [(4000, 5000), (7,)]
    rng = np.random.default_rng(931)
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck_pb = build_state_fast(ckpt)
    numel = [int(np.prod(s)) for s in shapes]
    with Engine(0) as eng:
        for cyc in range(3):
            diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(3)]
            inc = IncrementalCycle(eng, numel, slots=4, checkpoint=ck_pb)
            for w in range(4):
                inc.assigned(w)
            for w in (2, 1, 3):  # worker 0 never reports: all three rows fold at close
                inc.reported(w, build_state_fast(diffs[w - 1]))
            ck_pb = inc.close(ck_pb)
            ckpt = O.fedavg_mean(ckpt, diffs)
            _check(ck_pb, ckpt)


@pytest.mark.parametrize("mode", ["1", "0"], ids=["d2h-default", "PGH_D2H_STREAM=0"])
def test_report_time_close_first_in_a_fresh_process(mode):
    """The first report-time closes of a fresh process, the last D2H pieces right behind the FINAL
    ranges that wrote them: round 6's K6 k_copy_to_host (pieces copied out by a kernel on the D2H
    stream) read ranges there that had not run yet -- 1 close in ~40 with every piece by K6, most
    often a process's first (profiles/r06s/) -- and was removed.  Three fresh contexts x three
    chained closes of a 20 M-param shard (10 pieces, 8 cells) in a child process, every close's
    bytes compared with the oracle."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    r = subprocess.run([sys.executable, "-u", str(root / "tools" / "diag_d2h_race.py"), "3", mode],
                       capture_output=True, text=True, timeout=240, cwd=str(root))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "0 bad closes of 9" in r.stdout


def test_group_copy_threads_and_rccl_off(monkeypatch):
    """PGH_COPY_THREADS=2 split over a two-child group on GPU 0, PGH_RCCL=0 (peer copies)."""
    from pygrid_amd import Engine
    from pygrid_amd.cycle import CycleAggregator

    monkeypatch.setenv("PGH_COPY_THREADS", "2")
    monkeypatch.setenv("PGH_RCCL", "0")
    ckpt, diffs, ck_pb, d_pbs = _case(920)
    with Engine(devices=[0, 0]) as grp:
        _check(CycleAggregator(grp).average_plan_diffs({}, ck_pb, d_pbs), O.fedavg_mean(ckpt, diffs))
        grp.allgather_resident()
        assert grp.group_backend() == 0  # peer copies, never RCCL
