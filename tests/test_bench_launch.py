"""bench.py forms the N-rank world itself (no GPU: --dry-run uses gloo on the CPU).

The driver runs ``python bench.py --gpus N`` under torch.distributed.run for N > 1, but a plain
``python bench.py --gpus N`` must measure N ranks too, never one rank labelled N.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT


# the cpu_baseline children (a CPU torch loop of ~15 s each) stand in as stubs except where a test
# is about them (test_cpu_baseline_on_the_n8_line)
NO_CPU = "cpu_baseline=0"


def _env(env_extra=None) -> dict:
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    env["PGH_BENCH_STUB"] = ",".join(x for x in (env.get("PGH_BENCH_STUB"), NO_CPU) if x)
    return env


def _run(args, env_extra=None, timeout=240):
    env = _env(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=str(ROOT), env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


GROUP_DRY = {"dry_run": True, "n_gpus": 2, "backend": "gloo", "group": True, "workload": "resnet18-fedavg"}


def _has(rec: dict, sub: dict):
    assert {k: rec.get(k) for k in sub} == sub, rec


def _config_lines(rec: dict, n: int):
    """Configs 3, 4 and 5 ran as their own N-rank worlds, config 1
    on one GPU: the ranks, the collective backend and the --check request are on the line."""
    for key, wl, g in (("config1", "mnist-state", 1), ("config3", "resnet18-secagg", n), ("config4", "c4-stream", n),
                       ("config5", "c5-ingest", n)):
        _has(rec[key], {"dry_run": True, "n_gpus": g, "workload": wl, "dist_backend": "gloo" if g > 1 else None,
                        "rccl_ranks": 0, "check": True, "group": False})


def test_plain_bench_forms_two_ranks():
    """The per-rank world's line, with the one-process group over the same GPUs (what the node
    deploys) run after the ranks exit, in a fresh child, under `group`, and
    the config-4 / config-5 worlds over the same GPUs under `config4` / `config5`."""
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    _has(rec, {"dry_run": True, "n_gpus": 2, "backend": "gloo", "dist_backend": "gloo", "rccl_ranks": 0})
    _has(rec["group"], GROUP_DRY)
    _config_lines(rec, 2)


def test_config4_and_5_dry_runs_carry_ranks_backend_and_check():
    for wl in ("c4-stream", "c5-ingest"):
        r = _run(["--gpus", "2", "--dry-run", "--workload", wl, "--check"])
        assert r.returncode == 0, r.stderr
        rec = _json_line(r.stdout)
        _has(rec, {"workload": wl, "n_gpus": 2, "dist_backend": "gloo", "rccl_ranks": 0, "check": True,
                   "group": False})  # no group record: c4 / c5 run per rank only
        assert "config4" not in rec and "config5" not in rec


def test_group_line_can_be_skipped():
    r = _run(["--gpus", "2", "--dry-run", "--no-group-line", "--no-config-lines"])
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert not isinstance(rec["group"], dict) and "config4" not in rec


def test_plain_bench_forms_three_ranks():
    r = _run(["--gpus", "3", "--dry-run", "--no-config-lines"])
    assert r.returncode == 0, r.stderr
    assert _json_line(r.stdout)["n_gpus"] == 3


def test_single_rank_dry_run():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1
    _config_lines(rec, 1)


def test_launcher_world_mismatch_fails_loudly():
    # a launcher that formed 1 rank while --gpus says 2: exit non-zero, print no result line
    r = _run(["--gpus", "2", "--dry-run", "--no-config-lines"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE 1" in r.stderr


def test_torchrun_launch_forms_two_ranks():
    env = _env()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29517", str(ROOT / "bench.py"),
                        "--gpus", "2", "--dry-run"], cwd=str(ROOT), env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["backend"] == "gloo"
    _has(rec["group"], GROUP_DRY)  # rank 0 ran the group child itself after the world closed
    _config_lines(rec, 2)  # ... and the config-4 / config-5 worlds


def test_usable_cores_reports_a_positive_count():
    sys.path.insert(0, str(ROOT))
    import bench

    n, how = bench.usable_cores()
    assert n >= 1 and n <= len(os.sched_getaffinity(0))
    assert how in ("sched_getaffinity", "cgroup cpu quota")


def test_group_mode_is_one_process_over_n_gpus():
    r = _run(["--gpus", "4", "--group", "--dry-run"])
    assert r.returncode == 0, r.stderr
    _has(_json_line(r.stdout), {"dry_run": True, "n_gpus": 4, "backend": "gloo", "group": True})
    assert "config4" not in _json_line(r.stdout)


def test_roofline_quotes_live_traffic_over_the_committed_file(monkeypatch):
    """bench.py measures roofline.traffic itself (rocprofv3 --pmc passes before the timed run) and
    quotes it instead of profiles/pmc_traffic.json; a launch of another size gets the live ratio."""
    import importlib

    monkeypatch.setattr(sys, "argv", ["bench.py"])
    importlib.import_module("bench")
    bench = importlib.import_module("benchlib.roofline")
    monkeypatch.delenv("PGH_BENCH_LIVE_TRAFFIC", raising=False)
    st = {"kernel_launches": 2, "kernel_ms_total": 13.0, "kernel_bytes_total": 2 * 1000, "kernel_busy_ms_total": 13.0}
    monkeypatch.setattr(bench, "LIVE_TRAFFIC", (1001.0, 1000, "live: test"))
    r = bench.roofline_of(st, "resnet18-fedavg", 0, "k_fedavg")
    assert r["traffic"] == 1001.0 and r["traffic_source"] == "live: test"
    monkeypatch.setattr(bench, "LIVE_TRAFFIC", (1001.0, 500, "live: test"))
    r = bench.roofline_of(st, "resnet18-fedavg", 0, "k_fedavg")
    assert abs(r["traffic"] - 2002.0) < 1e-9 and "ratio" in r["traffic_source"]
    monkeypatch.setattr(bench, "LIVE_TRAFFIC", None)
    assert bench.roofline_of(st, "resnet18-fedavg", 0, "k_fedavg")["traffic_source"] != "live: test"


def test_live_traffic_is_skipped_under_a_profiler(monkeypatch):
    import importlib

    monkeypatch.setattr(sys, "argv", ["bench.py"])
    bench = importlib.import_module("bench")
    monkeypatch.setenv("ROCPROF_COUNTERS", "FETCH_SIZE")
    assert bench.under_profiler()


def test_check_leg_compares_bit_for_bit(monkeypatch):
    """bench.check_sampled (the --check leg) on one rank: equal values pass, one flipped low bit of
    one sampled param fails."""
    import importlib
    import types

    import numpy as np
    import torch

    monkeypatch.setattr(sys, "argv", ["bench.py"])
    bench = importlib.import_module("bench")
    ctx = types.SimpleNamespace(torch=torch, world=1, rank=0, dist=None)
    args = types.SimpleNamespace(seed=3)
    full = torch.arange(1000, dtype=torch.float32) * 0.5
    ok = bench.check_sampled(ctx, args, full, 0, 1000, lambda idx: idx.astype(np.float32) * np.float32(0.5))
    assert ok["bit_exact"] and ok["mismatches"] == 0 and ok["params_checked"] >= 2

    def off_by_one_ulp(idx):
        v = idx.astype(np.float32) * np.float32(0.5)
        v.view(np.uint32)[-1] ^= 1
        return v
    bad = bench.check_sampled(ctx, args, full, 0, 1000, off_by_one_ulp)
    assert not bad["bit_exact"] and bad["mismatches"] == 1


def test_headline_printed_inside_the_budget_when_a_child_overruns():
    """VERDICT r4 next #1, at the driver's N = 8 geometry (torch.distributed.run, 8 ranks, gloo):
    a config child that sleeps past its limit is killed at it and its slot holds the timeout, the
    children after it are skipped for lack of budget, and rank 0 still prints the headline line
    inside --budget-s."""
    import time

    env = _env({"PGH_BENCH_STUB": "config1=0,config4=1000,config5=0,config3=0,group=0"})
    budget = 75
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29531", str(ROOT / "bench.py"),
                        "--gpus", "8", "--dry-run", "--budget-s", str(budget), "--headline-reserve-s", "35"],
                       cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=240)
    wall = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 8 and rec["dist_backend"] == "gloo"
    assert rec["config1"] == {"dry_run": True, "stub": "config1"}
    assert rec["config4"]["error"].startswith("timeout after") and rec["config4"]["stage"] == "config4"
    for key in ("config5", "config3", "group"):
        assert rec[key]["error"].startswith("skipped") and rec[key]["stage"] == key, rec[key]
    assert rec["budget"]["budget_s"] <= budget and rec["budget"]["stages_s"]["config4"] >= 20
    assert wall < budget + 15, wall  # + the launcher's own start and teardown


def test_watchdog_prints_the_headline_line_when_the_headline_cannot_finish():
    import time

    t0 = time.time()
    r = _run(["--dry-run", "--no-config-lines", "--budget-s", "25"], {"PGH_BENCH_STUB": "headline=300"}, timeout=120)
    assert time.time() - t0 < 40
    assert r.returncode == 3
    rec = _json_line(r.stdout)
    assert rec["value"] is None and rec["metric"].startswith("client-diff GB/s") and rec["stage"] == "headline"
    assert "did not finish within" in rec["error"]


def test_spawned_ranks_line_survives_a_hung_headline():
    """Without a launcher: the parent (no GPU) runs the child lines, spawns the ranks, and prints
    rank 0's watchdog line with the child lines merged in."""
    r = _run(["--gpus", "2", "--dry-run", "--budget-s", "50", "--headline-reserve-s", "25"],
             {"PGH_BENCH_STUB": "config1=0,config4=0,config5=0,config3=0,group=0,headline=300"}, timeout=150)
    assert r.returncode != 0
    rec = _json_line(r.stdout)
    assert rec["value"] is None and "did not finish within" in rec["error"]
    assert rec["config4"] == {"dry_run": True, "stub": "config4"}


def test_cpu_baseline_on_the_n8_line():
    """the driver's N = 8 launch (torch.distributed.run, 8 ranks) carries a
    measured cpu_baseline -- timed by rank 0 before the world forms, at the node's 1 thread and on
    every usable core, with the core count and CPU model, its sample size and whether the close
    figures are extrapolated from it.  (A 20 K-param shard and 1 s of CPU work keep the test short;
    the driver's run times the 11.7 M-param shard for --cpu-seconds, default 12.)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.pop("PGH_BENCH_STUB", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", str(ROOT / "bench.py"),
                        "--gpus", "8", "--dry-run", "--no-config-lines", "--no-group-line", "--params", "20000",
                        "--cpu-seconds", "1"], cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 8 and rec["dist_backend"] == "gloo"
    cb = rec["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] == "port" and cb["cpu_model"], cb
    assert cb["all_cores"]["cores"] >= 1 and cb["all_cores"]["value"] > 0, cb
    assert cb["sample_clients"] == 32 and cb["workload_clients"] == 1000 and cb["extrapolated"] is True
    assert "8-GPU world" in cb["measured"] and "cycle_manager.py:276-296" in cb["sample"]
    assert rec["budget"]["stages_s"]["cpu_baseline"] > 0
