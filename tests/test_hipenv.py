"""hipenv.prepare: HIP hardware-queue count set before HIP initialises (profiles/r02u) -- only when
unset or asked for explicitly (PGH_HW_QUEUES), never on import."""
import os
import subprocess
import sys
from pathlib import Path

from pygrid_amd import hipenv

ROOT = Path(__file__).resolve().parent.parent


def test_sets_default_when_unset(monkeypatch):
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    monkeypatch.delenv("PGH_HW_QUEUES", raising=False)
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"


def test_keeps_an_operator_setting_lower_or_higher(monkeypatch):
    monkeypatch.delenv("PGH_HW_QUEUES", raising=False)
    for have in ("4", "24"):
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", have)
        hipenv.prepare()
        assert os.environ["GPU_MAX_HW_QUEUES"] == have


def test_explicit_request_wins_and_is_clamped(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    monkeypatch.setenv("PGH_HW_QUEUES", "4")
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"  # an explicit PGH_HW_QUEUES wins (A/B arms)
    monkeypatch.setenv("PGH_HW_QUEUES", "100")
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "32"


def test_bad_request_falls_back(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "x")
    monkeypatch.setenv("PGH_HW_QUEUES", "lots")
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"


def test_change_is_logged(monkeypatch, caplog):
    import logging

    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv("PGH_HW_QUEUES", "16")
    with caplog.at_level(logging.INFO, logger="pygrid_amd.hipenv"):
        hipenv.prepare()
    assert any("GPU_MAX_HW_QUEUES 4 -> 16" in r.getMessage() for r in caplog.records)


def test_bench_children_inherit():
    """bench.py asks for 16 queues at import (explicitly), before it spawns ranks or touches HIP."""
    env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "PGH_HW_QUEUES")}
    env["GPU_MAX_HW_QUEUES"] = "4"  # as on the GPU box
    code = "import sys, os; sys.argv = ['bench.py']; import bench; print(os.environ['GPU_MAX_HW_QUEUES'], bench.HW_QUEUES)"
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["16", "16"]


def test_import_leaves_the_process_alone():
    """`import pygrid_amd` changes neither GPU_MAX_HW_QUEUES nor glibc's mmap
    threshold.  The threshold is observed through its effect: a 47 MB allocation is mmapped by
    glibc's defaults (the program break does not move), carved from the heap once tuned."""
    code = ("import ctypes as C, os, sys\n"
            "libc = C.CDLL('libc.so.6'); libc.sbrk.restype = C.c_void_p; libc.sbrk.argtypes = [C.c_ssize_t]\n"
            "import pygrid_amd, pygrid_amd.cycle, pygrid_amd.incremental, pygrid_amd.node, pygrid_amd.report\n"
            "b0 = libc.sbrk(0); a = bytes(47_000_000); b1 = libc.sbrk(0); del a\n"
            "print(os.environ.get('GPU_MAX_HW_QUEUES', 'unset'), b1 - b0 >= 40_000_000)\n"
            "pygrid_amd.tune_process()\n"
            "b0 = libc.sbrk(0); a = bytes(47_000_000); b1 = libc.sbrk(0); del a\n"
            "print(os.environ.get('GPU_MAX_HW_QUEUES', 'unset'), b1 - b0 >= 40_000_000)\n")
    for have in (None, "4"):
        env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "PGH_HW_QUEUES", "PGH_MALLOC_TUNE")}
        if have:
            env["GPU_MAX_HW_QUEUES"] = have
        out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                             timeout=120)
        assert out.returncode == 0, out.stderr
        first, second = out.stdout.splitlines()
        assert first == f"{have or 'unset'} False"
        assert second == f"{have or '16'} True"  # tune_process: the operator's value kept, else 16
