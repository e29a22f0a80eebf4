"""hipenv.prepare: HIP hardware-queue count raised before HIP initialises (profiles/r02u)."""
import os
import subprocess
import sys
from pathlib import Path

from pygrid_amd import hipenv

ROOT = Path(__file__).resolve().parent.parent


def test_raises_default(monkeypatch):
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    monkeypatch.delenv("PGH_HW_QUEUES", raising=False)
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"


def test_raises_low_setting(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.delenv("PGH_HW_QUEUES", raising=False)
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"


def test_keeps_higher_setting(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    monkeypatch.delenv("PGH_HW_QUEUES", raising=False)
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "24"


def test_override_and_clamp(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    monkeypatch.setenv("PGH_HW_QUEUES", "4")
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"  # an explicit PGH_HW_QUEUES wins (A/B arms)
    monkeypatch.setenv("PGH_HW_QUEUES", "100")
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "32"


def test_bad_override_falls_back(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "x")
    monkeypatch.setenv("PGH_HW_QUEUES", "lots")
    hipenv.prepare()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"


def test_bench_children_inherit():
    """bench.py sets the variable at import, before it spawns ranks or touches HIP."""
    env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "PGH_HW_QUEUES")}
    code = "import sys, os; sys.argv = ['bench.py']; import bench; print(os.environ['GPU_MAX_HW_QUEUES'], bench.HW_QUEUES)"
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["16", "16"]
