"""CPU: the iterative fold's division shortcut (div_by_count in pgh_kernels.hip) equals IEEE
float32 division for every operand the fold can meet (tests/native/recip_div_check.c explains
why; here 2 x 10^7 random and adversarial pairs plus every 37th subnormal)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_reciprocal_multiply_equals_ieee_division(tmp_path):
    exe = tmp_path / "recip_div_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", str(ROOT / "tests" / "native" / "recip_div_check.c"), "-lm",
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "10000000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
