"""CPU: the host parsers of untrusted input (client State bytes, base64 diff text) fuzzed under
ASan + UBSan (GPU sanitizers are not available on the pool; these sources have no HIP)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_state_and_b64_parsers_fuzz_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "fuzz_host"
    csrc = ROOT / "pygrid_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", str(ROOT / "include"), str(ROOT / "tests" / "native" / "fuzz_host.cpp"),
                    str(csrc / "pgh_state.cpp"), str(csrc / "pgh_b64.cpp"), "-pthread", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
    parsed = int(out.stdout.split("parsed=")[1].split()[0])
    assert parsed > 1000  # the fuzzer exercised valid messages too
