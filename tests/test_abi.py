"""CPU: the C-ABI library builds, loads and exports every symbol include/pgh_api.h declares;
the host-only State codec works without a GPU; the engine refuses to run without one."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    text = (ROOT / "include" / "pgh_api.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pgh_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from pygrid_amd import _lib

    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signatures out of sync with the header"
    assert lib.pgh_abi_version() == _lib.ABI_VERSION == 10
    assert b"pgh_create_group" in (ROOT / "pygrid_amd" / "libpygrid_hip.so").read_bytes()


def test_library_exports_no_undeclared_c_symbol():
    """The only unmangled functions the library exports are the header's: internal helpers stay
    internal (helpers in anonymous namespaces inside an ``extern "C"`` block used to be exported)."""
    import shutil
    import subprocess

    if not shutil.which("nm"):
        pytest.skip("nm not installed")
    out = subprocess.run(["nm", "-D", "--defined-only", str(ROOT / "pygrid_amd" / "libpygrid_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[2] for ln in out.splitlines() if len(ln.split()) == 3 and ln.split()[1] == "T"}
    c_names = {s for s in exported if not s.startswith("_Z")}
    assert c_names == set(declared_symbols()), sorted(c_names ^ set(declared_symbols()))


def test_library_has_gfx950_code_object():
    data = (ROOT / "pygrid_amd" / "libpygrid_hip.so").read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_library_does_not_link_torch():
    import subprocess

    out = subprocess.run(["readelf", "-d", str(ROOT / "pygrid_amd" / "libpygrid_hip.so")],
                         capture_output=True, text=True).stdout
    # only the dependency and search-path entries (a hex address may happen to read "c10")
    deps = [ln for ln in out.splitlines() if "(NEEDED)" in ln or "PATH)" in ln]
    assert deps and not any("torch" in ln or "libc10" in ln for ln in deps), deps


def test_engine_without_gpu_raises():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from pygrid_amd import Engine, EngineUnavailableError, device_count

    assert device_count() == 0
    with pytest.raises(EngineUnavailableError):
        Engine(0)


def test_null_and_bad_arguments_return_status():
    from pygrid_amd import _lib

    lib = _lib.load()
    assert lib.pgh_create(0, 0, None) == -1
    assert lib.pgh_set_layout(None, 1, None) == -1
    assert lib.pgh_stats(None, None) == -1
    assert lib.pgh_last_error(None) is not None


def test_plain_c_consumer_compiles_links_and_runs(tmp_path):
    """The header is valid C99 and the library links from C (what a cgo / JNI / N-API binding sees)."""
    import subprocess

    exe = tmp_path / "consumer"
    lib_dir = ROOT / "pygrid_amd"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "c_abi_consumer.c"), "-L", str(lib_dir), "-lpygrid_hip",
                    f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True)
    import torch

    if torch.cuda.is_available():
        return  # the run below checks the no-GPU error path
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, (out.returncode, out.stdout, out.stderr)
    assert out.stdout.startswith("ok")
