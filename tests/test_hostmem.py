"""hostmem.tune: glibc mmap / trim thresholds for the node's 47 MB buffers (profiles/r02bk)."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(env_extra):
    code = ("import ctypes as C, pygrid_amd, pygrid_amd.hostmem as h; "
            "print(h.tune())")
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)


def test_tune_applies_on_glibc():
    r = _run({})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "True"


def test_opt_out():
    r = _run({"PGH_MALLOC_TUNE": "0"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "False"


def test_big_buffers_come_from_the_heap_after_tuning():
    """With the thresholds raised, a 47 MB bytes object is carved from the heap (the program
    break moves) and stays there when freed; without them glibc maps it on its own."""
    code = ("import ctypes as C, sys, pygrid_amd\n"
            "libc = C.CDLL('libc.so.6'); libc.sbrk.restype = C.c_void_p; libc.sbrk.argtypes = [C.c_ssize_t]\n"
            "b0 = libc.sbrk(0); a = bytes(47_000_000); b1 = libc.sbrk(0); del a\n"
            "print(b1 - b0 >= 47_000_000)")
    for tune, want in (("1", "True"), ("0", "False")):
        r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, PGH_MALLOC_TUNE=tune))
        assert r.returncode == 0, r.stderr
        assert r.stdout.strip() == want, tune
