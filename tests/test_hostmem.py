"""hostmem.tune: glibc mmap / trim thresholds for the node's 47 MB buffers (profiles/r02bk),
applied only through an explicit pygrid_amd.tune_process()."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(code, env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)


def test_tune_applies_on_glibc():
    r = _run("import pygrid_amd.hostmem as h; print(h.tune())", {})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "True"


def test_opt_out():
    r = _run("import pygrid_amd.hostmem as h; print(h.tune())", {"PGH_MALLOC_TUNE": "0"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "False"


def test_trim_threshold_fits_mallopts_int():
    """2 GiB passed through mallopt's int wraps to -2^31 (trimming off for good)."""
    from pygrid_amd import hostmem

    assert 0 < hostmem.TRIM_THRESHOLD <= 2**31 - 1
    assert 0 < hostmem.MMAP_THRESHOLD <= 2**31 - 1


def test_big_buffers_come_from_the_heap_after_tuning_and_heap_is_trimmed():
    """With the thresholds raised, a 47 MB bytes object is carved from the heap (the program break
    moves); without them glibc maps it on its own.  Freed heap above the trim threshold goes back
    to the OS (the break comes down), which the wrapped 2 GiB value never allowed."""
    code = ("import ctypes as C, sys, pygrid_amd\n"
            "pygrid_amd.tune_process(hw_queues=False)\n"
            "libc = C.CDLL('libc.so.6'); libc.sbrk.restype = C.c_void_p; libc.sbrk.argtypes = [C.c_ssize_t]\n"
            "b0 = libc.sbrk(0); a = bytes(47_000_000); b1 = libc.sbrk(0); del a\n"
            "big = [bytes(200_000_000) for _ in range(7)]; top = libc.sbrk(0); del big\n"
            "print(b1 - b0 >= 40_000_000, libc.sbrk(0) < top)")
    for tune, want in (("1", "True True"), ("0", "False")):
        r = _run(code, {"PGH_MALLOC_TUNE": tune})
        assert r.returncode == 0, r.stderr
        assert r.stdout.strip().startswith(want), (tune, r.stdout)
