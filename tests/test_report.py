"""CPU: native base64 decode of reported diffs equals Python's base64.b64decode
(fl_events.py:257), including its non-validating edge cases."""
import base64
import binascii

import numpy as np
import pytest

from pygrid_amd.report import b64decode

CASES = ["QQ==", "QQ===", "QUJD", "QUJD=", "QUJD====", "QQ==QUJD", "QUJDRA==", "QU JD\nRA==", "QU*JD",
         "QUI=", "====", "", "Zm9vYmFy", "Zm9v\r\nYmFy\n",
         # '=' the decoder skips (fewer than 2 characters of the quad), padding then more data
         "9zWv=UyDn", "6=Za3/x/z", "=itfetOos", "yKViQhM9=aJrR", "=*u3sw", "QUI=\n=", "QU=I="]
BAD = ["QQ", "QQ=", "Q", "QUJDRA", "QUJDRA=", "QUI"]


@pytest.mark.parametrize("s", CASES)
def test_matches_python_edge_cases(s):
    assert b64decode(s) == base64.b64decode(s)


@pytest.mark.parametrize("s", BAD)
def test_bad_padding_raises_like_python(s):
    with pytest.raises(binascii.Error):
        base64.b64decode(s)
    with pytest.raises(binascii.Error):
        b64decode(s)


def test_fuzz_matches_python():
    """CPython 3.10 a2b_base64 (non-strict) state machine, on random short strings."""
    rng = np.random.default_rng(7)
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
    junk = alpha + "===\n *"
    for _ in range(20000):
        n = int(rng.integers(0, 17))
        s = "".join(junk[rng.integers(len(junk))] if rng.random() < 0.4 else alpha[rng.integers(64)]
                    for _ in range(n))
        try:
            want = base64.b64decode(s)
        except binascii.Error:
            want = None
        try:
            got = b64decode(s)
        except binascii.Error:
            got = None
        assert got == want, s


@pytest.mark.parametrize("threads", [1, 5])
def test_mime_lines_and_junk_large(threads):
    """76-character lines (base64.encodebytes) and junk: the parallel compaction path."""
    data = np.random.default_rng(3).integers(0, 256, 3_000_001, dtype=np.uint8).tobytes()
    enc = base64.encodebytes(data)
    assert b64decode(enc, threads=threads) == data
    dirty = enc.replace(b"A", b"A*", 1000) + b"=\n==QUJD"
    assert b64decode(dirty, threads=threads) == base64.b64decode(dirty)


@pytest.mark.parametrize("seed", range(6))
def test_junk_multithreaded_matches_python(seed):
    """Large inputs (threaded path) with junk bursts, quads split across chunk edges, and '='
    tricks near the end, for several thread counts."""
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, int(rng.integers(200_000, 400_000)), dtype=np.uint8).tobytes()
    enc = bytearray(base64.b64encode(data).rstrip(b"="))
    for pos in sorted(rng.integers(0, len(enc), 300), reverse=True):
        enc[pos:pos] = bytes(rng.choice(list(b" \n\r*~\t"), int(rng.integers(1, 40))))
    enc = bytes(enc) + [b"", b"=", b"==", b"=\n=QUJD", b"Q=", b"QUJD=="][seed]
    try:
        want = base64.b64decode(enc)
    except binascii.Error:
        want = None
    for th in (2, 3, 7, 16):
        try:
            got = b64decode(enc, threads=th)
        except binascii.Error:
            got = None
        assert got == want, th


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 1000, 1 << 20, (3 << 20) + 1, 12_000_001])
def test_random_payloads(n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc = base64.b64encode(data)
    assert b64decode(enc) == data
    assert b64decode(enc, threads=3) == data


def test_state_diff_roundtrip():
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import MNIST_SHAPES

    rng = np.random.default_rng(2)
    pb = build_state_fast([rng.standard_normal(s).astype(np.float32) for s in MNIST_SHAPES])
    assert b64decode(base64.b64encode(pb).decode()) == pb


@pytest.mark.parametrize("size", [300, 90_000, 1_200_001])
def test_every_byte_value_inside_a_clean_string(size):
    """The AVX2 fast path (fixed quad positions, pshufb range check) must hand every character
    outside the alphabet to the general path: each of the 256 byte values planted in a clean
    string, at a SIMD-block edge and mid-block, single- and multi-threaded."""
    rng = np.random.default_rng(size)
    enc = base64.b64encode(rng.integers(0, 256, size, dtype=np.uint8).tobytes()).rstrip(b"=")
    for pos in (31, 32, 45, len(enc) // 2, len(enc) - 5):
        for b in range(256):
            s = enc[:pos] + bytes([b]) + enc[pos:]
            try:
                want = base64.b64decode(s)
            except binascii.Error:
                want = None
            for th in ((1, 7) if size > 1_000_000 else (1,)):
                try:
                    got = b64decode(s, threads=th)
                except binascii.Error:
                    got = None
                assert got == want, (pos, b, th)


def test_fast_and_general_paths_agree():
    """The clean (AVX2) route on plain base64 text, the general route on the same bytes with line
    breaks (``base64.encodebytes``: not clean, so decoded by the general route)."""
    rng = np.random.default_rng(11)
    for n in (0, 1, 2, 3, 23, 24, 25, 47, 48, 49, 196_607, 196_608, 196_609, 1_000_000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert b64decode(base64.b64encode(data)) == data
        assert b64decode(base64.encodebytes(data)) == data


def test_decode_into_capacity_and_clean_size():
    import ctypes as C

    from pygrid_amd import _lib

    lib = _lib.load()
    data = np.random.default_rng(5).integers(0, 256, 100_000, dtype=np.uint8).tobytes()
    enc = base64.b64encode(data)
    n = C.c_size_t(0)
    assert lib.pgh_b64_clean_size(enc, len(enc), C.byref(n)) == 0 and n.value == len(data)
    small = (C.c_uint8 * 10)()
    assert lib.pgh_b64_decode_clean(enc, len(enc), small, 10, C.byref(n), 1) == -3  # PGH_E_STATE: too small
    buf = (C.c_uint8 * len(data))()
    assert lib.pgh_b64_decode_clean(enc, len(enc), buf, len(data), C.byref(n), 4) == 0
    assert bytes(buf) == data and n.value == len(data)
    mime = base64.encodebytes(data)
    assert lib.pgh_b64_decode_clean(mime, len(mime), buf, len(data), C.byref(n), 4) == -3  # not clean
    for junk in (b"**\n", b"*\n\r*"):  # the clean size is only a guess: decode_into checks it
        dirty = enc[:1000] + junk + enc[1000:]
        assert b64decode(dirty) == data
    bad_tail = enc[:-2] + b"Q"  # one character over a multiple of 4
    assert lib.pgh_b64_clean_size(bad_tail, len(bad_tail), C.byref(n)) == -5
    with pytest.raises(binascii.Error):
        b64decode(bad_tail)


def test_str_text_is_decoded_in_place():
    """The report's JSON yields a str: decoded from the str's own ASCII buffer (no encode copy),
    same bytes as base64.b64decode; non-ASCII text raises ValueError as base64 does."""
    import base64

    from pygrid_amd.report import b64decode

    data = np.random.default_rng(3).integers(0, 256, 300_001, dtype=np.uint8).tobytes()
    text = base64.b64encode(data).decode("ascii")
    assert b64decode(text) == base64.b64decode(text) == data
    assert b64decode(text[:1000]) == base64.b64decode(text[:1000])
    with pytest.raises(ValueError):
        base64.b64decode("QUJDé")
    with pytest.raises(ValueError):
        b64decode("QUJDé")


class _FakePinnedLib:
    """pgh_host_alloc / pgh_host_free over ordinary ctypes buffers (no GPU here); every other
    entry point is the real library's."""

    def __init__(self, real):
        import ctypes as C

        self._real, self._C = real, C
        self.live = {}
        self.allocs = self.frees = 0

    def pgh_host_alloc(self, n, out):
        buf = self._C.create_string_buffer(n)
        addr = self._C.addressof(buf)
        self.live[addr] = buf
        out._obj.value = addr
        self.allocs += 1
        return 0

    def pgh_host_free(self, p):
        del self.live[p.value]
        self.frees += 1
        return 0

    def __getattr__(self, name):
        return getattr(self._real, name)


def test_pinned_pool_decodes_into_blocks_and_recycles_them(monkeypatch):
    """report.b64decode(into=pool): the diff lands in a pool block (a read-only memoryview); the
    block returns when the last view is gone, is reused for the next report, a report with every
    block taken falls back to bytes, and close() frees idle blocks and late returns."""
    import base64
    import gc

    from pygrid_amd import _lib, report

    fake = _FakePinnedLib(_lib.load())
    monkeypatch.setattr(report._lib, "load", lambda: fake)
    rng = np.random.default_rng(9)
    raws = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (300_000, 200_001, 3_000_000)]
    texts = [base64.b64encode(r).decode() for r in raws]
    pool = report.PinnedPool(max_blocks=2)
    a = report.b64decode(texts[0], into=pool)
    assert isinstance(a, memoryview) and a.readonly and bytes(a) == raws[0]
    b = report.b64decode(texts[1] + "\n", into=pool)  # the general route, into a second block
    assert isinstance(b, memoryview) and bytes(b) == raws[1] and pool.blocks == 2
    c = report.b64decode(texts[1], into=pool)  # every block in use: ordinary bytes
    assert isinstance(c, bytes) and c == raws[1] and pool.misses == 1
    held = np.frombuffer(a, np.uint8)  # another reference (the DB layer, a parked report ...)
    del a
    gc.collect()
    d = report.b64decode(texts[1], into=pool)
    assert isinstance(d, bytes)  # a's block is still referenced through `held`
    del held, d
    gc.collect()
    e = report.b64decode(texts[1], into=pool)
    assert isinstance(e, memoryview) and bytes(e) == raws[1] and fake.allocs == 2  # reused
    f = report.b64decode(texts[2], into=pool)  # no block fits and none idle: bytes
    assert isinstance(f, bytes)
    del e
    gc.collect()
    g = report.b64decode(texts[2], into=pool)  # the idle block is too small: replaced
    assert isinstance(g, memoryview) and bytes(g) == raws[2] and fake.frees == 1 and pool.blocks == 2
    h = report.b64decode(texts[0], into=pool)  # both blocks in use (b, g): bytes
    assert isinstance(h, bytes)
    pool.close()
    assert fake.frees == 1  # nothing idle to free yet
    del b, g
    gc.collect()
    assert fake.frees == 3 and not fake.live  # the late returns are freed, not pooled


def test_pinned_pool_without_a_gpu_falls_back_to_bytes():
    import base64

    from pygrid_amd import report

    raw = bytes(range(256)) * 1000
    pool = report.PinnedPool()
    got = report.b64decode(base64.b64encode(raw), into=pool)
    assert got == raw  # bytes on a box without HIP devices, a memoryview on the GPU box
