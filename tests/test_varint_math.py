"""CPU restatement of K4's arithmetic (pgh_kernels.hip: varint_at, term_mask16), checked against
the protobuf varint encoding of random int64 values of every length -- the identities the kernel
relies on, without a GPU:

* a value of `len` bytes b_0..b_{len-1} followed by arbitrary bytes: with raw = sum_{i<10} b_i 128^i
  (mod 2^64, bytes taken whole, continuation bits included), (raw - K10) mod 2^(7 len) is the
  value, K10 = sum_{j=1..9} 2^(7j); the kernel takes it as ((raw - K10) << cut) >> cut with
  cut = max(57 - 7 (len - 1), 0);
* raw as the kernel builds it: byte dot products (1, 128) over byte pairs, combined as
  a + (b << 28) + (c << 56) with a = p01 + (p23 << 14), b = p45 + (p67 << 14), c = p89;
* the terminator mask of 16 bytes as two pairs of byte dot products of ~v & 0x80808080.
"""
import numpy as np

from pygrid_amd.state_schema import varint_encode

M64 = (1 << 64) - 1
K10 = sum(1 << (7 * j) for j in range(1, 10))


def dot4(x: int, w: int, acc: int = 0) -> int:
    """v_dot4_u32_u8: sum of the four byte products plus acc, mod 2^32."""
    return (acc + sum(((x >> (8 * k)) & 0xFF) * ((w >> (8 * k)) & 0xFF) for k in range(4))) & 0xFFFFFFFF


def varint_at(buf: bytes, s: int, e: int) -> int:
    """The kernel's varint_at on bytes buf[s .. s + 12) (value bytes s..e, then what follows)."""
    w0, w1, w2 = (int.from_bytes(buf[s + 4 * k: s + 4 * k + 4], "little") for k in range(3))
    lo, hi = 0x00008001, 0x80010000
    a = (dot4(w0, lo) + (dot4(w0, hi) << 14)) & 0xFFFFFFFF
    b = (dot4(w1, lo) + (dot4(w1, hi) << 14)) & 0xFFFFFFFF
    c = dot4(w2, lo)
    raw = (a + (b << 28) + (c << 56)) & M64
    cut = max(57 - 7 * (e - s), 0)
    return ((((raw - K10) & M64) << cut) & M64) >> cut


def term_mask16(v: bytes) -> int:
    t = [~int.from_bytes(v[4 * k: 4 * k + 4], "little") & 0x80808080 for k in range(4)]
    m01 = dot4(t[0], 0x08040201, dot4(t[1], 0x80402010))
    m23 = dot4(t[2], 0x08040201, dot4(t[3], 0x80402010))
    return ((m01 >> 7) | (m23 << 1)) & 0xFFFF


def values_of_every_length(rng, n):
    bits = rng.integers(0, 65, n)
    v = [int(rng.integers(0, 1 << 62)) << 2 | int(rng.integers(0, 4)) for _ in range(n)]
    out = [x & ((1 << int(k)) - 1) for x, k in zip(v, bits)]
    return out + [0, 1, 127, 128, (1 << 56) - 1, 1 << 56, (1 << 63) - 1, 1 << 63, M64]


def test_varint_at_every_length_with_garbage_after():
    rng = np.random.default_rng(0)
    for u in values_of_every_length(rng, 3000):
        enc = varint_encode(np.array([u], dtype=np.uint64).view(np.int64))
        n = len(enc)
        assert 1 <= n <= 10
        tail = bytes(rng.integers(0, 256, 16, dtype=np.uint8))  # the next values' bytes
        lead = bytes(rng.integers(0, 256, 3, dtype=np.uint8))
        buf = lead + enc + tail
        s = len(lead)
        assert varint_at(buf, s, s + n - 1) == u, (hex(u), n)


def test_term_mask16_matches_bitwise():
    rng = np.random.default_rng(1)
    for _ in range(2000):
        v = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        want = sum(1 << k for k in range(16) if v[k] < 0x80)
        assert term_mask16(v) == want
