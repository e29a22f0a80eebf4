"""CPU: native base64 decode of reported diffs equals Python's base64.b64decode
(fl_events.py:257), including its non-validating edge cases."""
import base64
import binascii

import numpy as np
import pytest

from pygrid_amd.report import b64decode

CASES = ["QQ==", "QQ===", "QUJD", "QUJD=", "QUJD====", "QQ==QUJD", "QUJDRA==", "QU JD\nRA==", "QU*JD",
         "QUI=", "====", "", "Zm9vYmFy", "Zm9v\r\nYmFy\n"]
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
