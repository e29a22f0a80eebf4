"""CPU: the fresh checkpoint framing of serialize_model_params (model_manager.py:79-92) and the
shape walker it is built from (pygrid_amd/state_schema.py), against Google's protobuf runtime driven
by the restated schema (schema parity unpinned: DESIGN.md "State codec")."""
import numpy as np
import pytest

from pygrid_amd import state_schema as S
from pygrid_amd.state import serialize_fresh
from pygrid_amd.workloads import MNIST_SHAPES, RESNET18_SHAPES

F = np.float32


def reference_message(arrs, ids):
    """What syft's _bufferize of State(state_placeholders=[PlaceHolder().instantiate(p)]) holds,
    built field by field with google.protobuf."""
    st = S.classes()["State"]()
    for k, a in enumerate(arrs):
        ph = st.placeholders.add()
        ph.id.id_int = ids[2 * k]
        tt = st.tensors.add().torch_tensor
        tt.id.id_int = ids[2 * k + 1]
        tt.serializer = S.SERIALIZER_ALL
        tt.contents_data.shape.dims.extend(list(a.shape))
        tt.contents_data.dtype = "float32"
        tt.contents_data.contents_float32.extend(a.reshape(-1).tolist())
    return st.SerializeToString()


@pytest.mark.parametrize("shapes", [MNIST_SHAPES, RESNET18_SHAPES[:9], [(3,), (0,), (2, 0), (1,), (5, 1, 2)]])
def test_fresh_frame_is_byte_identical_to_protobuf(shapes):
    rng = np.random.default_rng(len(shapes))
    arrs = [rng.standard_normal(s).astype(F) for s in shapes]
    ids = S.syft_ids(2 * len(shapes), rng=__import__("random").Random(7))
    fresh = serialize_fresh(shapes, np.concatenate([a.reshape(-1) for a in arrs]), ids)
    assert fresh == reference_message(arrs, ids)
    total, pieces, spans = S.fresh_frame(shapes, ids)
    assert total == len(fresh) and len(spans) == len(shapes)
    for (off, n), a in zip(spans, arrs):
        assert fresh[off:off + n] == a.astype("<f4").tobytes()


def test_zero_ids_are_omitted_like_proto3_defaults():
    arrs = [np.ones((2, 2), F)]
    assert serialize_fresh([(2, 2)], arrs[0].reshape(-1), [0, 0]) == reference_message(arrs, [0, 0])


@pytest.mark.parametrize("as_param", [False, True])
def test_tensor_shapes_walker(as_param):
    rng = np.random.default_rng(3)
    shapes = [(7, 3), (3,), (0,), (2, 1, 4)]
    pb = S.build_state([rng.standard_normal(s).astype(F) for s in shapes], as_param=as_param)
    assert S.tensor_shapes(pb) == [tuple(s) for s in shapes]
    assert S.tensor_shapes(S.build_state_fast([np.zeros(s, F) for s in shapes])) == [tuple(s) for s in shapes]


def test_tensor_shapes_rejects_truncated_framing():
    pb = S.build_state_fast([np.zeros((4, 4), F)])
    with pytest.raises(ValueError):
        S.tensor_shapes(pb[:-3])


def test_syft_id_space():
    ids = S.syft_ids(1000)
    assert all(0 <= i < 10e10 for i in ids) and len(set(ids)) > 990


@pytest.mark.parametrize("shapes", [MNIST_SHAPES, RESNET18_SHAPES, [(3,), (0,), (2, 0), (1,), (5, 1, 2)]])
def test_native_fresh_frame_matches_the_restatement(shapes):
    """pgh_state_fresh (C++, the product path) == state_schema.fresh_frame (Python restatement)."""
    import ctypes as C

    from pygrid_amd.state import fresh_frame_bytes

    rng = np.random.default_rng(5)
    arrs = [rng.standard_normal(s).astype(F) for s in shapes]
    tmpl = S.build_state(arrs, as_param=True)  # the template's own framing differs (Parameters, tags)
    ids = S.syft_ids(2 * len(shapes))
    out, ptr = fresh_frame_bytes(tmpl, ids)
    total, pieces, spans = S.fresh_frame(shapes, ids)
    assert len(out) == total
    for (off, n), a in zip(spans, arrs):  # fill the payloads as the engine would
        C.memmove(ptr + off, a.astype("<f4").tobytes(), n)
    assert out == reference_message(arrs, ids)


def test_native_fresh_frame_rejects_bad_ids():
    from pygrid_amd import _lib

    import ctypes as C
    lib = _lib.load()
    tmpl = S.build_state_fast([np.zeros(3, F)])
    need = C.c_size_t(0)
    arr = (C.c_int64 * 1)(5)
    assert lib.pgh_state_fresh(tmpl, len(tmpl), arr, 1, None, 0, C.byref(need)) == -1  # 2 ids per tensor
