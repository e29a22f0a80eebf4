"""Build-owned restatement of the syft-proto 0.5.2 messages on the cycle-close path.

syft-proto (``apps/node/poetry.lock:1731-1734``) is not in the image and no ``.proto`` file
or serialized fixture exists under the reference, so these field numbers are the build's
restatement, flagged "parity unpinned" in DESIGN.md.  They must agree with the constants in
``csrc/pgh_state.h``; ``tests/test_host_logic.py`` checks the C++ walker against Google's
protobuf runtime driven by this schema.

``classes()`` builds the messages with ``google.protobuf`` at run time (the runtime is
importable here; ``protoc`` is not), which the tests use to produce State bytes the way a
client's syft stack would.
"""
from __future__ import annotations

# (message, [(field name, number, type, label, type_name)]) ; label 1 = optional, 3 = repeated
PACKAGE = "syft_proto_restated"
MESSAGES = {
    "Id": [("id_str", 1, "string", 1, None), ("id_int", 2, "int64", 1, None)],
    "Size": [("dims", 1, "int32", 3, None)],
    "TensorData": [
        ("shape", 1, "message", 1, "Size"),
        ("dtype", 2, "string", 1, None),
        ("is_quantized", 3, "bool", 1, None),
        ("scale", 4, "float", 1, None),
        ("zero_point", 5, "int32", 1, None),
        ("contents_int64", 10, "int64", 3, None),
        ("contents_float32", 12, "float", 3, None),
        ("contents_float64", 13, "double", 3, None),
    ],
    "TorchTensor": [
        ("id", 1, "message", 1, "Id"),
        ("serializer", 2, "int32", 1, None),
        ("contents_bin", 3, "bytes", 1, None),
        ("contents_data", 4, "message", 1, "TensorData"),
        ("tags", 5, "string", 3, None),
        ("description", 6, "string", 1, None),
    ],
    "Parameter": [
        ("id", 1, "message", 1, "Id"),
        ("tensor", 2, "message", 1, "TorchTensor"),
        ("requires_grad", 3, "bool", 1, None),
        ("grad", 4, "message", 1, "TorchTensor"),
    ],
    "Placeholder": [
        ("id", 1, "message", 1, "Id"),
        ("tags", 2, "string", 3, None),
        ("description", 3, "string", 1, None),
        ("expected_shape", 4, "message", 1, "Size"),
    ],
    "StateTensor": [
        ("torch_tensor", 1, "message", 1, "TorchTensor"),
        ("torch_param", 2, "message", 1, "Parameter"),
    ],
    "State": [
        ("placeholders", 1, "message", 3, "Placeholder"),
        ("tensors", 2, "message", 3, "StateTensor"),
    ],
}
SERIALIZER_ALL = 4

_CLASSES = None


def classes():
    """Message classes built with google.protobuf's runtime from MESSAGES (proto3)."""
    global _CLASSES
    if _CLASSES is not None:
        return _CLASSES
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    types = {"string": F.TYPE_STRING, "int64": F.TYPE_INT64, "int32": F.TYPE_INT32, "bool": F.TYPE_BOOL,
             "float": F.TYPE_FLOAT, "double": F.TYPE_DOUBLE, "bytes": F.TYPE_BYTES, "message": F.TYPE_MESSAGE}
    fdp = descriptor_pb2.FileDescriptorProto(name="syft_state_restated.proto", package=PACKAGE, syntax="proto3")
    for mname, fields in MESSAGES.items():
        m = fdp.message_type.add(name=mname)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=types[typ],
                            label=F.LABEL_REPEATED if label == 3 else F.LABEL_OPTIONAL)
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    _CLASSES = {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{PACKAGE}.{name}"))
                for name in MESSAGES}
    return _CLASSES


def build_state(tensors, ids=None, as_param=False) -> bytes:
    """State bytes for a list of float32 arrays, shaped like syft's
    ``State(state_placeholders=[PlaceHolder().instantiate(t) ...])`` (model_manager.py:82-90)."""
    import numpy as np

    cls = classes()
    st = cls["State"]()
    for k, t in enumerate(tensors):
        a = np.asarray(t, dtype=np.float32)
        tid = (ids[k] if ids is not None else 1000 + k)
        ph = st.placeholders.add()
        ph.id.id_int = tid
        ph.tags.append(f"#state-{k}")
        stt = st.tensors.add()
        tt = stt.torch_param.tensor if as_param else stt.torch_tensor
        if as_param:
            stt.torch_param.id.id_int = tid
            stt.torch_param.requires_grad = True
        tt.id.id_int = tid
        tt.serializer = SERIALIZER_ALL
        tt.contents_data.shape.dims.extend(list(a.shape))
        tt.contents_data.dtype = "float32"
        tt.contents_data.contents_float32.extend(a.reshape(-1).tolist())
    return st.SerializeToString()


def build_state_i64(tensors, ids=None) -> bytes:
    """State bytes of int64 share tensors (TensorData.contents_int64, packed varint) via
    google.protobuf: what a syft stack would send for one party's additive shares."""
    import numpy as np

    cls = classes()
    st = cls["State"]()
    for k, t in enumerate(tensors):
        a = np.asarray(t, dtype=np.int64)
        tid = (ids[k] if ids is not None else 2000 + k)
        ph = st.placeholders.add()
        ph.id.id_int = tid
        stt = st.tensors.add()
        tt = stt.torch_tensor
        tt.id.id_int = tid
        tt.serializer = SERIALIZER_ALL
        tt.contents_data.shape.dims.extend(list(a.shape))
        tt.contents_data.dtype = "int64"
        tt.contents_data.contents_int64.extend(a.reshape(-1).tolist())
    return st.SerializeToString()


def parse_state_i64(pb: bytes):
    """[int64 array] of a share State via google.protobuf (independent of the C++ walker and
    the GPU decoder)."""
    import numpy as np

    st = classes()["State"]()
    st.ParseFromString(pb)
    out = []
    for stt in st.tensors:
        tt = stt.torch_tensor if stt.HasField("torch_tensor") else stt.torch_param.tensor
        shape = tuple(tt.contents_data.shape.dims)
        out.append(np.asarray(tt.contents_data.contents_int64, dtype=np.int64).reshape(shape))
    return out


def varint_encode(values) -> bytes:
    """Packed-varint bytes of int64 values (two's complement as uint64: negatives take 10 bytes),
    vectorised with numpy."""
    import numpy as np

    v = np.ascontiguousarray(values, dtype=np.int64).reshape(-1).view(np.uint64)
    if v.size == 0:
        return b""
    nbits = np.zeros(v.size, dtype=np.int64)
    x = v.copy()
    for _ in range(10):  # bytes per value: ceil(bit length / 7), at least 1
        nz = x != 0
        nbits += nz
        x >>= np.uint64(7)
    nb = np.maximum(nbits, 1)
    starts = np.concatenate(([0], np.cumsum(nb)[:-1]))
    out = np.empty(int(nb.sum()), dtype=np.uint8)
    for j in range(10):
        sel = nb > j
        byte = ((v[sel] >> np.uint64(7 * j)) & np.uint64(0x7F)).astype(np.uint8)
        byte |= np.where(nb[sel] > j + 1, 0x80, 0).astype(np.uint8)
        out[starts[sel] + j] = byte
    return out.tobytes()


def build_state_i64_fast(tensors, ids=None) -> bytes:
    """Byte-identical to ``build_state_i64(tensors, ids)`` with the varint payload encoded by numpy
    (``varint_encode``): for building large share messages (bench, tests)."""
    import numpy as np

    parts = []
    for k, t in enumerate(tensors):
        tid = ids[k] if ids is not None else 2000 + k
        parts.append(_field(1, 2, _field(1, 2, _field(2, 0, value=tid) if tid else b"")))
    for k, t in enumerate(tensors):
        a = np.ascontiguousarray(t, dtype=np.int64)
        tid = ids[k] if ids is not None else 2000 + k
        dims = b"".join(_varint(d) for d in a.shape)
        td = (_field(1, 2, _field(1, 2, dims) if dims else b"") + _field(2, 2, b"int64")
              + (_field(10, 2, varint_encode(a)) if a.size else b""))
        tt = (_field(1, 2, _field(2, 0, value=tid) if tid else b"") + _field(2, 0, value=SERIALIZER_ALL)
              + _field(4, 2, td))
        parts.append(_field(2, 2, _field(1, 2, tt)))
    return b"".join(parts)


def parse_state(pb: bytes):
    """[(shape, float32 array)] via google.protobuf (independent of the C++ walker)."""
    import numpy as np

    st = classes()["State"]()
    st.ParseFromString(pb)
    out = []
    for stt in st.tensors:
        tt = stt.torch_tensor if stt.HasField("torch_tensor") else stt.torch_param.tensor
        shape = tuple(tt.contents_data.shape.dims)
        out.append(np.asarray(tt.contents_data.contents_float32, dtype=np.float32).reshape(shape))
    return out


def _varint(x: int) -> bytes:
    out = bytearray()
    x &= (1 << 64) - 1
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wt: int, payload: bytes = b"", value: int = None) -> bytes:
    key = _varint((num << 3) | wt)
    if wt == 0:
        return key + _varint(value)
    return key + _varint(len(payload)) + payload


def build_state_fast(tensors, ids=None) -> bytes:
    """Byte-identical to ``build_state(tensors, ids)`` (as_param=False) without going through
    per-element Python protobuf calls: the float payload is spliced in as raw little-endian
    bytes.  For building large synthetic diffs (bench, tests)."""
    import numpy as np

    parts = []
    for k, t in enumerate(tensors):
        tid = ids[k] if ids is not None else 1000 + k
        pid = _field(2, 0, value=tid) if tid else b""
        ph = _field(1, 2, pid) + _field(2, 2, f"#state-{k}".encode())
        parts.append(_field(1, 2, ph))
    for k, t in enumerate(tensors):
        a = np.ascontiguousarray(t, dtype="<f4")
        tid = ids[k] if ids is not None else 1000 + k
        dims = b"".join(_varint(d) for d in a.shape)
        td = (_field(1, 2, _field(1, 2, dims) if dims else b"") + _field(2, 2, b"float32")
              + (_field(12, 2, a.tobytes()) if a.size else b""))
        tt = (_field(1, 2, _field(2, 0, value=tid) if tid else b"") + _field(2, 0, value=SERIALIZER_ALL)
              + _field(4, 2, td))
        parts.append(_field(2, 2, _field(1, 2, tt)))
    return b"".join(parts)


# ---- fresh checkpoint framing (serialize_model_params, model_manager.py:79-92) ----------------------

def _read_varint(b, i: int):
    x, shift = 0, 0
    while True:
        if i >= len(b):
            raise ValueError("truncated varint")
        c = b[i]
        i += 1
        x |= (c & 0x7F) << shift
        if not c & 0x80:
            return x, i
        shift += 7
        if shift > 63:
            raise ValueError("varint longer than 10 bytes")


def _fields(b, a: int, z: int):
    """(field number, wire type, value-or-(start, end)) of the message bytes b[a:z], payloads skipped
    by length (nothing is decoded)."""
    i = a
    while i < z:
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
            yield num, wt, v
        elif wt == 2:
            n, i = _read_varint(b, i)
            if i + n > z:
                raise ValueError("length-delimited field runs past its message")
            yield num, wt, (i, i + n)
            i += n
        elif wt == 5:
            i += 4
            yield num, wt, None
        elif wt == 1:
            i += 8
            yield num, wt, None
        else:
            raise ValueError(f"unsupported wire type {wt}")
    if i != z:
        raise ValueError("message overruns its bytes")


def tensor_shapes(pb: bytes):
    """Shape of every tensor of a State message, State order, from the framing alone (the float
    payloads are skipped, not parsed): the shapes the new checkpoint keeps (cycle_manager.py:293-296
    subtracts elementwise)."""
    b = memoryview(pb)
    shapes = []
    for num, wt, v in _fields(b, 0, len(b)):
        if num != 2 or wt != 2:  # State.tensors
            continue
        tt = None
        for n2, w2, v2 in _fields(b, *v):
            if n2 == 1 and w2 == 2:  # StateTensor.torch_tensor
                tt = v2
            elif n2 == 2 and w2 == 2:  # StateTensor.torch_param -> Parameter.tensor
                for n3, w3, v3 in _fields(b, *v2):
                    if n3 == 2 and w3 == 2:
                        tt = v3
        dims = []
        if tt is not None:
            for n3, w3, v3 in _fields(b, *tt):
                if n3 == 4 and w3 == 2:  # TorchTensor.contents_data -> TensorData.shape -> Size.dims
                    for n4, w4, v4 in _fields(b, *v3):
                        if n4 == 1 and w4 == 2:
                            for n5, w5, v5 in _fields(b, *v4):
                                if n5 == 1 and w5 == 0:
                                    dims.append(v5)
                                elif n5 == 1 and w5 == 2:  # packed int32
                                    i, z = v5
                                    while i < z:
                                        d, i = _read_varint(b, i)
                                        dims.append(d)
        shapes.append(tuple(int(d) for d in dims))
    return shapes


def tensor_dtypes(pb: bytes):
    """Per tensor of a State message, State order: the TensorData dtype string and the numbers of the
    contents fields present (10 int64, 12 float32, 13 float64; 3 = TorchTensor.contents_bin, a
    serializer other than "all"), from the framing alone.  ValueError on bytes that are not a
    State."""
    b = memoryview(pb)
    out = []
    for num, wt, v in _fields(b, 0, len(b)):
        if num != 2 or wt != 2:  # State.tensors
            continue
        tt = None
        for n2, w2, v2 in _fields(b, *v):
            if n2 == 1 and w2 == 2:
                tt = v2
            elif n2 == 2 and w2 == 2:
                for n3, w3, v3 in _fields(b, *v2):
                    if n3 == 2 and w3 == 2:
                        tt = v3
        dtype, contents = "", set()
        if tt is not None:
            for n3, w3, v3 in _fields(b, *tt):
                if n3 == 3 and w3 == 2:  # TorchTensor.contents_bin
                    contents.add(3)
                elif n3 == 4 and w3 == 2:  # TorchTensor.contents_data -> TensorData
                    for n4, w4, v4 in _fields(b, *v3):
                        if n4 == 2 and w4 == 2:
                            dtype = bytes(b[v4[0]:v4[1]]).decode("utf-8", "replace")
                        elif n4 in (10, 12, 13):
                            contents.add(n4)
        out.append((dtype, frozenset(contents)))
    return out


def non_float32_tensors(pb: bytes):
    """Indices of the tensors of a State message that are well-formed but not float32 (another
    dtype, float64 / int64 contents, or a non-"all" serializer's binary blob): the reference
    averages those with torch's type promotion, the engine does not.  ValueError on bytes that are
    not a State."""
    bad = []
    for k, (dtype, contents) in enumerate(tensor_dtypes(pb)):
        if dtype not in ("", "float32", "torch.float32") or not contents <= {12}:
            bad.append(k)
    return bad


_ID_RNG = None


def syft_ids(n: int, rng=None):
    """n fresh object ids from syft 0.2.9's id space (random ints below 10e10,
    ``create_random_id``), as PlaceHolder().instantiate(...) and new tensors get them."""
    global _ID_RNG
    import os
    import random

    if rng is None:
        if _ID_RNG is None:
            _ID_RNG = random.Random(int.from_bytes(os.urandom(16), "little"))
        rng = _ID_RNG
    return [int(10e10 * rng.random()) for _ in range(n)]


def fresh_frame(shapes, ids):
    """Framing of ``State(state_placeholders=[PlaceHolder().instantiate(p) for p in params])`` for
    float32 params of ``shapes`` (model_manager.py:82-90): per param a placeholder {id} (no tags) and a
    StateTensor.torch_tensor {id, serializer, contents_data {shape, dtype "float32",
    contents_float32}} -- plain tensors, as the reference's ``model_param - diff_param`` are.
    ``ids`` holds 2 per param (placeholder, tensor).  Every float payload is the last field of its
    tensor entry, so the message is: placeholders, then per tensor (prefix bytes, payload).
    Returns (total bytes, [(offset, prefix bytes)], [(payload offset, payload bytes)])."""
    pieces, spans = [], []
    head = b"".join(_field(1, 2, _field(1, 2, _field(2, 0, value=ids[2 * k]) if ids[2 * k] else b""))
                    for k in range(len(shapes)))
    pieces.append((0, head))
    pos = len(head)
    for k, shape in enumerate(shapes):
        n = 1
        for d in shape:
            n *= int(d)
        payload = 4 * n
        dims = b"".join(_varint(int(d)) for d in shape)
        tid = ids[2 * k + 1]
        td_head = _field(1, 2, _field(1, 2, dims) if dims else b"") + _field(2, 2, b"float32")
        td_pay = (_varint((12 << 3) | 2) + _varint(payload)) if n else b""
        td_len = len(td_head) + len(td_pay) + (payload if n else 0)
        tt_head = (_field(1, 2, _field(2, 0, value=tid) if tid else b"") + _field(2, 0, value=SERIALIZER_ALL)
                   + _varint((4 << 3) | 2) + _varint(td_len))
        tt_len = len(tt_head) + td_len
        st_head = _varint((1 << 3) | 2) + _varint(tt_len)
        st_len = len(st_head) + tt_len
        prefix = _varint((2 << 3) | 2) + _varint(st_len) + st_head + tt_head + td_head + td_pay
        pieces.append((pos, prefix))
        pos += len(prefix)
        spans.append((pos, payload if n else 0))
        pos += payload if n else 0
    return pos, pieces, spans
