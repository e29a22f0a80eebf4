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
