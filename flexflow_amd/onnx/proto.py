"""Minimal reader for ONNX ModelProto files (protobuf wire format), so `ONNXModel("model.onnx")`
works without the `onnx` package (not installed in this image).

Only the fields the converter uses are decoded (onnx/onnx.proto numbering):
  ModelProto     1 ir_version, 2 producer_name, 7 graph, 8 opset_import
  GraphProto     1 node, 2 name, 5 initializer, 11 input, 12 output
  NodeProto      1 input, 2 output, 3 name, 4 op_type, 5 attribute, 7 domain
  AttributeProto 1 name, 2 f, 3 i, 4 s, 5 t, 7 floats, 8 ints, 9 strings, 20 type
  TensorProto    1 dims, 2 data_type, 4 float_data, 5 int32_data, 7 int64_data, 8 name, 9 raw_data,
                 10 double_data
  ValueInfoProto 1 name, 2 type -> TypeProto 1 tensor_type -> 1 elem_type, 2 shape -> 1 dim ->
                 1 dim_value | 2 dim_param
The result is plain Python objects with the same attribute names as the onnx classes
(`model.graph.node[i].op_type`, `tensor.dims`, ...); a TensorProto also carries `.array` (numpy).
Nothing from the file is executed: it is parsed as data only.
"""
from __future__ import annotations

import struct
from types import SimpleNamespace
from typing import Dict

import numpy as np

from ..utils.protowire import fields as _fields
from ..utils.protowire import packed_f32 as _packed_f32
from ..utils.protowire import packed_varints as _packed_varints
from ..utils.protowire import signed as _signed

# TensorProto.DataType -> numpy
ONNX_DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64,
               9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}


def parse_tensor(b: bytes):
    t = SimpleNamespace(dims=[], data_type=1, name="", raw_data=b"", float_data=[], int32_data=[], int64_data=[],
                        double_data=[])
    for f, wt, v in _fields(b):
        if f == 1:
            t.dims += _packed_varints(v, wt)
        elif f == 2:
            t.data_type = v
        elif f == 4:
            t.float_data += _packed_f32(v, wt)
        elif f == 5:
            t.int32_data += _packed_varints(v, wt)
        elif f == 7:
            t.int64_data += _packed_varints(v, wt)
        elif f == 8:
            t.name = v.decode()
        elif f == 9:
            t.raw_data = bytes(v)
        elif f == 10:
            t.double_data += list(struct.unpack(f"<{len(v) // 8}d", v)) if wt == 2 else [struct.unpack("<d", v)[0]]
    dt = ONNX_DTYPES.get(t.data_type, np.float32)
    shape = tuple(int(d) for d in t.dims)
    if t.raw_data:
        arr = np.frombuffer(t.raw_data, dtype=dt).copy()
    elif t.float_data:
        arr = np.asarray(t.float_data, dtype=dt)
    elif t.int64_data:
        arr = np.asarray(t.int64_data, dtype=dt)
    elif t.int32_data:
        arr = np.asarray(t.int32_data, dtype=dt)
    elif t.double_data:
        arr = np.asarray(t.double_data, dtype=dt)
    else:
        arr = np.zeros(shape, dtype=dt)
    t.array = arr.reshape(shape)
    return t


def _parse_attribute(b: bytes):
    a = SimpleNamespace(name="", f=None, i=None, s=None, t=None, floats=[], ints=[], strings=[], type=0)
    for f, wt, v in _fields(b):
        if f == 1:
            a.name = v.decode()
        elif f == 2:
            a.f = struct.unpack("<f", v)[0]
        elif f == 3:
            a.i = _signed(v)
        elif f == 4:
            a.s = bytes(v)
        elif f == 5:
            a.t = parse_tensor(v)
        elif f == 7:
            a.floats += _packed_f32(v, wt)
        elif f == 8:
            a.ints += _packed_varints(v, wt)
        elif f == 9:
            a.strings.append(bytes(v))
        elif f == 20:
            a.type = v
    return a


def _parse_node(b: bytes):
    n = SimpleNamespace(input=[], output=[], name="", op_type="", attribute=[], domain="")
    for f, wt, v in _fields(b):
        if f == 1:
            n.input.append(v.decode())
        elif f == 2:
            n.output.append(v.decode())
        elif f == 3:
            n.name = v.decode()
        elif f == 4:
            n.op_type = v.decode()
        elif f == 5:
            n.attribute.append(_parse_attribute(v))
        elif f == 7:
            n.domain = v.decode()
    return n


def _parse_value_info(b: bytes):
    vi = SimpleNamespace(name="", elem_type=0, shape=[])
    for f, wt, v in _fields(b):
        if f == 1:
            vi.name = v.decode()
        elif f == 2:  # TypeProto
            for f2, _, v2 in _fields(v):
                if f2 != 1:  # tensor_type
                    continue
                for f3, _, v3 in _fields(v2):
                    if f3 == 1:
                        vi.elem_type = v3
                    elif f3 == 2:  # TensorShapeProto
                        for f4, _, v4 in _fields(v3):
                            if f4 != 1:
                                continue
                            d = None
                            for f5, _, v5 in _fields(v4):
                                if f5 == 1:
                                    d = int(v5)
                                elif f5 == 2:
                                    d = v5.decode()
                            vi.shape.append(d)
    return vi


def _parse_graph(b: bytes):
    g = SimpleNamespace(node=[], name="", initializer=[], input=[], output=[])
    for f, wt, v in _fields(b):
        if f == 1:
            g.node.append(_parse_node(v))
        elif f == 2:
            g.name = v.decode()
        elif f == 5:
            g.initializer.append(parse_tensor(v))
        elif f == 11:
            g.input.append(_parse_value_info(v))
        elif f == 12:
            g.output.append(_parse_value_info(v))
    return g


def load_model(path_or_bytes) -> SimpleNamespace:
    """Parse an .onnx file (or its bytes) into a ModelProto-shaped object."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        b = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as f:
            b = f.read()
    m = SimpleNamespace(ir_version=0, producer_name="", graph=None, opset_import=[])
    for f, wt, v in _fields(b):
        if f == 1:
            m.ir_version = v
        elif f == 2:
            m.producer_name = v.decode()
        elif f == 7:
            m.graph = _parse_graph(v)
        elif f == 8:
            ver = dom = None
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    dom = v2.decode()
                elif f2 == 2:
                    ver = v2
            m.opset_import.append(SimpleNamespace(domain=dom or "", version=ver))
    if m.graph is None:
        raise ValueError("not an ONNX ModelProto (no graph)")
    return m


def input_shapes(model) -> Dict[str, list]:
    """Graph inputs that are not initializers -> declared shape."""
    inits = {t.name for t in model.graph.initializer}
    return {vi.name: vi.shape for vi in model.graph.input if vi.name not in inits}


# ------------------------------------------------------------------------------- writer
_NP_TO_ONNX = {"float32": 1, "uint8": 2, "int8": 3, "int32": 6, "int64": 7, "bool": 9, "float16": 10, "float64": 11}


def _enc_tensor(name, arr) -> bytes:
    import numpy as np
    from ..utils.protowire import enc_bytes, enc_int
    a = np.ascontiguousarray(arr)
    out = b"".join(enc_int(1, d) for d in a.shape)
    out += enc_int(2, _NP_TO_ONNX[str(a.dtype)]) + enc_bytes(8, name) + enc_bytes(9, a.tobytes())
    return out


def _enc_value_info(name, shape, elem=1) -> bytes:
    from ..utils.protowire import enc_bytes, enc_int
    dims = b"".join(enc_bytes(1, enc_int(1, d) if isinstance(d, int) and d >= 0 else enc_bytes(2, str(d)))
                    for d in shape)
    tensor_type = enc_int(1, elem) + enc_bytes(2, dims)
    return enc_bytes(1, name) + enc_bytes(2, enc_bytes(1, tensor_type))


def _enc_attr(name, v) -> bytes:
    from ..utils.protowire import enc_bytes, enc_f32, enc_int
    out = enc_bytes(1, name)
    if isinstance(v, bool) or isinstance(v, int):
        return out + enc_int(3, int(v)) + enc_int(20, 2)
    if isinstance(v, float):
        return out + enc_f32(2, v) + enc_int(20, 1)
    if isinstance(v, (str, bytes)):
        return out + enc_bytes(4, v) + enc_int(20, 3)
    if isinstance(v, (list, tuple)) and all(isinstance(x, int) for x in v):
        return out + b"".join(enc_int(8, x) for x in v) + enc_int(20, 7)
    if isinstance(v, (list, tuple)):
        return out + b"".join(enc_f32(7, x) for x in v) + enc_int(20, 6)
    raise TypeError(f"attribute {name}: unsupported value {v!r}")


def make_model_bytes(nodes, inputs, outputs, initializers=None, opset=13, name="graph") -> bytes:
    """Serialize a small ONNX ModelProto (no onnx package needed): nodes = [(op_type, [in], [out],
    {attr: value}), ...], inputs/outputs = {name: shape}, initializers = {name: ndarray}. Used to
    build test models and model-repository fixtures."""
    from ..utils.protowire import enc_bytes, enc_int
    g = b""
    for k, (op, ins, outs, attrs) in enumerate(nodes):
        nb = b"".join(enc_bytes(1, i) for i in ins) + b"".join(enc_bytes(2, o) for o in outs)
        nb += enc_bytes(3, f"{op}_{k}") + enc_bytes(4, op)
        nb += b"".join(enc_bytes(5, _enc_attr(a, v)) for a, v in (attrs or {}).items())
        g += enc_bytes(1, nb)
    g += enc_bytes(2, name)
    for n, a in (initializers or {}).items():
        g += enc_bytes(5, _enc_tensor(n, a))
    for n, shp in inputs.items():
        g += enc_bytes(11, _enc_value_info(n, shp))
    for n, shp in outputs.items():
        g += enc_bytes(12, _enc_value_info(n, shp))
    return enc_int(1, 7) + enc_bytes(2, "flexflow_amd") + enc_bytes(7, g) + enc_bytes(8, enc_bytes(1, "") +
                                                                                     enc_int(2, opset))
