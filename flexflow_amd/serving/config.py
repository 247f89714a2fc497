"""Model configuration (`config.pbtxt`) of a model repository, Triton-compatible.

The reference's serving prototype is a Triton Inference Server backend
(triton/src/backend.cc, model.cc: `LegionModelState` reads the model's `config.pbtxt` through
Triton's API, triton/qa/L0_e2e/models/*/config.pbtxt). Here the server is ours, so the protobuf
*text format* is parsed directly (no protobuf package): scalars, quoted strings, enum words,
`[ ... ]` lists, nested `{ ... }` messages and repeated fields.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

_TOKEN = re.compile(r'\s*(?:#[^\n]*\n?|("(?:[^"\\]|\\.)*"|\'(?:[^\'\\]|\\.)*\')|([{}\[\]:,])|([^\s{}\[\]:,#"\']+))')


def _tokens(text: str):
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                return
            raise ValueError(f"config.pbtxt: cannot parse near {text[pos:pos + 30]!r}")
        pos = m.end()
        if m.group(1) is not None:
            yield ("str", m.group(1)[1:-1].encode().decode("unicode_escape"))
        elif m.group(2) is not None:
            yield ("p", m.group(2))
        elif m.group(3) is not None:
            yield ("w", m.group(3))


def _scalar(kind, v):
    if kind == "str":
        return v
    if v in ("true", "True"):
        return True
    if v in ("false", "False"):
        return False
    try:
        return int(v)
    except ValueError:
        try:
            return float(v)
        except ValueError:
            return v  # enum identifier (TYPE_FP32, KIND_GPU, ...)


def parse_pbtxt(text: str) -> Dict[str, list]:
    """Parse protobuf text format into {field: [values...]} (every field treated as repeated;
    messages become nested dicts of the same shape)."""
    toks = list(_tokens(text))
    i = 0

    def value():
        nonlocal i
        kind, v = toks[i]
        if kind == "p" and v == "{":
            i += 1
            return message("}")
        if kind == "p" and v == "[":
            i += 1
            out = []
            while not (toks[i][0] == "p" and toks[i][1] == "]"):
                if toks[i][0] == "p" and toks[i][1] == ",":
                    i += 1
                    continue
                out.append(value())
            i += 1
            return out
        i += 1
        return _scalar(kind, v)

    def message(end):
        nonlocal i
        msg: Dict[str, list] = {}
        while i < len(toks):
            kind, v = toks[i]
            if kind == "p" and v == end:
                i += 1
                return msg
            if kind == "p" and v in (",", ";"):
                i += 1
                continue
            if kind != "w":
                raise ValueError(f"config.pbtxt: expected a field name, got {v!r}")
            name = v
            i += 1
            if toks[i][0] == "p" and toks[i][1] == ":":
                i += 1
            val = value()
            lst = msg.setdefault(name, [])
            if isinstance(val, list):
                lst.extend(val)  # `dims: [4, 2]` / `input [ {...}, {...} ]`
            else:
                lst.append(val)
        if end is not None:
            raise ValueError("config.pbtxt: unbalanced braces")
        return msg

    return message(None)


# Triton data types <-> numpy
TRITON_TO_NP = {"TYPE_BOOL": np.bool_, "TYPE_UINT8": np.uint8, "TYPE_INT8": np.int8, "TYPE_INT16": np.int16,
                "TYPE_INT32": np.int32, "TYPE_INT64": np.int64, "TYPE_FP16": np.float16, "TYPE_FP32": np.float32,
                "TYPE_FP64": np.float64}
# KServe v2 / Triton HTTP "datatype" strings
WIRE_TO_NP = {"BOOL": np.bool_, "UINT8": np.uint8, "INT8": np.int8, "INT16": np.int16, "INT32": np.int32,
              "INT64": np.int64, "FP16": np.float16, "FP32": np.float32, "FP64": np.float64}
NP_TO_WIRE = {np.dtype(v): k for k, v in WIRE_TO_NP.items()}


@dataclass
class TensorSpec:
    name: str
    data_type: str
    dims: List[int]

    @property
    def np_dtype(self):
        return np.dtype(TRITON_TO_NP[self.data_type])

    @property
    def wire_type(self) -> str:
        return self.data_type[len("TYPE_"):]


@dataclass
class ModelConfig:
    name: str
    backend: str = "flexflow_amd"
    max_batch_size: int = 0
    inputs: List[TensorSpec] = field(default_factory=list)
    outputs: List[TensorSpec] = field(default_factory=list)
    instance_kind: str = "KIND_GPU"
    dynamic_batching: bool = False
    preferred_batch_size: List[int] = field(default_factory=list)
    max_queue_delay_us: int = 0

    @staticmethod
    def parse(text: str, default_name: str = "") -> "ModelConfig":
        d = parse_pbtxt(text)

        def one(msg, k, default=None):
            v = msg.get(k)
            return v[0] if v else default

        def specs(key):
            return [TensorSpec(one(t, "name"), one(t, "data_type", "TYPE_FP32"), [int(x) for x in t.get("dims", [])])
                    for t in d.get(key, [])]

        cfg = ModelConfig(name=one(d, "name", default_name), backend=one(d, "backend", "flexflow_amd"),
                          max_batch_size=int(one(d, "max_batch_size", 0)), inputs=specs("input"),
                          outputs=specs("output"))
        ig = d.get("instance_group")
        if ig:
            cfg.instance_kind = one(ig[0], "kind", "KIND_GPU")
        db = d.get("dynamic_batching")
        if db is not None:
            cfg.dynamic_batching = True
            m = db[0] if db and isinstance(db[0], dict) else {}
            cfg.preferred_batch_size = [int(x) for x in m.get("preferred_batch_size", [])]
            cfg.max_queue_delay_us = int(one(m, "max_queue_delay_microseconds", 0))
        return cfg

    def to_json(self) -> dict:
        """Model metadata in the KServe v2 `GET /v2/models/{name}` shape."""
        def t(s, batch):
            return {"name": s.name, "datatype": s.wire_type, "shape": ([-1] if batch else []) + list(s.dims)}
        b = self.max_batch_size > 0
        return {"name": self.name, "platform": "onnx_flexflow_amd", "backend": self.backend,
                "inputs": [t(s, b) for s in self.inputs], "outputs": [t(s, b) for s in self.outputs]}


def find_spec(specs: List[TensorSpec], name: str) -> Optional[TensorSpec]:
    for s in specs:
        if s.name == name:
            return s
    return None
