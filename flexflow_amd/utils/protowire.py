"""Generic protobuf wire-format decoding (no generated classes, no protobuf runtime): the files we
read — ONNX models (flexflow_amd/onnx/proto.py) and the reference's legacy strategy files
(flexflow_amd/pcg/strategy.py: load_strategy_pb) — are parsed as data only."""
from __future__ import annotations

import struct
from typing import List, Tuple


def varint(b: bytes, i: int) -> Tuple[int, int]:
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, i
        s += 7


def fields(b: bytes) -> List[Tuple[int, int, object]]:
    """(field number, wire type, value) for every field of one message."""
    out, i, n = [], 0, len(b)
    while i < n:
        key, i = varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.append((f, wt, v))
    return out


def signed(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


def packed_varints(v, wt) -> List[int]:
    if wt == 0:
        return [signed(v)]
    vals, i = [], 0
    while i < len(v):
        x, i = varint(v, i)
        vals.append(signed(x))
    return vals


def packed_f32(v, wt) -> List[float]:
    if wt == 5:
        return [struct.unpack("<f", v)[0]]
    return list(struct.unpack(f"<{len(v) // 4}f", v))


# ------------------------------------------------------------------------------- encoding
def enc_varint(v: int) -> bytes:
    v &= (1 << 64) - 1  # negative int64 -> two's complement, 10 bytes
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def enc_key(field: int, wire_type: int) -> bytes:
    return enc_varint((field << 3) | wire_type)


def enc_int(field: int, v: int) -> bytes:
    return enc_key(field, 0) + enc_varint(int(v))


def enc_bytes(field: int, v) -> bytes:
    b = v.encode() if isinstance(v, str) else bytes(v)
    return enc_key(field, 2) + enc_varint(len(b)) + b


def enc_f32(field: int, v: float) -> bytes:
    import struct
    return enc_key(field, 5) + struct.pack("<f", float(v))
