"""Convert a TASO-format substitution rule collection (protobuf, GraphSubst.RuleCollection of the
reference's tools/protobuf_to_json/rules.proto) to the JSON rule format that
flexflow_amd.pcg.substitutions loads (--substitution-json).

    python -m flexflow_amd.tools.protobuf_to_json graph_subst.pb graph_subst.json

The file is decoded as data by flexflow_amd.utils.protowire (no protobuf runtime, no generated
code). The integer enums are the TASO rule numbering used inside those files, which differs from
the framework's OperatorType / PMParameter values.
"""
from __future__ import annotations

import json
import sys

from ..utils.protowire import fields, signed

# TASO rule-file numbering (operator types, parameter keys)
RULE_OP_TYPES = ["OP_INPUT", "OP_WEIGHT", "OP_ANY", "OP_CONV2D", "OP_DROPOUT", "OP_LINEAR", "OP_POOL2D_MAX",
                 "OP_POOL2D_AVG", "OP_RELU", "OP_SIGMOID", "OP_TANH", "OP_BATCHNORM", "OP_CONCAT", "OP_SPLIT",
                 "OP_RESHAPE", "OP_TRANSPOSE", "OP_EW_ADD", "OP_EW_MUL", "OP_MATMUL", "OP_MUL", "OP_ENLARGE",
                 "OP_MERGE_GCONV", "OP_CONSTANT_IMM", "OP_CONSTANT_ICONV", "OP_CONSTANT_ONE", "OP_CONSTANT_POOl",
                 "OP_PARTITION", "OP_COMBINE", "OP_REPLICATE", "OP_REDUCE", "OP_EMBEDDING"]
RULE_PARAMS = ["PM_OP_TYPE", "PM_NUM_INPUTS", "PM_NUM_OUTPUTS", "PM_GROUP", "PM_KERNEL_H", "PM_KERNEL_W",
               "PM_STRIDE_H", "PM_STRIDE_W", "PM_PAD", "PM_ACTI", "PM_NUMDIM", "PM_AXIS", "PM_PERM",
               "PM_OUTSHUFFLE", "PM_MERGE_GCONV_COUNT", "PM_PARALLEL_DIM", "PM_PARALLEL_DEGREE"]


def _name(table, v):
    return table[v] if 0 <= v < len(table) else v


def _parameter(b):
    key = value = 0
    for f, _, v in fields(b):
        if f == 1:
            key = signed(v)
        elif f == 2:
            value = signed(v)
    # values stay integers (activation / padding modes included), as in the reference's JSON files
    return {"_t": "Parameter", "key": _name(RULE_PARAMS, key), "value": value}


def _tensor(b):
    d = {"_t": "Tensor", "opId": 0, "tsId": 0}
    for f, _, v in fields(b):
        if f == 1:
            d["opId"] = signed(v)
        elif f == 2:
            d["tsId"] = signed(v)
    return d


def _operator(b):
    op = {"_t": "Operator", "input": [], "para": [], "type": None}
    for f, _, v in fields(b):
        if f == 1:
            op["type"] = _name(RULE_OP_TYPES, signed(v))
        elif f == 2:
            op["input"].append(_tensor(v))
        elif f == 3:
            op["para"].append(_parameter(v))
    return op


def _map_output(b):
    d = {"_t": "MapOutput", "dstOpId": 0, "dstTsId": 0, "srcOpId": 0, "srcTsId": 0}
    names = {1: "srcOpId", 2: "dstOpId", 3: "srcTsId", 4: "dstTsId"}
    for f, _, v in fields(b):
        if f in names:
            d[names[f]] = signed(v)
    return d


def convert(data: bytes) -> dict:
    rules = []
    for f, _, v in fields(data):
        if f != 1:
            continue
        r = {"_t": "Rule", "srcOp": [], "dstOp": [], "mappedOutput": []}
        for f2, _, v2 in fields(v):
            if f2 == 1:
                r["srcOp"].append(_operator(v2))
            elif f2 == 2:
                r["dstOp"].append(_operator(v2))
            elif f2 == 3:
                r["mappedOutput"].append(_map_output(v2))
        r["name"] = f"taso_rule_{len(rules)}"
        rules.append(r)
    return {"_t": "RuleCollection", "rule": rules}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2:
        print("usage: python -m flexflow_amd.tools.protobuf_to_json <input.pb> <output.json>", file=sys.stderr)
        return 1
    with open(argv[0], "rb") as f:
        out = convert(f.read())
    with open(argv[1], "w") as f:
        json.dump(out, f, indent=2)
    print(f"{len(out['rule'])} rules -> {argv[1]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
