"""Render substitution rules as Graphviz (reference tools/substitutions_to_dot).

    python -m flexflow_amd.tools.substitutions_to_dot rules.json RULE_NAME out.dot
    python -m flexflow_amd.tools.substitutions_to_dot rules.json --all out_dir/

rules.json is the JSON rule format (the reference's substitutions/*.json, or the output of
flexflow_amd.tools.protobuf_to_json)."""
from __future__ import annotations

import json
import os
import sys

from types import SimpleNamespace as _NS

from ..utils.dot import rule_to_dot


def _as_rule(r):
    """JSON rule dict -> the attribute view rule_to_dot reads (same fields as the native Rule)."""
    def op(o):
        return _NS(type=str(o["type"]),
                   params=[_NS(key=p["key"], value=p["value"]) for p in o.get("para", [])],
                   inputs=[_NS(op_id=t["opId"], ts_id=t["tsId"]) for t in o.get("input", [])])
    return _NS(name=r["name"], src=[op(o) for o in r["srcOp"]], dst=[op(o) for o in r["dstOp"]])


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 3:
        print(__doc__, file=sys.stderr)
        return 1
    path, which, out = argv
    with open(path) as f:
        rules = json.load(f)["rule"]
    if which == "--all":
        os.makedirs(out, exist_ok=True)
        for r in rules:
            rule_to_dot(_as_rule(r), os.path.join(out, f"{r['name']}.dot"))
        print(f"{len(rules)} rules -> {out}")
        return 0
    for r in rules:
        if r.get("name") == which:
            rule_to_dot(_as_rule(r), out)
            return 0
    print(f"no rule named {which}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
