"""tools/ (reference tools/protobuf_to_json, tools/substitutions_to_dot): the reference ships its
TASO rule collection both as protobuf and as JSON (substitutions/graph_subst_3_v2.{pb,json}); our
converter must reproduce the JSON exactly from the .pb, and the JSON must render as Graphviz."""
import json
import os

import pytest

from flexflow_amd.tools import protobuf_to_json, substitutions_to_dot

REF = "/root/reference/substitutions"
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "graph_subst_3_v2.pb")),
                                reason="reference substitution files not mounted")


def test_protobuf_to_json_reproduces_reference_json(tmp_path):
    out = tmp_path / "rules.json"
    assert protobuf_to_json.main([os.path.join(REF, "graph_subst_3_v2.pb"), str(out)]) == 0
    ours = json.loads(out.read_text())
    ref = json.load(open(os.path.join(REF, "graph_subst_3_v2.json")))
    assert len(ours["rule"]) == len(ref["rule"]) == 640
    assert ours == ref


def test_substitutions_to_dot(tmp_path):
    src = os.path.join(REF, "graph_subst_3_v2.json")
    dot = tmp_path / "r.dot"
    assert substitutions_to_dot.main([src, "taso_rule_0", str(dot)]) == 0
    text = dot.read_text()
    assert text.startswith("digraph") and "PARTITION" in text
    assert substitutions_to_dot.main([src, "--all", str(tmp_path / "all")]) == 0
    assert len(os.listdir(tmp_path / "all")) == 640
