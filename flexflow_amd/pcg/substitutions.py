"""Graph substitutions on the layer graph (reference Unity GraphXfer machinery:
src/runtime/substitution.cc, substitution_loader.cc; rule data substitutions/*.json).

Rules use the reference's JSON rule-collection format and are parsed + matched natively
(flexflow_amd._core.load_rules / match_rule over a typed graph). The layer graph is exported as
GNodes whose weight parameters appear as extra inputs, so TASO-style rules that treat weights as
tensors (OP_LINEAR with inputs (x, w)) bind our Parameters through their external tensor ids.

Two phases, as in the reference's search:
  * fusion rules (name prefix `fuse_`, shipped in substitutions/flexflow_amd_rules.json) are
    always profitable on MI355X — one kernel instead of two, one HBM round trip less — and are
    applied greedily to a fixed point;
  * every other rule (e.g. the 640 TASO rules of graph_subst_3_v2.json via --substitution-json)
    is applied only when the cost model says the rewritten graph is faster (best-first with the
    --search-alpha pruning of GraphSearchHelper::base_optimize), bounded by --budget.
Rewrites are materialised when every destination op maps onto an op we can build from the
matched ones (same type reusing its weights / attributes, activations folded into PM_ACTI,
parameter-free element-wise ops); others are skipped.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

from ..type import ActiMode, OperatorType

TASO_ACTI = {ActiMode.AC_MODE_NONE: 0, ActiMode.AC_MODE_SIGMOID: 1, ActiMode.AC_MODE_RELU: 2,
             ActiMode.AC_MODE_TANH: 3, ActiMode.AC_MODE_GELU: 4}
ACTI_FROM_TASO = {v: k for k, v in TASO_ACTI.items()}
WEIGHT_BASE = -1000000  # pseudo-node ids for weight parameters

BUILTIN = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                       "substitutions", "flexflow_amd_rules.json")


def _core():
    from flexflow_amd import _core
    return _core


def export_graph(layers):
    """layers -> (GNode list, weight id map). Inputs of op i: its tensors then its weights."""
    core = _core()
    owner = {}
    for i, L in enumerate(layers):
        for j, o in enumerate(L.outputs):
            owner[o.guid] = (i, j)
    widx: Dict[int, object] = {}
    nodes = []
    for i, L in enumerate(layers):
        g = core.GNode()
        g.type = L.op_type.name
        params = {}
        act = L.attrs.get("activation")
        if isinstance(act, ActiMode):
            params["PM_ACTI"] = TASO_ACTI.get(act, 0)
        if "axis" in L.attrs:
            params["PM_AXIS"] = int(L.attrs["axis"])
        if "num_heads" in L.attrs:
            params["PM_NUM_HEADS"] = int(L.attrs["num_heads"])
        g.params = params
        ins = []
        for t in L.inputs:
            ins.append(owner.get(t.guid, (-1 - (t.guid % 100000), 0)))
        for w in L.weights:
            wid = WEIGHT_BASE - (w.guid % 100000)
            widx[wid] = w
            ins.append((wid, 0))
        g.inputs = ins
        g.num_outputs = len(L.outputs)
        nodes.append(g)
    return nodes, widx


def load_rules(paths: List[str]):
    core = _core()
    rules = []
    for p in paths:
        if p and os.path.exists(p):
            rules += list(core.load_rules(p))
    return rules


def _tensor_of(layers, ref):
    node, idx = ref
    if node < 0:
        return None
    return layers[node].outputs[idx]


def apply_rule(model, rule, match) -> bool:
    """Materialise one match of `rule` in model.layers. Returns False if unsupported."""
    from ..core.layer import Layer
    layers = model.layers
    src_layers = [layers[i] for i in match.op_nodes]
    by_type: Dict[str, List] = {}
    for L in src_layers:
        by_type.setdefault(L.op_type.name, []).append(L)
    ext_t = {}
    for eid, ref in match.ext.items():
        if ref[0] <= WEIGHT_BASE + 100000 and ref[0] < -1000:
            continue
        t = _tensor_of(layers, ref)
        if t is None:  # graph input without producer
            return False
        ext_t[eid] = t
    # build destination layers
    new_layers = []
    used = {k: 0 for k in by_type}
    dst_out = {}
    for k, d in enumerate(rule.dst):
        try:
            op_type = OperatorType[d.type]
        except KeyError:
            return False
        tmpl_list = by_type.get(d.type, [])
        tmpl = tmpl_list[used.get(d.type, 0)] if used.get(d.type, 0) < len(tmpl_list) else None
        ins = []
        for t in d.inputs:
            if t.op_id >= 0:
                ins.append(dst_out[(t.op_id, t.ts_id)])
            elif t.op_id in ext_t:
                ins.append(ext_t[t.op_id])
            # weight tensors (bound to Parameters) are carried by the template layer
        if tmpl is not None:
            attrs = dict(tmpl.attrs)
            for p in d.params:
                if p.key == "PM_ACTI":
                    attrs["activation"] = ACTI_FROM_TASO.get(p.value, ActiMode.AC_MODE_NONE)
            if op_type == OperatorType.OP_LAYERNORM:
                n_in = len(ins)
                if n_in not in (1, 2):
                    return False
            elif len(ins) != len(tmpl.inputs):
                return False
            L = Layer(model, op_type, tmpl.name + "+", ins, attrs)
            if [w.dims for w in L.weights] != [w.dims for w in tmpl.weights]:
                return False
            L.weights = list(tmpl.weights)
            used[d.type] = used.get(d.type, 0) + 1
        else:
            # parameter-free op created by the rule
            if op_type.name in ("OP_RELU", "OP_SIGMOID", "OP_TANH", "OP_GELU", "OP_IDENTITY", "OP_EW_ADD",
                                "OP_EW_MUL", "OP_EW_SUB", "OP_CONCAT"):
                attrs = {}
                for p in d.params:
                    if p.key == "PM_AXIS":
                        attrs["axis"] = p.value
                L = Layer(model, op_type, None, ins, attrs)
            else:
                return False
        new_layers.append(L)
        for j, o in enumerate(L.outputs):
            dst_out[(k, j)] = o
    # rewire consumers of mapped outputs
    remap = {}
    for m in rule.mapped:
        old = src_layers[m.src_op].outputs[m.src_ts]
        new = dst_out[(m.dst_op, m.dst_ts)]
        if tuple(old.dims) != tuple(new.dims):
            return False
        remap[old.guid] = new
    removed = set(id(L) for L in src_layers)
    kept = [L for L in layers if id(L) not in removed]
    for L in kept:
        L.inputs = [remap.get(t.guid, t) for t in L.inputs]
    # tensors a user still holds (e.g. an ONNX graph output served by name) resolve through this
    getattr(model, "_tensor_remap", {}).update(remap)
    if model._output is not None and model._output.guid in remap:
        model._output = remap[model._output.guid]
    # the final output tensor object changes: keep `output_tensor()` pointing at the same role
    model.layers = _toposort(kept + new_layers)
    return True


def _toposort(layers):
    prod = {}
    for L in layers:
        for o in L.outputs:
            prod[o.guid] = L
    seen, out = set(), []

    def visit(L):
        if id(L) in seen:
            return
        seen.add(id(L))
        for t in L.inputs:
            p = prod.get(t.guid)
            if p is not None:
                visit(p)
        out.append(L)

    order = {id(L): i for i, L in enumerate(layers)}
    for L in sorted(layers, key=lambda x: order[id(x)]):
        visit(L)
    return out


def greedy_fusions(model, rules, max_rounds=10000) -> List[str]:
    applied = []
    core = _core()
    fuse = [r for r in rules if r.name.startswith("fuse_")]
    for _ in range(max_rounds):
        nodes, _ = export_graph(model.layers)
        done = False
        for r in fuse:
            for m in core.match_rule(r, nodes, 1):
                # output of the last matched op must stay the model output if it was
                if apply_rule(model, r, m):
                    applied.append(r.name)
                    done = True
                    break
            if done:
                break
        if not done:
            break
    return applied


def optimize_graph(model, cost_fn=None, budget: int = 0, alpha: float = 1.05) -> dict:
    """Apply greedy fusions, then (if cost_fn/budget) cost-checked general rules."""
    cfg = model.config
    paths = [BUILTIN]
    if cfg.substitution_json_path:
        paths.append(cfg.substitution_json_path)
    rules = load_rules(paths)
    report = {"rules_loaded": len(rules)}
    report["fusions"] = greedy_fusions(model, rules)
    if cost_fn is None or budget <= 0:
        return report
    core = _core()
    best = cost_fn(model)
    tried = accepted = 0
    others = [r for r in rules if not r.name.startswith("fuse_")]
    for r in others:
        if tried >= budget:
            break
        nodes, _ = export_graph(model.layers)
        for m in core.match_rule(r, nodes, 4):
            tried += 1
            snapshot = (list(model.layers), {id(L): list(L.inputs) for L in model.layers}, model._output)
            if not apply_rule(model, r, m):
                continue
            c = cost_fn(model)
            if c < best / alpha:
                best = c
                accepted += 1
                break
            model.layers, inputs, model._output = snapshot
            for L in model.layers:
                L.inputs = inputs[id(L)]
    report.update(tried=tried, accepted=accepted, best_ms=best)
    return report
