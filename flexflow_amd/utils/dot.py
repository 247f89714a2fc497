"""Graphviz export of the computation graph and of the per-device task graph (reference
include/flexflow/utils/dot/*, --compgraph / --taskgraph / --include-costs-dot-graph flags and
tools/substitutions_to_dot).

* computation graph: one node per layer, labelled with its op type, output shape and the chosen
  parallel config (degrees per op axis, devices); edges carry tensor shapes and, when the producer
  and consumer layouts differ, the transfer kind the runtime inserts (all_gather, reduce_scatter,
  all_reduce, local_slice, generic P2P). With costs, nodes show the cost model's fwd/bwd ms.
* task graph: the simulator's view — per-device forward/backward task nodes for every op shard,
  edges for data dependencies, and weight-sync nodes for replicated weights.
* rules: a substitution rule's source and destination patterns side by side.
"""
from __future__ import annotations

from typing import Dict, List, Optional


class DotFile:
    """Minimal record-style dot writer (reference utils/dot/dot_file.h)."""

    def __init__(self, name="G", rankdir="TB"):
        self.lines = [f'digraph "{name}" {{', f"  rankdir={rankdir};", '  node [shape=record, fontsize=10];']
        self._ids: Dict[object, str] = {}

    def node_id(self, key):
        if key not in self._ids:
            self._ids[key] = f"n{len(self._ids)}"
        return self._ids[key]

    @staticmethod
    def _esc(s):
        return str(s).replace("\\", "\\\\").replace('"', '\\"').replace("{", "\\{").replace("}", "\\}") \
            .replace("<", "\\<").replace(">", "\\>").replace("|", "\\|")

    def add_node(self, key, fields: List[str], **attrs):
        label = "{" + "|".join(self._esc(f) for f in fields) + "}"
        extra = "".join(f', {k}="{v}"' for k, v in attrs.items())
        self.lines.append(f'  {self.node_id(key)} [label="{label}"{extra}];')

    def add_edge(self, a, b, label: Optional[str] = None, **attrs):
        extra = f' [label="{self._esc(label)}"' + "".join(f', {k}="{v}"' for k, v in attrs.items()) + "]" \
            if label else ("" if not attrs else " [" + ", ".join(f'{k}="{v}"' for k, v in attrs.items()) + "]")
        self.lines.append(f"  {self.node_id(a)} -> {self.node_id(b)}{extra};")

    def subgraph(self, name, label):
        self.lines.append(f'  subgraph "cluster_{name}" {{ label="{self._esc(label)}";')

    def end_subgraph(self):
        self.lines.append("  }")

    def text(self):
        return "\n".join(self.lines + ["}"]) + "\n"

    def write(self, path):
        with open(path, "w") as f:
            f.write(self.text())
        return path


def export_computation_graph(model, path, include_costs=False):
    from ..pcg.strategy import op_layouts
    from ..parallel.comm import Transfer
    d = DotFile("computation_graph")
    strat = getattr(model, "strategy", None) or {}
    prod = {}
    for L in model.layers:
        for j, o in enumerate(L.outputs):
            prod[o.guid] = (L, j)
    costs = {}
    if include_costs and strat:
        from ..pcg import costmodel
        for L in model.layers:
            try:
                costs[L.name] = costmodel.op_cost(L, strat[L.name], model.config.compute_dtype, False, None)
            except Exception:  # noqa: BLE001 - costs are decoration only
                pass
    for L in model.layers:
        fields = [f"{L.name}", L.op_type.name.replace("OP_", ""),
                  " x ".join(str(s) for s in L.outputs[0].dims) if L.outputs else ""]
        c = strat.get(L.name)
        if c is not None:
            fields.append(f"degrees={list(c.degrees)} devices={list(c.devices)[:8]}{'...' if len(c.devices) > 8 else ''}")
        if L.name in costs:
            f, b = costs[L.name]
            fields.append(f"fwd {f:.3f} ms / bwd {b:.3f} ms")
        color = "lightgrey" if L.op_type.name == "OP_INPUT" else ("lightblue" if c is not None and any(
            dg > 1 for dg in c.degrees[1:]) else "white")
        d.add_node(L, fields, style="filled", fillcolor=color)
    for L in model.layers:
        for j, t in enumerate(L.inputs):
            if t.guid not in prod:
                continue
            P, pj = prod[t.guid]
            label = "x".join(str(s) for s in t.dims)
            if strat and P.name in strat and L.name in strat:
                try:
                    src = op_layouts(P, strat[P.name]).outputs[pj]
                    dst = op_layouts(L, strat[L.name]).inputs[j]
                    kind = Transfer(src, dst, src.partial, 0).kind
                    if kind != "identity":
                        label += f" [{kind}]"
                except Exception:  # noqa: BLE001
                    pass
            d.add_edge(P, L, label)
    return d.write(path)


def export_task_graph(model, path):
    """Per-device fwd/bwd tasks of every op shard (the simulator's task graph)."""
    from ..pcg.strategy import op_layouts
    d = DotFile("task_graph", rankdir="LR")
    strat = model.strategy
    prod = {}
    for L in model.layers:
        for o in L.outputs:
            prod[o.guid] = L
    devs_of = {L.name: sorted(set(strat[L.name].devices)) for L in model.layers}
    for L in model.layers:
        if L.op_type.name == "OP_INPUT":
            continue
        for dv in devs_of[L.name]:
            d.add_node(("f", L.name, dv), [f"{L.name} fwd", f"gpu {dv}"])
            d.add_node(("b", L.name, dv), [f"{L.name} bwd", f"gpu {dv}"], style="dashed")
            d.add_edge(("f", L.name, dv), ("b", L.name, dv))
        for t in L.inputs:
            P = prod.get(t.guid)
            if P is None or P.op_type.name == "OP_INPUT":
                continue
            for dv in devs_of[L.name]:
                src_devs = devs_of[P.name] if dv not in devs_of[P.name] else [dv]
                for sd in src_devs:
                    d.add_edge(("f", P.name, sd), ("f", L.name, dv))
                    d.add_edge(("b", L.name, dv), ("b", P.name, sd))
        lo = op_layouts(L, strat[L.name])
        for wi, wl in enumerate(lo.weights):
            if wl.replicas > 1:
                d.add_node(("sync", L.name, wi), [f"{L.name} weight {wi}", f"all-reduce x{wl.replicas}"],
                           shape="box", style="filled", fillcolor="orange")
                for dv in devs_of[L.name]:
                    d.add_edge(("b", L.name, dv), ("sync", L.name, wi))
    return d.write(path)


def rule_to_dot(rule, path):
    """A substitution rule's source and destination patterns (reference tools/substitutions_to_dot)."""
    d = DotFile(rule.name, rankdir="TB")
    for side, ops in (("src", rule.src), ("dst", rule.dst)):
        d.subgraph(side, f"{rule.name}: {side}")
        for i, op in enumerate(ops):
            params = ", ".join(f"{p.key}={p.value}" for p in op.params)
            d.add_node((side, i), [op.type.replace("OP_", ""), params] if params else [op.type.replace("OP_", "")])
        for i, op in enumerate(ops):
            for t in op.inputs:
                if t.op_id >= 0:
                    d.add_edge((side, t.op_id), (side, i), f"t{t.ts_id}")
                else:
                    d.add_node((side, "ext", t.op_id), [f"input {t.op_id}"], shape="ellipse")
                    d.add_edge((side, "ext", t.op_id), (side, i))
        d.end_subgraph()
    return d.write(path)
