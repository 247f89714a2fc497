"""Joint Unity search: best-first over rewritten graphs, each costed by the parallelization search
(reference GraphSearchHelper::graph_optimize / base_optimize, src/runtime/substitution.cc:1898-1945
and 2229-2320, with the generated xfers of substitution.cc:1750-1830 and 3041-3260).

A graph state is the layer list after a sequence of rewrites. Popping the cheapest state, every
xfer is matched on it; each rewritten graph is costed by the full strategy search on that graph
(pcg/unity.py: frontier DP over per-op configs + simulator refinement + resource splits) and
queued when its simulated step time beats the best so far by the --search-alpha factor, until
--budget graphs have been costed. The best graph is rebuilt from the ORIGINAL graph by replaying
its rewrite sequence, so every rank constructs it identically (names of rewritten layers derive
from the names they replace); rank 0 searches and broadcasts the sequence and the strategy.

Xfers (each `matches(model) -> [match]`, `apply(model, match) -> bool`; a match is a tuple of
layer names plus parameters, so it can be replayed on another process):
  * merge_siblings(OP_LINEAR / OP_CONV2D): two ops of the same kind reading the same tensor become
    one op with the output channels of both plus a Split (the TASO "concat of linears over a
    shared input" family; Inception's 1x1 tower heads, parallel MLP branches). One larger GEMM:
    fewer launches, fuller MFMA tiles, one all-reduce bucket instead of two.
  * pin_parallel(op, axis, degree): the reference's create_partition_linear_combine /
    create_replicate_linear_combine / create_partition_attention_combine. In the reference those
    xfers insert Repartition/Replicate before and Combine after an op; here the layouts around an
    op follow from its config (the executor's transfers are the Repartition/Combine data movement),
    so the xfer pins the op's degree on one axis for every op of the same signature (BERT's 24
    identical FFN layers move together: a coarse move the per-op DP + MCMC rarely reaches).
  * JSON rules (--substitution-json, non-fusion rules) through pcg/substitutions.apply_rule.
"""
from __future__ import annotations

import heapq
import os
import time
from typing import Dict, List, Optional, Tuple

from ..type import ActiMode, OperatorType


# ----------------------------------------------------------------------------- graph states
def snapshot(model):
    return (list(model.layers), {id(L): list(L.inputs) for L in model.layers}, model._output,
            dict(getattr(model, "_tensor_remap", {})), set(getattr(model, "_names", set())),
            dict(getattr(model, "_weight_alias", {})))


def stamp_init_slots(model):
    """Record each weight's (layer position, slot) in the graph as written: the seed of its default
    initializer. Rewrites move layers, and a rewritten graph must initialise like the original."""
    for li, L in enumerate(model.layers):
        for i, w in enumerate(L.weights):
            if getattr(w, "_init_slot", None) is None:
                w._init_slot = (li, i)


def restore(model, snap):
    layers, inputs, out, remap, names, alias = snap
    model._weight_alias = dict(alias)
    model.layers = list(layers)
    for L in model.layers:
        L.inputs = list(inputs[id(L)])
    model._output = out
    model._tensor_remap = dict(remap)
    model._names = set(names)


def graph_key(model) -> tuple:
    prod = {o.guid: L.name for L in model.layers for o in L.outputs}
    return tuple((L.name, L.op_type.value, tuple(prod.get(t.guid, "") for t in L.inputs)) for L in model.layers)


def _replace(model, removed: List, added: List, remap: Dict[int, object]):
    """Swap `removed` layers for `added` (inserted where the first removed one stood) and reroute
    every consumer of a remapped tensor."""
    ids = {id(L) for L in removed}
    pos = min(i for i, L in enumerate(model.layers) if id(L) in ids)
    kept = [L for L in model.layers if id(L) not in ids]
    before = sum(1 for L in model.layers[:pos] if id(L) not in ids)
    model.layers = kept[:before] + list(added) + kept[before:]
    for L in model.layers:
        L.inputs = [remap.get(t.guid, t) for t in L.inputs]
    model._tensor_remap.update(remap)
    if model._output is not None and model._output.guid in remap:
        model._output = remap[model._output.guid]
    from .substitutions import _toposort
    model.layers = _toposort(model.layers)
    for L in added:
        model._names.add(L.name)


def _users(model):
    users = {}
    for L in model.layers:
        for w in L.weights:
            users[id(w)] = users.get(id(w), 0) + 1
    return users


def _at(model, positions):
    """Layers at positions of model.layers (matches name layers by position: auto-generated names
    depend on how many layers a process built before, positions only on the graph)."""
    return [model.layers[p] if isinstance(p, int) and 0 <= p < len(model.layers) else None for p in positions]


# ----------------------------------------------------------------------------- xfers
class MergeSiblings:
    """op(x; W1) , op(x; W2)  ->  split(op(x; [W1; W2]))"""

    KEYS = {OperatorType.OP_LINEAR: ("activation", "use_bias", "data_type"),
            OperatorType.OP_CONV2D: ("kernel_h", "kernel_w", "stride_h", "stride_w", "padding_h", "padding_w",
                                     "activation", "groups", "use_bias")}

    def __init__(self, op_type: OperatorType):
        self.op_type = op_type
        self.name = f"merge_siblings_{op_type.name[3:].lower()}"

    def _out_attr(self):
        return "out_dim" if self.op_type == OperatorType.OP_LINEAR else "out_channels"

    def _ok(self, L, users, out_guid):
        if L.op_type != self.op_type or L.attrs.get("regularizer") is not None:
            return False
        if L.op_type == OperatorType.OP_CONV2D and L.attrs.get("groups", 1) != 1:
            return False
        if any(users.get(id(w), 0) != 1 for w in L.weights):
            return False  # shared weights (shared_op) keep their own layer
        return True

    def matches(self, model) -> List[tuple]:
        users = _users(model)
        groups: Dict[tuple, List] = {}
        out_guid = model._output.guid if model._output is not None else None
        for L in model.layers:
            if not self._ok(L, users, out_guid) or not L.inputs:
                continue
            sig = (L.inputs[0].guid,) + tuple(repr(L.attrs.get(k)) for k in self.KEYS[self.op_type])
            groups.setdefault(sig, []).append(L)
        out = []
        pos = {id(L): i for i, L in enumerate(model.layers)}
        for g in groups.values():
            for i in range(len(g) - 1):
                out.append((pos[id(g[i])], pos[id(g[i + 1])]))
        return out

    def apply(self, model, match) -> bool:
        from ..core.layer import Layer, op_class
        a, b = _at(model, match)
        if a is None or b is None or not self._ok(a, _users(model), None) or not self._ok(b, _users(model), None) \
                or a is b or not a.inputs or not b.inputs or a.inputs[0] is not b.inputs[0]:
            return False
        from ..core.initializers import BlockInitializer
        oa, ob = self._out_attr(), None
        attrs = dict(a.attrs)
        attrs[oa] = int(a.attrs[oa]) + int(b.attrs[oa])
        name = f"{a.name}&{b.name}"
        M = Layer(model, self.op_type, name, [a.inputs[0]], attrs)
        M.__class__ = op_class(self.op_type)
        if len(M.weights) != len(a.weights) or len(M.weights) != len(b.weights):
            return False
        # every weight of the merged op is the row-stack of the two originals: each block keeps its
        # original initializer / seed, and values set on the original Parameters (before or after
        # compile) are redirected into the block (FFModel._weight_alias)
        na, nb = int(a.attrs[oa]), int(b.attrs[oa])
        for wm, wa, wb in zip(M.weights, a.weights, b.weights):
            if wm.dims[0] != na + nb or tuple(wa.dims[1:]) != tuple(wm.dims[1:]) \
                    or tuple(wb.dims[1:]) != tuple(wm.dims[1:]):
                return False
            wm.initializer = BlockInitializer([(wa, 0, na), (wb, na, nb)])
        axis = -1 if self.op_type == OperatorType.OP_LINEAR else 1
        S = Layer(model, OperatorType.OP_SPLIT, f"split[{name}]", [M.outputs[0]],
                  {"sizes": [int(a.attrs[oa]), int(b.attrs[oa])], "axis": axis})
        S.__class__ = op_class(OperatorType.OP_SPLIT)
        if tuple(S.outputs[0].dims) != tuple(a.outputs[0].dims) or tuple(S.outputs[1].dims) != tuple(b.outputs[0].dims):
            return False
        alias = getattr(model, "_weight_alias", None)
        if alias is None:
            alias = model._weight_alias = {}
        for wm, wa, wb in zip(M.weights, a.weights, b.weights):
            alias[wa.guid] = (wm, 0, na)
            alias[wb.guid] = (wm, na, nb)
        _replace(model, [a, b], [M, S], {a.outputs[0].guid: S.outputs[0], b.outputs[0].guid: S.outputs[1]})
        return True


class PinParallel:
    """Fix the degree of one parallel axis (degree = all devices) for every op of one signature."""

    OPS = (OperatorType.OP_LINEAR, OperatorType.OP_MULTIHEAD_ATTENTION, OperatorType.OP_CONV2D,
           OperatorType.OP_EMBEDDING)
    LABEL = {"sample": "partition_{}_combine", "parameter": "replicate_{}_combine"}

    def __init__(self, num_devices: int, allowed=("sample", "parameter"), max_classes: int = 4):
        self.n = num_devices
        self.allowed = allowed
        self.max_classes = max_classes
        self.name = "pin_parallel"

    @staticmethod
    def signature(L) -> tuple:
        return (L.op_type.value, tuple(tuple(t.dims) for t in L.inputs), tuple(tuple(w.dims) for w in L.weights),
                repr(sorted((k, repr(v)) for k, v in L.attrs.items() if k != "pin")))

    def matches(self, model) -> List[tuple]:
        from .strategy import OpConfig, valid_config
        classes: Dict[tuple, List] = {}
        for L in model.layers:
            if L.op_type in self.OPS and "pin" not in L.attrs:
                classes.setdefault(self.signature(L), []).append(L)
        # the heaviest classes first (flops of one member x members)
        def weight(members):
            L = members[0]
            try:
                fl = L.impl.flops([t.dims for t in L.inputs], [o.dims for o in L.outputs], [w.dims for w in L.weights])
            except Exception:  # noqa: BLE001 - ops without a flop model rank last
                fl = 0.0
            return fl * len(members)
        out = []
        pos = {id(L): i for i, L in enumerate(model.layers)}
        for members in sorted(classes.values(), key=weight, reverse=True)[:self.max_classes]:
            L = members[0]
            kinds = L.impl.axis_kinds()
            sizes = L.impl.axis_sizes()
            for ax, k in enumerate(kinds):
                if k not in self.allowed or not L.impl.supports_axis(ax) or sizes[ax] % self.n:
                    continue
                degs = [1] * len(sizes)
                degs[ax] = self.n
                if not valid_config(L, OpConfig(tuple(degs), tuple(range(self.n)))):
                    continue
                label = self.LABEL[k].format(L.op_type.name[3:].lower())
                out.append((label, ax, tuple(pos[id(m)] for m in members)))
        return out

    def apply(self, model, match) -> bool:
        from ..core.layer import Layer, op_class
        label, ax, positions = match
        olds = _at(model, positions)
        if any(L is None or L.op_type not in self.OPS for L in olds):
            return False
        for L in olds:
            degs = [1] * len(L.impl.axis_sizes())
            degs[ax] = self.n
            attrs = dict(L.attrs)
            attrs["pin"] = tuple(degs)
            N = Layer(model, L.op_type, f"{L.name}@{label}", list(L.inputs), attrs)
            N.__class__ = op_class(L.op_type)
            if [w.dims for w in N.weights] != [w.dims for w in L.weights]:
                return False
            N.weights = list(L.weights)  # same parameters (and initial values) as the op it pins
            _replace(model, [L], [N], {o.guid: n for o, n in zip(L.outputs, N.outputs)})
        return True


class RuleXfer:
    """A non-fusion rule of a JSON rule collection (reference substitution_loader.cc format)."""

    def __init__(self, rule):
        self.rule = rule
        self.name = f"rule:{rule.name}"

    def matches(self, model) -> List[tuple]:
        from .substitutions import _core, export_graph
        nodes, _ = export_graph(model.layers)
        return [tuple(int(i) for i in m.op_nodes) for m in _core().match_rule(self.rule, nodes, 4)]

    def apply(self, model, match) -> bool:
        from .substitutions import _core, apply_rule, export_graph
        nodes, _ = export_graph(model.layers)
        for m in _core().match_rule(self.rule, nodes, 64):
            if tuple(int(i) for i in m.op_nodes) == tuple(match):
                return apply_rule(model, self.rule, m)
        return False


def build_xfers(model) -> List:
    cfg = model.config
    xs = [MergeSiblings(OperatorType.OP_LINEAR), MergeSiblings(OperatorType.OP_CONV2D)]
    if not cfg.only_data_parallel:
        from .unity import allowed_kinds
        xs.append(PinParallel(cfg.num_devices, tuple(k for k in allowed_kinds(cfg) if k in ("sample", "parameter"))))
    if cfg.substitution_json_path:
        from .substitutions import load_rules
        xs += [RuleXfer(r) for r in load_rules([cfg.substitution_json_path]) if not r.name.startswith("fuse_")]
    return xs


def replay(model, xfers, seq) -> List[str]:
    by = {x.name: x for x in xfers}
    done = []
    for name, match in seq:
        x = by.get(name)
        if x is None or not x.apply(model, tuple(match) if not isinstance(match, tuple) else match):
            raise RuntimeError(f"rewrite {name} {match} does not replay on this graph")
        done.append(name)
    return done


def _jsonable(match):
    return [list(m) if isinstance(m, tuple) else m for m in match]


def _tuple(match):
    return tuple(tuple(m) if isinstance(m, list) else m for m in match)


def joint_search(model, algo: str = "unity", budget: Optional[int] = None, alpha: Optional[float] = None):
    """Returns (strategy, report) for the best graph found; model.layers is left as that graph."""
    from .unity import search as param_search
    cfg = model.config
    if model._output is None:
        model._output = model.output_tensor()  # keep the model output's role stable under rewrites
    budget = budget if budget is not None else int(os.environ.get("FF_JOINT_BUDGET", str(
        cfg.search_budget if cfg.search_budget and cfg.search_budget > 0 and cfg.search_budget < 64 else 8)))
    alpha = alpha if alpha is not None else max(1.0, float(cfg.search_alpha or 1.0))
    xfers = build_xfers(model)
    t0 = time.perf_counter()
    stamp_init_slots(model)
    base = snapshot(model)
    strat0, rep0 = param_search(model, algo)
    best = [rep0["predicted_ms"], [], strat0, rep0]
    tried = []
    seen = {graph_key(model)}
    queue: List[Tuple[float, int, list]] = [(rep0["predicted_ms"], 0, [])]
    tick = 1
    evals = 1
    while queue and evals < budget:
        _, _, seq = heapq.heappop(queue)
        restore(model, base)
        replay(model, xfers, seq)
        cur = snapshot(model)
        cur_ids = {id(L) for L in model.layers}
        for x in xfers:
            if evals >= budget:
                break
            for m in x.matches(model)[:4]:
                if evals >= budget:
                    break
                restore(model, cur)
                if not x.apply(model, m):
                    continue
                key = graph_key(model)
                if key in seen:
                    continue
                seen.add(key)
                strat, rep = param_search(model, algo)
                evals += 1
                c = rep["predicted_ms"]
                step = (x.name, _tuple(m))
                tried.append({"xfer": x.name, "match": _jsonable(m), "after": [s[0] for s in seq],
                              "new_ops": [L.name for L in model.layers if id(L) not in cur_ids][:4],
                              "predicted_ms": round(c, 4)})
                if c < best[0]:
                    best = [c, seq + [step], strat, rep]
                if c < best[0] * alpha:
                    heapq.heappush(queue, (c, tick, seq + [step]))
                    tick += 1
    restore(model, base)
    replay(model, xfers, best[1])
    rep = dict(best[3])
    rep.update({"joint": True, "graphs_costed": evals, "joint_s": round(time.perf_counter() - t0, 3),
                "rewrites": [{"xfer": n, "match": _jsonable(m)} for n, m in best[1]],
                "start_graph_ms": round(rep0["predicted_ms"], 4),
                # speedup against data parallel on the graph as written (before any rewrite)
                "predicted_dp_ms": rep0["predicted_dp_ms"],
                "predicted_speedup_vs_dp": round(rep0["predicted_dp_ms"] / max(best[0], 1e-9), 4),
                "tried": tried[:64]})
    return best[2], rep, [(n, _jsonable(m)) for n, m in best[1]]


def replay_broadcast(model, seq):
    """Non-root ranks: rebuild rank 0's chosen graph from its rewrite sequence."""
    if model._output is None:
        model._output = model.output_tensor()
    xfers = build_xfers(model)
    stamp_init_slots(model)
    return replay(model, xfers, [(n, _tuple(m)) for n, m in seq])
