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
  * block pins (combine_inception / combine_concat) and leading_relu_branch_{combine,partition}
    (substitution.cc:3099-3167, 3463-3540): a fork's branches pinned to one sample degree so the
    fork tensor is re-laid-out once (or not at all) instead of once per branch.
  * JSON rules (--substitution-json, non-fusion rules) through pcg/substitutions.apply_rule.
"""
from __future__ import annotations

import heapq
import math
import os
import sys
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


def _weight(members):
    L = members[0]
    try:
        fl = L.impl.flops([t.dims for t in L.inputs], [o.dims for o in L.outputs], [w.dims for w in L.weights])
    except Exception:  # noqa: BLE001 - ops without a flop model rank last
        fl = 0.0
    return fl * len(members)


def signature(L) -> tuple:
    return (L.op_type.value, tuple(tuple(t.dims) for t in L.inputs), tuple(tuple(w.dims) for w in L.weights),
            repr(sorted((k, repr(v)) for k, v in L.attrs.items() if k != "pin")))


def _pin_ok(L, degs) -> bool:
    from .strategy import OpConfig, valid_config
    return valid_config(L, OpConfig(tuple(degs), tuple(range(int(math.prod(degs))))))


def _pin_layers(model, olds, degs_of, label) -> bool:
    """Replace each layer by a copy whose degrees are fixed to degs_of(L) (same parameters)."""
    from ..core.layer import Layer, op_class
    for L in olds:
        attrs = dict(L.attrs)
        attrs["pin"] = tuple(degs_of(L))
        N = Layer(model, L.op_type, f"{L.name}@{label}", list(L.inputs), attrs)
        N.__class__ = op_class(L.op_type)
        if [w.dims for w in N.weights] != [w.dims for w in L.weights]:
            return False
        N.weights = list(L.weights)  # same parameters (and initial values) as the op it pins
        _replace(model, [L], [N], {o.guid: n for o, n in zip(L.outputs, N.outputs)})
    return True


class PinAxis:
    """One of the reference's generated parallelization xfers (substitution.cc:1726-1850) at one
    degree: Repartition/Replicate before, the op with one axis split `degree` ways, Combine/Reduction
    after. Here the data movement around an op follows from its config (the executor's transfers
    are the parallel ops), so the xfer pins that axis's degree — for every op of one signature at
    once (BERT's 24 identical FFNs move together, a coarse move the per-op DP + MCMC rarely make).

    family: the reference's name (partition_linear_combine, replicate_attention_reduce, ...);
    axis_of(layer) -> parallel axis of the op (None: not applicable)."""

    def __init__(self, family: str, op_types, axis_of, degree: int, max_classes: int = 4):
        self.family = family
        self.op_types = tuple(op_types)
        self.axis_of = axis_of
        self.degree = degree
        self.max_classes = max_classes
        self.name = f"{family}[{degree}]"

    def _degs(self, L):
        ax = self.axis_of(L)
        if ax is None:
            return None
        sizes = L.impl.axis_sizes()
        if ax >= len(sizes) or not L.impl.supports_axis(ax) or sizes[ax] % self.degree:
            return None
        degs = [1] * len(sizes)
        degs[ax] = self.degree
        return degs if _pin_ok(L, degs) else None

    def matches(self, model) -> List[tuple]:
        classes: Dict[tuple, List] = {}
        for L in model.layers:
            if L.op_type in self.op_types and "pin" not in L.attrs:
                classes.setdefault(signature(L), []).append(L)
        pos = {id(L): i for i, L in enumerate(model.layers)}
        out = []
        for members in sorted(classes.values(), key=_weight, reverse=True):
            if len(out) >= self.max_classes:
                break
            degs = self._degs(members[0])
            if degs is None:
                continue
            out.append((self.family, tuple(degs), tuple(pos[id(m)] for m in members)))
        return out

    def apply(self, model, match) -> bool:
        _, degs, positions = match
        olds = _at(model, positions)
        if any(L is None or L.op_type not in self.op_types or "pin" in L.attrs for L in olds):
            return False
        if any(len(L.impl.axis_sizes()) != len(degs) or not _pin_ok(L, degs) for L in olds):
            return False
        return _pin_layers(model, olds, lambda L: degs, f"{self.family}{self.degree}")


class BlockPin:
    """create_combine_inception / create_combine_concat (substitution.cc:3099-3167): the Combine that
    ends a sample-partitioned region is moved past an Inception block, so the block's branches and
    its Concat all run sample-parallel `degree` ways with no re-layout in between. Here: every op
    of the region (all ops between the block's fork and the Concat; for combine_concat the Concat
    and its producers) is pinned to sample degree `degree`."""

    def __init__(self, family: str, degree: int, whole_block: bool, max_blocks: int = 4):
        self.family = family
        self.degree = degree
        self.whole = whole_block
        self.max_blocks = max_blocks
        self.name = f"{family}[{degree}]"

    def _region(self, model, C):
        prod = {o.guid: L for L in model.layers for o in L.outputs}
        heads = [prod.get(t.guid) for t in C.inputs]
        if len(heads) < 2 or any(h is None for h in heads):
            return None
        if not self.whole:
            return heads + [C]
        pos = {id(L): i for i, L in enumerate(model.layers)}
        anc_cache: Dict[int, set] = {}

        def anc(L):  # ids of L and all its ancestors
            k = id(L)
            if k not in anc_cache:
                a = {k}
                for t in L.inputs:
                    p = prod.get(t.guid)
                    if p is not None:
                        a |= anc(p)
                anc_cache[k] = a
            return anc_cache[k]

        common = set.intersection(*[anc(h) for h in heads])
        if not common:
            return None
        fork = max(common, key=lambda k: pos.get(k, -1))
        fork_anc = anc(next(L for L in model.layers if id(L) == fork))
        region = set().union(*[anc(h) for h in heads]) - fork_anc
        if len(region) > 64:
            return None
        return [L for L in model.layers if id(L) in region] + [C]

    def matches(self, model) -> List[tuple]:
        from ..type import OperatorType as OT
        pos = {id(L): i for i, L in enumerate(model.layers)}
        out = []
        for C in model.layers:
            if C.op_type != OT.OP_CONCAT or "pin" in C.attrs:
                continue
            reg = self._region(model, C)
            if not reg or any("pin" in L.attrs or L.op_type == OT.OP_INPUT for L in reg):
                continue
            if not all(self._degs(L) is not None for L in reg):
                continue
            out.append((self.family, tuple(pos[id(L)] for L in reg)))
        # the biggest blocks first
        out.sort(key=lambda m: -len(m[1]))
        return out[:self.max_blocks]

    def _degs(self, L):
        sizes = L.impl.axis_sizes()
        if not sizes or L.impl.axis_kinds()[0] != "sample" or sizes[0] % self.degree:
            return None
        degs = [1] * len(sizes)
        degs[0] = self.degree
        return degs if _pin_ok(L, degs) else None

    def apply(self, model, match) -> bool:
        _, positions = match
        olds = _at(model, positions)
        if any(L is None or "pin" in L.attrs for L in olds):
            return False
        degs = {id(L): self._degs(L) for L in olds}
        if any(d is None for d in degs.values()):
            return False
        return _pin_layers(model, olds, lambda L: degs[id(L)], f"{self.family}{self.degree}")


class LeadingBranch:
    """leading_relu_branch_combine / leading_relu_branch_partition (substitution.cc:3463-3540,
    generated at 1839-1841 for num_combines 1..4 on the sample dim). In the reference a tensor that
    fans out (Inception's ReLU'd tower inputs, a residual fork) feeds one branch through a
    Repartition and `num` sibling branches through Combines (or one through a Combine and `num`
    through Repartitions); the rewrite keeps the leading branch's re-layout and turns the `num`
    siblings' into no-ops, so those branches consume the fork tensor as it is laid out.

    Here a layout change on an edge is implied by the degrees of its two ends, so the two forms
    become pins on a fork F -> consumers c0 (the leading branch), c1..c_num:
      * combine[d, num]: c0..c_num all sample-parallel `d` ways — the leading branch's
        re-layout of F serves every sibling (one transfer of F instead of num + 1);
      * partition[d, num]: F's producer and c1..c_num sample-parallel `d` ways — the siblings
        read F where it is produced (no transfer on those edges); c0 keeps its own layout.
    Forks are ranked by the flops of the ops they pin; at most `max_forks` matches."""

    def __init__(self, family: str, degree: int, num: int, max_forks: int = 2):
        assert family in ("leading_relu_branch_combine", "leading_relu_branch_partition")
        self.family = family
        self.degree = degree
        self.num = num
        self.max_forks = max_forks
        self.name = f"{family}[{degree},{num}]"

    def _degs(self, L):
        sizes = L.impl.axis_sizes()
        if not sizes or L.impl.axis_kinds()[0] != "sample" or sizes[0] % self.degree:
            return None
        degs = [1] * len(sizes)
        degs[0] = self.degree
        return degs if _pin_ok(L, degs) else None

    def _pinned(self, prod, consumers):
        if self.family == "leading_relu_branch_combine":
            return consumers[:self.num + 1]
        return [prod] + consumers[1:self.num + 1]

    def matches(self, model) -> List[tuple]:
        from ..type import OperatorType as OT
        pos = {id(L): i for i, L in enumerate(model.layers)}
        readers: Dict[int, List] = {}
        for L in model.layers:
            for t in {t.guid: t for t in L.inputs}.values():
                readers.setdefault(t.guid, []).append(L)
        out = []
        for P in model.layers:
            if P.op_type == OT.OP_INPUT or not P.outputs:
                continue
            cons = readers.get(P.outputs[0].guid, [])
            if len(cons) < self.num + 1:
                continue
            pins = self._pinned(P, cons)
            if any("pin" in L.attrs or L.op_type == OT.OP_INPUT or self._degs(L) is None for L in pins):
                continue
            w = sum(_weight([L]) for L in pins)
            out.append((w, (self.family, self.degree, self.num, tuple(pos[id(L)] for L in pins))))
        out.sort(key=lambda m: -m[0])
        return [m for _, m in out[:self.max_forks]]

    def apply(self, model, match) -> bool:
        _, _, _, positions = match
        olds = _at(model, positions)
        if any(L is None or "pin" in L.attrs for L in olds):
            return False
        degs = {id(L): self._degs(L) for L in olds}
        if any(d is None for d in degs.values()):
            return False
        return _pin_layers(model, olds, lambda L: degs[id(L)], f"lrb{self.family[20]}{self.degree}x{self.num}")


class LinearReluMerge:
    """create_linear_relu_merge (substitution.cc:1790-1793): Linear (no activation) followed by its
    only consumer ReLU becomes one Linear with a fused ReLU epilogue (same parameters)."""

    name = "linear_relu_merge"

    def matches(self, model) -> List[tuple]:
        from ..type import OperatorType as OT
        users: Dict[int, List] = {}
        for L in model.layers:
            for t in L.inputs:
                users.setdefault(t.guid, []).append(L)
        out_guid = model._output.guid if model._output is not None else None
        pos = {id(L): i for i, L in enumerate(model.layers)}
        out = []
        for L in model.layers:
            if L.op_type != OT.OP_LINEAR or L.attrs.get("activation", ActiMode.AC_MODE_NONE) != ActiMode.AC_MODE_NONE:
                continue
            us = users.get(L.outputs[0].guid, [])
            if len(us) == 1 and us[0].op_type == OT.OP_RELU and L.outputs[0].guid != out_guid:
                out.append((pos[id(L)], pos[id(us[0])]))
        return out

    def apply(self, model, match) -> bool:
        from ..core.layer import Layer, op_class
        from ..type import OperatorType as OT
        lin, relu = _at(model, match)
        if lin is None or relu is None or lin.op_type != OT.OP_LINEAR or relu.op_type != OT.OP_RELU \
                or relu.inputs[0].guid != lin.outputs[0].guid:
            return False
        attrs = dict(lin.attrs)
        attrs["activation"] = ActiMode.AC_MODE_RELU
        M = Layer(model, OT.OP_LINEAR, f"{lin.name}+relu", list(lin.inputs), attrs)
        M.__class__ = op_class(OT.OP_LINEAR)
        if [w.dims for w in M.weights] != [w.dims for w in lin.weights]:
            return False
        M.weights = list(lin.weights)
        _replace(model, [lin, relu], [M], {lin.outputs[0].guid: M.outputs[0], relu.outputs[0].guid: M.outputs[0]})
        return True


def _axis_last_param(L):
    kinds = L.impl.axis_kinds()
    n = len(L.outputs[0].dims)
    return n - 1 if kinds[n - 1] == "parameter" else None


def _linear_red_axis(L):
    return len(L.outputs[0].dims)


def _axis(i):
    return lambda L: i


def parallel_xfers(cfg) -> List:
    """The reference's generate_all_pcg_xfers (substitution.cc:1726-1850) for this machine: every
    parallel degree that divides the GPUs of a node, plus node multiples (all_parallel_degrees);
    the replicate (parameter-parallel) families only within a node (single_node_parallel_degrees)."""
    from .unity import allowed_kinds
    OT = OperatorType
    n = cfg.num_devices
    gpn = max(1, min(cfg.search_num_workers or cfg.local_world_size or n, n))
    nodes = max(1, n // gpn)
    single = [d for d in range(2, gpn + 1) if gpn % d == 0]
    every = single + [k * gpn for k in range(2, nodes + 1) if nodes % k == 0]
    kinds = allowed_kinds(cfg)
    xs: List = []
    for d in every:
        xs += [PinAxis("partition_linear_combine", [OT.OP_LINEAR], _axis(0), d),
               PinAxis("partition_attention_combine", [OT.OP_MULTIHEAD_ATTENTION], _axis(0), d),
               PinAxis("partition_add_combine", [OT.OP_EW_ADD], _axis(0), d),
               PinAxis("partition_relu_combine", [OT.OP_RELU], _axis(0), d),
               PinAxis("partition_softmax_combine", [OT.OP_SOFTMAX], _axis(0), d),
               PinAxis("partition_concat_combine", [OT.OP_CONCAT], _axis(0), d),
               # create_mapping_xfers<Conv2D / Pool2D / Flat>: the sample mapping at every degree
               PinAxis("partition_conv2d_combine", [OT.OP_CONV2D], _axis(0), d),
               PinAxis("partition_pool2d_combine", [OT.OP_POOL2D], _axis(0), d),
               PinAxis("partition_flat_combine", [OT.OP_FLAT], _axis(0), d),
               BlockPin("combine_inception", d, True), BlockPin("combine_concat", d, False)]
        # generate_all_pcg_xfers' loop over num_combines 1..4 (substitution.cc:1839-1841)
        for num in range(1, 5):
            xs += [LeadingBranch("leading_relu_branch_combine", d, num),
                   LeadingBranch("leading_relu_branch_partition", d, num)]
        if "attribute" in kinds:  # spatial mappings (halo exchange) only with attribute parallelism
            for ax in (2, 3):
                xs += [PinAxis(f"partition_conv2d_combine_dim{ax}", [OT.OP_CONV2D], _axis(ax), d),
                       PinAxis(f"partition_pool2d_combine_dim{ax}", [OT.OP_POOL2D], _axis(ax), d)]
    if "parameter" in kinds:
        for d in single:
            xs += [PinAxis("replicate_linear_combine", [OT.OP_LINEAR], _axis_last_param, d),
                   PinAxis("partition_linear_reduce", [OT.OP_LINEAR], _linear_red_axis, d),
                   PinAxis("replicate_attention_reduce", [OT.OP_MULTIHEAD_ATTENTION], _axis(3), d),
                   PinAxis("replicate_conv2d_combine", [OT.OP_CONV2D], _axis(1), d),
                   PinAxis("replicate_embedding_combine", [OT.OP_EMBEDDING], _axis_last_param, d),
                   PinAxis("partition_embedding_reduce", [OT.OP_EMBEDDING], _linear_red_axis, d)]
    return xs


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
                try:
                    return apply_rule(model, self.rule, m)
                except (IndexError, KeyError, ValueError, AssertionError):
                    return False  # a destination op our layer types cannot express
        return False


def build_xfers(model) -> List:
    """Sibling merges and linear_relu_merge always; the reference's generated parallelization
    xfers at every parallel degree unless --only-data-parallel; JSON rule collections given with
    --substitution-json. (The TASO collection graph_subst_3_v2 is not loaded by default: its 640
    rules rewrite explicit Partition / Combine / Replicate / Reduce ops, which this layer graph
    does not contain — parallelism is an op's config here — and none of them matches the zoo's
    graphs once those are removed: scripts/taso_rule_coverage.py.)"""
    cfg = model.config
    xs = [MergeSiblings(OperatorType.OP_LINEAR), MergeSiblings(OperatorType.OP_CONV2D), LinearReluMerge()]
    if not cfg.only_data_parallel:
        xs += parallel_xfers(cfg)
    if cfg.substitution_json_path:
        from .substitutions import load_rules
        xs += [RuleXfer(r) for r in load_rules([cfg.substitution_json_path]) if not r.name.startswith("fuse_")]
    return xs


def _xfer_from_name(name: str):
    """A parallelization xfer named by a rewrite sequence that this process's machine did not
    generate (a plan for 8 devices replayed by a 1-process reference run): rebuilt from its name."""
    if "[" not in name or not name.endswith("]"):
        return None
    fam, deg = name[:-1].split("[", 1)
    if fam.startswith("leading_relu_branch_"):
        d, num = (deg.split(",") + [""])[:2]
        return LeadingBranch(fam, int(d), int(num)) if d.isdigit() and num.isdigit() else None
    if not deg.isdigit():
        return None
    if fam in ("combine_inception", "combine_concat"):
        return BlockPin(fam, int(deg), fam == "combine_inception")
    for x in parallel_xfers(_AllKinds(int(deg))):
        if isinstance(x, PinAxis) and x.family == fam:
            return PinAxis(fam, x.op_types, x.axis_of, int(deg))
    return None


class _AllKinds:
    """A config stand-in under which parallel_xfers generates every family at one degree."""

    def __init__(self, d):
        self.num_devices = d
        self.search_num_workers = d
        self.local_world_size = d
        self.only_data_parallel = False
        self.enable_attribute_parallel = True


def replay(model, xfers, seq) -> List[str]:
    by = {x.name: x for x in xfers}
    done = []
    for name, match in seq:
        x = by.get(name) or _xfer_from_name(name)
        if x is None or not x.apply(model, tuple(match) if not isinstance(match, tuple) else match):
            raise RuntimeError(f"rewrite {name} {match} does not replay on this graph")
        done.append(name)
    return done


def _jsonable(match):
    return [list(m) if isinstance(m, tuple) else m for m in match]


def _tuple(match):
    return tuple(tuple(m) if isinstance(m, list) else m for m in match)


def _class_key(x, match) -> tuple:
    """What a rewrite acts on, independent of the graph state it was applied to: the xfer and the
    signature class / layer names of its match (a pin that did not pay off once is not re-tried
    after unrelated rewrites: the additive cost of one op class does not depend on them)."""
    return (x.name, repr(match))


def joint_search(model, algo: str = "unity", budget: Optional[int] = None, alpha: Optional[float] = None):
    """Best-first over rewritten graphs (reference GraphSearchHelper::base_optimize,
    substitution.cc:2229-2320). `budget` has the reference's meaning (--budget): the number of
    graphs popped from the queue; every xfer is matched on each popped graph. Candidate graphs are
    ranked by the DP's predicted step time (no MCMC / resource-split refinement: that runs once,
    on the best graph, at the end); FF_JOINT_MAX_GRAPHS bounds the graphs costed in all.
    Returns (strategy, report, rewrite sequence); model.layers is left as the best graph."""
    from .unity import search as param_search
    cfg = model.config
    if model._output is None:
        model._output = model.output_tensor()  # keep the model output's role stable under rewrites
    if budget is None:
        env = os.environ.get("FF_JOINT_BUDGET")
        budget = int(env) if env else (cfg.search_budget if cfg.search_budget and cfg.search_budget > 0 else 8)
    max_graphs = int(os.environ.get("FF_JOINT_MAX_GRAPHS", "64"))
    alpha = alpha if alpha is not None else max(1.0, float(cfg.search_alpha or 1.0))
    xfers = build_xfers(model)
    t0 = time.perf_counter()
    stamp_init_slots(model)
    base = snapshot(model)
    _, rep0 = param_search(model, algo, quick=True)
    best = [rep0["predicted_ms"], []]
    tried = []
    seen = {graph_key(model)}
    queue: List[Tuple[float, int, list]] = [(rep0["predicted_ms"], 0, [])]
    tick = 1
    evals = 1
    pops = 0
    rejected = set()  # rewrites that did not beat the graph they were applied to
    tlimit = float(getattr(cfg, "search_time_s", 0) or 0)
    timed_out = False

    def out_of_time():
        return tlimit > 0 and time.perf_counter() - t0 > tlimit

    while queue and pops < budget and evals < max_graphs:
        if out_of_time():
            timed_out = True
            break
        cost, _, seq = heapq.heappop(queue)
        pops += 1
        if cost > best[0] * alpha:
            continue
        restore(model, base)
        replay(model, xfers, seq)
        cur = snapshot(model)
        cur_ids = {id(L) for L in model.layers}
        for x in xfers:
            if evals >= max_graphs or timed_out:
                break
            for m in x.matches(model)[:4]:
                if evals >= max_graphs:
                    break
                if out_of_time():
                    timed_out = True
                    break
                ck = _class_key(x, m)
                if ck in rejected:
                    continue
                restore(model, cur)
                if not x.apply(model, m):
                    continue
                key = graph_key(model)
                if key in seen:
                    continue
                seen.add(key)
                _, rep = param_search(model, algo, quick=True)
                evals += 1
                c = rep["predicted_ms"]
                if os.environ.get("FF_SEARCH_PROGRESS") == "1":
                    print(f"[joint] graph {evals}: {x.name} -> {c:.4f} ms (best {best[0]:.4f})", file=sys.stderr,
                          flush=True)
                step = (x.name, _tuple(m))
                tried.append({"xfer": x.name, "match": _jsonable(m), "after": [s_[0] for s_ in seq],
                              "new_ops": [L.name for L in model.layers if id(L) not in cur_ids][:4],
                              "predicted_ms": round(c, 4)})
                if c >= cost:
                    rejected.add(ck)
                if c < best[0]:
                    best = [c, seq + [step]]
                if c < best[0] * alpha:
                    heapq.heappush(queue, (c, tick, seq + [step]))
                    tick += 1
    restore(model, base)
    strat0 = rep_full0 = None
    if best[1]:  # the rewritten graph must also win under the full search
        strat0, rep_full0 = param_search(model, algo)
        replay(model, xfers, best[1])
    strat, rep = param_search(model, algo)  # full search (simulator refinement, resource splits)
    if rep_full0 is not None and rep_full0["predicted_ms"] <= rep["predicted_ms"]:
        restore(model, base)
        strat, rep, best = strat0, rep_full0, [rep_full0["predicted_ms"], []]
    rep = dict(rep)
    # the starting graph's full search result, for the report's speedup against data parallel
    rep.update({"joint": True, "graphs_costed": evals, "graphs_popped": pops, "budget": budget,
                "time_limit_s": tlimit, "timed_out": timed_out,
                "xfers": len(xfers), "joint_s": round(time.perf_counter() - t0, 3),
                "rewrites": [{"xfer": n, "match": _jsonable(m)} for n, m in best[1]],
                "start_graph_ms": round(rep0["predicted_ms"], 4),
                "predicted_dp_ms": rep0["predicted_dp_ms"],
                "predicted_speedup_vs_dp": round(rep0["predicted_dp_ms"] / max(rep["predicted_ms"], 1e-9), 4),
                "tried": tried[:128]})
    return strat, rep, [(n, _jsonable(m)) for n, m in best[1]]


def replay_broadcast(model, seq):
    """Non-root ranks: rebuild rank 0's chosen graph from its rewrite sequence."""
    if model._output is None:
        model._output = model.output_tensor()
    xfers = build_xfers(model)
    stamp_init_slots(model)
    return replay(model, xfers, [(n, _tuple(m)) for n, m in seq])
