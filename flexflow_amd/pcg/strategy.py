"""Parallelization strategies: per-op parallel configs, their tensor layouts, and strategy files.

An `OpConfig` assigns a degree to every parallel axis of an op (its output dims + op-specific
reduction axes, see ops/base.py) and a device for every part — the reference's
ParallelConfig/MachineView pair (include/flexflow/machine_view.h, parallel_tensor.h). From it the
layouts of every input requirement, weight shard and output follow mechanically
(`op_layouts`), which is what both the executor and the cost model consume.

Strategy files are JSON (`{"version": 1, "num_devices": N, "ops": {layer_name: {"degrees": [...],
"devices": [...]}}}`), written by `--export-strategy` and read by `--import-strategy` — the
reference parses these flags but never uses them (model.cc:2812-2815); here they round-trip.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from ..parallel.layout import Layout
from ..type import OperatorType


@dataclass(frozen=True)
class OpConfig:
    degrees: Tuple[int, ...]
    devices: Tuple[int, ...]

    @property
    def num_parts(self) -> int:
        return int(math.prod(self.degrees))

    def coords(self, p: int) -> Tuple[int, ...]:
        cs = []
        for d in reversed(self.degrees):
            cs.append(p % d)
            p //= d
        return tuple(reversed(cs))

    def part(self, coords: Sequence[int]) -> int:
        p = 0
        for c, d in zip(coords, self.degrees):
            p = p * d + c
        return p

    def to_json(self):
        return {"degrees": list(self.degrees), "devices": list(self.devices)}

    @staticmethod
    def from_json(d):
        return OpConfig(tuple(d["degrees"]), tuple(d["devices"]))


def tensor_layout(shape, dim_axes, cfg: OpConfig, partial_axes=(), halo=None) -> Layout:
    """Layout of a tensor whose dim i is partitioned along op axis dim_axes[i] (None = whole).
    Op axes with degree > 1 that the tensor does not map become its replica dims (in axis order)."""
    nax = len(cfg.degrees)
    mapped = [a for a in dim_axes if a is not None]
    degrees = tuple(cfg.degrees[a] if a is not None else 1 for a in dim_axes)
    rep_axes = [a for a in range(nax) if a not in mapped and cfg.degrees[a] > 1]
    replicas = int(math.prod(cfg.degrees[a] for a in rep_axes)) if rep_axes else 1
    nblocks = int(math.prod(degrees))
    devices = [0] * (nblocks * replicas)
    for p in range(cfg.num_parts):
        c = cfg.coords(p)
        block = [c[a] if a is not None else 0 for a in dim_axes]
        r = 0
        for a in rep_axes:
            r = r * cfg.degrees[a] + c[a]
        b = 0
        for bc, d in zip(block, degrees):
            b = b * d + bc
        devices[b * replicas + r] = cfg.devices[p]
    partial = bool(partial_axes) and any(cfg.degrees[a] > 1 for a in partial_axes)
    if partial:
        assert set(rep_axes) <= set(partial_axes), "outputs may only be replicated over partial-sum axes"
    return Layout(tuple(shape), degrees, replicas, tuple(devices), partial, halo)


@dataclass
class OpLayouts:
    inputs: List[Layout]
    weights: List[Layout]
    outputs: List[Layout]


def op_layouts(layer, cfg: OpConfig) -> OpLayouts:
    impl = layer.impl
    ins = []
    for i, (t, m) in enumerate(zip(layer.inputs, impl.input_maps())):
        halo = impl.input_halo(i, cfg.degrees) if len(cfg.degrees) > 0 else None
        if halo is not None and not any(halo):
            halo = None
        ins.append(tensor_layout(t.dims, m, cfg, halo=halo))
    ws = [tensor_layout(w.dims, m, cfg) for w, m in zip(layer.weights, impl.weight_maps())]
    pax = impl.partial_axes()
    outs = [tensor_layout(o.dims, m, cfg, partial_axes=pax) for o, m in zip(layer.outputs, impl.output_maps())]
    return OpLayouts(ins, ws, outs)


def valid_config(layer, cfg: OpConfig) -> bool:
    impl = layer.impl
    sizes = impl.axis_sizes()
    if len(cfg.degrees) != len(sizes) or len(cfg.devices) != cfg.num_parts:
        return False
    if len(set(cfg.devices)) != len(cfg.devices):
        return False
    kinds = impl.axis_kinds()
    for a, (d, s) in enumerate(zip(cfg.degrees, sizes)):
        if d == 1:
            continue
        if s % d != 0 or kinds[a] == "none" or not impl.supports_axis(a):
            return False
    # every tensor dim must divide
    try:
        op_layouts(layer, cfg)
    except AssertionError:
        return False
    return True


def divisors(n: int) -> List[int]:
    return [d for d in range(1, n + 1) if n % d == 0]


def machine_device_sets(num_devices: int, gpus_per_node: Optional[int] = None) -> Dict[int, List[Tuple[int, ...]]]:
    """parts -> device tuples of every machine view of the machine (native MachineResource:
    aligned contiguous blocks `i | N` as the reference's register_all_machine_views,
    graph.cc:2329-2360, plus whole-node 2-D grids and one-GPU-per-node strided views on multi-node
    machines). Falls back to contiguous aligned blocks when the native core is not built."""
    gpn = max(1, min(gpus_per_node or num_devices, num_devices))
    nodes = max(1, num_devices // gpn)
    out: Dict[int, List[Tuple[int, ...]]] = {}
    try:
        from flexflow_amd import _core
        res = _core.MachineResource(num_nodes=nodes, gpus_per_node=gpn)
        for v in res.enumerate_views():
            ids = tuple(v.device_ids())
            out.setdefault(len(ids), [])
            if ids not in out[len(ids)]:
                out[len(ids)].append(ids)
    except ImportError:
        for p in divisors(num_devices):
            out[p] = [tuple(range(st, st + p)) for st in range(0, num_devices, p)]
    return out


def enumerate_configs(layer, num_devices: int, allow_kinds=("sample", "attribute", "parameter"),
                      max_configs: int = 64, contiguous_starts: bool = True,
                      device_sets: Optional[Dict[int, List[Tuple[int, ...]]]] = None) -> List[OpConfig]:
    """Candidate parallelizations of one op: degree combos over its allowed axes whose product
    divides the device count, each placed on every machine view with that many parts
    (machine_device_sets; contiguous_starts=False keeps only the view starting at device 0)."""
    impl = layer.impl
    pin = getattr(impl, "pinned_config", None)
    if pin is not None:  # explicit parallel ops (ops/parallel_ops.py) fix their output layout
        return [pin(num_devices)]
    sizes = impl.axis_sizes()
    kinds = impl.axis_kinds()
    axes = [a for a, k in enumerate(kinds) if k in allow_kinds and impl.supports_axis(a)]
    out: List[OpConfig] = []
    degs = [1] * len(sizes)
    if device_sets is None:
        device_sets = machine_device_sets(num_devices)

    def rec(i, prod):
        if i == len(axes):
            P = prod
            sets = device_sets.get(P, [tuple(range(P))])
            if not contiguous_starts:
                sets = [s for s in sets if s[0] == 0][:1] or sets[:1]
            for devs in sets:
                cfg = OpConfig(tuple(degs), tuple(devs))
                if valid_config(layer, cfg):
                    out.append(cfg)
            return
        a = axes[i]
        for d in divisors(num_devices // prod):
            if sizes[a] % d:
                continue
            degs[a] = d
            rec(i + 1, prod * d)
        degs[a] = 1

    rec(0, 1)
    pinned = layer.attrs.get("pin")
    if pinned is not None and math.prod(pinned) > num_devices:
        pinned = None  # a plan for more devices replayed on fewer (e.g. a 1-process reference run)
    if pinned is not None:  # a parallelization rewrite (pcg/joint.py) fixed this op's degrees
        out = [c for c in out if tuple(c.degrees) == tuple(pinned)] or \
            [OpConfig(tuple(pinned), tuple(range(int(math.prod(pinned)))))]
    return _cap_candidates(out, max_configs)


def _cap_candidates(cands: List[OpConfig], max_configs: int) -> List[OpConfig]:
    """Cap the candidate list with a quota per part count (1, 2, 4, 8, ... devices), each quota
    filled round-robin over the machine views of that size. Sorting by part count and truncating
    (round 2) dropped every placement on fewer devices at 8 GPUs — a Linear has 34 configs using
    8/4/2 devices — so operator placement and branch-parallel resource splits never reached the
    DP. Any budget a small group leaves unused goes to the larger part counts."""
    if len(cands) <= max_configs:
        return sorted(cands, key=lambda c: (-c.num_parts, c.devices[0], c.degrees))
    groups: Dict[int, List[OpConfig]] = {}
    for c in sorted(cands, key=lambda c: (c.degrees, c.devices)):
        groups.setdefault(c.num_parts, []).append(c)
    for P, lst in groups.items():  # interleave the views: every device block shows up early
        by_view: Dict[Tuple[int, ...], List[OpConfig]] = {}
        for c in lst:
            by_view.setdefault(c.devices, []).append(c)
        views = sorted(by_view, key=lambda v: v[0])
        inter = []
        for k in range(max(len(v) for v in by_view.values())):
            inter += [by_view[v][k] for v in views if k < len(by_view[v])]
        groups[P] = inter
    order = sorted(groups, reverse=True)
    quota = max(1, max_configs // len(order))
    take = {P: min(quota, len(groups[P])) for P in order}
    spare = max_configs - sum(take.values())
    for P in order:
        extra = min(spare, len(groups[P]) - take[P])
        take[P] += extra
        spare -= extra
    out = [c for P in order for c in groups[P][:take[P]]]
    return out


def data_parallel_config(layer, num_devices: int) -> OpConfig:
    """Reference --only-data-parallel: partition the sample dim over all devices when legal,
    otherwise run the op on device 0 (degree 1)."""
    pin = getattr(layer.impl, "pinned_config", None)
    if pin is not None:
        return pin(num_devices)
    if layer.attrs.get("pin") is not None and math.prod(layer.attrs["pin"]) <= num_devices:
        degs = tuple(layer.attrs["pin"])  # pinned by a joint-search rewrite: its only layout
        return OpConfig(degs, tuple(range(int(math.prod(degs)))))
    sizes = layer.impl.axis_sizes()
    n = len(sizes)
    for d in sorted(divisors(num_devices), reverse=True):
        degs = [1] * n
        degs[0] = d
        cfg = OpConfig(tuple(degs), tuple(range(d)))
        if layer.impl.axis_kinds()[0] == "sample" and valid_config(layer, cfg):
            return cfg
    return OpConfig(tuple([1] * n), (0,))


def data_parallel_strategy(layers, num_devices: int) -> Dict[str, OpConfig]:
    return {l.name: data_parallel_config(l, num_devices) for l in layers}


def save_strategy(path: str, strategy: Dict[str, OpConfig], num_devices: int, extra: Optional[dict] = None):
    doc = {"version": 1, "num_devices": num_devices, "ops": {k: v.to_json() for k, v in strategy.items()}}
    if extra:
        doc.update(extra)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)


def load_strategy(path: str) -> Tuple[Dict[str, OpConfig], int]:
    with open(path) as f:
        doc = json.load(f)
    return {k: OpConfig.from_json(v) for k, v in doc["ops"].items()}, int(doc.get("num_devices", 1))


def load_strategy_pb(path: str, layers, num_devices: int) -> Dict[str, OpConfig]:
    """The reference's legacy protobuf strategy files (src/runtime/strategy.proto: Strategy { repeated
    Op ops = 1 }, Op { name = 1; device_type = 2; repeated dims = 3; repeated device_ids = 4 }, e.g.
    examples/cpp/DLRM/strategies/*.pb), read as data with our wire decoder.

    `dims` are per-output-dim parallel degrees in Legion order (innermost first); `device_ids` the
    devices of the parts. An entry applies to the layer of that exact name, else to the k-th layer of
    that type when named "<type><k>" (the reference named its ops "embedding0", "embedding1", ...),
    else to every layer of that type when named by the bare type ("linear", "concat"). Layers with
    no entry, or whose entry is not a valid config for them here, are left out (data parallel)."""
    from ..utils.protowire import fields, packed_varints
    with open(path, "rb") as f:
        data = f.read()
    table = {}
    for fno, _, v in fields(data):
        if fno != 1:
            continue
        name, dims, devs = "", [], []
        for f2, wt2, v2 in fields(v):
            if f2 == 1:
                name = v2.decode()
            elif f2 == 3:
                dims += packed_varints(v2, wt2)
            elif f2 == 4:
                devs += packed_varints(v2, wt2)
        table[name] = (dims, devs)
    return _table_configs(table, layers, num_devices)


def load_strategy_text(path: str, layers, num_devices: int) -> Dict[str, OpConfig]:
    """The text strategy files of the reference's Triton backend (triton/src/strategy.cc
    `PartitionStrategy::LoadStrategy`; e.g. triton/qa/L0_e2e/models/add/1/model.strategy):

        <num_ops>
        <op_name> <device_type 0=GPU|1=CPU> <ndims> <dim_{n-1}> ... <dim_0> <num_ids> <id> ...

    The dims are listed outermost first (the loader fills dim[n-1] first). Same per-layer matching
    and validation as the protobuf form."""
    with open(path) as f:
        tok = f.read().split()
    pos = 0

    def nxt():
        nonlocal pos
        pos += 1
        return tok[pos - 1]

    table = {}
    for _ in range(int(nxt())):
        name = nxt()
        dev_type = int(nxt())
        if dev_type not in (0, 1):
            raise ValueError(f"{path}: unsupported device type {dev_type} for {name}")
        nd = int(nxt())
        outer_first = [int(nxt()) for _ in range(nd)]
        nids = int(nxt())
        ids = [int(nxt()) for _ in range(nids)]
        if nids and nids != math.prod(outer_first):
            raise ValueError(f"{path}: {name} lists {nids} devices for {math.prod(outer_first)} parts")
        table[name] = (list(reversed(outer_first)), ids)  # Legion order, like the protobuf files
    return _table_configs(table, layers, num_devices)


def _table_configs(table, layers, num_devices: int) -> Dict[str, OpConfig]:
    out: Dict[str, OpConfig] = {}
    per_type: Dict[str, int] = {}
    for L in layers:
        base = L.op_type.name[3:].lower()
        k = per_type.get(base, 0)
        per_type[base] = k + 1
        ent = table.get(L.name) or table.get(f"{base}{k}") or table.get(base)
        if ent is None:
            continue
        dims, devs = ent
        n_axes = len(data_parallel_config(L, num_devices).degrees)
        n_out = len(L.outputs[0].dims) if L.outputs else n_axes
        outer_first = list(reversed(dims))
        deg = [1] * n_axes
        if outer_first:
            deg[0] = int(outer_first[0])  # sample dim
            inner = outer_first[1:]
            for j, d in enumerate(reversed(inner)):  # innermost dims align with our last output dims
                if n_out - 1 - j >= 1:
                    deg[n_out - 1 - j] = int(d)
        cfg = OpConfig(tuple(deg), tuple(int(d) for d in devs[:math.prod(deg)]))
        if len(cfg.devices) == cfg.num_parts and all(0 <= d < num_devices for d in cfg.devices) and \
                valid_config(L, cfg):
            out[L.name] = cfg
    return out
