"""Per-rank SPMD executor (replaces the reference's Legion index-task launches, mapper and
region-based data movement: FFModel::forward/backward/update, model.cc:2401-2474, and
FFMapper, src/mapper/mapper.cc).

Every rank runs the same program: for each op in topological order, the edge transfers that
bring its inputs into the layouts its parallel config requires (collectives over RCCL), then —
iff the rank owns a part of the op — the op's HIP kernels on its local shards. The backward pass
mirrors it with the dual transfers; weight gradients land in flat fp32 arenas whose buckets are
all-reduced asynchronously as they complete (overlapping the rest of the backward), and `update`
applies one fused optimizer kernel per arena.

Static, step-invariant structure (layouts, transfers, process groups, weight arenas, input
staging buffers) is built once in `__init__`, so a whole forward+backward step can be captured
into a hipGraph (runtime/graph.py) when the strategy has no in-step collectives.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import kernels as K
from ..ops import OpCtx, torch_dtype
from ..parallel.comm import Communicator, GradBucketer, Transfer
from ..parallel.layout import Layout, rel_slices
from ..pcg.strategy import OpConfig, op_layouts
from ..type import ActiMode, DataType, LossType, MetricsType, OperatorType
from ..ops.elementwise import BINARY as _BINARY

BINARY_OPS = frozenset(_BINARY.keys())


class WeightArena:
    """Flat storage for all local weight shards sharing one replica (gradient-sync) group."""

    def __init__(self, group: tuple, device, lowp_dtype):
        self.group = group
        self.device = device
        self.lowp_dtype = lowp_dtype
        self.entries = []  # (param, offset, numel, shape)
        self.size = 0
        self.acc_end = 0   # entries [0, acc_end) accumulate their gradient (+=): zeroed every step
        self.master = self.grad = self.lowp = None

    def add(self, param, shape):
        n = int(math.prod(shape))
        # 16-byte align every shard so vector kernels / GEMM operand loads stay aligned
        self.entries.append((param, self.size, n, tuple(shape)))
        self.size += (n + 7) // 8 * 8

    def materialize(self):
        self.master = torch.zeros(max(self.size, 8), dtype=torch.float32, device=self.device)
        self.grad = torch.zeros_like(self.master)
        if self.lowp_dtype is not None:
            self.lowp = torch.zeros(max(self.size, 8), dtype=self.lowp_dtype, device=self.device)

    def views(self, i):
        _, off, n, shape = self.entries[i]
        m = self.master[off:off + n].view(shape)
        g = self.grad[off:off + n].view(shape)
        c = self.lowp[off:off + n].view(shape) if self.lowp is not None else m
        return m, g, c


def _device_for(config):
    if torch.cuda.is_available() and not getattr(config, "cpu_only", False):
        return torch.device("cuda", config.local_rank % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


class Executor:
    def __init__(self, model, strategy: Dict[str, OpConfig], loss_type: Optional[LossType], metrics, training=True):
        self.model = model
        cfg = model.config
        self.config = cfg
        self.hooks = []  # per-op context managers: OpProfiler, NonFiniteGuard (runtime/profiler.py, health.py)
        self.rank, self.world = cfg.rank, cfg.world_size
        if torch.cuda.is_available() and os.environ.get("FF_CONV_BENCHMARK", "0") == "1":
            # opt-in MIOpen find mode (time every solver once per convolution shape). Off by
            # default: its exhaustive search ran > 3 min for ResNet-50's shapes on a fresh box,
            # while immediate mode measured the same AlexNet step time (7.0 ms at batch 256)
            torch.backends.cudnn.benchmark = True
        self.device = _device_for(cfg)
        self.training = training
        self.cdt = DataType.DT_BF16 if cfg.compute_dtype == DataType.DT_BF16 else DataType.DT_FLOAT
        self.ctorch = torch.bfloat16 if self.cdt == DataType.DT_BF16 else torch.float32
        self.layers = list(model.layers)
        self.strategy = strategy
        self.loss_type = loss_type
        self.metrics = list(metrics or [])
        self.step_idx = 0
        self.comm = Communicator(self.rank, self.world)

        self.lay = {L.name: op_layouts(L, strategy[L.name]) for L in self.layers}
        self.local: Dict[str, bool] = {}
        self.ctx: Dict[str, OpCtx] = {}
        for L in self.layers:
            scfg = strategy[L.name]
            mine = [p for p, d in enumerate(scfg.devices) if d == self.rank]
            self.local[L.name] = bool(mine)
            if mine:
                self.ctx[L.name] = OpCtx(layer=L, part_coords=scfg.coords(mine[0]), degrees=scfg.degrees,
                                         compute_dtype=self.cdt, training=training, seed=cfg.seed)
        self.producer_layout: Dict[int, Layout] = {}
        for L in self.layers:
            for o, lo in zip(L.outputs, self.lay[L.name].outputs):
                self.producer_layout[o.guid] = lo

        # model output / loss plumbing
        self.output_tensor = model.output_tensor()
        self._build_grad_reachability()
        self._build_transfers()
        self._alloc_weights()
        self._setup_loss()
        self.values: Dict[int, Optional[torch.Tensor]] = {}
        self.inputs: Dict[int, torch.Tensor] = {}
        self._metric_acc = torch.zeros(8, dtype=torch.float32, device=self.device)
        self.last_loss = None
        self.comm.ensure_groups(self._rank_sets)

    # ------------------------------------------------------------------ static analysis
    def _build_grad_reachability(self):
        need = {self.output_tensor.guid} if self.output_tensor is not None else set()
        self.layer_bwd: Dict[str, bool] = {}
        for L in reversed(self.layers):
            nb = any(o.guid in need for o in L.outputs) and L.op_type != OperatorType.OP_INPUT
            self.layer_bwd[L.name] = nb and self.training
            if nb:
                for j, t in enumerate(L.inputs):
                    if L.impl.needs_input_grad(j) and t.data_type in (DataType.DT_FLOAT, DataType.DT_HALF,
                                                                        DataType.DT_DOUBLE, DataType.DT_BF16):
                        need.add(t.guid)
        self.tensor_needs_grad = need
        # a grad only has to flow into an input whose producer (or its ancestors) owns weights
        has_w = set()
        for L in self.layers:
            if L.weights or any(t.guid in has_w for t in L.inputs):
                for o in L.outputs:
                    has_w.add(o.guid)
        self.grad_useful = has_w

    def _build_transfers(self):
        self.fwd_tx: Dict[Tuple[str, int], Transfer] = {}
        self.bwd_tx: Dict[Tuple[str, int], Transfer] = {}
        self.in_grad: Dict[Tuple[str, int], bool] = {}
        rank_sets = []
        for L in self.layers:
            if L.op_type == OperatorType.OP_INPUT:
                continue
            for j, t in enumerate(L.inputs):
                src = self.producer_layout[t.guid]
                dst = self.lay[L.name].inputs[j]
                tx = Transfer(src, dst, src.partial, self.rank)
                self.fwd_tx[(L.name, j)] = tx
                rank_sets += tx.rank_sets()
                ig = (self.layer_bwd[L.name] and t.guid in self.tensor_needs_grad and t.guid in self.grad_useful
                      and L.impl.needs_input_grad(j))
                self.in_grad[(L.name, j)] = ig
                if ig:
                    btx = Transfer(dst.with_(partial=False), src.with_(partial=False),
                                   dst.replicas > 1 or dst.halo is not None, self.rank)
                    self.bwd_tx[(L.name, j)] = btx
                    rank_sets += btx.rank_sets()
            if L.name in self.ctx:
                # first Linear-like ops whose input needs no grad skip the dgrad GEMM
                self.ctx[L.name].extra["need_dx0"] = bool(L.inputs) and self.in_grad.get((L.name, 0), False)
                lo = self.lay[L.name]
                if lo.inputs:
                    p = lo.inputs[0].parts_on(self.rank)
                    if p:
                        self.ctx[L.name].extra["in_region0"] = lo.inputs[0].region(p[0])
                if lo.outputs:
                    p = lo.outputs[0].parts_on(self.rank)
                    if p:
                        self.ctx[L.name].extra["out_region"] = lo.outputs[0].region(p[0])
        self._rank_sets = rank_sets
        # forward consumers of every tensor, in layer order (the order every rank issues the
        # prefetched transfers in: collectives must be issued in the same order on all ranks)
        self._consumers: Dict[int, List[Tuple[str, int]]] = {}
        for L in self.layers:
            if L.op_type == OperatorType.OP_INPUT:
                continue
            seen = set()
            for j, t in enumerate(L.inputs):
                k = (t.guid, self.lay[L.name].inputs[j].key())
                if k in seen:
                    continue  # a repeated (tensor, layout) input is moved once (forward's cache)
                seen.add(k)
                self._consumers.setdefault(t.guid, []).append((L.name, j))
        self.overlap_comm = os.environ.get("FF_OVERLAP_COMM", "1") != "0"
        self.comm_trace = None  # list of (event, kind, edge, op counter) when tracing (profiler / tests)
        self._op_counter = 0

    def _alloc_weights(self):
        lowp = torch.bfloat16 if self.cdt == DataType.DT_BF16 else None
        self.arenas: Dict[tuple, WeightArena] = {}
        self.weight_loc: Dict[int, Tuple[WeightArena, int]] = {}
        self.weight_layout: Dict[int, Layout] = {}
        self.weight_users: Dict[int, int] = {}
        for L in self.layers:
            for w in L.weights:
                if self.layer_bwd.get(L.name) and self.local.get(L.name):
                    self.weight_users[w.guid] = self.weight_users.get(w.guid, 0) + 1
        # Gradients an op fully OVERWRITES (a weight GEMM with beta = 0: Linear / attention / LSTM
        # matrices whose layer is the weights' only user) need no zeroing between steps; every other
        # gradient is accumulated into (+=: biases, norms, embeddings, shared weights). Each arena
        # lays out its accumulated entries first, so zero_gradients() clears one prefix instead of
        # the whole ~1.5 GB fp32 arena of BERT-Large. Within each group the order stays backward-
        # completion order (reverse layers) for the bucketed all-reduce.
        placed = []
        for L in reversed(self.layers):  # backward completion order
            single = bool(L.weights) and all(self.weight_users.get(w.guid, 1) == 1 for w in L.weights)
            for i, (w, wl) in enumerate(zip(L.weights, self.lay[L.name].weights)):
                if w.guid in self.weight_layout:  # shared weight (shared_op): allocated once
                    assert self.weight_layout[w.guid].key() == wl.key(), "shared weights need equal layouts"
                    continue
                self.weight_layout[w.guid] = wl
                parts = wl.parts_on(self.rank)
                if not parts:
                    continue
                p = parts[0]
                grp = tuple(sorted(wl.replica_group(wl.coords(p)[0])))
                ow = single and self.training and L.impl.overwrites_wgrad(i)
                placed.append((ow, grp, w, wl.local_shape(p)))
        for ow_pass in (False, True):
            for ow, grp, w, shape in placed:
                if ow != ow_pass:
                    continue
                ar = self.arenas.setdefault(grp, WeightArena(grp, self.device, lowp))
                ar.add(w, shape)
                self.weight_loc[w.guid] = (ar, len(ar.entries) - 1)
                if not ow:
                    ar.acc_end = ar.size
        # ZeRO-1 sharded optimizer (opt-in --zero / FF_ZERO=1): replicated (data-parallel) arenas
        # reduce-SCATTER their gradient buckets, each rank runs the optimizer on its 1/R chunk of
        # every bucket, and the updated compute copy is all-gathered back, per bucket, while the
        # next forward runs (each layer waits only for the buckets holding its weights)
        self.zero = bool(getattr(self.config, "zero_optimizer", False) or os.environ.get("FF_ZERO") == "1") \
            and self.comm.distributed
        for grp, ar in self.arenas.items():
            if self.zero and len(grp) > 1:
                unit = 16 * len(grp)
                ar.size = (ar.size + unit - 1) // unit * unit
            ar.materialize()
        # process groups are created collectively: every rank must list EVERY gradient-sync group
        # (also those it is not part of) in the same order, not just its own arenas' groups —
        # otherwise ranks call new_group on different sets and a strategy with replica subgroups
        # smaller than the world (e.g. sample 2 x parameter 4 on 8 ranks) deadlocks at compile
        all_groups = set()
        for wl in self.weight_layout.values():
            for blk in wl.blocks():
                all_groups.add(tuple(sorted(wl.replica_group(blk))))
        self._rank_sets += sorted(all_groups)
        bucket_bytes = int(self.config.grad_bucket_mb * (1 << 20))
        cdt = torch.bfloat16 if getattr(self.config, "grad_comm_dtype", "fp32") == "bf16" else None
        self.bucketer = GradBucketer(self.comm, bucket_bytes, cdt)
        self.zero_buckets = {}  # arena group -> sharded buckets
        self._w_buckets = {}    # weight guid -> [(arena group, bucket index)]
        self._ag_pending = {}   # (arena group, bucket index) -> async all-gather handle
        self._master_stale = False
        for grp, ar in self.arenas.items():
            segs = [(w.guid, off, off + n) for (w, off, n, _) in ar.entries]
            if self.zero and len(grp) > 1:
                bs = self.bucketer.add_sharded_arena(grp, ar.grad, segs, self.rank)
                self.zero_buckets[grp] = bs
                for key, lo, hi in segs:
                    self._w_buckets[key] = [(grp, i) for i, b in enumerate(bs) if lo < b["hi"] and hi > b["lo"]]
            else:
                self.bucketer.add_arena(grp, ar.grad, segs)
        # overlapped update (config.overlap_update, train_step only): bucket -> arena, side stream
        self._bucket_arena = {id(b): self.arenas[grp] for grp, _, bs in self.bucketer.arenas for b in bs}
        self._upd_stream = None
        self._upd_done = set()
        self._overlap_active = False
        self._opt_next_done = None  # the optimizer whose next() the overlapped backward already ran
        self._bwd_since_update = 0   # backward passes since the last update (row-sparse SGD guard)
        self.bucketer.on_ready = self._on_bucket_ready
        # workgroup cap of the overlapped update launches (FF_UPD_BLOCKS; 0 = the full 2048-block
        # sweep; < 0 = short-lived workgroups of -N float4 groups per thread, see optimizer.hip)
        self._upd_blocks = int(os.environ.get("FF_UPD_BLOCKS", "0"))
        self._sparse, self._sparse_key = {}, None  # row-sparse SGD plan (_sparse_plan)
        self._sparse_cleared = {}  # arena group -> [(lo, hi)] whose gradient the sparse update cleared
        self._marks = {}           # weight guid -> int32 [rows] scratch of the sparse update
        for L in self.layers:
            if L.name in self.ctx:
                self.ctx[L.name].extra["wgrad_overwrite"] = bool(L.weights) and all(
                    self.weight_users.get(w.guid, 1) == 1 for w in L.weights)
                self.ctx[L.name].wgrads = [self.weight_loc[w.guid][0].views(self.weight_loc[w.guid][1])[1]
                                           if w.guid in self.weight_loc else None for w in L.weights]

    def init_weights(self, seed_base: int, only=None):
        """Deterministic global init, each rank keeping its shard (only: re-initialise just these
        layers, the reference's Op.init)."""
        from ..core.initializers import BlockInitializer, default_initializer

        def resolve(w, li=None, i=None):
            # model-local seed (layer position, weight slot): identical in every process and
            # independent of how many models were built before. Graph rewrites stamp the slot of
            # the graph as written (w._init_slot) so that rewritten graphs initialise identically.
            slot = getattr(w, "_init_slot", None) or (li, i)
            seed = seed_base + 1009 * slot[0] + slot[1]
            init = w.initializer or default_initializer(getattr(w, "short_name", w.name), seed)
            if getattr(init, "seed", 0) is None:  # an explicit initializer asking for the model-local seed
                import copy
                init = copy.copy(init)
                init.seed = seed
            if isinstance(init, BlockInitializer):
                init.resolve = resolve
            return init

        done = set()
        for li, L in enumerate(self.layers):
            if only is not None and L not in only:
                continue
            for i, w in enumerate(L.weights):
                if w.guid not in self.weight_loc or w.guid in done:
                    continue
                done.add(w.guid)
                ar, idx = self.weight_loc[w.guid]
                m, _, c = ar.views(idx)
                init = resolve(w, li, i)
                full = torch.empty(w.dims, dtype=torch.float32, device=self.device)
                init.fill_full(full, w.dims)
                wl = self.weight_layout[w.guid]
                p = wl.parts_on(self.rank)[0]
                m.copy_(full[rel_slices(wl.region(p), tuple((0, s) for s in w.dims))])
                if c is not m:
                    c.copy_(m)

    def weight_tensor(self, w):
        ar, idx = self.weight_loc[w.guid]
        return ar.views(idx)[2]

    # ------------------------------------------------------------------ loss
    def _setup_loss(self):
        self.loss_layout = None
        self.label_layout = None
        self.softmax_fused = False  # inference-only models (no loss) keep plain softmax outputs
        self._softmax_last_dim = False
        self._fwd_training = self.training
        out = self.output_tensor
        if out is None or self.loss_type is None:
            return
        pl = self.producer_layout[out.guid]
        d0 = pl.degrees[0]
        devs = []
        for b in range(d0):
            blk = [b] + [0] * (pl.ndim - 1)
            devs.append(pl.devices[pl.part_index(blk, 0)])
        self.loss_layout = Layout(pl.shape, (d0,) + (1,) * (pl.ndim - 1), 1, tuple(devs))
        lab = self.model.label_tensor
        self.label_layout = Layout(tuple(lab.dims), (d0,) + (1,) * (len(lab.dims) - 1), 1, tuple(devs))
        self.loss_fwd_tx = Transfer(pl, self.loss_layout, pl.partial, self.rank)
        self.loss_bwd_tx = Transfer(self.loss_layout, pl.with_(partial=False), False, self.rank)
        self._rank_sets += self.loss_fwd_tx.rank_sets() + self.loss_bwd_tx.rank_sets()
        owner = out.owner_layer
        self.softmax_fused = (owner.op_type == OperatorType.OP_SOFTMAX and self.loss_type in (
            LossType.LOSS_CATEGORICAL_CROSSENTROPY, LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY))
        if self.softmax_fused and owner.name in self.ctx:
            self.ctx[owner.name].extra["loss_fused"] = True
        self._softmax_last_dim = self.softmax_fused and (owner.attrs.get("dim", -1) % len(out.dims) == len(out.dims) - 1)
        self._fwd_training = self.training

    def _softmax_emitted_logits(self) -> bool:
        """The fused softmax emits raw logits in training forwards (see ops/softmax.py)."""
        return self._softmax_last_dim and self._fwd_training

    # ------------------------------------------------------------------ inputs
    def input_layout(self, t) -> Layout:
        if t.guid in self.producer_layout:
            return self.producer_layout[t.guid]
        if self.model.label_tensor is not None and t.guid == self.model.label_tensor.guid:
            return self.label_layout
        raise KeyError(t)

    def feed(self, t, value):
        """Stage the global value of an input/label tensor: keep this rank's shard in a persistent
        device buffer (stable address for graph replay)."""
        lay = self.input_layout(t)
        parts = lay.parts_on(self.rank)
        if not parts:
            return
        reg = lay.region(parts[0])
        full = tuple((0, s) for s in lay.shape)
        if isinstance(value, np.ndarray):
            src = torch.from_numpy(np.ascontiguousarray(value[rel_slices(reg, full)]))
        else:
            src = value[rel_slices(reg, full)]
        is_float = t.data_type in (DataType.DT_FLOAT, DataType.DT_HALF, DataType.DT_DOUBLE, DataType.DT_BF16)
        dt = self.ctorch if is_float else torch_dtype(t.data_type)
        buf = self.inputs.get(t.guid)
        if buf is None or tuple(buf.shape) != tuple(src.shape) or buf.dtype != dt:
            buf = torch.empty(tuple(src.shape), dtype=dt, device=self.device)
            self.inputs[t.guid] = buf
        if src.device.type == "cpu" and self.device.type == "cuda":
            src = src.pin_memory() if not src.is_pinned() else src
            buf.copy_(src.to(dt) if src.dtype != dt and not is_float else src, non_blocking=True)
        else:
            buf.copy_(src)

    # ------------------------------------------------------------------ execution
    def _like(self, t):
        is_float = t.data_type in (DataType.DT_FLOAT, DataType.DT_HALF, DataType.DT_DOUBLE, DataType.DT_BF16)
        return torch.empty(0, dtype=self.ctorch if is_float else torch_dtype(t.data_type), device=self.device)

    def forward_layer(self, L, training: bool = False):
        """Run one layer on the current values of its inputs (the reference's Op.forward); its
        outputs replace the stored values."""
        vals = self.values
        if L.op_type == OperatorType.OP_INPUT:
            return
        xs = [self.fwd_tx[(L.name, j)].run(self.comm, vals.get(t.guid, self.inputs.get(t.guid)), self._like(t))
              for j, t in enumerate(L.inputs)]
        if self.local[L.name]:
            ctx = self.ctx[L.name]
            ctx.training = training
            outs = L.impl.forward(ctx, xs, [self.weight_tensor(w) for w in L.weights])
            if not training:
                ctx.saved.clear()
            for o, v in zip(L.outputs, outs):
                vals[o.guid] = v

    def _trace(self, event, kind, edge):
        if self.comm_trace is not None:
            self.comm_trace.append((event, kind, edge, self._op_counter))
        for h in self.hooks:
            if hasattr(h, "comm_event"):
                h.comm_event(event, kind, edge)

    def _prefetch(self, L, inflight):
        """Start the forward transfers of L's outputs to every consumer right after L ran (every
        rank, layer order): with RCCL the collective runs on the process group's stream while the
        compute stream goes on with the ops in between; the consumer waits only for its own input."""
        if not self.overlap_comm:
            return
        vals = self.values
        for o in L.outputs:
            for cname, j in self._consumers.get(o.guid, ()):
                tx = self.fwd_tx[(cname, j)]
                if tx.kind in ("identity", "local_slice"):
                    continue
                p = inflight[(cname, j)] = tx.start(self.comm, vals.get(o.guid), self._like(o))
                p.edge = ("fwd", cname, j)
                self._trace("issue", tx.kind, p.edge)

    def forward(self, training: Optional[bool] = None):
        tr = self.training if training is None else training
        self._fwd_training = tr
        # every registered transposed weight copy (kernels.weight_t) in one launch; a sharded
        # optimizer's weights still arrive by all-gather during the forward, so those ops refresh
        # their own copies (weight_t outside a batched forward)
        batched = bool(tr and self.device.type == "cuda" and not self._ag_pending
                       and os.environ.get("FF_WT_BATCH", "1") != "0")
        if batched:
            stores = [st for c in self.ctx.values() for k, st in c.extra.items() if k.startswith("wt_store")]
            K.wt_refresh_all(stores, self.__dict__.setdefault("_wt_batch", {}))
        K.wt_forward(batched)
        try:
            return self._forward(tr)
        finally:
            K.wt_forward(False)

    def _forward(self, tr):
        vals = self.values
        inflight = {}
        for L in self.layers:
            if L.op_type == OperatorType.OP_INPUT:
                o = L.outputs[0]
                vals[o.guid] = self.inputs.get(o.guid) if self.local[L.name] else None
                self._prefetch(L, inflight)
                continue
            xs, cache = [], {}
            for j, t in enumerate(L.inputs):
                key = (t.guid, self.lay[L.name].inputs[j].key())
                if key not in cache:
                    p = inflight.pop((L.name, j), None)
                    if p is not None:
                        cache[key] = p.wait()
                        self._trace("wait", p.kind, p.edge)
                    else:
                        cache[key] = self.fwd_tx[(L.name, j)].run(self.comm, vals.get(t.guid), self._like(t))
                xs.append(cache[key])
            if self.local[L.name]:
                ctx = self.ctx[L.name]
                ctx.training = tr
                ctx.step = self.step_idx
                if self._ag_pending:
                    self._wait_weights(L)
                ws = [self.weight_tensor(w) for w in L.weights]
                if self.hooks:
                    with self._hooked(L, "fwd"):
                        outs = L.impl.forward(ctx, xs, ws)
                        for o, v in zip(L.outputs, outs):
                            vals[o.guid] = v
                else:
                    outs = L.impl.forward(ctx, xs, ws)
                    for o, v in zip(L.outputs, outs):
                        vals[o.guid] = v
            else:
                for o in L.outputs:
                    vals[o.guid] = None
            self._op_counter += 1
            self._prefetch(L, inflight)
        for p in inflight.values():  # outputs nobody consumed (e.g. the model output's own edges)
            p.wait()

    def compute_loss_grad(self):
        """Loss gradient w.r.t. the model output (reference Loss::backward, scale 1/batch or
        2/volume for MSE-avg), seeded in the producer's layout."""
        out = self.output_tensor
        v = self.loss_fwd_tx.run(self.comm, self.values.get(out.guid), self._like(out))
        g = None
        if v is not None:
            lt = self.loss_type
            B = out.dims[0]
            lab = self.inputs.get(self.model.label_tensor.guid)
            rows = v.reshape(v.shape[0], -1) if lt != LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY else \
                v.reshape(-1, v.shape[-1])
            logits = not self.softmax_fused or self._softmax_emitted_logits()
            if lt == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
                labels = lab.reshape(-1).to(torch.int32)
                if not logits:
                    g, lrow = K.xent_grad(rows.contiguous(), labels, None, 1.0 / B, True)
                    self._metric_acc[0] += lrow.sum()
                else:  # fused softmax + cross-entropy (+ accuracy/CE metrics) straight from the logits
                    acc3 = torch.zeros(3, dtype=torch.float32, device=rows.device)
                    g, lrow = K.softmax_xent(rows.contiguous(), labels, 1.0 / B, acc3)
                    self._metric_acc[0] += acc3[1]
                    self._xent_acc3 = acc3
                self._lrow = lrow
            elif lt == LossType.LOSS_CATEGORICAL_CROSSENTROPY:
                oh = lab.reshape(rows.shape).to(rows.dtype)
                if self.softmax_fused:
                    g, lrow = K.xent_grad(rows.contiguous(), None, oh, 1.0 / B, False)
                else:
                    g = ((torch.softmax(rows.float(), -1) - oh.float()) / B).to(rows.dtype)
                    lrow = -(oh.float() * torch.log_softmax(rows.float(), -1)).sum(-1)
                self._metric_acc[0] += lrow.sum()
            elif lt in (LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, LossType.LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE):
                vol = math.prod(out.dims)
                sc = 2.0 / vol if lt == LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE else 1.0 / B
                g, l2 = K.mse_grad(v.contiguous(), lab.reshape(v.shape), sc)
                self._metric_acc[0] += l2.sum()
            else:  # identity
                g = torch.full_like(v, 1.0 / B)
                self._metric_acc[0] += v.float().sum()
            g = g.reshape(v.shape)
            self._metric_acc[7] += v.shape[0]
            self._accumulate_metrics(v, lab)
        return self.loss_bwd_tx.run(self.comm, g, self._like(out))

    def _accumulate_metrics(self, v, lab):
        mets = set(self.metrics)
        if not mets:
            return
        lt = self.loss_type
        if MetricsType.METRICS_ACCURACY in mets or MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY in mets \
                or MetricsType.METRICS_CATEGORICAL_CROSSENTROPY in mets:
            rows = v.reshape(-1, v.shape[-1])
            if lt == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
                labels = lab.reshape(-1).to(torch.int32)
            elif lab.shape[-1] == v.shape[-1] and v.shape[-1] > 1:
                labels = lab.reshape(rows.shape).float().argmax(-1).to(torch.int32)
            else:
                labels = None
            acc3 = getattr(self, "_xent_acc3", None)
            if acc3 is not None:  # already folded into the fused softmax-xent pass
                self._xent_acc3 = None
                self._metric_acc[1] += acc3[0]
                self._metric_acc[2] += acc3[1]
                self._metric_acc[3] += acc3[2]
            elif labels is not None and rows.shape[0] == labels.shape[0]:
                have_probs = self.softmax_fused and not self._softmax_emitted_logits()
                acc3 = torch.zeros(3, dtype=torch.float32, device=v.device)
                # argmax of logits == argmax of probabilities: accuracy needs no softmax pass
                K.metrics_classify(rows.contiguous(), labels, acc3)
                self._metric_acc[1] += acc3[0]
                self._metric_acc[3] += acc3[2]
                if have_probs:
                    self._metric_acc[2] += acc3[1]
                elif lt == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY and getattr(self, "_lrow", None) is not None:
                    self._metric_acc[2] += self._lrow.sum()
        if MetricsType.METRICS_MEAN_SQUARED_ERROR in mets or MetricsType.METRICS_ROOT_MEAN_SQUARED_ERROR in mets \
                or MetricsType.METRICS_MEAN_ABSOLUTE_ERROR in mets:
            if lab.numel() == v.numel():
                d = v.float() - lab.reshape(v.shape).float()
                self._metric_acc[4] += (d * d).sum()
                self._metric_acc[5] += d.abs().sum()
                self._metric_acc[6] += d.numel()

    def _overlap_possible(self):
        opt = self.model.optimizer
        from ..core.optimizers import Optimizer
        ranged = opt is not None and getattr(type(opt), "step_range", None) not in (None, Optimizer.step_range)
        return (self.training and ranged and not self.zero
                and not self._sparse_plan(opt)
                and not self.hooks and self.device.type == "cuda"
                and not torch.cuda.is_current_stream_capturing()
                and not any(L.attrs.get("regularizer") is not None for L in self.layers))

    def _on_bucket_ready(self, b, handle):
        """Overlapped update: bucket b's gradients are final (all-reduced when handle is set), so
        its slice of the fused optimizer runs now on a side stream while the backward continues.
        A bucket completes only after the backward of every op using its weights was issued (the
        executor marks a weight ready after its last user), so no later backward op reads the
        weights this overwrites. Memory-bound Adam beside compute-bound GEMMs: on BERT-Large about
        half of the ~2.5 ms pass overlaps the backward (step profile: busy exceeds span by
        ~1.3 ms, profiles/bert_large_b32_r3_w4_steps.txt); same-box A/B -0.2 ms/step."""
        if not self._overlap_active or b.get("sharded"):
            return
        if handle is not None and dist.get_backend(self.comm.group(b["group"])) != "nccl":
            return  # gloo's wait() blocks the host: leave this bucket to update()
        ar = self._bucket_arena.get(id(b))
        if ar is None or b["hi"] <= b["lo"]:
            return
        if self._upd_stream is None:
            self._upd_stream = self._make_upd_stream()
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self._upd_stream):
            self._upd_stream.wait_event(ev)
            if handle is not None:
                handle.wait()  # the side stream waits for the bucket's all-reduce
            # the bucket's update as launches of at most FF_UPD_CHUNK elements (default 4 Mi = 16 MB
            # per fp32 stream, ~23 us): each full-grid sweep holds every wave slot of every CU until
            # it ends, so a compute-stream kernel queued behind it waited out the whole 64 MiB
            # bucket (~93 us: col_reduce 5 -> 68 us, the persistent wgrad GEMM 125 -> 200 us);
            # between shorter launches the backward's kernels get the CUs. Same-box A/B, BERT-Large:
            # 43.76 -> 43.43 ms (1 Mi: no gain, 8 Mi: -0.1; profiles/update_interference_r6.txt); 0 = whole bucket
            ch = int(os.environ.get("FF_UPD_CHUNK", "4194304")) // 8 * 8
            pieces = [(a, min(a + ch, b["hi"])) for a in range(b["lo"], b["hi"], ch)] if ch > 0 else \
                [(b["lo"], b["hi"])]
            for lo, hi in pieces:
                if self._upd_blocks:
                    self.model.optimizer.step_range(ar, lo, hi, max_blocks=self._upd_blocks)
                else:  # plain call: user optimizers may implement step_range(arena, lo, hi) only
                    self.model.optimizer.step_range(ar, lo, hi)
        self._upd_done.add(id(b))

    def _make_upd_stream(self):
        """The overlapped update's side stream. FF_UPD_PRIO=low puts it at the lowest priority the
        device offers (torch's default streams sit at 0), so that when both streams have work ready
        the hardware scheduler hands freed CU slots to the backward's kernels first; "default" (the
        default) or an integer priority otherwise."""
        prio = os.environ.get("FF_UPD_PRIO", "default")
        p = 0
        if prio == "low":
            try:
                least, greatest = torch.cuda.Stream.priority_range()
                p = max(least, greatest)  # numerically larger = lower priority
            except Exception:
                p = 0
        elif prio != "default":
            p = int(prio)
        return torch.cuda.Stream(device=self.device, priority=p)

    def backward(self, overlap_update: bool = False):
        """overlap_update: update each gradient bucket as soon as it is final (see
        _on_bucket_ready); only train_step passes it, because the weights then change during
        backward() — the separate backward()/update() API keeps the reference's semantics.

        FF_DEFER_FOLDS=1 (with the overlapped update on one rank): the slab folds that finish
        parameter gradients (bias / LayerNorm column sums, split-K weight-gradient slabs) run on the
        update's side stream, ahead of the bucket updates that read them
        (kernels.set_reduce_stream); every reader of gradients on the compute stream joins that
        stream first (_join_folds). Off by default: same-box A/B at BERT-Large b32 measured no step
        gain (45.74-45.75 vs 45.78-45.83 ms, profiles/defer_folds_ab_r4.txt) — the folds are
        bandwidth-light but launch-bound, and running them beside the backward stretched them
        (col_reduce 1.4 -> 6.4 ms of busy time per step, bert_large_b32_r4_v2_steps.txt)."""
        defer = (bool(overlap_update) and not self.comm.distributed and self._overlap_possible()
                 and os.environ.get("FF_DEFER_FOLDS", "0") == "1")
        if defer:
            if self._upd_stream is None:
                self._upd_stream = self._make_upd_stream()
            K.set_reduce_stream(self._upd_stream)
            self._folds_pending = True
        # batched folds (kernels.fold_flush): the bias / LayerNorm gradient folds of the backward
        # queue up and launch a few per kernel, before each gradient bucket is reduced or updated
        # and at the end; not under per-op timing hooks (they would book the folds elsewhere)
        batch = (not defer and self.training and self.device.type == "cuda" and not self.hooks
                 and os.environ.get("FF_FOLD_BATCH", "1") != "0")
        if batch:
            K.set_fold_batching(True)
            self.bucketer.before_launch = K.fold_flush
        try:
            return self._backward(overlap_update)
        finally:
            if batch:
                K.fold_flush()
                K.set_fold_batching(False)
                self.bucketer.before_launch = None
            K.set_reduce_stream(None)

    def _join_folds(self):
        if getattr(self, "_folds_pending", False):
            torch.cuda.current_stream(self.device).wait_stream(self._upd_stream)
            self._folds_pending = False

    def _backward(self, overlap_update: bool = False):
        if self._ag_pending:  # sharded optimizer: weights of layers this rank did not run
            self.wait_all_gathers()
        self.bucketer.reset()
        self._upd_done = set()
        self._overlap_active = bool(overlap_update) and self._overlap_possible()
        self._opt_next_done = None
        self._bwd_since_update += 1
        if self._overlap_active:
            self.model.optimizer.next()  # this step's bias-corrected scalars, before any bucket update
            self._opt_next_done = self.model.optimizer
        self._wdone = {}
        grads: Dict[int, torch.Tensor] = {}
        gpend: Dict[int, list] = {}  # tensor guid -> in-flight gradient transfers (summed on use)

        def resolve(guid):
            for p in gpend.pop(guid, ()):
                v = p.wait()
                self._trace("wait", p.kind, p.edge)
                if v is None:
                    continue
                prev = grads.get(guid)
                grads[guid] = v if (prev is None or prev is v) else prev + v

        if self.output_tensor is not None and self.loss_type is not None:
            owner = self.output_tensor.owner_layer
            if self.softmax_fused and self.hooks and owner is not None:
                # the fused softmax-cross-entropy pass IS the output softmax's work (the simulator
                # books it there: pcg/costmodel.fused_xent_cost): profile it under that op
                with self._hooked(owner, "fwd"):
                    g = self.compute_loss_grad()
            else:
                g = self.compute_loss_grad()
            if g is not None:
                grads[self.output_tensor.guid] = g
        for L in reversed(self.layers):
            if not self.layer_bwd.get(L.name):
                continue
            dxs = None
            early = {}
            if self.local[L.name]:
                for o in L.outputs:
                    resolve(o.guid)
                douts = [grads.pop(o.guid, None) for o in L.outputs]
                if any(d is not None for d in douts):
                    ref = [d for d in douts if d is not None][0]
                    vals = [self.values.get(o.guid) for o in L.outputs]
                    douts = [d if d is not None else (torch.zeros_like(v) if v is not None else None)
                             for d, v in zip(douts, vals)]
                    ctx = self.ctx[L.name]
                    for t in L.inputs:
                        resolve(t.guid)  # in-place dgrad accumulation needs the concrete tensor
                    ctx.extra["dx_accum"] = self._accum_targets(L, grads, douts)
                    ctx.extra["dx_ready"] = self._dx_ready_cb(L, early) if self.overlap_comm else None
                    if self.hooks:
                        with self._hooked(L, "bwd"):
                            dxs = L.impl.backward(ctx, douts)
                    else:
                        dxs = L.impl.backward(ctx, douts)
                    ctx.extra["dx_accum"] = None
                    ctx.extra["dx_ready"] = None
                for w in L.weights:
                    self._wdone[w.guid] = self._wdone.get(w.guid, 0) + 1
                    if self._wdone[w.guid] == self.weight_users.get(w.guid, 1):
                        self.bucketer.mark_ready(w.guid)
            else:
                for o in L.outputs:
                    resolve(o.guid)
                    grads.pop(o.guid, None)
            self._op_counter += 1
            pending = {}
            for j, t in enumerate(L.inputs):
                if not self.in_grad.get((L.name, j)):
                    continue
                key = (t.guid, self.lay[L.name].inputs[j].key())
                gj = dxs[j] if dxs is not None and j < len(dxs) else None
                if key in pending:
                    if gj is not None:
                        prev = pending[key][2]
                        pending[key][2] = gj if prev is None else prev + gj
                else:
                    pending[key] = [t, j, gj]
            for key, (t, j, gj) in pending.items():
                tx = self.bwd_tx[(L.name, j)]
                p = early.pop(j, None)
                same = p is not None and gj is not None and p[1].data_ptr() == gj.data_ptr() and \
                    p[1].shape == gj.shape
                if not same:
                    if p is not None:
                        p[0].wait()  # superseded (the op changed the tensor after announcing it)
                    if tx.kind == "identity" or not self.overlap_comm:
                        gp = tx.run(self.comm, gj, self._like(t))
                        if gp is not None:
                            prev = grads.get(t.guid)
                            grads[t.guid] = gp if (prev is None or prev is gp) else prev + gp
                        continue
                    p = (tx.start(self.comm, gj, self._like(t)), gj)
                    p[0].edge = ("bwd", L.name, j)
                    self._trace("issue", tx.kind, p[0].edge)
                gpend.setdefault(t.guid, []).append(p[0])
        for guid in list(gpend):
            resolve(guid)

    def _dx_ready_cb(self, L, early):
        """Callback an op's backward may call as soon as input j's gradient is final (Linear: after
        the dgrad GEMM, before the wgrad GEMM): the gradient's transfer (e.g. the all-reduce of a
        row-parallel layer's partial dx) starts then and runs beside the wgrad GEMM."""
        counts = {}
        for t in L.inputs:
            counts[t.guid] = counts.get(t.guid, 0) + 1

        def ready(j, g):
            t = L.inputs[j]
            tx = self.bwd_tx.get((L.name, j))
            if (tx is None or not self.in_grad.get((L.name, j)) or counts[t.guid] != 1
                    or tx.kind == "identity" or j in early or g is None):
                return
            early[j] = (tx.start(self.comm, g, self._like(t)), g)
            early[j][0].edge = ("bwd", L.name, j)
            self._trace("issue", tx.kind, early[j][0].edge)
        return ready

    def _plan_inplace(self):
        """Reference in-place optimisation (model.cc:2885-2919): an element-wise op whose gradient
        needs only its output overwrites its input when that input has no other reader — one
        consumer, not a model input or output, the producer's backward does not read it, and the
        edge is the identity transfer on this rank."""
        consumers = {}
        for L in self.layers:
            for t in L.inputs:
                consumers[t.guid] = consumers.get(t.guid, 0) + 1
        prod = {}
        for L in self.layers:
            for o in L.outputs:
                prod[o.guid] = L
        out_guid = self.output_tensor.guid if self.output_tensor is not None else None
        n = 0
        for L in self.layers:
            if not L.impl.can_inplace() or len(L.inputs) != 1 or not self.local.get(L.name):
                continue
            t = L.inputs[0]
            P = prod.get(t.guid)
            if P is None or P.op_type == OperatorType.OP_INPUT or consumers.get(t.guid, 0) != 1:
                continue
            if t.guid == out_guid or P.impl.saves_output() or len(P.outputs) != 1:
                continue
            if self.fwd_tx[(L.name, 0)].kind != "identity" or t.data_type != L.outputs[0].data_type:
                continue
            self.ctx[L.name].extra["inplace"] = True
            n += 1
        return n

    def _plan_binary_relu(self):
        """A ReLU whose input is the output of an element-wise binary op (ResNet's residual add)
        and nothing else reads (the in-place conditions of _plan_inplace) is applied inside that
        op's kernel: one pass over the activation instead of two. The ReLU's backward is unchanged
        (it needs only the output)."""
        if os.environ.get("FF_NO_BINARY_RELU") == "1":
            return 0
        prod = {}
        for L in self.layers:
            for o in L.outputs:
                prod[o.guid] = L
        n = 0
        for L in self.layers:
            if L.op_type != OperatorType.OP_RELU or not self.ctx[L.name].extra.get("inplace"):
                continue
            P = prod.get(L.inputs[0].guid)
            if P is None or P.op_type not in BINARY_OPS or not self.local.get(P.name):
                continue
            self.ctx[P.name].extra["fused_relu"] = True
            self.ctx[L.name].extra["fused_into_producer"] = True
            n += 1
        return n

    def _plan_bias_grad_fusion(self):
        """Cross-op fusion for the backward: a LayerNorm whose input comes straight (same layout,
        sole consumer) from a Linear without activation — or the output projection of a
        multi-head attention — computes that producer's bias gradient, colsum(dx), inside its own
        backward kernel (ops/norm.py -> csrc/kernels/norm.hip ln_bwd_kernel). The producer then
        skips its separate column-reduction pass over the same [tokens, hidden] gradient (BERT:
        the out-projection and FFN2 biases of every layer)."""
        if not self.training or os.environ.get("FF_NO_BIAS_FUSION") == "1":
            return 0
        consumers = {}
        for L in self.layers:
            for t in L.inputs:
                consumers[t.guid] = consumers.get(t.guid, 0) + 1
        prod = {o.guid: L for L in self.layers for o in L.outputs}
        out_guid = self.output_tensor.guid if self.output_tensor is not None else None
        n = 0
        for L in self.layers:
            if L.op_type != OperatorType.OP_LAYERNORM or L.name not in self.ctx or not self.layer_bwd.get(L.name):
                continue
            for j, t in enumerate(L.inputs):
                P = prod.get(t.guid)
                if P is None or P.name not in self.ctx or consumers.get(t.guid, 0) != 1 or t.guid == out_guid:
                    continue
                if not self.in_grad.get((L.name, j)) or self.fwd_tx[(L.name, j)].kind != "identity":
                    continue
                pctx = self.ctx[P.name]
                db = None
                if P.op_type == OperatorType.OP_LINEAR and P.impl.act == K.ACT_NONE and len(P.weights) > 1:
                    db = pctx.wgrads[1] if pctx.wgrads and len(pctx.wgrads) > 1 else None
                elif P.op_type == OperatorType.OP_MULTIHEAD_ATTENTION:
                    gi = P.impl._grad_index()
                    if "o_bias" in gi and pctx.wgrads:
                        db = pctx.wgrads[gi["o_bias"]]
                if db is None or db.dtype != torch.float32 or db.numel() != t.dims[-1]:
                    continue
                self.ctx[L.name].extra["colsum_out"] = db.reshape(-1)
                pctx.extra["bias_grad_fused"] = True
                n += 1
                break
        return n

    def _plan_dact_fusion(self):
        """Cross-op fusion for the backward: a Linear whose input comes straight (identity transfer,
        sole consumer) from a Linear with an activation computes the producer's pre-activation
        gradient in its own dgrad GEMM epilogue, dx * act'(z), together with the producer's bias
        gradient (kernels.gemm_dact). The producer's backward then skips its bias_act_bwd pass,
        which re-read and re-wrote the whole [tokens, ffn] gradient (BERT: FFN2's dgrad carries
        FFN1's GELU')."""
        if not self.training or os.environ.get("FF_NO_DACT_FUSION") == "1":
            return 0
        consumers = {}
        for L in self.layers:
            for t in L.inputs:
                consumers[t.guid] = consumers.get(t.guid, 0) + 1
        prod = {o.guid: L for L in self.layers for o in L.outputs}
        out_guid = self.output_tensor.guid if self.output_tensor is not None else None
        n = 0
        # Conv -> Conv fusion is opt-in (FF_CONV_DACT_FUSION=1): bench-neutral to slightly slower on
        # Inception-v3 / ResNet-50 (profiles/conv_dact_ab_r5.txt) — most consumer dgrads there run
        # as 1x1 GEMMs or MIOpen, which keep the separate mask pass, and the fused sites pay a slab
        # clear and a fold launch
        conv_ok = os.environ.get("FF_CONV_DACT_FUSION", "0") == "1"
        for L in self.layers:
            if L.name not in self.ctx or not self.layer_bwd.get(L.name):
                continue
            t = L.inputs[0] if L.inputs else None
            P = prod.get(t.guid) if t is not None else None
            if P is None or P.name not in self.ctx:
                continue
            if L.op_type == OperatorType.OP_LINEAR:
                if P.op_type != OperatorType.OP_LINEAR or P.impl.act == K.ACT_NONE:
                    continue
            elif L.op_type == OperatorType.OP_CONV2D and conv_ok:
                # Conv -> Conv: the consumer's dgrad epilogue applies the producer's ReLU and sums its
                # bias gradient (conv.hip IGemmArgs.dmask); no spatial split on either side (a halo'd
                # block's dx is cropped and scattered, not the producer's output layout)
                if P.op_type != OperatorType.OP_CONV2D or \
                        P.attrs.get("activation", ActiMode.AC_MODE_NONE) != ActiMode.AC_MODE_RELU:
                    continue
                if any(d > 1 for d in list(self.ctx[L.name].degrees)[2:4] + list(self.ctx[P.name].degrees)[2:4]):
                    continue
            else:
                continue
            if consumers.get(t.guid, 0) != 1 or t.guid == out_guid or not self.layer_bwd.get(P.name):
                continue
            if not self.in_grad.get((L.name, 0)) or self.fwd_tx[(L.name, 0)].kind != "identity":
                continue
            if self.bwd_tx[(L.name, 0)].kind != "identity":
                continue
            pctx = self.ctx[P.name]
            if pctx.wgrads and len(pctx.wgrads) > 1 and pctx.wgrads[1].dtype != torch.float32:
                continue
            self.ctx[L.name].extra["dact_src"] = (pctx, getattr(P.impl, "act", K.ACT_RELU))
            pctx.extra["dact_fused"] = True
            n += 1
        return n

    def _hooked(self, L, phase):
        """Nest every attached hook's op(L, phase) context (profiler, non-finite guard)."""
        from contextlib import ExitStack
        st = ExitStack()
        for h in self.hooks:
            st.enter_context(h.op(L, phase))
        return st

    def _accum_targets(self, L, grads, douts):
        """Input slots whose existing gradient the op may accumulate into in place (a dgrad GEMM
        with beta = 1 instead of a separate add): the tensor already has a gradient from another
        consumer, the backward transfer is the identity, and no other live gradient (or this op's
        own output gradient) aliases that buffer."""
        if not L.impl.accumulates_dx():
            return None
        out = {}
        for j, t in enumerate(L.inputs):
            prev = grads.get(t.guid)
            if prev is None or not self.in_grad.get((L.name, j)) or self.bwd_tx[(L.name, j)].kind != "identity":
                continue
            if any(u.guid == t.guid for u in L.inputs[:j]):
                continue  # offered to the first slot only; the op returns None for the repeats
            sp = prev.untyped_storage().data_ptr()
            if any(g is not None and g.untyped_storage().data_ptr() == sp for k, g in grads.items() if k != t.guid) \
                    or (not L.impl.accum_may_alias_douts()
                        and any(d is not None and d.untyped_storage().data_ptr() == sp for d in douts)) \
                    or not L.impl.accum_target_ok(prev):
                continue
            out[j] = prev
        return out or None

    def zero_gradients(self):
        self._join_folds()
        # tables updated by the row-sparse SGD had their touched gradient rows cleared by it
        skip = self._sparse_cleared if os.environ.get("FF_ZERO_ALL_GRADS") != "1" else {}
        self._sparse_cleared = {}
        for grp, ar in self.arenas.items():
            if ar.acc_end >= ar.size or os.environ.get("FF_ZERO_ALL_GRADS") == "1":
                end = ar.size
            else:
                end = ar.acc_end
            if not end:
                continue
            holes = sorted(skip.get(grp, ()))
            if not holes:
                if end >= ar.size:
                    ar.grad.zero_()
                else:
                    ar.grad[:end].zero_()
                continue
            lo = 0
            for a, b in holes:
                if a > lo:
                    ar.grad[lo:min(a, end)].zero_()
                lo = max(lo, b)
            if lo < end:
                ar.grad[lo:end].zero_()

    def _sparse_plan(self, optimizer):
        """Embedding tables the optimizer may update row-sparsely: plain SGD (momentum 0, no weight
        decay), so a row no id touched keeps a zero gradient and would not move; the table is
        this rank's alone (no gradient all-reduce), its layer is its only user and carries no
        regularizer. {arena group: [(entry index, layer name)]}. FF_SPARSE_EMB=0 disables."""
        # hyper-parameters are part of the key: setting momentum / weight decay on the same
        # optimizer object after the first update must switch the tables back to the dense step
        key = (id(optimizer), getattr(optimizer, "momentum", None), getattr(optimizer, "weight_decay", None),
               getattr(optimizer, "nesterov", None))
        if self._sparse_key == key:
            return self._sparse
        plan = {}
        from ..core.optimizers import SGDOptimizer
        if (isinstance(optimizer, SGDOptimizer) and not optimizer.momentum and not optimizer.weight_decay
                and os.environ.get("FF_SPARSE_EMB", "1") != "0" and not self.zero):
            for L in self.layers:
                if L.op_type != OperatorType.OP_EMBEDDING or L.name not in self.ctx or not self.layer_bwd.get(L.name):
                    continue
                if L.attrs.get("regularizer") is not None or not L.weights:
                    continue
                w = L.weights[0]
                if w.guid not in self.weight_loc or self.weight_users.get(w.guid, 1) != 1:
                    continue
                ar, i = self.weight_loc[w.guid]
                if len(ar.group) > 1 or len(ar.entries[i][3]) != 2:
                    continue
                plan.setdefault(ar.group, []).append((i, L.name))
        self._sparse, self._sparse_key = plan, key
        return plan

    def _apply_regularizers(self):
        """Keras-style weight regularizers (layer attr 'regularizer' with l1/l2): grad += 2*l2*w +
        l1*sign(w) on the fp32 master copy, after the gradient all-reduce (the reference keeps the
        regularizer on the layer but applies none)."""
        for L in self.layers:
            reg = L.attrs.get("regularizer")
            if reg is None or not L.weights:
                continue
            l1, l2 = reg.grad_terms() if hasattr(reg, "grad_terms") else (0.0, float(reg))
            w = L.weights[0]
            if w.guid not in self.weight_loc:
                continue
            m, g, _ = self.weight_loc[w.guid][0].views(self.weight_loc[w.guid][1])
            if l2:
                g.add_(m, alpha=2.0 * l2)
            if l1:
                g.add_(torch.sign(m), alpha=l1)

    def update(self, optimizer):
        self._join_folds()
        if self._ag_pending:
            self.wait_all_gathers()
        self.bucketer.flush()
        self._apply_regularizers()
        if self._opt_next_done is not optimizer:
            optimizer.next()
        self._master_stale = False
        overlapped = self._overlap_active and optimizer is self.model.optimizer
        # the row-sparse update only knows the rows of the LAST backward's ids: after several
        # backward passes without an update the accumulated table gradient can hold other rows too,
        # so this update runs dense (and zero_gradients then clears the whole table)
        multi_bwd = self._bwd_since_update > 1
        self._bwd_since_update = 0
        for grp, ar in self.arenas.items():
            if not ar.size:
                continue
            bs = self.zero_buckets.get(grp)
            sparse = self._sparse_plan(optimizer).get(grp) if bs is None and not multi_bwd else None
            if sparse:
                self._sparse_update(optimizer, grp, ar, sparse)
                continue
            if bs is None:
                if overlapped:  # the buckets the backward did not complete (e.g. frozen weights)
                    for _, flat, buckets in self.bucketer.arenas:
                        if flat is ar.grad:
                            for b in buckets:
                                if id(b) not in self._upd_done:
                                    optimizer.step_range(ar, b["lo"], b["hi"])
                else:
                    optimizer.step(ar)
                continue
            g = self.comm.group(grp)
            for i, b in enumerate(bs):
                lo, hi = b["own"]
                optimizer.step_range(ar, lo, hi)
                # the compute copy (bf16, or the fp32 master itself) of the whole bucket, in place
                src = ar.lowp if ar.lowp is not None else ar.master
                self._ag_pending[(grp, i)] = dist.all_gather_into_tensor(src[b["lo"]:b["hi"]], src[lo:hi], group=g,
                                                                          async_op=True)
            self._master_stale |= ar.lowp is not None
        if self._upd_stream is not None and self._upd_done:
            torch.cuda.current_stream(self.device).wait_stream(self._upd_stream)
        self._upd_done = set()
        self._overlap_active = False
        self._opt_next_done = None
        self.step_idx += 1

    def _sparse_update(self, optimizer, grp, ar, sparse):
        """Dense SGD over the arena minus the sparse tables, then each table's touched rows only
        (kernels.sgd_sparse_rows, which also clears those gradient rows)."""
        holes = sorted((ar.entries[i][1], ar.entries[i][1] + ar.entries[i][2], i, name) for i, name in sparse)
        lo = 0
        for a, b, _, _ in holes:
            if a > lo:
                optimizer.step_range(ar, lo, a)
            lo = max(lo, b)
        if lo < ar.size:
            optimizer.step_range(ar, lo, ar.size)
        cleared = []
        for a, b, i, name in holes:
            idx = self.ctx[name].extra.get("touched_idx")
            m, g, c = ar.views(i)
            if idx is None:  # the table's layer did not run backward: its gradient is whatever it was
                continue
            w = ar.entries[i][0]
            mark = self._marks.get(w.guid)
            if mark is None:
                mark = self._marks[w.guid] = torch.empty(m.shape[0], dtype=torch.int32, device=m.device)
            K.sgd_sparse_rows(idx, mark, m, g, c if ar.lowp is not None else None, optimizer.lr)
            cleared.append((a, b))
        self._sparse_cleared[grp] = cleared

    def _wait_weights(self, L):
        """Sharded optimizer: the all-gathers of the buckets holding L's weights must land first."""
        for w in L.weights:
            for k in self._w_buckets.get(w.guid, ()):
                h = self._ag_pending.pop(k, None)
                if h is not None:
                    h.wait()

    def wait_all_gathers(self):
        for h in self._ag_pending.values():
            h.wait()
        self._ag_pending = {}

    def sync_master(self):
        """Sharded optimizer: rank r's fp32 master is current only on its chunks; gather the full
        master before reading weights (get_weights, checkpoints)."""
        self.wait_all_gathers()
        if not self._master_stale:
            return
        for grp, bs in self.zero_buckets.items():
            ar = self.arenas[grp]
            g = self.comm.group(grp)
            for b in bs:
                dist.all_gather_into_tensor(ar.master[b["lo"]:b["hi"]], ar.master[b["own"][0]:b["own"][1]], group=g)
        self._master_stale = False

    def sync_optimizer_state(self, optimizer):
        """Sharded optimizer: each rank's Adam m/v (SGD momentum) is current only on its own chunk
        of every bucket; gather the full state so a checkpoint does not depend on the sharding
        (world size, --grad-bucket-mb, --zero on or off at resume time)."""
        self.wait_all_gathers()
        for grp, bs in self.zero_buckets.items():
            ar = self.arenas[grp]
            st = getattr(optimizer, "state", {}).get(id(ar))
            if st is None:
                continue
            g = self.comm.group(grp)
            for t in (st if isinstance(st, (tuple, list)) else (st,)):
                for b in bs:
                    dist.all_gather_into_tensor(t[b["lo"]:b["hi"]], t[b["own"][0]:b["own"][1]], group=g)

    def init_optimizer(self, optimizer):
        for ar in self.arenas.values():
            optimizer.init_state(ar)

    # ------------------------------------------------------------------ value access
    def gather_full(self, t, local: Optional[torch.Tensor], layout: Layout,
                    dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """Full logical value on every rank (for get_tensor / get_weights). `dtype` is the element
        type the holders send (weights: their fp32 master copy); ranks that hold no part of the
        tensor receive into a buffer of that type, so every rank posts the same message sizes."""
        if not self.comm.distributed:
            assert layout.num_parts == 1 or layout.device_set() == (self.rank,), layout
            return local
        dst = Layout(layout.shape, (1,) * layout.ndim, self.world, tuple(range(self.world)))
        tx = Transfer(layout, dst, layout.partial, self.rank)
        self.comm.ensure_groups(tx.rank_sets())
        like = self._like(t) if dtype is None else torch.empty(0, dtype=dtype, device=self.device)
        return tx.run(self.comm, local, like)

    def get_value(self, t):
        if self.model.label_tensor is not None and t.guid == self.model.label_tensor.guid:
            return self.gather_full(t, self.inputs.get(t.guid), self.label_layout)
        lay = self.producer_layout[t.guid]
        full = self.gather_full(t, self.values.get(t.guid), lay)
        if (self.output_tensor is not None and t.guid == self.output_tensor.guid and self.softmax_fused
                and self._softmax_emitted_logits()):
            full = torch.softmax(full.float(), -1).to(full.dtype)  # probabilities on demand
        return full

    def get_weight(self, w):
        if self.zero:
            self.sync_master()
        loc = self.weight_tensor(w) if w.guid in self.weight_loc else None
        if loc is not None and w.guid in self.weight_loc:
            loc = self.weight_loc[w.guid][0].views(self.weight_loc[w.guid][1])[0]
        return self.gather_full(w, loc, self.weight_layout[w.guid].with_(partial=False), dtype=torch.float32)

    def get_weight_grad(self, w):
        self._join_folds()
        loc = None
        if w.guid in self.weight_loc:
            loc = self.weight_loc[w.guid][0].views(self.weight_loc[w.guid][1])[1]
        return self.gather_full(w, loc, self.weight_layout[w.guid].with_(partial=False), dtype=torch.float32)

    def set_weight(self, w, value: np.ndarray):
        if self.zero:
            self.sync_master()
        if w.guid not in self.weight_loc:
            return
        ar, idx = self.weight_loc[w.guid]
        m, _, c = ar.views(idx)
        wl = self.weight_layout[w.guid]
        p = wl.parts_on(self.rank)[0]
        sl = rel_slices(wl.region(p), tuple((0, s) for s in w.dims))
        m.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(value, dtype=np.float32)[sl])))
        if c is not m:
            c.copy_(m)

    def metrics_snapshot(self) -> np.ndarray:
        acc = self._metric_acc.clone()
        if self.comm.distributed:
            dist.all_reduce(acc)
        return acc.cpu().numpy()

    def reset_metrics(self):
        self._metric_acc.zero_()
