"""Operator cost model for the search (reference Simulator::measure_operator_cost,
src/runtime/simulator.cu:58 — profiles each op with per-shard shapes on GPU 0, warmup 5 /
repeat 10 — plus the hard-coded ~2019-GPU machine constants of machine_model.cc:67-69).

Two sources, same interface (`op_cost(layer, cfg) -> (fwd_ms, bwd_ms, mem_bytes)`):
  * measured: run the op's real forward+backward (our HIP kernels) on the local GPU with the
    per-part shard shapes of the config; cached per (op, attributes, shard shapes) so BERT's 24
    identical layers cost one measurement per distinct config;
  * analytic: an MI355X roofline — MFMA ops at a shape-dependent fraction of the 2.5 PF/s dense
    bf16 peak (tile wave-quantization over 256 CUs), memory-bound ops at ~5.5 TB/s HBM3E.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Tuple

import torch

from ..parallel.layout import Layout
from ..type import DataType, OperatorType
from .strategy import OpConfig, op_layouts

PEAK_BF16 = 2.5e15
PEAK_FP32 = 1.5e14
HBM = 5.5e12
LAUNCH_S = 4e-6

_measured: Dict[tuple, Tuple[float, float]] = {}


def _local_shape(lay: Layout, rank_part: int = 0):
    return lay.local_shape(rank_part)


def _gemm_eff(M, N, K):
    tiles = math.ceil(M / 256) * math.ceil(N / 128)
    waves = math.ceil(tiles / 256)
    quant = tiles / (waves * 256)
    kfac = min(1.0, K / 2048) ** 0.25
    return max(0.05, 0.42 * quant * kfac)


def analytic_cost(layer, cfg: OpConfig, compute_dtype: DataType) -> Tuple[float, float]:
    lo = op_layouts(layer, cfg)
    ins = [l.local_shape(0) for l in lo.inputs]
    outs = [l.local_shape(0) for l in lo.outputs]
    ws = [l.local_shape(0) for l in lo.weights]
    impl = layer.impl
    elem = 2 if compute_dtype == DataType.DT_BF16 else 4
    fl = impl.flops(ins, outs, ws)
    by = impl.mem_bytes(ins, outs, ws, elem)
    if impl.uses_mfma():
        if compute_dtype == DataType.DT_BF16:
            # representative GEMM dims for the tile-quantization term
            out0 = outs[0] if outs else (1,)
            M = max(1, int(math.prod(out0[:-1])))
            N = max(1, int(out0[-1]))
            K = max(1, int(fl / max(1, 2 * M * N)))
            peak = PEAK_BF16 * _gemm_eff(M, N, K)
        else:
            peak = PEAK_FP32 * 0.6
        t = max(fl / peak, by / HBM) + LAUNCH_S * 2
        return t * 1e3, 2.0 * t * 1e3
    t = by / HBM + LAUNCH_S
    return t * 1e3, 2.0 * t * 1e3


def measure_cost(layer, cfg: OpConfig, compute_dtype: DataType, device, reps: int = 10) -> Tuple[float, float]:
    """Time the op's own forward/backward on this GPU with the shard shapes of `cfg`."""
    from ..ops import OpCtx
    lo = op_layouts(layer, cfg)
    key = (layer.op_type, layer.impl.params_key(), tuple(l.local_shape(0) for l in lo.inputs),
           tuple(l.local_shape(0) for l in lo.weights), cfg.degrees, compute_dtype)
    if key in _measured:
        return _measured[key]
    ct = torch.bfloat16 if compute_dtype == DataType.DT_BF16 else torch.float32
    xs = []
    for t, l in zip(layer.inputs, lo.inputs):
        shp = l.local_shape(0)
        if t.data_type in (DataType.DT_INT32, DataType.DT_INT64):
            hi = 2
            if layer.op_type == OperatorType.OP_EMBEDDING:
                hi = layer.attrs["num_entries"] // max(1, cfg.degrees[-1])
            xs.append(torch.randint(0, max(1, hi), shp, device=device, dtype=torch.int32))
        else:
            xs.append(torch.randn(shp, device=device, dtype=ct))
    # identical tensors in the graph stay identical (fused self-attention)
    seen = {}
    for i, t in enumerate(layer.inputs):
        if t.guid in seen and lo.inputs[i].key() == lo.inputs[seen[t.guid]].key():
            xs[i] = xs[seen[t.guid]]
        else:
            seen.setdefault(t.guid, i)
    ws = [torch.randn(l.local_shape(0), device=device, dtype=ct) * 0.02 for l in lo.weights]
    ctx = OpCtx(layer=layer, part_coords=(0,) * len(cfg.degrees), degrees=cfg.degrees, compute_dtype=compute_dtype)
    ctx.wgrads = [torch.zeros(w.shape, device=device, dtype=torch.float32) for w in ws]
    ctx.extra["need_dx0"] = True
    impl = layer.impl

    def fwd():
        return impl.forward(ctx, xs, ws)

    try:
        outs = fwd()
        douts = [torch.randn_like(o) if o.is_floating_point() else None for o in outs]
        impl.backward(ctx, douts)
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(reps):
            fwd()
            ctx.saved.clear()
        en.record()
        en.synchronize()
        tf = st.elapsed_time(en) / reps
        st.record()
        for _ in range(reps):
            fwd()
            impl.backward(ctx, douts)
        en.record()
        en.synchronize()
        tb = max(st.elapsed_time(en) / reps - tf, 0.0)
    except Exception:
        tf, tb = analytic_cost(layer, cfg, compute_dtype)
    _measured[key] = (tf, tb)
    return tf, tb


def mem_bytes(layer, cfg: OpConfig, compute_dtype: DataType, training: bool = True) -> float:
    lo = op_layouts(layer, cfg)
    elem = 2 if compute_dtype == DataType.DT_BF16 else 4
    act = sum(math.prod(l.local_shape(0)) for l in lo.outputs) * elem
    act += sum(math.prod(l.local_shape(0)) for l in lo.inputs) * elem if training else 0
    w = sum(math.prod(l.local_shape(0)) for l in lo.weights)
    # fp32 master + fp32 grad + bf16 copy + Adam m, v
    wbytes = w * (4 + 4 + (2 if compute_dtype == DataType.DT_BF16 else 0) + 8) if training else w * elem
    return float(act + wbytes)


def _loss_fused_softmax(layer) -> bool:
    """The model's output softmax under a cross-entropy loss: the executor runs it as ONE fused
    softmax-cross-entropy pass over the logits inside the loss (ops/softmax.py emits the logits
    unchanged), so its standalone softmax forward/backward never runs."""
    from ..type import LossType
    m = getattr(layer, "model", None)
    if m is None or layer.op_type != OperatorType.OP_SOFTMAX:
        return False
    if getattr(m, "loss_type", None) not in (LossType.LOSS_CATEGORICAL_CROSSENTROPY,
                                             LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY):
        return False
    out = m.output_tensor()
    n = len(layer.outputs[0].dims)
    return out is not None and out.guid == layer.outputs[0].guid and layer.attrs.get("dim", -1) % n == n - 1


def fused_xent_cost(layer, cfg: OpConfig, compute_dtype: DataType, measure: bool, device=None):
    """Cost of the fused softmax-cross-entropy pass on this config's shard (forward + backward in
    one kernel: read the logits, write their gradient), charged to the forward."""
    lo = op_layouts(layer, cfg)
    shp = lo.inputs[0].local_shape(0)
    V = shp[-1]
    rows = int(math.prod(shp[:-1]))
    if measure and device is not None and device.type == "cuda" and compute_dtype == DataType.DT_BF16:
        key = ("xent", rows, V)
        if key not in _measured:
            from .. import kernels as K
            x = torch.randn(rows, V, device=device, dtype=torch.bfloat16)
            lab = torch.randint(0, V, (rows,), device=device, dtype=torch.int32)
            acc = torch.zeros(3, device=device, dtype=torch.float32)
            K.softmax_xent(x, lab, 1.0, acc)
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(5):
                K.softmax_xent(x, lab, 1.0, acc)
            en.record()
            en.synchronize()
            _measured[key] = (st.elapsed_time(en) / 5, 0.0)
        return _measured[key]
    elem = 2 if compute_dtype == DataType.DT_BF16 else 4
    t = 2.0 * rows * V * elem / HBM + LAUNCH_S
    return t * 1e3, 0.0


def op_cost(layer, cfg: OpConfig, compute_dtype: DataType, measure: bool, device=None):
    if layer.op_type == OperatorType.OP_INPUT:
        return 0.0, 0.0
    if _loss_fused_softmax(layer):
        return fused_xent_cost(layer, cfg, compute_dtype, measure, device)
    if measure and device is not None and device.type == "cuda":
        return measure_cost(layer, cfg, compute_dtype, device)
    return analytic_cost(layer, cfg, compute_dtype)
