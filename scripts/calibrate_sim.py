#!/usr/bin/env python3
"""Simulator calibration at N = 1: the search's prediction of a data-parallel step (op costs
measured on this GPU by pcg/costmodel.measure_cost, scheduled by the native simulator) against the
measured step, per op class.

usage: calibrate_sim.py [model=bert-large] [batch=32] [steps=6]
Prints a table (op class: predicted fwd/bwd ms vs measured fwd/bwd ms, error) and the whole-step
prediction error, as JSON on the last line.
"""
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "bert-large"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6


def build(profiling):
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert
    flags = ["--dtype", "bf16", "--no-hip-graphs"] + (["--profiling"] if profiling else [])
    cfg = FFConfig(flags)
    cfg.batch_size = batch
    ff = FFModel(cfg)
    rng = np.random.default_rng(0)
    if model.startswith("bert"):
        bc = {"bert-large": BertConfig.large, "bert-base": BertConfig.base}[model](512)
        ids, pos, _ = build_bert(ff, batch, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-4)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (batch, bc.seq), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (batch, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (batch, bc.seq, 1), dtype=np.int32))
    else:
        from flexflow_amd.models import build as zoo
        inputs, _, loss, mets, make_batch = zoo(model, ff, batch)
        ff.optimizer = AdamOptimizer(ff, 1e-4)
        ff.compile(loss_type=loss, metrics=mets)
        arrs, lab = make_batch(rng)
        for t, a in zip(inputs, arrs):
            t.set_tensor(ff, a)
        ff.label_tensor.set_tensor(ff, lab)
    return ff


# ---- measured: whole step (as bench.py: eager, overlapped update) and per op (profiler)
ff = build(False)
for _ in range(3):
    ff.train_step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    ff.train_step()
torch.cuda.synchronize()
step_ms = (time.perf_counter() - t0) / steps * 1e3
print(f"measured step {step_ms:.3f} ms", flush=True)

ffp = build(True)
for _ in range(2):
    ffp.train_step()
ffp.profiler.records.clear()
for _ in range(steps):
    ffp.train_step()
    ffp.profiler.next_step()
meas = ffp.profiler.summary()
torch.cuda.synchronize()

# ---- predicted: the search problem with measured op costs, data-parallel plan at N = 1
from flexflow_amd import _core  # noqa: E402
from flexflow_amd.pcg.strategy import data_parallel_config  # noqa: E402
from flexflow_amd.pcg.unity import build_problem  # noqa: E402

prob, cands = build_problem(ffp, 1, True)
choice = [cands[i].index(data_parallel_config(L, 1)) for i, L in enumerate(ffp.layers)]
sim = _core.simulate(prob, choice)
pred = {}
for i, L in enumerate(ffp.layers):
    c = prob.nodes[i].cands[choice[i]]
    pred[L.name] = (L.op_type.name, c.fwd_ms, c.bwd_ms)

rows = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0])
for name, (op, f, b) in pred.items():
    m = meas.get(name, {"fwd_ms": 0.0, "bwd_ms": 0.0})
    r = rows[op]
    r[0] += f
    r[1] += b
    r[2] += m["fwd_ms"]
    r[3] += m["bwd_ms"]
    r[4] += 1
tot_pred_ops = sum(r[0] + r[1] for r in rows.values())
tot_meas_ops = sum(r[2] + r[3] for r in rows.values())
print(f"{'op class':28s} {'n':>4s} {'pred fwd':>9s} {'meas fwd':>9s} {'pred bwd':>9s} {'meas bwd':>9s} {'err':>7s}")
for op, r in sorted(rows.items(), key=lambda kv: -(kv[1][2] + kv[1][3])):
    err = (r[0] + r[1]) / max(r[2] + r[3], 1e-9) - 1
    print(f"{op:28s} {r[4]:4d} {r[0]:9.3f} {r[2]:9.3f} {r[1]:9.3f} {r[3]:9.3f} {100 * err:6.1f}%")
upd_pred = sim.makespan_ms - tot_pred_ops
print(f"{'ops total':28s} {'':4s} {tot_pred_ops:9.3f} {tot_meas_ops:9.3f}  (fwd+bwd, pred vs measured per-op sums)")
print(f"simulated step {sim.makespan_ms:.3f} ms (ops {tot_pred_ops:.3f} + update/sync {upd_pred:.3f}) "
      f"vs measured step {step_ms:.3f} ms: error {100 * (sim.makespan_ms / step_ms - 1):+.1f}%")
# per-op detail: the largest absolute disagreements (what a per-class error is made of)
det = []
for name, (op, f, b) in pred.items():
    m = meas.get(name, {"fwd_ms": 0.0, "bwd_ms": 0.0})
    det.append((abs(f - m["fwd_ms"]) + abs(b - m["bwd_ms"]), name, op, f, m["fwd_ms"], b, m["bwd_ms"]))
det.sort(reverse=True)
print("largest per-op disagreements (ms): name op pred_fwd meas_fwd pred_bwd meas_bwd")
for d, name, op, f, mf, b, mb in det[:12]:
    print(f"  {name:34s} {op:24s} {f:8.3f} {mf:8.3f} {b:8.3f} {mb:8.3f}")
# the 20 largest ops by measured time, per-op fwd / bwd error
big = sorted(pred.items(), key=lambda kv: -(meas.get(kv[0], {}).get("fwd_ms", 0.0) + meas.get(kv[0], {}).get("bwd_ms", 0.0)))
print("20 largest ops (measured): name op pred_fwd meas_fwd err_fwd pred_bwd meas_bwd err_bwd")
worst = 0.0
for name, (op, f, b) in big[:20]:
    m = meas.get(name, {"fwd_ms": 0.0, "bwd_ms": 0.0})
    ef = 100 * (f / max(m["fwd_ms"], 1e-9) - 1)
    eb = 100 * (b / max(m["bwd_ms"], 1e-9) - 1) if m["bwd_ms"] > 0 else 0.0
    worst = max(worst, abs(ef), abs(eb))
    print(f"  {name:34s} {op:24s} {f:8.3f} {m['fwd_ms']:8.3f} {ef:+6.1f}% {b:8.3f} {m['bwd_ms']:8.3f} {eb:+6.1f}%")
print(f"worst per-op error among the 20 largest: {worst:.1f}%")
print(json.dumps({"model": model, "batch": batch, "measured_step_ms": round(step_ms, 3),
                  "worst_top20_op_error_pct": round(worst, 1),
                  "simulated_step_ms": round(sim.makespan_ms, 3),
                  "error_pct": round(100 * (sim.makespan_ms / step_ms - 1), 2),
                  "pred_ops_ms": round(tot_pred_ops, 3), "measured_ops_ms": round(tot_meas_ops, 3),
                  "per_class": {op: {"n": r[4], "pred_fwd": round(r[0], 3), "meas_fwd": round(r[2], 3),
                                     "pred_bwd": round(r[1], 3), "meas_bwd": round(r[3], 3)}
                                for op, r in rows.items()}}))
