#!/usr/bin/env python3
"""Flagship benchmark: BERT-Large training throughput (samples/s) under the auto-searched
parallelization strategy, one process per MI355X (torchrun), bf16 compute, synthetic data.

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

Per-GPU batch is fixed (weak scaling): global_batch = batch_per_gpu * N (default 32 sequences
of 512 tokens per GPU: MI355X has 288 GB of HBM, and at 16 the step is too short to amortise the
optimizer pass and the small-GEMM tails). Every timed step is a
full training iteration (forward, backward, gradient all-reduce, optimizer update). Rank 0 prints
ONE JSON line; the step time is the MAX over ranks of the time between two barrier+synchronize
fences around exactly K steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_METRIC = "samples/sec under auto-searched strategy at 1/2/4/8 MI355X; speedup vs DP"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="bert-large",
                    help="bert-large | bert-base | bert-tiny | any flexflow_amd.models.MODELS entry "
                         "(alexnet, resnet50, inception_v3, dlrm, ...)")
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="default 32 for BERT (HBM-sized: 288 GB/GPU), 64 for the other models")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--pad-vocab", type=int, default=int(os.environ.get("FF_PAD_VOCAB", "64")),
                    help="BERT: pad the MLM decoder width to a multiple of this with masked logits (0: off)")
    ap.add_argument("--search", default="unity", help="unity | mcmc | dp")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--optimizer", default="adam", choices=["adam", "sgd"])
    ap.add_argument("--no-hip-graphs", action="store_true")
    ap.add_argument("--zero", action="store_true",
                    help="ZeRO-1 sharded optimizer on data-parallel weights (reduce-scatter + all-gather)")
    ap.add_argument("--compare-dp", action="store_true", help="also time pure data parallel (speedup vs DP)")
    ap.add_argument("--verify-steps", type=int, default=4,
                    help="N>1: time the searched strategy and data parallel for this many steps each and keep "
                         "the faster (measurement-verified search; 0 disables)")
    return ap.parse_args()


def build(args, search):
    """Returns (ff, global_batch, info); info = {seq, flops_per_sample, params, extra config fields}."""
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexflow_amd.models import build as build_model
    from flexflow_amd.models.bert import BertConfig, build_bert
    world = int(os.environ.get("WORLD_SIZE", "1"))
    flags = ["--dtype", args.dtype, "--search", search]
    if args.no_hip_graphs:
        flags.append("--no-hip-graphs")
    if args.zero:
        flags.append("--zero")
    cfg = FFConfig(flags)
    bert = args.model.startswith("bert")
    bpg = args.batch_per_gpu or (32 if bert else 64)
    gb = bpg * world
    cfg.batch_size = gb
    ff = FFModel(cfg)
    rng = np.random.default_rng(1234)
    if bert:
        bc = {"bert-large": BertConfig.large, "bert-base": BertConfig.base, "bert-tiny": BertConfig.tiny}[args.model](args.seq)
        bc.seq = args.seq
        bc.max_pos = max(bc.max_pos, args.seq)
        # MLM decoder width padded to a multiple of 64 (30522 -> 30528) with masked (-1e9 bias)
        # columns: identical loss / gradients, every vocab GEMM on aligned tiles
        bc.pad_vocab_multiple = args.pad_vocab
        ids, pos, out = build_bert(ff, gb, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-4) if args.optimizer == "adam" else SGDOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (gb, bc.seq), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (gb, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (gb, bc.seq, 1), dtype=np.int32))
        info = {"seq": bc.seq, "flops_per_sample": bc.train_flops_per_seq(), "params": bc.params(),
                "extra": {"hidden": bc.hidden, "layers": bc.layers, "heads": bc.heads, "vocab": bc.vocab,
                          "vocab_padded": bc.padded_vocab()}}
        return ff, gb, info
    inputs, out, loss, mets, make_batch = build_model(args.model, ff, gb)
    ff.optimizer = AdamOptimizer(ff, 1e-4) if args.optimizer == "adam" else SGDOptimizer(ff, 1e-3)
    ff.compile(loss_type=loss, metrics=mets)
    arrs, lab = make_batch(rng)
    for t, a in zip(inputs, arrs):
        t.set_tensor(ff, a)
    ff.label_tensor.set_tensor(ff, lab)
    params = sum(int(np.prod(w.dims)) for L in ff.layers for w in L.weights)
    return ff, gb, {"seq": None, "flops_per_sample": None, "params": params, "extra": {}}


def describe(ff, world):
    """Short parallelism label: dpN when every op is sample-partitioned N ways."""
    strat = ff.strategy
    kinds = set()
    for L in ff.layers:
        c = strat[L.name]
        if c.num_parts == 1:
            kinds.add("single")
            continue
        ax = [i for i, d in enumerate(c.degrees) if d > 1]
        kinds.add("dp" if ax == [0] else "hybrid")
    if world == 1:
        return "single"
    if kinds == {"dp"}:
        return f"dp{world}"
    return f"searched-hybrid{world}"


def timed(ff, steps, warmup, world):
    for _ in range(warmup):
        ff.train_step()
    sync(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        ff.train_step()
    sync(world)
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def sync(world):
    if world > 1:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    verify = None
    t_start = time.perf_counter()
    if world > 1 and args.search not in ("dp", "none") and args.verify_steps > 0:
        # measurement-verified search: the simulator's pick is timed against data parallel on the
        # real machine and the faster one is kept (FlexFlow's search also trusts measured op costs)
        ff, gb, info = build(args, args.search)
        label = describe(ff, world)
        if label.startswith("dp"):
            verify = {"searched": label, "chosen": label}
        else:
            t_s = timed(ff, args.verify_steps, 2, world) / args.verify_steps
            ff_dp, _, _ = build(args, "dp")
            t_d = timed(ff_dp, args.verify_steps, 2, world) / args.verify_steps
            keep_dp = t_d < t_s
            verify = {"searched": label, "searched_ms": round(t_s * 1e3, 3), "dp_ms": round(t_d * 1e3, 3),
                      "chosen": f"dp{world}" if keep_dp else label}
            if keep_dp:
                del ff
                ff = ff_dp
            else:
                del ff_dp
    else:
        ff, gb, info = build(args, args.search)
    setup_s = time.perf_counter() - t_start  # build(s) + compile + search + verification
    el = timed(ff, args.steps, args.warmup, world)
    ms = el / args.steps * 1e3
    sps = gb * args.steps / el
    res = {
        "metric": BASELINE_METRIC,
        "value": round(sps, 3),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (random inputs / labels, random-init weights)",
        "config": dict({"model": args.model, "global_batch": gb, "seq_len": info["seq"],
                        "parallelism": describe(ff, world), "search": (ff.search_report or {}).get("algo"),
                        "optimizer": args.optimizer, "params": info["params"]}, **info["extra"]),
    }
    res["setup_s"] = round(setup_s, 1)
    sg = getattr(ff, "_step_graph", None)
    res["hip_graph"] = bool(sg is not None and sg.graph is not None)  # step replayed from a hipGraph
    if info["flops_per_sample"]:
        res["model_tflops_per_gpu"] = round(info["flops_per_sample"] * sps / world / 1e12, 2)
    rep = ff.search_report or {}
    if rep.get("predicted_speedup_vs_dp") is not None:
        res["search"] = {k: rep[k] for k in ("predicted_ms", "predicted_dp_ms", "predicted_speedup_vs_dp",
                                             "candidates", "search_s", "search_wall_s", "graphs_costed",
                                             "timed_out", "measured_costs", "cost_lookups") if k in rep}
    if verify is not None:
        res["search_verification"] = verify
        if "dp_ms" in verify:
            res["speedup_vs_dp"] = round(verify["dp_ms"] / (ms if verify["chosen"] != f"dp{world}" else
                                                             verify["dp_ms"]), 4)
    if args.compare_dp and world > 1 and "speedup_vs_dp" not in res:
        del ff
        ff2, _, _ = build(args, "dp")
        el2 = timed(ff2, args.steps, args.warmup, world)
        res["dp_samples_per_s"] = round(gb * args.steps / el2, 3)
        res["speedup_vs_dp"] = round(el2 / el, 4)
    if rank == 0:
        print(json.dumps(res), flush=True)
        if os.environ.get("FF_TUNE_LOG"):
            from flexflow_amd import kernels as K
            with open(os.environ["FF_TUNE_LOG"], "w") as f:
                json.dump(K.TUNE_LOG, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
