#!/usr/bin/env python3
"""Plan bench.py's flagship (BERT-Large, 32 sequences of 512 per GPU, MLM vocab padded to 64) for N
devices in ONE process on one GPU, the way rank 0 of `bench.py --gpus N` does: graph passes, then
the joint Unity search with measured op costs. Prints one JSON line per N (predicted times, search
wall time, graphs costed).

  FF_COST_CACHE=flexflow_amd/pcg/data/op_costs_mi355x.json python scripts/cost_table.py 2 4 8
      fills the shipped measured-cost table (so bench's N > 1 search times nothing on the box);
  FF_COST_CACHE=0 python scripts/cost_table.py 8 8
      two independent measurement passes of the same plan (determinism of the measured costs).

usage: cost_table.py N [N ...] [--model bert-large] [--batch-per-gpu 32]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="+")
ap.add_argument("--model", default="bert-large")
ap.add_argument("--batch-per-gpu", type=int, default=32)
ap.add_argument("--seq", type=int, default=512)
a = ap.parse_args()

from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel  # noqa: E402
from flexflow_amd.models.bert import BertConfig, build_bert  # noqa: E402
from flexflow_amd.pcg import costmodel  # noqa: E402
from flexflow_amd.pcg.search import choose_strategy  # noqa: E402
from flexflow_amd.pcg.substitutions import optimize_graph  # noqa: E402

for n in a.n:
    costmodel._measured.clear()  # every N (and every repeat) measures or reads the table afresh
    costmodel._disk["table"] = None
    costmodel.STATS.update(table_hits=0, timed=0, timed_s=0.0)
    cfg = FFConfig(["--dtype", "bf16", "--search", "unity", "--search-num-workers", str(n)])
    gb = a.batch_per_gpu * n
    cfg.batch_size = gb
    ff = FFModel(cfg)
    bc = {"bert-large": BertConfig.large, "bert-base": BertConfig.base, "bert-tiny": BertConfig.tiny}[a.model](a.seq)
    bc.seq = a.seq
    bc.max_pos = max(bc.max_pos, a.seq)
    bc.pad_vocab_multiple = 64
    build_bert(ff, gb, bc)
    ff.optimizer = AdamOptimizer(ff, 1e-4)
    t0 = time.perf_counter()
    optimize_graph(ff)
    strat, rep = choose_strategy(ff)
    wall = time.perf_counter() - t0
    multi = sorted({tuple(c.degrees) for c in strat.values() if c.num_parts > 1 and
                    [i for i, d in enumerate(c.degrees) if d > 1] != [0]})
    print(json.dumps({"n": n, "model": a.model, "global_batch": gb, "wall_s": round(wall, 1),
                      "cost_cache": os.environ.get("FF_COST_CACHE", "(shipped, read-only)"),
                      **{k: rep.get(k) for k in ("predicted_ms", "predicted_dp_ms", "predicted_speedup_vs_dp",
                                                 "graphs_costed", "timed_out", "search_wall_s", "measured_costs",
                                                 "cost_lookups")},
                      "rewrites": len(rep.get("rewrites") or []), "non_dp_degree_vectors": [list(d) for d in multi][:8]}),
          flush=True)
