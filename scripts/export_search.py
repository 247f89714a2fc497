#!/usr/bin/env python3
"""Run the strategy search for a model in ONE process planning for N devices and export the chosen
strategy (+ search report) as a strategy file, e.g. to replay a GPU-measured search on CPU ranks.
usage: export_search.py MODEL N OUT.json [search] [batch] [extra FFConfig flags...]
(MODEL: bert-tiny-test | zoo name)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType  # noqa: E402

name, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
algo = sys.argv[4] if len(sys.argv) > 4 else "unity"
batch = int(sys.argv[5]) if len(sys.argv) > 5 else 8
cfg = FFConfig(["--dtype", "bf16", "--search", algo, "--search-num-workers", str(n), "--export-strategy", out]
               + sys.argv[6:])
cfg.batch_size = batch
ff = FFModel(cfg)
if name == "bert-tiny-test":
    from flexflow_amd.models.bert import BertConfig, build_bert
    bc = BertConfig(hidden=256, heads=4, layers=2, ffn=1024, vocab=512, max_pos=128, seq=128)
    build_bert(ff, batch, bc)
    loss, mets = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, [MetricsType.METRICS_ACCURACY]
else:
    from flexflow_amd.models import build
    _, _, loss, mets, _ = build(name, ff, batch)
ff.optimizer = AdamOptimizer(ff, 1e-3)
if int(os.environ.get("WORLD_SIZE", "1")) >= n:
    ff.compile(loss_type=loss, metrics=mets)
    report = ff.search_report
else:
    # one process planning for N devices: run compile()'s graph passes and the search only (an
    # executor for N ranks cannot be built here), then export the strategy
    import time
    from flexflow_amd.pcg.search import choose_strategy
    from flexflow_amd.pcg.strategy import save_strategy
    from flexflow_amd.pcg.substitutions import optimize_graph
    t0 = time.perf_counter()
    subst = optimize_graph(ff)
    strat, report = choose_strategy(ff)
    report = dict(report or {}, substitutions=subst, wall_s=round(time.perf_counter() - t0, 2))
    save_strategy(out, strat, n, {k: v for k, v in report.items() if k != "measured_costs"})
    multi = sorted({tuple(c.degrees) for c in strat.values() if c.num_parts > 1})
    report["distinct_degree_vectors"] = [list(d) for d in multi][:20]
print(json.dumps({k: v for k, v in (report or {}).items() if k != "measured_costs"}, default=str)[:4000])
