#!/usr/bin/env python3
"""Run the strategy search for a model in ONE process planning for N devices and export the chosen
strategy (+ search report) as a strategy file, e.g. to replay a GPU-measured search on CPU ranks.
usage: export_search.py MODEL N OUT.json [search] [batch]   (MODEL: bert-tiny-test | zoo name)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType  # noqa: E402

name, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
algo = sys.argv[4] if len(sys.argv) > 4 else "unity"
batch = int(sys.argv[5]) if len(sys.argv) > 5 else 8
cfg = FFConfig(["--dtype", "bf16", "--search", algo, "--search-num-workers", str(n), "--export-strategy", out])
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
ff.compile(loss_type=loss, metrics=mets)
print(json.dumps({k: v for k, v in (ff.search_report or {}).items() if k != "measured_costs"}, default=str)[:2000])
