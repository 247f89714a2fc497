"""Shared driver for the model-zoo examples (alexnet / resnet / resnext50 / inception / dlrm / xdl /
candle_uno / transformer / mlp_unify / mixture_of_experts): builds the flexflow_amd.models builder
of the reference example into an FFModel, feeds synthetic batches of the model's shapes and times
training iterations (reference examples/cpp/*/ top_level_task loops, examples/python/native/*).

    python examples/python/native/alexnet.py -b 64 --iterations 20 [--small] [--search unity]
    python -m flexflow_amd.run --nproc 8 examples/python/native/inception.py -b 512 --search mcmc
"""
import argparse
import sys

import _args  # noqa: F401  (puts the repo root on sys.path)
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.models import build


def run(name, argv=None):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--small", action="store_true", help="reduced widths / image sizes (CPU runs)")
    args, rest = ap.parse_known_args(sys.argv[1:] if argv is None else argv)
    ffconfig = FFConfig(rest)
    ffmodel = FFModel(ffconfig)
    inputs, out, loss, mets, make_batch = build(name, ffmodel, ffconfig.batch_size, small=args.small)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.001)
    ffmodel.compile(loss_type=loss, metrics=mets)
    rng = np.random.default_rng(0)
    arrs, lab = make_batch(rng)
    for t, a in zip(inputs, arrs):
        t.set_tensor(ffmodel, a)
    ffmodel.label_tensor.set_tensor(ffmodel, lab)
    ffmodel.init_layers()
    ffmodel.train_step()  # warm-up (kernel autotuning, hipGraph capture)
    ffmodel.reset_metrics()
    ts = ffconfig.get_current_time()
    for _ in range(args.iterations):
        ffconfig.begin_trace(111)
        ffmodel.train_step()
        ffconfig.end_trace(111)
    pm = ffmodel.get_perf_metrics()  # host read-back: waits for the device
    run_time = 1e-6 * (ffconfig.get_current_time() - ts)
    print("%s: ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s, strategy %s" %
          (name, run_time, ffconfig.batch_size * args.iterations / run_time,
           (ffmodel.search_report or {}).get("algo")))
    return pm
