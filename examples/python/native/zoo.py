"""Shared timing loop for the synthetic-data examples (inception / resnext50 / dlrm / xdl / candle_uno /
transformer / mlp_unify / mixture_of_experts / nmt). Each example builds its own network with the
FFModel API and hands its input tensors, output and loss here; this module feeds random batches of
those shapes and times training iterations inside begin_trace / end_trace (reference
examples/cpp/*/ top_level_task loops, examples/python/native/*).

    python examples/python/native/inception.py -b 64 --iterations 20 [--small] [--search unity]
    python -m flexflow_amd.run --nproc 8 examples/python/native/inception.py -b 512 --search mcmc
"""
import argparse
import sys

import _args  # noqa: F401  (puts the repo root on sys.path)
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403

SCCE = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
MSE = LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
ACC = [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY]


def setup(argv=None):
    """Parse --iterations / --small; return (ffconfig, ffmodel, small, iterations)."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--small", action="store_true", help="reduced widths / image sizes (CPU runs)")
    args, rest = ap.parse_known_args(sys.argv[1:] if argv is None else argv)
    ffconfig = FFConfig(rest)
    return ffconfig, FFModel(ffconfig), args.small, args.iterations


def random_batch(inputs, out, loss, index_range=None, seed=0):
    """Synthetic batch: normal floats, integer ids below index_range[guid] (default 2), and labels
    (class ids for cross entropy, normal targets of the output's shape for MSE)."""
    rng = np.random.default_rng(seed)
    arrs = []
    for t in inputs:
        if t.data_type in (DataType.DT_INT32, DataType.DT_INT64):
            hi = (index_range or {}).get(t.guid, 2)
            arrs.append(rng.integers(0, hi, tuple(t.dims)).astype(
                np.int64 if t.data_type == DataType.DT_INT64 else np.int32))
        else:
            arrs.append(rng.standard_normal(tuple(t.dims)).astype(np.float32))
    if loss == SCCE:
        lab = rng.integers(0, out.dims[-1], tuple(out.dims[:-1]) + (1,)).astype(np.int32)
    else:
        lab = rng.standard_normal(tuple(out.dims)).astype(np.float32)
    return arrs, lab


def train(name, ffconfig, ffmodel, inputs, out, loss, metrics, iterations, index_range=None, optimizer=None):
    """Compile with SGD (or `optimizer`), load one synthetic batch, and time `iterations` steps."""
    ffmodel.optimizer = optimizer or SGDOptimizer(ffmodel, 0.001)
    ffmodel.compile(loss_type=loss, metrics=metrics)
    arrs, lab = random_batch(inputs, out, loss, index_range)
    for t, a in zip(inputs, arrs):
        t.set_tensor(ffmodel, a)
    ffmodel.label_tensor.set_tensor(ffmodel, lab)
    ffmodel.init_layers()
    ffmodel.train_step()  # warm-up (kernel autotuning, hipGraph capture)
    ffmodel.reset_metrics()
    ts = ffconfig.get_current_time()
    for _ in range(iterations):
        ffconfig.begin_trace(111)
        ffmodel.train_step()
        ffconfig.end_trace(111)
    pm = ffmodel.get_perf_metrics()  # host read-back: waits for the device
    run_time = 1e-6 * (ffconfig.get_current_time() - ts)
    print("%s: ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s, strategy %s" %
          (name, run_time, ffconfig.batch_size * iterations / run_time,
           (ffmodel.search_report or {}).get("algo")))
    return pm
