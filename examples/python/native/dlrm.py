"""DLRM (reference examples/cpp/DLRM/dlrm.cc, examples/python/native/dlrm.py): a bottom MLP over the
dense features, one sum-pooled embedding bag per sparse feature (bf16 tables, the reference's
half-precision tables), concatenation, and a top MLP ending in a sigmoid; MSE loss. Defaults: 4 tables
of 1,000,000 x 64, bottom 4-64-64, top 64-64-2 (1000-row tables with --small). Tables can be placed
one per GPU by the search (`--search unity`) or an imported strategy; the exchange back to data
parallel is an all-to-all.

    python examples/python/native/dlrm.py -b 2048 --iterations 20
"""
import math

import zoo
from flexflow_amd.core import *  # noqa: F401,F403


def mlp(ff, t, widths, sigmoid_at, seed):
    """Bias-free denses with Glorot-normal weights; ReLU except a sigmoid on layer `sigmoid_at`."""
    for i, (fan_in, fan_out) in enumerate(zip(widths[:-1], widths[1:])):
        act = ActiMode.AC_MODE_SIGMOID if i == sigmoid_at else ActiMode.AC_MODE_RELU
        init = NormInitializer(seed + i, 0.0, math.sqrt(2.0 / (fan_in + fan_out)))
        t = ff.dense(t, fan_out, act, use_bias=False, kernel_initializer=init)
    return t


def dlrm(ff, dense, sparse, rows, dim=64, bottom=(4, 64, 64), top=(64, 64, 2)):
    x = mlp(ff, dense, list(bottom), -1, 1)
    bags = []
    for i, (ids, n) in enumerate(zip(sparse, rows)):
        bound = math.sqrt(1.0 / n)
        e = ff.embedding(ids, n, dim, AggrMode.AGGR_MODE_SUM, dtype=DataType.DT_HALF,
                         kernel_initializer=UniformInitializer(1000 + i, -bound, bound))
        bags.append(ff.cast(e, DataType.DT_FLOAT))
    z = ff.concat([x] + bags, -1)
    return mlp(ff, z, [z.dims[-1]] + list(top[1:]), len(top) - 2, 100)


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    rows = [1000] * 4 if small else [1000000] * 4
    b = ffconfig.batch_size
    sparse = [ffmodel.create_tensor([b, 1], DataType.DT_INT64) for _ in rows]
    dense = ffmodel.create_tensor([b, 4], DataType.DT_FLOAT)
    out = dlrm(ffmodel, dense, sparse, rows)
    zoo.train("dlrm", ffconfig, ffmodel, sparse + [dense], out, zoo.MSE,
              [MetricsType.METRICS_MEAN_SQUARED_ERROR], iterations,
              index_range={t.guid: n for t, n in zip(sparse, rows)})
