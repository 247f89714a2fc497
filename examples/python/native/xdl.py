"""XDL (reference examples/cpp/XDL/xdl.cc): sum-pooled embedding bags for every sparse feature,
concatenated and fed to a 256-256-256-2 MLP with a sigmoid output; MSE loss. 4 tables of
1,000,000 x 64 (1000 rows with --small).

    python examples/python/native/xdl.py -b 2048 --iterations 20
"""
import math

import zoo
from flexflow_amd.core import *  # noqa: F401,F403


def xdl(ff, sparse, rows, dim=64, top=(256, 256, 256, 2)):
    bags = []
    for i, (ids, n) in enumerate(zip(sparse, rows)):
        bound = math.sqrt(1.0 / n)
        bags.append(ff.embedding(ids, n, dim, AggrMode.AGGR_MODE_SUM,
                                 kernel_initializer=UniformInitializer(1000 + i, -bound, bound)))
    t = ff.concat(bags, -1)
    for i, w in enumerate(top):
        last = i + 1 == len(top)
        std = math.sqrt(2.0 / (t.dims[-1] + w))
        t = ff.dense(t, w, ActiMode.AC_MODE_SIGMOID if last else ActiMode.AC_MODE_RELU, use_bias=False,
                     kernel_initializer=NormInitializer(200 + i, 0.0, std))
    return t


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    rows = [1000] * 4 if small else [1000000] * 4
    sparse = [ffmodel.create_tensor([ffconfig.batch_size, 1], DataType.DT_INT64) for _ in rows]
    out = xdl(ffmodel, sparse, rows)
    zoo.train("xdl", ffconfig, ffmodel, sparse, out, zoo.MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR],
              iterations, index_range={t.guid: n for t, n in zip(sparse, rows)})
