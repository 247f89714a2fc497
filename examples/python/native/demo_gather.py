"""Gather neighbour rows with an attached index tensor, trained with MSE against an attached label
(reference examples/python/native/demo_gather.py)."""
from _args import parse  # noqa: I001
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def top_level_task(argv=None, iters=100):
    ffconfig = FFConfig(argv)
    bs = ffconfig.batch_size
    ffmodel = FFModel(ffconfig)
    neighbors = np.array([[[0], [5], [3], [3], [7], [9]]]).repeat(bs, 0).repeat(5, 2).astype(np.int32)
    x = np.full((bs, 16, 5), 0.01, np.float32)
    inp = ffmodel.create_tensor([bs, 16, 5], DataType.DT_FLOAT)
    index = ffmodel.create_tensor([bs, 6, 5], DataType.DT_INT32)
    x0 = ffmodel.dense(inp, 5, ActiMode.AC_MODE_NONE, False)
    ffmodel.gather(x0, index, 1)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ffmodel.init_layers()
    inp.attach_numpy_array(ffmodel, ffconfig, x)
    index.attach_numpy_array(ffmodel, ffconfig, neighbors)
    y = np.random.default_rng(0).random((bs, 6, 5)).astype("float32")
    ffmodel.label_tensor.attach_numpy_array(ffmodel, ffconfig, y)
    for _ in range(iters):
        ffmodel.forward()
        ffmodel.zero_gradients()
        ffmodel.backward()
        ffmodel.update()
    print("mse", ffmodel.get_perf_metrics().get_mse_loss() if hasattr(ffmodel.get_perf_metrics(), "get_mse_loss")
          else ffmodel.get_perf_metrics())


if __name__ == "__main__":
    args, rest = parse(0)
    top_level_task(rest)
