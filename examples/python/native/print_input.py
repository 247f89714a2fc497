"""Map input tensors on the host, write them, then inspect layer inputs / outputs / weights by id
(reference examples/python/native/print_input.py)."""
from _args import parse  # noqa: I001
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def top_level_task(argv=None):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input1 = ffmodel.create_tensor([ffconfig.batch_size, 3, 64, 64], DataType.DT_FLOAT)
    input2 = ffmodel.create_tensor([ffconfig.batch_size, 256], DataType.DT_FLOAT)
    input1.inline_map(ffconfig)
    a1 = input1.get_array(ffconfig)
    print(hex(a1.__array_interface__["data"][0]), a1.shape)
    input1.inline_unmap(ffconfig)
    input2.inline_map(ffconfig)
    a2 = input2.get_array(ffconfig)
    a2 *= 0
    a2 += 2.2
    print(a2.shape, a2.reshape(-1)[:4])
    input2.inline_unmap(ffconfig)
    t1 = ffmodel.conv2d(input1, 64, 11, 11, 4, 4, 2, 2)
    t2 = ffmodel.dense(input2, 128, ActiMode.AC_MODE_RELU)
    t2 = ffmodel.dense(t2, 128, ActiMode.AC_MODE_RELU)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    ffmodel.init_layers()
    ffmodel.forward()
    dense1 = ffmodel.get_layer_by_id(1)  # op ids skip inputs: conv2d = 0, first dense = 1
    x = dense1.get_input_tensor().get_tensor(ffmodel)
    assert np.allclose(x, 2.2), x.reshape(-1)[:4]
    y = dense1.get_output_tensor().get_tensor(ffmodel)
    w = dense1.get_weight_tensor().get_weights(ffmodel)
    print("dense1 in", x.shape, "out", y.shape, "kernel", w.shape)
    print("conv out", t1.get_tensor(ffmodel).shape)


if __name__ == "__main__":
    args, rest = parse(0)
    top_level_task(rest)
