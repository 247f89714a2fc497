"""Read a layer's weight tensor after init (reference examples/python/native/print_weight.py)."""
from _args import parse  # noqa: I001
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def top_level_task(argv=None):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input_tensor = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    t = ffmodel.dense(input_tensor, 512, ActiMode.AC_MODE_RELU, kernel_initializer=UniformInitializer(12, -1, 1))
    t = ffmodel.dense(t, 512, ActiMode.AC_MODE_RELU)
    ffmodel.softmax(ffmodel.dense(t, 10))
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    ffmodel.init_layers()
    dense1 = ffmodel.get_layer_by_id(0)
    print(dense1)
    w = dense1.get_weight_tensor()
    arr = np.asarray(w.get_weights(ffmodel))
    print(w, arr.shape, float(arr.min()), float(arr.max()))
    assert arr.min() >= -1 and arr.max() <= 1  # UniformInitializer(12, -1, 1)


if __name__ == "__main__":
    args, rest = parse(0)
    top_level_task(rest)
