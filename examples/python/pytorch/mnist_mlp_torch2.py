"""MNIST MLP built straight from the nn.Module with PyTorchModel.torch_to_ff (no .ff file;
reference examples/python/pytorch/mnist_mlp_torch2.py)."""
from _args import parse  # noqa: I001
import numpy as np
from accuracy import ModelAccuracy
from mnist_mlp_torch import MLP

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.torch import PyTorchModel


def top_level_task(argv=None, num_samples=60000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input_tensor = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    PyTorchModel(MLP()).torch_to_ff(ffmodel, [input_tensor])
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x, y), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x = x.reshape(num_samples, 784).astype("float32") / 255
    y = np.reshape(y.astype("int32"), (num_samples, 1))
    dl_x = ffmodel.create_data_loader(input_tensor, x)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y)
    ffmodel.init_layers()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    return ffmodel.get_perf_metrics().get_accuracy()


if __name__ == "__main__":
    args, rest = parse(60000)
    acc = top_level_task(rest, args.samples)
    if args.test_acc:
        assert acc >= ModelAccuracy.MNIST_MLP.value, acc
