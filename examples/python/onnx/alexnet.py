"""Train AlexNet imported from ONNX on CIFAR-10 upscaled to 229x229 by nearest neighbour
(reference examples/python/onnx/alexnet.py; --small: 67x67 inputs for CPU tests)."""
from _args import parse  # noqa: I001
import argparse
import os

import numpy as np

from flexflow_amd.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.onnx.model import ONNXModel


def upscale(x, size):
    idx = (np.arange(size) * x.shape[-1] // size).astype(np.int64)
    return x[:, :, idx][:, :, :, idx]


def top_level_task(argv, num_samples=10000, size=229):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    inp = ffmodel.create_tensor([ffconfig.batch_size, 3, size, size], DataType.DT_FLOAT)
    path = f"alexnet_{size}.onnx"
    if not os.path.exists(path):
        import alexnet_pt
        alexnet_pt.export(path, size)
    ONNXModel(path).apply(ffmodel, {"input.1": inp})
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x = upscale(x_train[:num_samples], size).astype(np.float32) / 255
    y = y_train[:num_samples].astype("int32")
    ffmodel.fit(x=ffmodel.create_data_loader(inp, x), y=ffmodel.create_data_loader(ffmodel.label_tensor, y),
                epochs=ffconfig.epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--small", action="store_true")
    a2, rest = ap.parse_known_args(rest)
    top_level_task(rest, args.samples, 67 if a2.small else 229)
