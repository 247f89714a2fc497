"""Train ResNet-18 imported from ONNX on CIFAR-10 upscaled to 224x224 (reference
examples/python/onnx/resnet.py; --small: 64x64 inputs and quarter widths for CPU tests)."""
from _args import parse  # noqa: I001
import argparse
import os

import numpy as np
from alexnet import upscale

from flexflow_amd.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.onnx.model import ONNXModel


def top_level_task(argv, num_samples=10000, size=224, small=False):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    inp = ffmodel.create_tensor([ffconfig.batch_size, 3, size, size], DataType.DT_FLOAT)
    path = f"resnet18_{size}{'_small' if small else ''}.onnx"
    if not os.path.exists(path):
        import resnet_pt
        resnet_pt.export(path, size, (16, 32, 64, 128) if small else (64, 128, 256, 512))
    t = ONNXModel(path).apply(ffmodel, {"input.1": inp})
    ffmodel.softmax(t)
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
    top_level_task(rest, args.samples, 64 if a2.small else 224, a2.small)
