"""Train the CIFAR-10 CNN imported from ONNX (reference examples/python/onnx/cifar10_cnn.py):
--test_type 1 = torch export, 0 = Keras export."""
from _args import parse  # noqa: I001
import argparse
import os

import numpy as np

from flexflow_amd.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.onnx.model import ONNXModel, ONNXModelKeras


def top_level_task(argv, test_type=1, num_samples=10000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    inp = ffmodel.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    if test_type == 1:
        if not os.path.exists("cifar10_cnn_pt.onnx"):
            import cifar10_cnn_pt
            cifar10_cnn_pt.export()
        om = ONNXModel("cifar10_cnn_pt.onnx")
        om.apply(ffmodel, {"input.1": inp})
    else:
        if not os.path.exists("cifar10_cnn_keras.onnx"):
            import cifar10_cnn_keras
            cifar10_cnn_keras.export(batch=ffconfig.batch_size)
        om = ONNXModelKeras("cifar10_cnn_keras.onnx", ffconfig, ffmodel)
        om.apply(ffmodel, {"input_1": inp})
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    om.load_initializers(ffmodel)
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x = x_train[:num_samples].astype("float32") / 255
    y = y_train[:num_samples].astype("int32")
    ffmodel.fit(x=ffmodel.create_data_loader(inp, x), y=ffmodel.create_data_loader(ffmodel.label_tensor, y),
                epochs=ffconfig.epochs)
    return ffmodel.get_perf_metrics().get_accuracy()


if __name__ == "__main__":
    args, rest = parse(10000)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--test_type", type=int, choices=[0, 1], default=1)
    a2, rest = ap.parse_known_args(rest)
    top_level_task(rest, a2.test_type, args.samples)
