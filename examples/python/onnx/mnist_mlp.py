"""Train the MNIST MLP imported from ONNX (reference examples/python/onnx/mnist_mlp.py):
--test_type 1 loads the torch export (mnist_mlp_pt.onnx, input "input.1"), 0 the Keras export
(mnist_mlp_keras.onnx through ONNXModelKeras, input "input_1"). Missing files are exported first."""
from _args import parse  # noqa: I001
import argparse
import os
import sys

import numpy as np
from accuracy import ModelAccuracy

from flexflow_amd.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.onnx.model import ONNXModel, ONNXModelKeras


def top_level_task(argv, test_type=1, num_samples=60000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input1 = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    if test_type == 1:
        if not os.path.exists("mnist_mlp_pt.onnx"):
            import mnist_mlp_pt
            mnist_mlp_pt.export()
        t = ONNXModel("mnist_mlp_pt.onnx").apply(ffmodel, {"input.1": input1})
    else:
        if not os.path.exists("mnist_mlp_keras.onnx"):
            import mnist_mlp_keras
            mnist_mlp_keras.export(batch=ffconfig.batch_size)
        om = ONNXModelKeras("mnist_mlp_keras.onnx", ffconfig, ffmodel)
        t = om.apply(ffmodel, {"input_1": input1})
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    if test_type == 0:
        om.load_initializers(ffmodel)
    (x_train, y_train), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x_train = x_train.reshape(num_samples, 784).astype("float32") / 255
    y_train = np.reshape(y_train.astype("int32"), (num_samples, 1))
    dl_x = ffmodel.create_data_loader(input1, x_train)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y_train)
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    run = 1e-6 * (ffconfig.get_current_time() - ts)
    print(f"epochs {ffconfig.epochs}, ELAPSED TIME = {run:.4f}s, THROUGHPUT = "
          f"{num_samples * ffconfig.epochs / run:.2f} samples/s")
    return ffmodel.get_perf_metrics().get_accuracy()


if __name__ == "__main__":
    args, rest = parse(60000)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--test_type", type=int, choices=[0, 1], default=1)
    a2, rest = ap.parse_known_args(rest)
    acc = top_level_task(rest, a2.test_type, args.samples)
    if args.test_acc and acc < ModelAccuracy.MNIST_MLP.value:
        sys.exit(f"accuracy {acc} below {ModelAccuracy.MNIST_MLP.value}")
