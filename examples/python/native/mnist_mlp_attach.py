"""MNIST MLP fed batch by batch with set_tensor instead of a data loader (reference
examples/python/native/mnist_mlp_attach.py)."""
from _args import parse  # noqa: I001
import numpy as np
from accuracy import ModelAccuracy

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import mnist


def top_level_task(argv=None, num_samples=60000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input_tensor = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    (x_train, y_train), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x_train = x_train.reshape(num_samples, 784).astype("float32") / 255
    y_train = np.reshape(y_train.astype("int32"), (num_samples, 1))
    t = ffmodel.dense(input_tensor, 512, ActiMode.AC_MODE_RELU)
    t = ffmodel.dense(t, 512, ActiMode.AC_MODE_RELU)
    ffmodel.softmax(ffmodel.dense(t, 10))
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    label_tensor = ffmodel.label_tensor
    bs = ffconfig.batch_size
    ffmodel.init_layers()
    ts0 = ffconfig.get_current_time()
    for epoch in range(ffconfig.epochs):
        ffmodel.reset_metrics()
        for it in range(num_samples // bs):
            input_tensor.set_tensor(ffmodel, x_train[it * bs:(it + 1) * bs])
            label_tensor.set_tensor(ffmodel, y_train[it * bs:(it + 1) * bs])
            ffconfig.begin_trace(111)
            ffmodel.forward()
            ffmodel.zero_gradients()
            ffmodel.backward()
            ffmodel.update()
            ffconfig.end_trace(111)
        print(f"epoch {epoch}: {ffmodel.get_perf_metrics()}")
    run = 1e-6 * (ffconfig.get_current_time() - ts0)
    print(f"epochs {ffconfig.epochs}, ELAPSED TIME = {run:.4f}s, THROUGHPUT = "
          f"{num_samples * ffconfig.epochs / run:.2f} samples/s")
    return ffmodel.get_perf_metrics().get_accuracy()


if __name__ == "__main__":
    args, rest = parse(60000)
    acc = top_level_task(rest, args.samples)
    if args.test_acc:
        assert acc >= ModelAccuracy.MNIST_MLP.value, acc
