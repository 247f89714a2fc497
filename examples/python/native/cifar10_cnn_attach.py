"""CIFAR-10 CNN fed by attaching each batch's numpy arrays to the input and label tensors
(reference examples/python/native/cifar10_cnn_attach.py)."""
from _args import parse  # noqa: I001

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import cifar10


def top_level_task(argv=None, num_samples=10000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    bs = ffconfig.batch_size
    input_tensor = ffmodel.create_tensor([bs, 3, 32, 32], DataType.DT_FLOAT)
    t = ffmodel.conv2d(input_tensor, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.pool2d(ffmodel.conv2d(t, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU), 2, 2, 2, 2, 0, 0)
    t = ffmodel.conv2d(t, 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.pool2d(ffmodel.conv2d(t, 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU), 2, 2, 2, 2, 0, 0)
    t = ffmodel.softmax(ffmodel.dense(ffmodel.dense(ffmodel.flat(t), 512, ActiMode.AC_MODE_RELU), 10))
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x = x_train[:num_samples].astype("float32") / 255
    y = y_train[:num_samples].astype("int32")
    ffmodel.init_layers()
    for epoch in range(ffconfig.epochs):
        ffmodel.reset_metrics()
        for it in range(num_samples // bs):
            input_tensor.attach_numpy_array(ffmodel, ffconfig, x[it * bs:(it + 1) * bs])
            ffmodel.label_tensor.attach_numpy_array(ffmodel, ffconfig, y[it * bs:(it + 1) * bs])
            ffmodel.forward()
            ffmodel.zero_gradients()
            ffmodel.backward()
            ffmodel.update()
            input_tensor.detach_numpy_array(ffconfig)
            ffmodel.label_tensor.detach_numpy_array(ffconfig)
        print(f"epoch {epoch}: {ffmodel.get_perf_metrics()}")


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(rest, args.samples)
