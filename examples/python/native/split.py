"""Three convolutions concatenated, split back into three, one branch trained on (reference
examples/python/native/split.py)."""
from _args import parse  # noqa: I001

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import cifar10


def top_level_task(argv=None, num_samples=10000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input_tensor = ffmodel.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    ts = [ffmodel.conv2d(input_tensor, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU) for _ in range(3)]
    t = ffmodel.concat(ts, 1)
    ts = ffmodel.split(t, 3, 1)
    t = ffmodel.conv2d(ts[1], 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = ffmodel.conv2d(t, 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.conv2d(t, 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.flat(ffmodel.pool2d(t, 2, 2, 2, 2, 0, 0))
    t = ffmodel.softmax(ffmodel.dense(ffmodel.dense(t, 512, ActiMode.AC_MODE_RELU), 10))
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x = x_train[:num_samples].astype("float32") / 255
    y = y_train[:num_samples].astype("int32")
    dl_x = ffmodel.create_data_loader(input_tensor, x)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y)
    ffmodel.init_layers()
    ts0 = ffconfig.get_current_time()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    run = 1e-6 * (ffconfig.get_current_time() - ts0)
    print(f"epochs {ffconfig.epochs}, ELAPSED TIME = {run:.4f}s, THROUGHPUT = "
          f"{dl_x.num_samples * ffconfig.epochs / run:.2f} samples/s")


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(rest, args.samples)
