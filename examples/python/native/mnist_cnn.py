"""MNIST CNN (reference examples/python/native/mnist_cnn.py): conv-conv-pool-flat-dense-dense."""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import mnist


def top_level_task(argv=None, num_samples=60000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    x = ffmodel.create_tensor([ffconfig.batch_size, 1, 28, 28], DataType.DT_FLOAT)
    t = ffmodel.conv2d(x, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.conv2d(t, 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ffmodel.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = ffmodel.flat(t)
    t = ffmodel.dense(t, 128, ActiMode.AC_MODE_RELU)
    t = ffmodel.dense(t, 10)
    t = ffmodel.softmax(t)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x_train = x_train.reshape(num_samples, 1, 28, 28).astype("float32") / 255
    y_train = y_train.astype("int32").reshape(num_samples, 1)
    dl_x = ffmodel.create_data_loader(x, x_train)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y_train)
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    run_time = 1e-6 * (ffconfig.get_current_time() - ts)
    print("epochs %d, ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" %
          (ffconfig.epochs, run_time, num_samples * ffconfig.epochs / run_time))
    return ffmodel.get_perf_metrics()


if __name__ == "__main__":
    args, rest = parse(60000)
    pm = top_level_task(rest, args.samples)
    if args.test_acc:
        assert pm.get_accuracy() >= ModelAccuracy.MNIST_CNN.value, pm.get_accuracy()
