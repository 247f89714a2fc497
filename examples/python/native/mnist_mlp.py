"""MNIST MLP through the native FFModel API (reference examples/python/native/mnist_mlp.py).

    python examples/python/native/mnist_mlp.py -b 64 -e 2 [--samples N] [-a]
    python -m flexflow_amd.run --nproc 8 examples/python/native/mnist_mlp.py   # data parallel, 8 GPUs
"""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import mnist


def top_level_task(argv=None, num_samples=60000):
    ffconfig = FFConfig(argv)
    print("Python API batchSize(%d) workersPerNodes(%d) numNodes(%d)" %
          (ffconfig.batch_size, ffconfig.workers_per_node, ffconfig.num_nodes))
    ffmodel = FFModel(ffconfig)
    input_tensor = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    kernel_init = UniformInitializer(12, -1, 1)
    t = ffmodel.dense(input_tensor, 512, ActiMode.AC_MODE_RELU, kernel_initializer=kernel_init)
    t = ffmodel.dense(t, 512, ActiMode.AC_MODE_RELU)
    t = ffmodel.dense(t, 10)
    t = ffmodel.softmax(t)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x_train = x_train.reshape(num_samples, 784).astype("float32") / 255
    y_train = y_train.astype("int32").reshape(num_samples, 1)
    dl_x = ffmodel.create_data_loader(input_tensor, x_train)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y_train)
    ffmodel.init_layers()
    ts_start = ffconfig.get_current_time()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    ffmodel.eval(x=dl_x, y=dl_y)
    run_time = 1e-6 * (ffconfig.get_current_time() - ts_start)
    print("epochs %d, ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" %
          (ffconfig.epochs, run_time, num_samples * ffconfig.epochs / run_time))
    return ffmodel.get_perf_metrics()


if __name__ == "__main__":
    args, rest = parse(60000)
    pm = top_level_task(rest, args.samples)
    if args.test_acc:
        assert pm.get_accuracy() >= ModelAccuracy.MNIST_MLP.value, pm.get_accuracy()
