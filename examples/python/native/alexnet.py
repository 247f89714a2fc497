"""AlexNet on CIFAR-10 images resized to 229 x 229 (reference examples/python/native/alexnet.py and
examples/cpp/AlexNet): the network is spelled out with the FFModel builder API, the data goes through
SingleDataLoaders and `fit`. Offline, `flexflow_amd.keras.datasets.cifar10` serves deterministic
synthetic images of CIFAR-10's shapes.

    python examples/python/native/alexnet.py -b 64 -e 1 --samples 2048
    python examples/python/native/alexnet.py -b 4 --iterations 1 --small     # CPU smoke run
"""
import argparse

from _args import parse  # noqa: I001  (puts the repo root on sys.path)
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import cifar10


def alexnet(ff, x, classes=10):
    """The reference layer stack: five convolutions (the first with Glorot-uniform weights and zero
    bias), three max pools, two 4096-wide ReLU dense layers and a softmax classifier."""
    t = ff.conv2d(x, 64, 11, 11, 4, 4, 2, 2, ActiMode.AC_MODE_RELU, 1, True, None,
                  GlorotUniformInitializer(123), ZeroInitializer())
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = ff.conv2d(t, 192, 5, 5, 1, 1, 2, 2, ActiMode.AC_MODE_RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    for ch in (384, 256, 256):
        t = ff.conv2d(t, ch, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = ff.flat(t)
    t = ff.dense(t, 4096, ActiMode.AC_MODE_RELU)
    t = ff.dense(t, 4096, ActiMode.AC_MODE_RELU)
    return ff.softmax(ff.dense(t, classes))


def resize_nearest(images, size):
    """[N, C, H, W] uint8 -> [N, C, size, size] float32 in [0, 1], nearest-neighbour sampling."""
    h, w = images.shape[2:]
    rows = (np.arange(size) * h // size).astype(np.int64)
    cols = (np.arange(size) * w // size).astype(np.int64)
    return images[:, :, rows][:, :, :, cols].astype(np.float32) / 255.0


def top_level_task(argv, num_samples, iterations=None, small=False):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    side = 67 if small else 229  # --small: the smallest input the layer stack accepts
    x = ffmodel.create_tensor([ffconfig.batch_size, 3, side, side], DataType.DT_FLOAT)
    alexnet(ffmodel, x)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples=num_samples, num_test=16)
    images = resize_nearest(x_train, side)
    labels = y_train.astype(np.int32).reshape(num_samples, 1)
    dl_x = ffmodel.create_data_loader(x, images)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, labels)
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    if iterations is None:
        ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
        seen = num_samples * ffconfig.epochs
    else:  # a fixed number of traced iterations, as the reference C++ driver loops
        dl_x.reset()
        dl_y.reset()
        for _ in range(iterations):
            dl_x.next_batch(ffmodel)
            dl_y.next_batch(ffmodel)
            ffconfig.begin_trace(111)
            ffmodel.forward()
            ffmodel.zero_gradients()
            ffmodel.backward()
            ffmodel.update()
            ffconfig.end_trace(111)
        seen = ffconfig.batch_size * iterations
    pm = ffmodel.get_perf_metrics()  # host read-back: waits for the device
    run_time = 1e-6 * (ffconfig.get_current_time() - ts)
    print("alexnet: ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s, accuracy %.2f%%" %
          (run_time, seen / run_time, pm.get_accuracy()))
    return pm


if __name__ == "__main__":
    args, rest = parse(2048)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--iterations", type=int, default=None)
    ap.add_argument("--small", action="store_true")
    extra, rest = ap.parse_known_args(rest)
    top_level_task(rest, min(args.samples, 64) if extra.small else args.samples, extra.iterations, extra.small)
