"""ResNet-50 (bottleneck blocks 3-4-6-3) on CIFAR-10 images resized to 229 x 229 (reference
examples/python/native/resnet.py and examples/cpp/ResNet), spelled out with the FFModel builder API.
The residual add and the ReLU after it run as one element-wise pass at compile time
(Executor._plan_binary_relu). Offline, the CIFAR-10 loader serves synthetic images of its shapes.

    python examples/python/native/resnet.py -b 64 -e 1 --samples 1024
    python examples/python/native/resnet.py -b 4 --iterations 1 --small     # CPU smoke run
"""
import argparse

from _args import parse  # noqa: I001  (puts the repo root on sys.path)
import numpy as np

from alexnet import resize_nearest
from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import cifar10


def bottleneck(ff, x, width, stride):
    """1x1 reduce -> 3x3 (carries the stride) -> 1x1 expand to 4*width, each followed by batch norm;
    a projection shortcut when the shape changes; then add and ReLU."""
    t = ff.batch_norm(ff.conv2d(x, width, 1, 1, 1, 1, 0, 0, ActiMode.AC_MODE_NONE))
    t = ff.batch_norm(ff.conv2d(t, width, 3, 3, stride, stride, 1, 1, ActiMode.AC_MODE_NONE))
    t = ff.batch_norm(ff.conv2d(t, 4 * width, 1, 1, 1, 1, 0, 0), False)
    if stride > 1 or x.dims[1] != 4 * width:
        x = ff.batch_norm(ff.conv2d(x, 4 * width, 1, 1, stride, stride, 0, 0, ActiMode.AC_MODE_NONE), False)
    return ff.relu(ff.add(x, t))


def resnet(ff, x, stages=(3, 4, 6, 3), classes=10):
    t = ff.batch_norm(ff.conv2d(x, 64, 7, 7, 2, 2, 3, 3))
    t = ff.pool2d(t, 3, 3, 2, 2, 1, 1)
    for i, (blocks, width) in enumerate(zip(stages, (64, 128, 256, 512))):
        for b in range(blocks):
            t = bottleneck(ff, t, width, 2 if (b == 0 and i > 0) else 1)
    side = t.dims[2]
    t = ff.pool2d(t, side, side, 1, 1, 0, 0, PoolType.POOL_AVG)  # global average pool
    return ff.softmax(ff.dense(ff.flat(t), classes))


def top_level_task(argv, num_samples, iterations=None, small=False):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    side = 64 if small else 229
    x = ffmodel.create_tensor([ffconfig.batch_size, 3, side, side], DataType.DT_FLOAT)
    resnet(ffmodel, x, stages=(1, 1, 1, 1) if small else (3, 4, 6, 3))
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.001)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples=num_samples, num_test=16)
    dl_x = ffmodel.create_data_loader(x, resize_nearest(x_train, side))
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y_train.astype(np.int32).reshape(num_samples, 1))
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    if iterations is None:
        ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
        seen = num_samples * ffconfig.epochs
    else:
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
    pm = ffmodel.get_perf_metrics()
    run_time = 1e-6 * (ffconfig.get_current_time() - ts)
    print("resnet: ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s, accuracy %.2f%%" %
          (run_time, seen / run_time, pm.get_accuracy()))
    return pm


if __name__ == "__main__":
    args, rest = parse(1024)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--iterations", type=int, default=None)
    ap.add_argument("--small", action="store_true")
    extra, rest = ap.parse_known_args(rest)
    top_level_task(rest, min(args.samples, 64) if extra.small else args.samples, extra.iterations, extra.small)
