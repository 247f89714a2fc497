"""Data preparation shared by the keras examples (mnist / cifar10 synthetic stand-ins, as in the
reference's `mnist.load_data()` / `cifar10.load_data(num_samples)` preambles)."""
import numpy as np

from flexflow_amd.keras.datasets import cifar10, mnist


def mnist_flat(n):
    (x, y), _ = mnist.load_data(num_train=n, num_test=16)
    return x.reshape(n, 784).astype("float32") / 255, np.reshape(y.astype("int32"), (n, 1))


def mnist_images(n):
    (x, y), _ = mnist.load_data(num_train=n, num_test=16)
    return x.reshape(n, 1, 28, 28).astype("float32") / 255, np.reshape(y.astype("int32"), (n, 1))


def cifar(n):
    (x, y), _ = cifar10.load_data(n, num_test=16)
    return x[:n].astype("float32") / 255, y[:n].astype("int32")
