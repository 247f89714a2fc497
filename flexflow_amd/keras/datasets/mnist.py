"""MNIST: (x_train [60000,28,28] uint8, y_train), (x_test [10000,28,28], y_test)."""
import numpy as np

from . import _local, synthetic_images


def load_data(path="mnist.npz", num_train=60000, num_test=10000):
    p = _local(path)
    if p:
        with np.load(p, allow_pickle=False) as f:
            return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    x, y = synthetic_images(num_train + num_test, (28, 28), 10, seed=28)
    return (x[:num_train], y[:num_train]), (x[num_train:], y[num_train:])
