"""CIFAR-10: (x_train [50000,3,32,32] uint8 channels-first, y_train [50000,1]), (x_test, y_test)."""
import numpy as np

from . import _local, synthetic_images


def load_data(num_samples=50000, num_test=10000):
    p = _local("cifar10.npz")
    if p:
        with np.load(p, allow_pickle=False) as f:
            return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    x, y = synthetic_images(num_samples + num_test, (3, 32, 32), 10, seed=32)
    y = y.reshape(-1, 1)
    return (x[:num_samples], y[:num_samples]), (x[num_samples:], y[num_samples:])
