import numpy as np


def to_categorical(y, num_classes=None, dtype="float32"):
    y = np.asarray(y, dtype=np.int64).reshape(-1)
    n = int(num_classes or (y.max() + 1))
    out = np.zeros((y.shape[0], n), dtype=dtype)
    out[np.arange(y.shape[0]), y] = 1
    return out


def normalize(x, axis=-1, order=2):
    n = np.atleast_1d(np.linalg.norm(x, order, axis))
    n[n == 0] = 1
    return x / np.expand_dims(n, axis)
