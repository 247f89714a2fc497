"""Keras-style datasets (reference keras/datasets/{mnist,cifar10,reuters}.py).

There is no network: `load_data()` reads a local copy when one exists (FF_DATASETS_DIR or
~/.keras/datasets, standard npz/pickle-free formats only) and otherwise returns a deterministic
SYNTHETIC dataset of the same shapes and dtypes whose labels are a fixed function of the inputs
(nearest random class prototype), so models can actually learn it and accuracy tests mean something.
"""
from __future__ import annotations

import os

import numpy as np


def _local(name):
    for d in (os.environ.get("FF_DATASETS_DIR"), os.path.expanduser("~/.keras/datasets")):
        if d and os.path.exists(os.path.join(d, name)):
            return os.path.join(d, name)
    return None


def synthetic_images(n, shape, num_classes, seed, noise=48.0):
    """uint8 images around per-class prototypes + labels (deterministic)."""
    rng = np.random.default_rng(seed)
    protos = rng.integers(0, 256, (num_classes,) + tuple(shape)).astype(np.float32)
    y = rng.integers(0, num_classes, n)
    x = protos[y] + rng.normal(0, noise, (n,) + tuple(shape)).astype(np.float32)
    return np.clip(x, 0, 255).astype(np.uint8), y.astype(np.uint8)
