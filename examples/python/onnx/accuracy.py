"""Accuracy floors the example tests assert (reference examples/python/native/accuracy.py).

The datasets are the offline synthetic stand-ins of flexflow_amd.keras.datasets (class prototypes +
noise, labels a fixed function of the inputs), so a model that trains reaches these floors quickly."""
from enum import Enum


class ModelAccuracy(Enum):
    MNIST_MLP = 90
    MNIST_CNN = 90
    REUTERS_MLP = 90
    CIFAR10_CNN = 90
    CIFAR10_ALEXNET = 90
