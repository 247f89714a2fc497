"""Bootcamp Keras CNN: Sequential conv / pool / dense / dropout network on CIFAR-10 (synthetic
stand-in data) with `fit(batch_size=64)` (reference bootcamp_demo/keras_cnn_cifar10.py).

    python examples/python/bootcamp_demo/keras_cnn_cifar10.py [--samples N] [--epochs E]
"""
import argparse
import sys

import _path  # noqa: F401,I001
from _common import cifar

from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Dropout, Flatten, MaxPooling2D
from flexflow_amd.keras.models import Sequential
from flexflow_amd.keras.optimizers import SGD


def top_level_task(num_samples=10000, epochs=4):
    x, y = cifar(num_samples)
    model = Sequential()
    model.add(Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding="valid",
                     activation="relu"))
    model.add(Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu"))
    model.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"))
    model.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu"))
    model.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding="valid"))
    model.add(Activation("relu"))
    model.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"))
    model.add(Flatten())
    model.add(Dense(512))
    model.add(Activation("relu"))
    model.add(Dropout(0.5))
    model.add(Dense(10))
    model.add(Activation("softmax"))
    model.compile(optimizer=SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit(x, y, batch_size=64, epochs=epochs)


if __name__ == "__main__":
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--epochs", type=int, default=4)
    a, _ = ap.parse_known_args(sys.argv[1:])
    print("Sequential API, cifar10 cnn")
    top_level_task(a.samples, a.epochs)
