"""Functional AlexNet on CIFAR-10 upscaled to 229x229 (reference
examples/python/keras/func_cifar10_alexnet.py; --small: 67x67 and a narrower classifier for CPU tests)."""
from _args import parse  # noqa: I001
import argparse

import numpy as np
from _common import cifar

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras.models import Model


def top_level_task(num_samples=10000, epochs=1, size=229, fc=4096):
    x, y = cifar(num_samples)
    idx = (np.arange(size) * 32 // size).astype(np.int64)
    x = x[:, :, idx][:, :, :, idx]
    inp = Input(shape=(3, size, size), dtype="float32")
    t = Conv2D(filters=64, kernel_size=(11, 11), strides=(4, 4), padding=(2, 2), activation="relu")(inp)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=192, kernel_size=(5, 5), strides=(1, 1), padding=(2, 2), activation="relu")(t)
    t = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=384, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=256, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=256, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Flatten()(MaxPooling2D(pool_size=(3, 3), strides=(2, 2), padding="valid")(t))
    t = Dense(fc, activation="relu")(t)
    t = Dense(fc, activation="relu")(t)
    model = Model(inp, Activation("softmax")(Dense(10)(t)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.001), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--small", action="store_true")
    a2, rest = ap.parse_known_args(rest)
    top_level_task(args.samples, size=67 if a2.small else 229, fc=256 if a2.small else 4096)
