"""keras_exp: four nested two-layer towers over two inputs, concatenated (reference
examples/python/keras_exp/func_mnist_mlp_concat.py)."""
from _args import parse  # noqa: I001

import numpy as np

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.keras.layers import Activation, Concatenate, Dense, Input
from flexflow_amd.keras_exp.models import Model


def tower(name):
    i = Input(shape=(784,))
    t = Dense(512, activation="relu", name=f"dense{name}")(i)
    t = Dense(512, activation="relu", name=f"dense{name}{name}")(t)
    return Model(i, t)


def top_level_task(num_samples=60000, epochs=1):
    (x_train, y_train), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x_train = x_train.reshape(num_samples, 784).astype("float32") / 255
    y_train = np.reshape(y_train.astype("int32"), (len(y_train), 1))
    m1, m2, m3, m4 = (tower(k) for k in "1234")
    in1, in2 = Input(shape=(784,)), Input(shape=(784,))
    out = Concatenate(axis=1)([m1(in1), m2(in1), m3(in2), m4(in2)])
    out = Activation("softmax")(Dense(10)(out))
    model = Model({5: in1, 6: in2}, out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"], batch_size=64)
    return model.fit([x_train, x_train], y_train, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples)
