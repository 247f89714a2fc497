"""Add / subtract merge layers over two towers, compiled and initialised (reference
examples/python/keras/unary.py)."""
import _args  # noqa: F401,I001

import flexflow_amd.keras.optimizers
from flexflow_amd.keras.layers import Add, Dense, Input, subtract
from flexflow_amd.keras.models import Model


def _towers():
    input1 = Input(shape=(16,), dtype="float32")
    input2 = Input(shape=(32,), dtype="float32")
    return input1, input2, Dense(8, activation="relu")(input1), Dense(8, activation="relu")(input2)


def add_test():
    i1, i2, x1, x2 = _towers()
    model = Model([i1, i2], Dense(4)(Add()([x1, x2])))
    model.compile(optimizer=flexflow_amd.keras.optimizers.SGD(learning_rate=0.01),
                  loss="sparse_categorical_crossentropy", metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    model.ffmodel.init_layers()


def subtract_test():
    i1, i2, x1, x2 = _towers()
    model = Model([i1, i2], Dense(4)(subtract([x1, x2])))
    model.compile(optimizer=flexflow_amd.keras.optimizers.SGD(learning_rate=0.01),
                  loss="sparse_categorical_crossentropy", metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    model.ffmodel.init_layers()


if __name__ == "__main__":
    add_test()
    subtract_test()
