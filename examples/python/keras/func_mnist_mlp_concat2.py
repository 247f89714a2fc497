"""MNIST MLP with three towers concatenated twice (reference examples/python/keras/func_mnist_mlp_concat2.py)."""
from _args import parse  # noqa: I001
from _common import mnist_flat

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Dense, Input, concatenate
from flexflow_amd.keras.models import Model


def top_level_task(num_samples=60000, epochs=1):
    x, y = mnist_flat(num_samples)
    inp1, inp2, inp3 = Input(shape=(784,)), Input(shape=(784,)), Input(shape=(784,))
    t1 = Dense(512, activation="relu")(inp1)
    t2 = Dense(512, activation="relu")(inp2)
    t3 = Dense(512, activation="relu")(inp3)
    t = concatenate([t1, t2], axis=1)
    t = Dense(512, activation="relu")(t)
    t = concatenate([t, t3], axis=1)
    model = Model([inp1, inp2, inp3], Activation("softmax")(Dense(10)(Dense(512, activation="relu")(t))))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit([x, x, x], y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples)
