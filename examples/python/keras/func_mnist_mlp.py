"""Functional MNIST MLP (reference examples/python/keras/func_mnist_mlp.py)."""
from _args import parse  # noqa: I001
from _common import mnist_flat
from accuracy import ModelAccuracy

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.callbacks import EpochVerifyMetrics, VerifyMetrics
from flexflow_amd.keras.layers import Activation, Dense, Input
from flexflow_amd.keras.models import Model


def top_level_task(num_samples=60000, epochs=10, verify=False):
    x, y = mnist_flat(num_samples)
    inp = Input(shape=(784,), dtype="float32")
    t = Dense(512, input_shape=(784,), activation="relu")(inp)
    t = Dense(512, activation="relu")(t)
    model = Model(inp, Activation("softmax")(Dense(10)(t)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    cbs = [VerifyMetrics(ModelAccuracy.MNIST_MLP), EpochVerifyMetrics(ModelAccuracy.MNIST_MLP)] if verify else []
    return model.fit(x, y, epochs=epochs, callbacks=cbs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples, verify=args.test_acc)
