"""Functional CIFAR-10 CNN with three convolution branches over two inputs (the second input
feeds two branches) concatenated on channels, then a second two-branch concat (reference
examples/python/keras/func_cifar10_cnn_concat.py)."""
from _args import parse  # noqa: I001
from _common import cifar

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Concatenate, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras.models import Model


def conv3(filters, name=None):
    return Conv2D(filters=filters, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu", name=name)


def branch(x, tag):
    return conv3(32, f"conv2d_1_{tag}")(conv3(32, f"conv2d_0_{tag}")(x))


def top_level_task(num_samples=10000, epochs=1):
    x, y = cifar(num_samples)
    in1 = Input(shape=(3, 32, 32), dtype="float32", name="input1")
    in2 = Input(shape=(3, 32, 32), dtype="float32", name="input2")
    t = Concatenate(axis=1)([branch(in1, 1), branch(in2, 2), branch(in2, 3)])
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Concatenate(axis=1)([conv3(64, "conv2d_0_4")(t), conv3(64, "conv2d_1_4")(t)])
    t = conv3(64)(t)
    t = Flatten()(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t))
    out = Activation("softmax")(Dense(10)(Dense(512, activation="relu")(t)))
    model = Model([in1, in2], out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit([x, x], y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples)
