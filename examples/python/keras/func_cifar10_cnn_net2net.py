"""Functional CIFAR-10 CNN teacher -> student (reference examples/python/keras/func_cifar10_cnn_net2net.py)."""
from _args import parse  # noqa: I001
from _common import cifar
from _net2net import transfer

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras.models import Model


def cnn():
    convs = [Conv2D(filters=f, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")
             for f in (32, 32, 64, 64)]
    dense = [Dense(512, activation="relu"), Dense(10)]
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(convs[1](convs[0](inp)))
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(convs[3](convs[2](t)))
    t = dense[1](dense[0](Flatten()(t)))
    m = Model(inp, Activation("softmax")(t))
    m.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
              metrics=["accuracy", "sparse_categorical_crossentropy"])
    return m, convs + dense


def top_level_task(num_samples=10000, epochs=1):
    x, y = cifar(num_samples)
    teacher, tl = cnn()
    teacher.fit(x, y, epochs=epochs)
    student, sl = cnn()
    transfer(tl, teacher, sl, student)
    return student.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples)
