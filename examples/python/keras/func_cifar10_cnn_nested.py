"""CIFAR-10 CNN assembled from two nested functional models (reference
examples/python/keras/func_cifar10_cnn_nested.py)."""
from _args import parse  # noqa: I001
from _common import cifar

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras.models import Model


def top_level_task(num_samples=10000, epochs=1):
    x, y = cifar(num_samples)
    i1 = Input(shape=(3, 32, 32), dtype="float32")
    t1 = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(i1)
    t1 = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t1)
    model1 = Model(i1, MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t1))
    i2 = Input(shape=(32, 16, 16), dtype="float32")
    t2 = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(i2)
    t2 = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t2)
    t2 = Flatten()(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t2))
    model2 = Model(i2, Activation("softmax")(Dense(10)(Dense(512, activation="relu")(t2))))
    i3 = Input(shape=(3, 32, 32), dtype="float32")
    model = Model(i3, model2(model1(i3)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples)
