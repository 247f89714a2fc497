"""MNIST CNN with two convolution branches concatenated (reference
examples/python/keras/func_mnist_cnn_concat.py)."""
from _args import parse  # noqa: I001
from _common import mnist_images

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D, concatenate
from flexflow_amd.keras.models import Model


def top_level_task(num_samples=60000, epochs=1):
    x, y = mnist_images(num_samples)
    inp = Input(shape=(1, 28, 28), dtype="float32")
    t1 = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(inp)
    t2 = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(inp)
    t = concatenate([t1, t2], axis=1)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Dense(128, activation="relu")(Flatten()(t))
    model = Model(inp, Activation("softmax")(Dense(10)(t)))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples)
