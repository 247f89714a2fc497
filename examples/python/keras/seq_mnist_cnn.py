"""Sequential MNIST CNN (reference examples/python/keras/seq_mnist_cnn.py)."""
from _args import parse  # noqa: I001
from _common import mnist_images

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, MaxPooling2D
from flexflow_amd.keras.models import Sequential


def build():
    model = Sequential()
    model.add(Conv2D(filters=32, input_shape=(1, 28, 28), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                     activation="relu"))
    model.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu"))
    model.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"))
    model.add(Flatten())
    model.add(Dense(128, activation="relu"))
    model.add(Dense(10))
    model.add(Activation("softmax"))
    return model


def top_level_task(num_samples=60000, epochs=1):
    x, y = mnist_images(num_samples)
    model = build()
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples)
