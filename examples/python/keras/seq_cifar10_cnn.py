"""Sequential CIFAR-10 CNN (reference examples/python/keras/seq_cifar10_cnn.py)."""
from _args import parse  # noqa: I001
from _common import cifar

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, MaxPooling2D
from flexflow_amd.keras.models import Sequential


def top_level_task(num_samples=10000, epochs=1):
    x, y = cifar(num_samples)
    model = Sequential()
    model.add(Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                     activation="relu"))
    model.add(Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu"))
    model.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"))
    model.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu"))
    model.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu"))
    model.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"))
    model.add(Flatten())
    model.add(Dense(512, activation="relu"))
    model.add(Dense(10))
    model.add(Activation("softmax"))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples)
