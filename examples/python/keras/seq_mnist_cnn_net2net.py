"""Sequential MNIST CNN teacher -> student, convolution and dense weights transferred (reference
examples/python/keras/seq_mnist_cnn_net2net.py)."""
from _args import parse  # noqa: I001
from _common import mnist_images
from _net2net import transfer

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, MaxPooling2D
from flexflow_amd.keras.models import Sequential


def cnn():
    c1 = Conv2D(filters=32, input_shape=(1, 28, 28), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                activation="relu")
    c2 = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")
    d1, d2 = Dense(128, activation="relu"), Dense(10)
    m = Sequential([c1, c2, MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"), Flatten(), d1, d2,
                    Activation("softmax")])
    m.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
              metrics=["accuracy", "sparse_categorical_crossentropy"])
    return m, [c1, c2, d1, d2]


def top_level_task(num_samples=60000, epochs=1):
    x, y = mnist_images(num_samples)
    teacher, tl = cnn()
    teacher.fit(x, y, epochs=epochs)
    student, sl = cnn()
    transfer(tl, teacher, sl, student)
    return student.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples)
