"""Sequential MNIST MLP teacher -> student (reference examples/python/keras/seq_mnist_mlp_net2net.py)."""
from _args import parse  # noqa: I001
from _common import mnist_flat
from _net2net import transfer

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Dense
from flexflow_amd.keras.models import Sequential


def mlp():
    ds = [Dense(512, input_shape=(784,), activation="relu"), Dense(512, activation="relu"), Dense(10)]
    m = Sequential(ds + [Activation("softmax")])
    m.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
              metrics=["accuracy", "sparse_categorical_crossentropy"])
    return m, ds


def top_level_task(num_samples=60000, epochs=2):
    x, y = mnist_flat(num_samples)
    teacher, td = mlp()
    teacher.fit(x, y, epochs=epochs)
    student, sd = mlp()
    transfer(td, teacher, sd, student)
    return student.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    top_level_task(args.samples)
