"""Functional MNIST MLP with two towers joined by concatenate, built as a nested Model
(reference examples/python/keras/func_mnist_mlp_concat.py / func_mnist_mlp_concat2.py)."""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.keras import layers, optimizers
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.keras.models import Model


def top_level_task(argv=None, num_samples=60000, epochs=2):
    (x, y), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x = x.reshape(num_samples, 784).astype("float32") / 255
    y = y.astype("int32").reshape(num_samples, 1)
    inp = layers.Input(shape=(784,))
    a = layers.Dense(256, activation="relu")(inp)
    b = layers.Dense(256, activation="relu")(inp)
    tower = Model(inp, layers.concatenate([a, b], axis=1))
    inp2 = layers.Input(shape=(784,))
    t = layers.Dense(10)(tower(inp2))
    model = Model(inp2, layers.Activation("softmax")(t))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy"], batch_size=64)
    hist = model.fit(x, y, epochs=epochs)
    model.evaluate(x, y)
    return hist


if __name__ == "__main__":
    args, rest = parse(60000)
    hist = top_level_task(rest, args.samples)
    if args.test_acc:
        assert hist.history["accuracy"][-1] >= ModelAccuracy.MNIST_MLP.value
