"""Sequential MNIST MLP through flexflow_amd.keras (reference examples/python/keras/seq_mnist_mlp.py).

    python examples/python/keras/seq_mnist_mlp.py [-b 64] [--samples N] [-a]
"""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.keras import callbacks, layers, optimizers
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.keras.models import Sequential


def top_level_task(argv=None, num_samples=60000, epochs=2):
    (x, y), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x = x.reshape(num_samples, 784).astype("float32") / 255
    y = y.astype("int32").reshape(num_samples, 1)
    model = Sequential([layers.Dense(512, input_shape=(784,), activation="relu"),
                        layers.Dense(512, activation="relu"),
                        layers.Dense(10),
                        layers.Activation("softmax")])
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"], batch_size=64)
    print(model.summary())
    return model.fit(x, y, epochs=epochs, callbacks=[callbacks.VerifyMetrics(ModelAccuracy.MNIST_MLP.value)])


if __name__ == "__main__":
    args, rest = parse(60000)
    hist = top_level_task(rest, args.samples)
    if args.test_acc:
        assert hist.history["accuracy"][-1] >= ModelAccuracy.MNIST_MLP.value
