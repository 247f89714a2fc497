"""Functional CIFAR-10 CNN with a concat of two convolution branches (reference
examples/python/keras/func_cifar10_cnn.py and func_cifar10_cnn_concat.py)."""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.keras import callbacks, layers, optimizers
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.keras.models import Model


def top_level_task(argv=None, num_samples=50000, epochs=2):
    (x, y), _ = cifar10.load_data(num_samples=num_samples, num_test=16)
    x = x.astype("float32") / 255
    y = y.astype("int32")
    inp = layers.Input(shape=(3, 32, 32), dtype="float32")
    a = layers.Conv2D(32, (3, 3), padding=(1, 1), activation="relu")(inp)
    b = layers.Conv2D(32, (5, 5), padding="same", activation="relu")(inp)
    t = layers.concatenate([a, b], axis=1)
    t = layers.MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = layers.Conv2D(64, (3, 3), padding=(1, 1), activation="relu")(t)
    t = layers.MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = layers.Flatten()(t)
    t = layers.Dense(512, activation="relu")(t)
    out = layers.Activation("softmax")(layers.Dense(10)(t))
    model = Model(inp, out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"], batch_size=64)
    return model.fit(x, y, epochs=epochs, callbacks=[callbacks.EpochVerifyMetrics(ModelAccuracy.CIFAR10_CNN.value)])


if __name__ == "__main__":
    args, rest = parse(50000)
    hist = top_level_task(rest, args.samples)
    if args.test_acc:
        assert hist.history["accuracy"][-1] >= ModelAccuracy.CIFAR10_CNN.value
