"""keras_exp functional MNIST MLP: the Keras graph goes through ONNX (keras2onnx conventions) into
FFModel (reference examples/python/keras_exp/func_mnist_mlp.py, there from tf.keras)."""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)

import numpy as np

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.keras.layers import Activation, Dense, Input
from flexflow_amd.keras_exp.models import Model


def top_level_task(num_samples=60000, epochs=1):
    (x_train, y_train), _ = mnist.load_data(num_train=num_samples, num_test=16)
    x_train = x_train.reshape(num_samples, 784).astype("float32") / 255
    y_train = np.reshape(y_train.astype("int32"), (len(y_train), 1))
    input_tensor = Input(shape=(784,))
    output = Dense(512, activation="relu")(input_tensor)
    output = Dense(512, activation="relu")(output)
    output = Dense(10)(output)
    output = Activation("softmax")(output)
    model = Model(inputs={1: input_tensor}, outputs=output)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"], batch_size=64)
    return model.fit(x_train, y_train, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(60000)
    hist = top_level_task(args.samples, epochs=2 if args.test_acc else 1)
    if args.test_acc:
        assert hist.history["accuracy"][-1] >= 90, hist.history
