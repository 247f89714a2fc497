"""Export the CIFAR-10 CNN from Keras to cifar10_cnn_keras.onnx (reference
examples/python/onnx/cifar10_cnn_keras.py)."""
import _args  # noqa: F401,I001

from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras.models import Model
from flexflow_amd.keras_exp import export_keras_model


def export(path="cifar10_cnn_keras.onnx", batch=64):
    inp = Input(shape=(3, 32, 32))
    t = Conv2D(32, (3, 3), activation="relu")(inp)
    t = MaxPooling2D((2, 2), (2, 2))(Conv2D(32, (3, 3), activation="relu")(t))
    t = Conv2D(64, (3, 3), activation="relu")(t)
    t = MaxPooling2D((2, 2), (2, 2))(Conv2D(64, (3, 3), activation="relu")(t))
    t = Dense(512, activation="relu")(Flatten()(t))
    out = Activation("softmax")(Dense(10)(t))
    with open(path, "wb") as f:
        f.write(export_keras_model(Model(inp, out), [1], batch))
    return path


if __name__ == "__main__":
    print(export())
