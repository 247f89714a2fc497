"""Export the MNIST MLP from Keras to mnist_mlp_keras.onnx (reference
examples/python/onnx/mnist_mlp_keras.py: tf.keras + keras2onnx; here our keras2onnx-convention exporter)."""
import _args  # noqa: F401,I001

from flexflow_amd.keras.layers import Activation, Dense, Input
from flexflow_amd.keras.models import Model
from flexflow_amd.keras_exp import export_keras_model


def export(path="mnist_mlp_keras.onnx", batch=64):
    inp = Input(shape=(784,))
    t = Dense(512, activation="relu")(inp)
    t = Dense(512, activation="relu")(t)
    out = Activation("softmax")(Dense(10)(t))
    with open(path, "wb") as f:
        f.write(export_keras_model(Model(inp, out), [1], batch))
    return path


if __name__ == "__main__":
    print(export())
