"""keras_exp CIFAR-10 CNN through ONNX (reference examples/python/keras_exp/func_cifar10_cnn.py)."""
from _args import parse  # noqa: I001

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras_exp.models import Model


def top_level_task(num_samples=10000, epochs=1):
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x_train = x_train[:num_samples].astype("float32") / 255
    y_train = y_train[:num_samples].astype("int32")
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding="valid",
               activation="relu")(inp)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Activation("softmax")(Dense(10)(t))
    model = Model({1: inp}, t)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"], batch_size=64)
    return model.fit(x_train, y_train, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples)
