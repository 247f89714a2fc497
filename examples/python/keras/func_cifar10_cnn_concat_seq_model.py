"""Two Sequential branch models concatenated through their outputs (reference
examples/python/keras/func_cifar10_cnn_concat_seq_model.py)."""
from _args import parse  # noqa: I001
from _common import cifar

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Concatenate, Conv2D, Dense, Flatten, MaxPooling2D
from flexflow_amd.keras.models import Model, Sequential


def branch(k):
    m = Sequential()
    m.add(Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                 activation="relu", name=f"conv2d_0_{k}"))
    m.add(Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu",
                 name=f"conv2d_1_{k}"))
    return m


def top_level_task(num_samples=10000, epochs=1):
    x, y = cifar(num_samples)
    m1, m2 = branch(0), branch(1)
    t = Concatenate(axis=1)([m1.output, m2.output])
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Flatten()(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t))
    out = Activation("softmax")(Dense(10)(Dense(512, activation="relu")(t)))
    model = Model([m1.input[0], m2.input[0]], out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    model.summary()
    return model.fit([x, x], y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples)
