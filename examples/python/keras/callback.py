"""LearningRateScheduler and accuracy-verifying callbacks on a CIFAR-10 CNN (reference
examples/python/keras/callback.py)."""
from _args import parse  # noqa: I001
from _common import cifar
from accuracy import ModelAccuracy

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.callbacks import EpochVerifyMetrics, LearningRateScheduler, VerifyMetrics
from flexflow_amd.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow_amd.keras.models import Model

SEEN_LR = []


def lr_scheduler(epoch):
    lr = 0.01 if epoch == 0 else 0.02
    SEEN_LR.append(lr)
    return lr


def top_level_task(num_samples=10000, epochs=80, verify=False):
    x, y = cifar(num_samples)
    inp = Input(shape=(3, 32, 32), dtype="float32")
    t = Conv2D(filters=32, input_shape=(3, 32, 32), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
               activation="relu")(inp)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu")(t)
    t = Flatten()(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t))
    model = Model(inp, Activation("softmax")(Dense(10)(Dense(512, activation="relu")(t))))
    model.compile(optimizer=optimizers.SGD(learning_rate=0.02), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    cbs = [LearningRateScheduler(lr_scheduler)]
    if verify:
        cbs += [VerifyMetrics(ModelAccuracy.CIFAR10_CNN), EpochVerifyMetrics(ModelAccuracy.CIFAR10_CNN)]
    hist = model.fit(x, y, epochs=epochs, callbacks=cbs)
    assert SEEN_LR[:2] == [0.01, 0.02][:len(SEEN_LR[:2])]
    return hist


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(args.samples, epochs=2 if not args.test_acc else 80, verify=args.test_acc)
