"""Maximum / Minimum merge layers (reference examples/python/keras/elementwise_max_min.py)."""
import _args  # noqa: F401,I001
import numpy as np

import flexflow_amd.keras.optimizers
from flexflow_amd.keras.layers import Dense, Input, Maximum, Minimum
from flexflow_amd.keras.models import Model


def _run(layer):
    input0 = Input(shape=(16 * 2,), dtype="float32")
    input1 = Input(shape=(10 * 1,), dtype="float32")
    f0 = layer()([Dense(20, activation="relu")(input0), Dense(20, activation="relu")(input1)])
    model = Model([input0, input1], Dense(1)(f0))
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.fit(x=[np.random.randn(300, 32).astype(np.float32), np.random.randn(300, 10).astype(np.float32)],
              y=np.random.randn(300, 1).astype(np.float32), epochs=2)


def elementwise_max():
    _run(Maximum)


def elementwise_min():
    _run(Minimum)


if __name__ == "__main__":
    elementwise_max()
    elementwise_min()
