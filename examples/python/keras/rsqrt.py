"""rsqrt of a tensor sum written with `+` (reference examples/python/keras/rsqrt.py)."""
import _args  # noqa: F401,I001
import numpy as np

import flexflow_amd.keras.optimizers
from flexflow_amd.keras.backend.internal import rsqrt
from flexflow_amd.keras.layers import Dense, Input
from flexflow_amd.keras.models import Model


def test_rsqrt():
    inp1 = Input(shape=(32,), dtype="float32")
    inp2 = Input(shape=(20,), dtype="float32")
    x = Dense(20, activation="relu")(inp1)
    out = rsqrt(x + inp2)
    model = Model([inp1, inp2], out)
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.summary()
    return model.fit(x=[np.random.randn(300, 32).astype(np.float32), np.ones((300, 20)).astype(np.float32)],
                     y=np.random.randn(300, 20).astype(np.float32), epochs=2)


if __name__ == "__main__":
    test_rsqrt()
