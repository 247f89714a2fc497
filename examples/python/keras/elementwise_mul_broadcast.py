"""Multiply with broadcasting ([B,10,1] x [B,10,2], both operand orders) (reference
examples/python/keras/elementwise_mul_broadcast.py)."""
import _args  # noqa: F401,I001
import numpy as np

import flexflow_amd.keras.optimizers
from flexflow_amd.keras.layers import Dense, Input, Multiply, Reshape
from flexflow_amd.keras.models import Model


def _broadcast(swap):
    input0 = Input(shape=(16 * 2,), dtype="float32")
    input1 = Input(shape=(10 * 1,), dtype="float32")
    nx0 = Reshape((10, 2))(Dense(20, activation="relu")(input0))  # B, 10, 2
    nx1 = Reshape((10, 1))(Dense(10, activation="relu")(input1))  # B, 10, 1
    m0 = Multiply()([nx0, nx1] if swap else [nx1, nx0])           # B, 10, 2
    out = Dense(1)(Reshape((20,))(m0))
    model = Model([input0, input1], out)
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.summary()
    model.fit(x=[np.random.randn(300, 32).astype(np.float32), np.random.randn(300, 10).astype(np.float32)],
              y=np.random.randn(300, 1).astype(np.float32), epochs=2)


def broadcast1():
    _broadcast(False)


def broadcast2():
    _broadcast(True)


if __name__ == "__main__":
    broadcast1()
    broadcast2()
