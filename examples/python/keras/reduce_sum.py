"""keras backend sum over one axis, two axes, and with keepdims (reference
examples/python/keras/reduce_sum.py)."""
import _args  # noqa: F401,I001
import numpy as np

import flexflow_amd.keras.backend as K
import flexflow_amd.keras.optimizers
from flexflow_amd.keras.layers import Dense, Input, Reshape
from flexflow_amd.keras.models import Model


def _run(axis, keepdims, yshape):
    input0 = Input(shape=(32,), dtype="float32")
    nx0 = Reshape((10, 2))(Dense(20, activation="relu")(input0))  # B, 10, 2
    out = K.sum(nx0, axis=axis, keepdims=keepdims)
    model = Model(input0, out)
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.summary()
    model.fit(x=np.random.randn(300, 32).astype(np.float32), y=np.random.randn(300, *yshape).astype(np.float32),
              epochs=2)


def test_reduce_sum1():
    _run(1, False, (2,))       # B, 2


def test_reduce_sum2():
    _run([1, 2], False, ())    # B


def test_reduce_sum3():
    _run([1, 2], True, (1, 1))  # B, 1, 1


if __name__ == "__main__":
    test_reduce_sum1()
    test_reduce_sum2()
    test_reduce_sum3()
