"""Gather along axis 1 with torch.gather index semantics (reference examples/python/keras/gather.py)."""
import _args  # noqa: F401,I001  (repo root on sys.path)
import numpy as np

import flexflow_amd.keras.optimizers
from flexflow_amd.keras.backend.internal import gather
from flexflow_amd.keras.layers import Dense, Input, Reshape
from flexflow_amd.keras.models import Model


def get_modified_idx(idx, hidden_shape):
    return idx.reshape(-1, 1).repeat(hidden_shape, 1).astype(np.int32)


def gather_example(samples=300):
    h = 3
    idx = get_modified_idx(np.array([[5, 7, 10], [8, 4, 0]]), h)  # 6, 3
    input0 = Input(shape=(10,), dtype="float32")
    input1 = Input(shape=idx.shape, dtype="int32")
    x0 = Reshape((20, h))(Dense(60, activation="relu")(input0))  # B, 20, 3
    f0 = Reshape((18,))(gather(x0, input1, axis=1))             # B, 6, 3 -> B, 18
    out = Dense(1)(f0)
    model = Model([input0, input1], out)
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.summary()
    return model.fit(x=[np.random.randn(samples, 10).astype(np.float32),
                        idx[None, ...].repeat(samples, 0).astype(np.int32)],
                     y=np.random.randn(samples, 1).astype(np.float32), epochs=2)


if __name__ == "__main__":
    gather_example()
