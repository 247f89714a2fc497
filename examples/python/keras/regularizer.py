"""L2 kernel regularizer on a Dense layer (reference examples/python/keras/regularizer.py)."""
import _args  # noqa: F401,I001
import numpy as np

import flexflow_amd.keras as keras
import flexflow_amd.keras.optimizers
from flexflow_amd.keras.layers import Dense, Input
from flexflow_amd.keras.models import Model


def regularizer_example():
    input0 = Input(shape=(10,), dtype="float32")
    x0 = Dense(16, activation="relu", kernel_regularizer=keras.regularizers.L2(0.001))(input0)
    model = Model(input0, Dense(1)(x0))
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.001), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    return model.fit(x=np.random.randn(300, 10).astype(np.float32), y=np.random.randn(300, 1).astype(np.float32),
                     epochs=2)


if __name__ == "__main__":
    regularizer_example()
