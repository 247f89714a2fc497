"""'identity' loss over a reduced output (reference examples/python/keras/identity_loss.py)."""
import _args  # noqa: F401,I001
import numpy as np

import flexflow_amd.keras.backend as K
import flexflow_amd.keras.optimizers
from flexflow_amd.keras.layers import Dense, Input
from flexflow_amd.keras.models import Model


def test_identity_loss():
    input0 = Input(shape=(32,), dtype="float32")
    out = K.sum(Dense(20, activation="relu")(input0), axis=1)  # B
    model = Model(input0, out)
    model.compile(optimizer=flexflow_amd.keras.optimizers.Adam(learning_rate=0.01), loss="identity",
                  metrics=["mean_absolute_error"])
    model.summary()
    return model.fit(x=np.random.randn(300, 32).astype(np.float32), y=np.zeros((300)).astype(np.float32), epochs=2)


if __name__ == "__main__":
    test_identity_loss()
