"""CANDLE Uno drug-response regression in the Keras API (reference
examples/python/keras/candle_uno/candle_uno.py + uno_default_model.txt): per-feature-type encoder
submodels (dense 1000x3 on cell RNA-seq and drug descriptor / fingerprint inputs), concatenated with
the dose inputs, then dense 1000x5 and a scalar output, MSE loss. The reference loads the CANDLE
dataset (downloaded); offline, synthetic features of the same shapes stand in."""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import _args  # noqa: F401,E402,I001  (repo root on sys.path)
import numpy as np  # noqa: E402

from flexflow_amd.keras import optimizers  # noqa: E402
from flexflow_amd.keras.layers import Concatenate, Dense, Dropout, Input  # noqa: E402
from flexflow_amd.keras.models import Model  # noqa: E402

FEATURE_SHAPES = {"dose": (1,), "cell.rnaseq": (942,), "drug.descriptors": (5270,), "drug.fingerprints": (2048,)}
INPUT_FEATURES = {"dose1": "dose", "dose2": "dose", "cell.rnaseq": "cell.rnaseq",
                  "drug1.descriptors": "drug.descriptors", "drug1.fingerprints": "drug.fingerprints",
                  "drug2.descriptors": "drug.descriptors", "drug2.fingerprints": "drug.fingerprints"}


def build_feature_model(input_shape, name="", dense_layers=(1000, 1000, 1000), activation="relu", dropout_rate=0.0):
    x_input = Input(shape=input_shape)
    h = x_input
    for layer in dense_layers:
        h = Dense(layer, activation=activation)(h)
        if dropout_rate > 0:
            h = Dropout(dropout_rate)(h)
    return Model(x_input, h, name=name)


def build_model(dense_feature_layers, dense, dropout_rate=0.0):
    encoders = {t: build_feature_model(s, t, dense_feature_layers, dropout_rate=dropout_rate)
                for t, s in FEATURE_SHAPES.items() if t.split(".")[0] in ("cell", "drug")}
    inputs, encoded = [], []
    for fea_name, fea_type in INPUT_FEATURES.items():
        inp = Input(FEATURE_SHAPES[fea_type], name="input." + fea_name)
        inputs.append(inp)
        encoded.append(encoders[fea_type](inp) if fea_type in encoders else inp)
    h = Concatenate(axis=1)(encoded)
    for layer in dense:
        h = Dense(layer, activation="relu")(h)
        if dropout_rate > 0:
            h = Dropout(dropout_rate)(h)
    return Model(inputs, Dense(1)(h))


def top_level_task(num_samples=1024, epochs=1, small=False):
    fl, dl = ((64, 64, 64), (64,) * 5) if small else ((1000, 1000, 1000), (1000,) * 5)
    model = build_model(fl, dl)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="mean_squared_error",
                  metrics=["mean_squared_error"])
    model.summary()
    rng = np.random.default_rng(0)
    xs = [rng.standard_normal((num_samples,) + FEATURE_SHAPES[t]).astype(np.float32) for t in INPUT_FEATURES.values()]
    y = (xs[0] * 0.5 - xs[1] * 0.25 + 0.1 * xs[2][:, :1]).astype(np.float32)
    return model.fit(xs, y, epochs=epochs)


if __name__ == "__main__":
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--small", action="store_true")
    a, rest = ap.parse_known_args(sys.argv[1:])
    top_level_task(a.samples, small=a.small)
