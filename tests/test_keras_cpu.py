"""flexflow_amd.keras frontend (reference python/flexflow/keras + examples/python/keras/*):
Sequential / functional / nested models, merge layers, callbacks, regularizers, datasets."""
import numpy as np
import pytest

from flexflow_amd.keras import backend as K
from flexflow_amd.keras import callbacks, layers, losses, metrics, optimizers, regularizers
from flexflow_amd.keras.datasets import cifar10, mnist, reuters
from flexflow_amd.keras.models import Model, Sequential
from flexflow_amd.keras.preprocessing.text import Tokenizer
from flexflow_amd.keras.utils import to_categorical


def _mnist(n=1024, flat=True):
    (x, y), _ = mnist.load_data(num_train=n, num_test=16)
    x = x.astype("float32") / 255
    x = x.reshape(n, 784) if flat else x.reshape(n, 1, 28, 28)
    return x, y.astype("int32").reshape(n, 1)


def test_seq_mnist_mlp_learns():
    x, y = _mnist()
    model = Sequential([layers.Dense(128, input_shape=(784,), activation="relu"),
                        layers.Dense(10), layers.Activation("softmax")])
    model.compile(optimizer=optimizers.SGD(learning_rate=0.05), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"], batch_size=64)
    assert "dense" in model.summary()
    hist = model.fit(x, y, epochs=3, verbose=0, callbacks=[callbacks.VerifyMetrics(50.0)])
    assert hist.history["accuracy"][-1] > 50.0
    p = model.predict(x[:128])
    assert p.shape == (128, 10) and np.allclose(p.sum(1), 1.0, atol=1e-3)
    logs = model.evaluate(x, y, verbose=0)
    assert logs["accuracy"] > 50.0


def test_functional_cnn_concat_nested():
    x, y = _mnist(256, flat=False)
    inp = layers.Input(shape=(1, 28, 28), dtype="float32")
    a = layers.Conv2D(8, (3, 3), padding=(1, 1), activation="relu")(inp)
    b = layers.Conv2D(8, (5, 5), padding="same", activation="relu")(inp)
    t = layers.concatenate([a, b], axis=1)
    t = layers.MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    inner = Model(inp, layers.Flatten()(t))
    inp2 = layers.Input(shape=(1, 28, 28), dtype="float32")
    h = inner(inp2)  # nested model used as a layer
    h = layers.Dense(32, activation="relu", kernel_regularizer=regularizers.L2(1e-4))(h)
    h = layers.Dropout(0.1)(h)
    out = layers.Activation("softmax")(layers.Dense(10)(h))
    model = Model(inp2, out)
    model.compile(optimizer=optimizers.Adam(learning_rate=0.002), loss=losses.SparseCategoricalCrossentropy(),
                  metrics=[metrics.Accuracy()], batch_size=32)
    sched = callbacks.LearningRateScheduler(lambda ep: 0.002 * (0.5 ** ep))
    stop = callbacks.EpochVerifyMetrics(0.0)  # reached immediately -> stops after one epoch
    hist = model.fit(x, y, epochs=4, verbose=0, callbacks=[sched, stop])
    assert len(hist.epoch) == 1
    assert np.isfinite(hist.history["loss"][0])
    assert len(model.get_layer(index=0).get_weights()) >= 1


def test_merge_layers_and_backend():
    n = 128
    rng = np.random.default_rng(0)
    x1 = rng.standard_normal((n, 16)).astype("float32")
    x2 = rng.standard_normal((n, 16)).astype("float32")
    yv = (x1 * x2).sum(1, keepdims=True).astype("float32")
    i1 = layers.Input(shape=(16,))
    i2 = layers.Input(shape=(16,))
    m = layers.multiply([i1, i2])
    s = layers.add([layers.subtract([m, i1]), i1])
    s = layers.maximum([s, layers.minimum([s, m])])
    e = K.exp(K.sin(s) * 0 if False else K.cos(s))
    r = K.sum(e, axis=1, keepdims=True)
    out = layers.Dense(1)(layers.concatenate([r, s], axis=1))
    model = Model([i1, i2], out)
    model.compile(optimizer="sgd", loss="mean_squared_error", metrics=["mean_squared_error"], batch_size=32)
    hist = model.fit([x1, x2], yv, epochs=2, verbose=0)
    assert np.isfinite(hist.history["loss"]).all()


def test_reuters_mlp_and_utils():
    (xtr, ytr), _ = reuters.load_data(num_words=256, n=512)
    tok = Tokenizer(num_words=256)
    x = tok.sequences_to_matrix(xtr, mode="binary")
    y = ytr.astype("int32").reshape(-1, 1)
    oh = to_categorical(ytr, 46)
    assert oh.shape == (len(ytr), 46) and oh.sum() == len(ytr)
    model = Sequential()
    model.add(layers.Input(shape=(256,)))
    model.add(layers.Dense(64, activation="relu"))
    model.add(layers.Dense(46, activation="softmax"))
    model.compile(optimizer=optimizers.SGD(0.1), loss="sparse_categorical_crossentropy", metrics=["accuracy"],
                  batch_size=32)
    hist = model.fit(x, y, epochs=3, verbose=0)
    assert hist.history["accuracy"][-1] > hist.history["accuracy"][0] or hist.history["accuracy"][-1] > 20


def test_cifar_shapes_and_errors():
    (x, y), (xt, yt) = cifar10.load_data(num_samples=64, num_test=8)
    assert x.shape == (64, 3, 32, 32) and y.shape == (64, 1) and x.dtype == np.uint8
    with pytest.raises(ValueError):
        Sequential([layers.Dense(4)])  # first layer without input shape


def test_keras_shared_layer_and_submodel_reuse():
    """A layer (or nested model) called on two inputs lowers to two FFModel ops that SHARE weights
    (Keras semantics, FFModel shared_op), with unique op names; training runs through both uses."""
    import numpy as np
    from flexflow_amd.keras import optimizers
    from flexflow_amd.keras.layers import Concatenate, Dense, Input
    from flexflow_amd.keras.models import Model
    from flexflow_amd.type import OperatorType
    sub_in = Input(shape=(6,))
    enc = Model(sub_in, Dense(4, activation="relu", name="enc_dense")(sub_in))
    a, b = Input(shape=(6,)), Input(shape=(6,))
    out = Dense(1, name="head")(Concatenate(axis=1)([enc(a), enc(b)]))
    model = Model([a, b], out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.01), loss="mean_squared_error",
                  metrics=["mean_squared_error"], batch_size=8)
    lin = [L for L in model.ffmodel.layers if L.op_type == OperatorType.OP_LINEAR and L.name.startswith("enc_dense")]
    assert len(lin) == 2 and len({L.name for L in lin}) == 2
    assert [w.guid for w in lin[0].weights] == [w.guid for w in lin[1].weights]
    x = np.random.default_rng(0).standard_normal((32, 6)).astype(np.float32)
    hist = model.fit([x, x[::-1].copy()], x[:, :1].copy(), epochs=2)
    assert np.isfinite(hist.history["loss"][-1])
