"""keras_exp (reference python/flexflow/keras_exp): Keras graph -> ONNX in keras2onnx conventions
-> ONNXModelKeras -> FFModel. The exported file holds MatMul+Add pairs that the importer fuses into
dense layers with bias, and the compiled model's forward equals a numpy evaluation of the ONNX
graph with its own initializers."""
import numpy as np

from flexflow_amd.keras import optimizers
from flexflow_amd.keras.layers import Activation, Concatenate, Dense, Input
from flexflow_amd.keras_exp.models import Model, Sequential
from flexflow_amd.onnx.proto import load_model
from flexflow_amd.type import OperatorType


def test_keras_exp_mlp_matches_onnx_numpy():
    inp = Input(shape=(12,))
    t = Dense(16, activation="relu")(inp)
    t = Dense(5)(t)
    out = Activation("softmax")(t)
    model = Model(inputs={1: inp}, outputs=out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.0), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy"], batch_size=8)
    g = load_model(model.onnx_model).graph
    ops = [n.op_type for n in g.node]
    assert ops == ["MatMul", "Add", "Relu", "MatMul", "Add", "Softmax"], ops
    assert [vi.name for vi in g.input] == ["input_1"]
    ff = model.ffmodel
    dense = [L for L in ff.layers if L.op_type == OperatorType.OP_LINEAR]
    assert len(dense) == 2 and all(len(L.weights) == 2 for L in dense)  # MatMul+Add fused, bias kept
    inits = {t.name: t.array for t in g.initializer}
    mm = [n for n in g.node if n.op_type == "MatMul"]
    ad = [n for n in g.node if n.op_type == "Add"]
    x = np.random.default_rng(0).standard_normal((8, 12)).astype(np.float32)
    h = np.maximum(x @ inits[mm[0].input[1]] + inits[ad[0].input[1]], 0)
    z = h @ inits[mm[1].input[1]] + inits[ad[1].input[1]]
    ref = np.exp(z - z.max(1, keepdims=True))
    ref /= ref.sum(1, keepdims=True)
    got = model.predict(x, batch_size=8)
    np.testing.assert_allclose(np.asarray(got).reshape(ref.shape), ref, rtol=1e-4, atol=1e-5)


def test_keras_exp_nested_concat_and_sequential_train():
    rng = np.random.default_rng(1)
    i1 = Input(shape=(6,))
    tower = Model(i1, Dense(8, activation="relu")(i1))
    a, b = Input(shape=(6,)), Input(shape=(6,))
    out = Activation("softmax")(Dense(3)(Concatenate(axis=1)([tower(a), tower(b)])))
    model = Model({5: a, 6: b}, out)
    model.compile(optimizer=optimizers.SGD(learning_rate=0.05), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy"], batch_size=16)
    g = load_model(model.onnx_model).graph
    assert [vi.name for vi in g.input] == ["input_5", "input_6"]
    assert sum(n.op_type == "Concat" for n in g.node) == 1
    x = rng.standard_normal((64, 6)).astype(np.float32)
    y = (x[:, :1] > 0).astype(np.int32) + (x[:, 1:2] > 0).astype(np.int32)
    hist = model.fit([x, x], y, epochs=3)
    assert np.isfinite(hist.history["loss"][-1])
    seq = Sequential([Dense(8, activation="relu", input_shape=(6,)), Dense(3), Activation("softmax")])
    seq.compile(optimizer=optimizers.SGD(learning_rate=0.05), loss="sparse_categorical_crossentropy",
                metrics=["accuracy"], batch_size=16)
    seq.fit(x, y, epochs=1)
    assert [n.op_type for n in load_model(seq.onnx_model).graph.node][:2] == ["MatMul", "Add"]
