"""Inference server (flexflow_amd/serving) against the reference Triton backend's QA model
repository (triton/qa/L0_e2e/models: config.pbtxt + 1/model.onnx + 1/model.strategy, read as data)
with the checks of its end-to-end test (triton/qa/L0_e2e/operator_test.py: same inputs, same
expected outputs), through our client over HTTP, JSON and binary tensors. Plus the native dynamic
batcher, a max_batch_size model built here, and the text strategy loader."""
import os
import shutil
import threading

import numpy as np
import pytest

from flexflow_amd.serving import InferenceServer, InferenceServerClient, InferInput, InferRequestedOutput
from flexflow_amd.serving.client import InferenceServerException
from flexflow_amd.serving.config import ModelConfig

REPO = "/root/reference/triton/qa/L0_e2e/models"
pytestmark = pytest.mark.skipif(not os.path.isdir(REPO), reason="reference Triton QA models not mounted")


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    root = tmp_path_factory.mktemp("repo")
    for m in os.listdir(REPO):  # a private copy (the reference tree is read-only data)
        shutil.copytree(os.path.join(REPO, m), root / m)
    srv = InferenceServer(str(root), port=0, ff_flags=["--device", "cpu", "--no-hip-graphs"]).start()
    yield srv
    srv.stop()


@pytest.fixture
def client(server):
    return InferenceServerClient(server.url)


def _infer(client, model, feeds, out="output", binary=True):
    ins = []
    for name, a in feeds.items():
        i = InferInput(name, list(a.shape), "FP32")
        i.set_data_from_numpy(a, binary_data=binary)
        ins.append(i)
    r = client.infer(model_name=model, inputs=ins, outputs=[InferRequestedOutput(out, binary_data=binary)])
    return r.as_numpy(out)


def softmax(x, axis):
    e = np.exp(x - np.max(x, axis, keepdims=True))
    return e / np.sum(e, axis, keepdims=True)


def test_health_and_index(client, server):
    assert client.is_server_live() and client.is_server_ready()
    idx = {e["name"]: e for e in client.get_model_repository_index()}
    assert set(idx) == set(os.listdir(REPO))
    not_ready = {n: e for n, e in idx.items() if e["state"] != "READY"}
    assert not not_ready, not_ready
    md = client.get_model_metadata("add")
    assert [i["name"] for i in md["inputs"]] == ["input0", "input1"] and md["outputs"][0]["shape"] == [4, 2]
    assert client.is_model_ready("add") and not client.is_model_ready("nope")


@pytest.mark.parametrize("binary", [True, False])
def test_operator_models(client, binary):
    """The reference QA's per-operator checks (operator_test.py), one request each."""
    a = np.arange(8, dtype=np.float32).reshape(4, 2)
    np.testing.assert_array_equal(_infer(client, "add", {"input0": a, "input1": a}, binary=binary), a + a)
    np.testing.assert_array_equal(_infer(client, "mul", {"input0": a, "input1": a}, binary=binary), a * a)
    ones = np.ones((4, 2), np.float32)
    np.testing.assert_array_equal(_infer(client, "sub", {"input0": ones, "input1": a}, binary=binary), ones - a)
    ident = np.arange(100, dtype=np.float32).reshape(4, 1, 5, 5)
    np.testing.assert_array_equal(_infer(client, "identity", {"input": ident}, binary=binary), ident)
    t = np.arange(3, dtype=np.float32).reshape(3, 1)
    np.testing.assert_allclose(_infer(client, "tanh", {"input": t}, binary=binary), np.tanh(t), rtol=1e-6)
    np.testing.assert_allclose(_infer(client, "sqrt", {"input": t}, binary=binary), np.sqrt(t), rtol=1e-6)
    r = np.linspace(0, .1, 3, dtype=np.float32).reshape(1, 3)  # the QA test's input (1/0 = inf included)
    with np.errstate(divide="ignore"):
        np.testing.assert_array_equal(_infer(client, "reciprocal", {"input": r}, binary=binary), np.reciprocal(r))
    c = _infer(client, "cast", {"input": r}, binary=binary)
    assert c.dtype == np.float64 and np.array_equal(c, r.astype(np.float64))
    s = np.arange(3, dtype=np.float32).reshape(3, 1)
    # softmax: axis 0 (model "softmax", opset default of its file) and axis 1 ("softmax1") per the QA test
    np.testing.assert_allclose(_infer(client, "softmax", {"input": s}, binary=binary), softmax(s, 0), rtol=1e-5)
    np.testing.assert_allclose(_infer(client, "softmax1", {"input": s}, binary=binary), softmax(s, 1), rtol=1e-5)


def test_bad_requests_are_400(client):
    a = np.zeros((3, 2), np.float32)  # wrong shape for "add" ([4, 2])
    with pytest.raises(InferenceServerException) as e:
        _infer(client, "add", {"input0": a, "input1": a})
    assert e.value.status == 400
    with pytest.raises(InferenceServerException) as e:
        _infer(client, "add", {"input0": np.zeros((4, 2), np.float32)})  # missing input1
    assert e.value.status == 400
    with pytest.raises(InferenceServerException) as e:
        _infer(client, "no_such_model", {"input": a})
    assert e.value.status == 404
    # the model keeps serving after bad requests
    x = np.ones((4, 2), np.float32)
    np.testing.assert_array_equal(_infer(client, "add", {"input0": x, "input1": x}), 2 * x)


def test_unload_load(client):
    client.unload_model("tanh")
    assert not client.is_model_ready("tanh")
    client.load_model("tanh")
    assert client.is_model_ready("tanh")


def _gemm_model(root, mbs, delay_us):
    """A Gemm+Relu ONNX model with a batch dim and dynamic batching, serialized by our own ONNX
    writer (flexflow_amd/onnx/proto.py make_model_bytes; the onnx package is not installed)."""
    from flexflow_amd.onnx.proto import make_model_bytes
    rng = np.random.default_rng(0)
    w = rng.standard_normal((6, 4)).astype(np.float32)
    b = rng.standard_normal(6).astype(np.float32)
    d = root / "mlp"
    (d / "1").mkdir(parents=True)
    (d / "1" / "model.onnx").write_bytes(make_model_bytes(
        nodes=[("Gemm", ["x", "w", "b"], ["h"], {"transB": 1}), ("Relu", ["h"], ["y"], {})],
        inputs={"x": [mbs, 4]}, outputs={"y": [mbs, 6]}, initializers={"w": w, "b": b}))
    (d / "config.pbtxt").write_text(
        f'name: "mlp"\nmax_batch_size: {mbs}\ninput [{{ name: "x" data_type: TYPE_FP32 dims: [ 4 ] }}]\n'
        f'output [{{ name: "y" data_type: TYPE_FP32 dims: [ 6 ] }}]\n'
        f'dynamic_batching {{ preferred_batch_size: [ {mbs} ] max_queue_delay_microseconds: {delay_us} }}\n')
    return w, b


def test_dynamic_batching(tmp_path):
    w, b = _gemm_model(tmp_path, 8, 200000)
    srv = InferenceServer(str(tmp_path), port=0, ff_flags=["--device", "cpu", "--no-hip-graphs"]).start()
    try:
        cl = InferenceServerClient(srv.url)
        xs = [np.random.default_rng(i).standard_normal((2, 4)).astype(np.float32) for i in range(4)]
        res = [None] * 4

        def go(i):
            res[i] = _infer(cl, "mlp", {"x": xs[i]}, out="y")
        th = [threading.Thread(target=go, args=(i,)) for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for x, r in zip(xs, res):
            np.testing.assert_allclose(r, np.maximum(x @ w.T + b, 0), rtol=1e-5, atol=1e-5)
        st = cl.get_inference_statistics("mlp")["model_stats"][0]
        assert st["inference_count"] == 4
        # 4 requests x 2 rows reach the preferred size 8: fewer executions than requests
        assert st["batcher"]["requests"] == 4 and st["batcher"]["batches"] < 4, st
    finally:
        srv.stop()


def test_request_queue_policy():
    from flexflow_amd import _core
    q = _core.RequestQueue(8, 10_000_000, [4])
    assert q.push(1, 2) and q.push(2, 2)
    assert q.pop(0) == [1, 2]              # preferred size 4 reached: no waiting
    assert q.push(3, 3) and q.push(4, 6)
    assert q.pop(0) == [3]                 # 3 + 6 > 8: full, never split a request
    assert not q.push(5, 9)                # larger than max_rows
    q.close()
    assert q.pop(0) == [4]                 # closed: drain what is queued
    assert q.pop(-1) == []
    assert q.stats() == [3, 4, 13]


def test_pbtxt_and_text_strategy(tmp_path):
    from flexflow_amd.core import FFConfig, FFModel
    from flexflow_amd.pcg.strategy import load_strategy_text
    from flexflow_amd.type import DataType
    c = ModelConfig.parse(open(os.path.join(REPO, "identity", "config.pbtxt")).read())
    assert c.name == "identity" and c.inputs[0].dims == [4, 1, 5, 5] and c.instance_kind == "KIND_MODEL"
    ff = FFModel(FFConfig(["--device", "cpu"]))
    x = ff.create_tensor([4, 8], DataType.DT_FLOAT)
    ff.dense(x, 6, name="Gemm_0")
    p = tmp_path / "m.strategy"
    p.write_text("1\nGemm_0 0 2 2 1 2 0 1\n")  # batch split 2 ways over devices 0, 1
    st = load_strategy_text(str(p), ff.layers, 2)
    assert st["Gemm_0"].degrees[0] == 2 and st["Gemm_0"].devices == (0, 1)
