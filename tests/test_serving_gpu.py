"""The inference server on the GPU: the reference Triton QA models and a dynamically batched
Gemm+Relu model served from cuda:0 (fp32, and bf16 compute with --dtype bf16)."""
import os
import shutil
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = "/root/reference/triton/qa/L0_e2e/models"


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_serve_on_gpu(tmp_path, dtype):
    import torch
    from flexflow_amd.serving import InferenceServer, InferenceServerClient
    from test_serving_cpu import _gemm_model, _infer
    assert torch.cuda.is_available()
    w, b = _gemm_model(tmp_path, 8, 100000)
    if os.path.isdir(REPO):
        shutil.copytree(os.path.join(REPO, "add"), tmp_path / "add")
    srv = InferenceServer(str(tmp_path), port=0, ff_flags=["--dtype", dtype]).start()
    try:
        m = srv.repo.get("mlp")
        assert m.ff.executor.device.type == "cuda"
        cl = InferenceServerClient(srv.url)
        xs = [np.random.default_rng(i).standard_normal((2, 4)).astype(np.float32) for i in range(4)]
        res = [None] * 4
        th = [threading.Thread(target=lambda i=i: res.__setitem__(i, _infer(cl, "mlp", {"x": xs[i]}, out="y")))
              for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        tol = 1e-4 if dtype == "fp32" else 5e-2
        for x, r in zip(xs, res):
            np.testing.assert_allclose(r, np.maximum(x @ w.T + b, 0), rtol=tol, atol=tol)
        if os.path.isdir(REPO):
            a = np.arange(8, dtype=np.float32).reshape(4, 2)
            np.testing.assert_allclose(_infer(cl, "add", {"input0": a, "input1": a}), a + a)
    finally:
        srv.stop()
