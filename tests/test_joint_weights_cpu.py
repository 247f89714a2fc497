"""Graph rewrites keep the user's weights (pcg/joint.py MergeSiblings).

Two sibling Linears reading one tensor are stacked into one Linear by merge_siblings_linear. The
rewritten graph must start from exactly the values the graph as written starts from: each row block
keeps its own initializer, fans and seed, values set on the original Parameters before compile land
in their block, and get/set on an original Parameter after compile address its block.
"""
import json
import os
import tempfile

import numpy as np

B = 4


def _build(ff):
    from flexflow_amd.core import ActiMode, DataType
    from flexflow_amd.core.initializers import UniformInitializer, ZeroInitializer
    x = ff.create_tensor([B, 12], DataType.DT_FLOAT, name="x")
    a = ff.dense(x, 8, ActiMode.AC_MODE_RELU, name="da", kernel_initializer=UniformInitializer(5, -0.3, 0.3),
                 bias_initializer=ZeroInitializer())
    b = ff.dense(x, 6, ActiMode.AC_MODE_RELU, name="db", bias_initializer=ZeroInitializer())
    t = ff.concat([a, b], 1, name="cat")
    ff.dense(t, 5, name="head")
    return x, a, b


def _run(rewrites=None, set_before=None, set_after=None):
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    flags = ["--no-hip-graphs"]
    if rewrites is not None:
        fd, path = tempfile.mkstemp(suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(rewrites, f)
        flags += ["--import-rewrites", path]
    cfg = FFConfig(flags)
    cfg.batch_size = B
    ff = FFModel(cfg)
    x, a, b = _build(ff)
    la = ff.get_layer_by_name("da")
    lb = ff.get_layer_by_name("db")
    if set_before is not None:
        la.weights[0].set_weights(ff, set_before)
    ff.optimizer = SGDOptimizer(ff, 0.0)
    ff.compile()
    if set_after is not None:
        lb.weights[0].set_weights(ff, set_after)
    x.set_tensor(ff, np.random.default_rng(0).standard_normal((B, 12)).astype(np.float32))
    ff.forward()
    out = np.asarray(ff._get_tensor_value(ff.output_tensor()), dtype=np.float32)
    return ff, la, lb, out


def _merge_match():
    from flexflow_amd.core import FFConfig, FFModel
    from flexflow_amd.pcg.joint import MergeSiblings
    from flexflow_amd.type import OperatorType
    cfg = FFConfig([])
    cfg.batch_size = B
    ff = FFModel(cfg)
    _build(ff)
    m = MergeSiblings(OperatorType.OP_LINEAR).matches(ff)
    assert len(m) == 1, m
    return [["merge_siblings_linear", list(m[0])]]


def test_merged_siblings_initialise_like_the_written_graph():
    rw = _merge_match()
    ff0, la0, lb0, out0 = _run()
    ff1, la1, lb1, out1 = _run(rw)
    assert any("&" in L.name for L in ff1.layers), [L.name for L in ff1.layers]
    np.testing.assert_allclose(out1, out0, rtol=1e-5, atol=1e-6)
    for L0, L1 in ((la0, la1), (lb0, lb1)):
        for w0, w1 in zip(L0.weights, L1.weights):
            np.testing.assert_array_equal(w1.get_weights(ff1), w0.get_weights(ff0))


def test_merged_siblings_keep_values_set_before_and_after_compile():
    rw = _merge_match()
    rng = np.random.default_rng(7)
    ka = rng.standard_normal((8, 12)).astype(np.float32)
    kb = rng.standard_normal((6, 12)).astype(np.float32)
    ff0, la0, lb0, out0 = _run(set_before=ka, set_after=kb)
    ff1, la1, lb1, out1 = _run(rw, set_before=ka, set_after=kb)
    np.testing.assert_allclose(la1.weights[0].get_weights(ff1), ka, rtol=0, atol=0)
    np.testing.assert_allclose(lb1.weights[0].get_weights(ff1), kb, rtol=0, atol=0)
    np.testing.assert_allclose(out1, out0, rtol=1e-5, atol=1e-6)
