"""Aux subsystems: per-op profiling + Chrome trace, non-finite detection, watchdog, determinism
(race) check, checkpoint/resume, dot export of the computation / task graph and of rules."""
import json
import os

import numpy as np
import pytest

from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, SGDOptimizer
from flexflow_amd.models import build
from flexflow_amd.runtime.health import NonFiniteError, determinism_check


def _model(flags=(), name="mnist_mlp", opt="adam", batch=8):
    cfg = FFConfig(["--no-hip-graphs"] + list(flags))
    cfg.batch_size = batch
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build(name, ff, batch, small=True)
    ff.optimizer = AdamOptimizer(ff, 1e-3) if opt == "adam" else SGDOptimizer(ff, 0.05)
    ff.compile(loss_type=loss, metrics=mets)
    arrs, lab = make_batch(np.random.default_rng(0))
    for t, a in zip(inputs, arrs):
        t.set_tensor(ff, a)
    ff.label_tensor.set_tensor(ff, lab)
    return ff, inputs


def test_profiler_and_trace(tmp_path):
    ff, _ = _model(["--profiling", "--trace-dir", str(tmp_path)])
    for _ in range(2):
        ff.train_step()
    rep = ff.profile_report()
    assert "forward" in rep and "OP_LINEAR" in rep
    tr = json.load(open(tmp_path / "trace_rank0.json"))
    names = {e["name"] for e in tr["traceEvents"]}
    assert any(n.endswith(" fwd") for n in names) and any(n.endswith(" bwd") for n in names)


def test_nonfinite_guard_names_the_op(monkeypatch):
    monkeypatch.setenv("FF_DEBUG_NAN", "1")
    ff, inputs = _model(["--check-nan", "1"])
    x = np.zeros(tuple(inputs[0].dims), np.float32)
    x[0, 0] = np.nan
    inputs[0].set_tensor(ff, x)
    with pytest.raises(NonFiniteError, match="output of"):
        ff.train_step()


def test_watchdog_arms_and_disarms():
    ff, _ = _model(["--watchdog", "30"])
    ff.train_step()
    assert ff.watchdog is not None


def test_determinism_check():
    ff, _ = _model()
    ff.train_step()
    assert determinism_check(ff, steps=2)


def test_checkpoint_resume_matches_uninterrupted(tmp_path):
    ff, _ = _model(opt="adam")
    for _ in range(2):
        ff.train_step()
    ff.save_checkpoint(str(tmp_path / "ck"))
    for _ in range(2):
        ff.train_step()
    w_ref = [np.asarray(w.get_weights(ff)).copy() for L in ff.layers for w in L.weights]
    ff2, _ = _model(opt="adam")
    step = ff2.load_checkpoint(str(tmp_path / "ck"))
    assert step == 2
    for _ in range(2):
        ff2.train_step()
    w2 = [np.asarray(w.get_weights(ff2)).copy() for L in ff2.layers for w in L.weights]
    for a, b in zip(w_ref, w2):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    meta = json.load(open(tmp_path / "ck" / "meta.json"))
    assert meta["step"] == 2 and "strategy" in meta


def test_dot_exports(tmp_path):
    cg, tg = tmp_path / "cg.dot", tmp_path / "tg.dot"
    ff, _ = _model(["--compgraph", str(cg), "--taskgraph", str(tg), "--include-costs-dot-graph"])
    t = cg.read_text()
    assert t.startswith('digraph') and "LINEAR" in t and "->" in t
    assert "fwd" in tg.read_text()
    from flexflow_amd import _core
    from flexflow_amd.pcg.substitutions import BUILTIN
    from flexflow_amd.utils.dot import rule_to_dot
    r = _core.load_rules(BUILTIN)[0]
    assert "digraph" in open(rule_to_dot(r, str(tmp_path / "r.dot"))).read()


def test_inplace_plan_same_results(monkeypatch):
    """In-place element-wise ops (add -> relu in ResNet blocks) change memory, not math."""
    def run():
        ff, _ = _model(name="resnet50", batch=1, opt="sgd")
        ff.train_step()
        ff.train_step()
        return ff, [np.asarray(w.get_weights(ff)).copy() for L in ff.layers for w in L.weights]
    ff1, w1 = run()
    n = sum(1 for L in ff1.layers if ff1.executor.ctx.get(L.name) is not None
            and ff1.executor.ctx[L.name].extra.get("inplace"))
    assert n >= 10
    monkeypatch.setenv("FF_NO_INPLACE", "1")
    _, w2 = run()
    for a, b in zip(w1, w2):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_launcher_argv():
    from flexflow_amd.run import build_argv
    a = build_argv(["-ll:gpu", "4", "train.py", "--epochs", "2"])
    assert a[:2] == ["--nproc-per-node", "4"] and "127.0.0.1" in a and a[-3:] == ["train.py", "--epochs", "2"]
    b = build_argv(["--nproc=2", "--master-addr", "10.0.0.1", "x.py"])
    assert "127.0.0.1" not in b and b[-1] == "x.py"


def test_checkpoint_from_training_loads_into_inference_model(tmp_path):
    """Arena order differs between a training and an inference compile (accumulated gradients
    first); the loader maps every weight by (layer position, slot), not by flat arena offset."""
    ff, _ = _model(opt="adam")
    ff.train_step()
    ff.save_checkpoint(str(tmp_path / "ck"))
    w_ref = [np.asarray(w.get_weights(ff)).copy() for L in ff.layers for w in L.weights]
    cfg = FFConfig(["--no-hip-graphs"])
    cfg.batch_size = 8
    ff2 = FFModel(cfg)
    build("mnist_mlp", ff2, 8, small=True)
    ff2.optimizer = AdamOptimizer(ff2, 1e-3)
    from flexflow_amd.type import CompMode
    ff2.compile(comp_mode=CompMode.INFERENCE)
    assert not ff2.executor.training
    ff2.load_checkpoint(str(tmp_path / "ck"), strict=False)
    w2 = [np.asarray(w.get_weights(ff2)).copy() for L in ff2.layers for w in L.weights]
    assert len(w_ref) == len(w2)
    for a, b in zip(w_ref, w2):
        np.testing.assert_array_equal(a, b)


def test_checkpoint_rejects_mismatched_shapes(tmp_path):
    ff, _ = _model(opt="adam")
    ff.save_checkpoint(str(tmp_path / "ck"))
    ff2, _ = _model(name="mlp_unify", opt="adam")
    with pytest.raises(ValueError):
        ff2.load_checkpoint(str(tmp_path / "ck"), strict=False)


def test_update_with_other_optimizer_runs_its_next():
    """backward(overlap_update) ran next() for the model's optimizer; an update() with another
    optimizer object must still advance that optimizer's own Adam step."""
    ff, _ = _model(opt="adam")
    other = AdamOptimizer(ff, 1e-3)
    ff.executor.init_optimizer(other)
    ff.executor.zero_gradients()
    ff.executor.forward()
    ff.executor.backward(overlap_update=True)
    t0 = other.beta1_t
    ff.executor.update(other)
    assert other.beta1_t != t0


def test_model_repository_rejects_path_escape(tmp_path):
    from flexflow_amd.serving.repository import ModelRepository
    root = tmp_path / "repo"
    root.mkdir()
    (tmp_path / "evil").mkdir()
    (tmp_path / "evil" / "config.pbtxt").write_text('name: "evil"')
    repo = ModelRepository(str(root))
    for name in ("../evil", "..", str(tmp_path / "evil")):
        with pytest.raises(KeyError):
            repo.load(name)


def test_checkpoint_without_entry_layout_loads_when_arenas_match(tmp_path):
    """Shards written before the per-entry arena layout existed still load when the arena sizes
    match this job's and strict=True checked world size and strategy; otherwise
    they are rejected."""
    from safetensors.torch import load_file, save_file
    ff, _ = _model(opt="adam")
    ff.train_step()
    ck = tmp_path / "ck"
    ff.save_checkpoint(str(ck))
    fn = str(ck / "rank0.safetensors")
    save_file(load_file(fn), fn)  # drop the metadata: the old format
    w_ref = [np.asarray(w.get_weights(ff)).copy() for L in ff.layers for w in L.weights]
    ff2, _ = _model(opt="adam")
    with pytest.raises(ValueError):  # equal sizes alone do not prove equal contents
        ff2.load_checkpoint(str(ck), strict=False)
    assert ff2.load_checkpoint(str(ck)) == 1
    w2 = [np.asarray(w.get_weights(ff2)).copy() for L in ff2.layers for w in L.weights]
    for a, b in zip(w_ref, w2):
        np.testing.assert_array_equal(a, b)
    ff3, _ = _model(name="mlp_unify", opt="adam")
    with pytest.raises(ValueError):
        ff3.load_checkpoint(str(ck), strict=False)
