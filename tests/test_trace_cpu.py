"""begin_trace / end_trace bookkeeping on the host (runtime/trace.py): sequences are recorded,
an iteration body that changes turns the trace off, and on CPU every call runs eagerly with the
same results as an untraced loop."""
import numpy as np

from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
from flexflow_amd.models import build


def _model():
    cfg = FFConfig(["--device", "cpu"])
    cfg.batch_size = 16
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build("dlrm", ff, 16, small=True)
    ff.optimizer = SGDOptimizer(ff, 0.05)
    ff.compile(loss_type=loss, metrics=mets)
    return cfg, ff, inputs, make_batch


def _loop(trace, body):
    cfg, ff, inputs, make_batch = _model()
    rng = np.random.default_rng(0)
    for it in range(4):
        arrs, lab = make_batch(rng)
        for t, a in zip(inputs, arrs):
            t.set_tensor(ff, a)
        ff.label_tensor.set_tensor(ff, lab)
        if trace:
            cfg.begin_trace(7)
        body(ff, it)
        if trace:
            cfg.end_trace(7)
    return cfg, [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]


def _std(ff, it):
    ff.forward()
    ff.zero_gradients()
    ff.backward()
    ff.update()


def test_trace_runs_eagerly_on_cpu_with_same_results():
    cfg, a = _loop(True, _std)
    st = cfg._trace_state[7]
    assert st.graph is None and st.off  # nothing to capture on the host
    _, b = _loop(False, _std)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-6)


def test_trace_records_sequence_and_detects_changes(monkeypatch):
    import flexflow_amd.runtime.graph as g
    monkeypatch.setattr(g, "capturable", lambda m: False)

    def changing(ff, it):
        ff.forward()
        if it != 1:
            ff.zero_gradients()
        ff.backward()
        ff.update()

    cfg, _ = _loop(True, changing)
    st = cfg._trace_state[7]
    assert st.off and st.iters == 4 and st.graph is None


def test_trace_policy_and_replay_bookkeeping():
    """The trace graph follows the train_step graph's timing policy, and a replay does the host
    bookkeeping its eager calls would have done (backward count for the sparse-SGD guard)."""
    from types import SimpleNamespace

    from flexflow_amd.runtime import trace as T
    cfg = SimpleNamespace(hip_graphs="auto", graph_min_step_ms=12.0, graph_trial_max_ms=30.0)
    ex = SimpleNamespace(_bwd_since_update=0)
    st = T._Trace(SimpleNamespace(config=cfg, executor=ex))
    st.seq = ["zero_gradients", "forward", "backward"]
    T._replay_bookkeeping(st)
    T._replay_bookkeeping(st)
    assert ex._bwd_since_update == 2
    if T._timing_wanted(st):  # device: the eager timings decide
        st.eager_ms = [5.0]
        assert T._decide(st) is True
        st.eager_ms = [20.0]
        assert T._decide(st) == "trial"
        st.eager_ms = [50.0]
        assert T._decide(st) is False
    else:  # CPU never captures: nothing to time, the default is to capture when capturable
        assert T._decide(st) is True
