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
