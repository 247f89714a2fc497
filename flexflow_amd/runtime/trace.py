"""FFConfig.begin_trace / end_trace as hipGraphs (reference: Legion tracing of the iteration body,
`ffconfig.begin_trace(111) ... ffconfig.end_trace(111)` in examples/cpp/* and
python/flexflow/core/flexflow_cffi.py begin_trace/end_trace).

Between begin_trace(id) and end_trace(id) the FFModel calls forward / zero_gradients / backward
are recorded by name. Once two consecutive iterations of a trace id made the same sequence, the
third captures that sequence (up to the first update(), whose bias-corrected scalars are host
values) into one hipGraph; from then on the first recorded call of an iteration replays the whole
graph and the following recorded calls return at once. update(), and any call that departs from
the recorded sequence, runs eagerly. A trace whose iterations do not repeat, or a model that
cannot be captured (CPU, ZeRO, per-op hooks, multi-rank without FF_GRAPH_COLLECTIVES=1), runs
eagerly throughout — the reference's semantics: tracing only ever changes how an iteration is
issued, not what it computes.
"""
from __future__ import annotations

import torch

TRACED = ("forward", "zero_gradients", "backward")


class _Trace:
    def __init__(self, model):
        self.model = model
        self.iters = 0
        self.prev = None   # call sequence of the previous iteration
        self.cur = []      # call sequence of this iteration (recording)
        self.seq = None    # captured prefix
        self.graph = None
        self.pos = 0       # replay: next recorded call of this iteration
        self.off = False


def _state(model):
    cfg = model.config
    tid = getattr(cfg, "_trace_active", None)
    if tid is None:
        return None
    st = cfg._trace_state.get(tid)
    if st is None:
        st = cfg._trace_state[tid] = _Trace(model)
    if st.model is not model:  # one trace id drives one model
        st.off = True
    return st


def traced_call(model, name: str, run) -> None:
    """Runs `run()` (the eager body of FFModel.<name>) or its share of the trace's graph."""
    st = _state(model)
    if st is None or st.off:
        run()
        return
    if st.graph is None:
        st.cur.append(name)
        if st.iters >= 2 and st.seq and len(st.cur) == 1 and name == st.seq[0]:
            from .graph import capturable
            if capturable(model):
                g = torch.cuda.CUDAGraph()
                try:
                    torch.cuda.synchronize()
                    with torch.cuda.graph(g):
                        for n in st.seq:
                            getattr(model, "_eager_" + n)()
                except Exception as e:  # fall back to eager, loudly
                    st.off = True
                    print(f"[flexflow_amd] trace capture failed ({e}); running eagerly", flush=True)
                    torch.cuda.synchronize()
                    run()
                    return
                st.graph = g
                g.replay()
                st.pos = 1
                return
            st.off = True
        run()
        return
    if st.pos == 0 and name == st.seq[0]:
        st.graph.replay()
        st.pos = 1
        return
    if 0 < st.pos < len(st.seq) and name == st.seq[st.pos]:
        st.pos += 1  # already issued by this iteration's replay
        return
    run()


def note_update(model) -> None:
    st = _state(model)
    if st is not None and not st.off:
        if st.graph is None:
            st.cur.append("update")
        else:
            st.pos = len(st.seq)  # recorded calls after an update run eagerly


def begin(cfg, trace_id) -> None:
    cfg._trace_active = trace_id
    st = cfg._trace_state.get(trace_id)
    if st is not None:
        st.cur, st.pos = [], 0


def end(cfg, trace_id) -> None:
    st = cfg._trace_state.get(trace_id)
    cfg._trace_active = None
    if st is None:
        return
    st.iters += 1
    if st.graph is None and not st.off:
        if st.prev is not None and st.prev != st.cur:
            st.off = True  # the iteration body changes: no stable sequence to capture
        pre = []
        for n in st.cur:
            if n == "update":
                break
            pre.append(n)
        st.seq = pre if pre else None
        st.prev, st.cur = st.cur, []
    elif st.graph is not None and 0 < st.pos < len(st.seq):
        # an iteration ended before issuing all of its recorded calls after the replay
        st.off = True
        st.graph = None
