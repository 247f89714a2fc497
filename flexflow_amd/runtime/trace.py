"""FFConfig.begin_trace / end_trace as hipGraphs (reference: Legion tracing of the iteration body,
`ffconfig.begin_trace(111) ... ffconfig.end_trace(111)` in examples/cpp/* and
python/flexflow/core/flexflow_cffi.py begin_trace/end_trace).

Between begin_trace(id) and end_trace(id) the FFModel calls forward / zero_gradients / backward
are recorded by name. Once two consecutive iterations of a trace id made the same sequence, the
third captures that sequence (up to the first update(), whose bias-corrected scalars are host
values) into one hipGraph; from then on the first recorded call of an iteration replays the whole
graph and the following recorded calls return at once. update(), and any call that departs from
the recorded sequence, runs eagerly. A trace whose iterations do not repeat, or a model that
cannot be captured (CPU, ZeRO, per-op hooks, more than one backward per update, a row-sparse SGD
plan), runs eagerly throughout — the reference's semantics: tracing only ever changes how an
iteration is issued, not what it computes. The eager iterations 2 and 3 are timed and the
train_step graph's policy applies (runtime/graph.py): long bodies stay eager, mid-length ones are
captured on trial and kept only when two timed replays beat the eager time.
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
        # the train_step graph's timing policy (runtime/graph.py): eager iterations are timed, a
        # long body stays eager, a mid-length one is captured on trial and kept only if faster
        self.ev = None       # (start event) of the iteration being timed
        self.eager_ms = []
        self.graph_ms = []
        self.decision = None  # True: keep the graph, "trial": replaying while timing it
        self.replays = 0


def _timing_wanted(st) -> bool:
    return torch.cuda.is_available() and st.model.config.hip_graphs == "auto"


def _start_timer(st):
    torch.cuda.synchronize()
    st.ev = torch.cuda.Event(enable_timing=True)
    st.ev.record()


def _stop_timer(st):
    if st.ev is None:
        return None
    en = torch.cuda.Event(enable_timing=True)
    en.record()
    en.synchronize()
    ms = st.ev.elapsed_time(en)
    st.ev = None
    return ms


def _decide(st):
    """True / "trial" / False from the timed eager iterations (graph.StepGraph's thresholds)."""
    if not _timing_wanted(st) or not st.eager_ms:
        return True
    cfg = st.model.config
    best = min(st.eager_ms)
    if best < float(cfg.graph_min_step_ms):
        return True
    if best < float(getattr(cfg, "graph_trial_max_ms", 30.0)):
        return "trial"
    return False


def _replay_bookkeeping(st):
    """Host-side state the replayed calls would have updated eagerly."""
    ex = st.model.executor
    ex._bwd_since_update += sum(1 for n in st.seq if n == "backward")


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
        if len(st.cur) == 1 and st.iters in (1, 2) and _timing_wanted(st):
            _start_timer(st)  # eager iterations 2 and 3 are timed (the first pays autotuning)
        # capture in iteration 4 (iters == 3): eager iterations 2 and 3 have both been timed
        if st.iters >= 3 and st.seq and len(st.cur) == 1 and name == st.seq[0]:
            import torch.distributed as dist

            from .graph import _agree, capturable
            ex = model.executor
            decision = _decide(st)
            # one graph per update: the row-sparse SGD plan and several backward passes per update
            # depend on host bookkeeping a replay would skip
            if (capturable(model) and decision is not False and st.seq.count("backward") <= 1
                    and not ex._sparse_plan(model.optimizer)):
                st.ev = None
                g = torch.cuda.CUDAGraph()
                err = None
                try:
                    torch.cuda.synchronize()
                    with torch.cuda.graph(g):
                        for n in st.seq:
                            getattr(model, "_eager_" + n)()
                except Exception as e:  # noqa: BLE001 - fall back to eager, loudly
                    err = e
                # every rank replays or none does (graph.StepGraph agrees the same way)
                if _agree(ex, 0.0 if err is not None else 1.0, dist.ReduceOp.MIN) < 0.5:
                    st.off = True
                    why = err if err is not None else "a peer rank's capture failed"
                    print(f"[flexflow_amd] trace capture failed ({why}); running eagerly", flush=True)
                    torch.cuda.synchronize()
                    run()
                    return
                st.graph = g
                st.decision = decision
                g.replay()
                _replay_bookkeeping(st)
                st.replays = 1
                st.pos = 1
                return
            st.ev = None
            st.off = True
        run()
        return
    if st.pos == 0 and name == st.seq[0]:
        if st.decision == "trial" and st.replays >= 1:
            _start_timer(st)  # the first replay pays first-use costs
        st.graph.replay()
        _replay_bookkeeping(st)
        st.replays += 1
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
    ms = _stop_timer(st)
    if ms is not None:
        # every rank takes the same decision: the world's slowest timing counts
        import torch.distributed as dist

        from .graph import _agree
        ms = _agree(st.model.executor, ms, dist.ReduceOp.MAX)
    if st.graph is not None and st.decision == "trial" and ms is not None:
        st.graph_ms.append(ms)
        if len(st.graph_ms) >= 2:
            import torch.distributed as dist

            from .graph import _agree
            keep = float(min(st.graph_ms) < 0.98 * min(st.eager_ms))
            if _agree(st.model.executor, keep, dist.ReduceOp.MIN) > 0.5:
                st.decision = True
            else:  # replay is not faster: eager for good (releases the graph's pool)
                st.graph, st.off = None, True
                return
    elif st.graph is None and ms is not None:
        st.eager_ms.append(ms)
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
