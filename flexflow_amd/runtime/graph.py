"""hipGraph capture of the training step (replaces the reference's Legion tracing,
`begin_trace/end_trace` around forward/backward, examples/cpp/*).

A BERT-Large step is ~1.5k kernel launches; eager Python dispatch would dominate the GPU time.
After three eager warm-up steps (so every buffer of the torch caching allocator exists), the
zero-grad + forward + backward of one step is captured once into a hipGraph and replayed; the
optimizer update (one fused kernel per arena, with host-side bias-corrected scalars) runs after
the replay. Multi-rank steps are captured only on request (FF_GRAPH_COLLECTIVES=1; RCCL supports
stream capture): the activation collectives and the bucketed gradient all-reduces are then part of
the graph, joined back into the captured stream before it ends, and the timing decision below is
agreed over all ranks. By default (FF_GRAPH_COLLECTIVES=0) multi-rank steps run eagerly with the
backward-overlapped bucketed all-reduce; a capture error falls back to eager loudly.

Policy (config.hip_graphs = "auto", the default): the eager warm-up steps are timed; a step whose
GPU work is long (>= config.graph_min_step_ms, e.g. BERT-Large: 55 ms) keeps running eagerly —
measured on MI355X, replaying its ~800-node graph took 58.7 ms/step against 55.1 ms eager (the
graph's per-node dispatch costs more than the host's launch stream, which runs far ahead of the
GPU) — while short steps (DLRM, small CNNs), where host launch latency dominates, are captured.
Steps in between (config.graph_min_step_ms <= eager < config.graph_trial_max_ms, e.g. Inception-v3
with ~1k kernels per step) are captured on trial: two replays are timed and the graph is kept only
if it beats the eager step, else dropped for good.
"""
from __future__ import annotations

import os

import torch


def _collectives_capturable(ex, default: str) -> bool:
    """Multi-rank steps: RCCL collectives can be captured (RCCL supports stream capture); gloo
    (the CPU multi-rank tests) cannot. FF_GRAPH_COLLECTIVES=0 keeps every multi-rank step eager."""
    if not ex.comm.distributed:
        return True
    if os.environ.get("FF_GRAPH_COLLECTIVES", default) != "1":
        return False
    return ex.comm.is_nccl


def capturable(model) -> bool:
    """Whether the model's iteration can be captured into a hipGraph at all (shared by the
    train_step graph below and begin_trace / end_trace, runtime/trace.py). A trace body ends at a
    backward() whose bucket all-reduces are waited for by the later update(): at N > 1 it is
    captured only on request (FF_GRAPH_COLLECTIVES=1); the train_step graph joins them itself."""
    ex = model.executor
    if getattr(ex, "zero", False) or ex.hooks:
        return False
    if not (model.config.hip_graphs and torch.cuda.is_available() and ex.device.type == "cuda"):
        return False
    return _collectives_capturable(ex, "0")


def _agree(ex, value: float, op) -> float:
    """Every rank takes the same graph decision: the timings are reduced over the world (a rank
    capturing while another runs its collectives eagerly would leave the two out of step)."""
    if not ex.comm.distributed:
        return value
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64,
                     device=ex.device if ex.comm.is_nccl else "cpu")
    dist.all_reduce(t, op=op)
    return float(t.item())


class StepGraph:
    def __init__(self, model):
        self.model = model
        self.graph = None
        self.warm = 0
        self.failed = False
        self.eager_ms = []  # timed eager warm-up steps ("auto" policy)
        self.graph_ms = []  # timed replays of a trial capture
        self.trial = 0
        self.decision = None  # True: replay, False: eager, "trial": replay while timing it

    def enabled(self) -> bool:
        m = self.model
        ex = m.executor
        # ZeRO-1: update() leaves async all-gathers of the compute copy in flight and forward waits
        # for them layer by layer from Python; a replayed graph would never run those waits
        if getattr(ex, "zero", False):
            return False
        if not (m.config.hip_graphs and torch.cuda.is_available() and ex.device.type == "cuda"):
            return False
        if self.decision is False:
            return False
        if self.failed or ex.hooks:  # per-op hooks time / inspect individual ops: run eagerly
            return False
        # multi-rank: captured over RCCL only with FF_GRAPH_COLLECTIVES=1 (the bucket all-reduces
        # are then joined inside the graph, see step()); every decision is agreed over all ranks
        return _collectives_capturable(ex, "0")

    def _full_step(self, m, ex) -> bool:
        """Capture the optimizer update too (its overlapped per-bucket launches on the side stream
        included): one process, Adam (its launches read the per-step alpha_t from a device scalar
        that next() refreshes before each replay). Other optimizers and multi-rank steps keep
        update() eager after the replay. Opt-in (FF_GRAPH_UPDATE=1): same-box A/B AlexNet 1.665-1.671
        vs 1.670-1.682 ms, ResNet-50 7.58-7.60 vs 7.60 ms (profiles/graph_update_ab_r5.txt) — the
        eager update after the replay was not exposed enough for the overlap to pay."""
        import torch.distributed as dist
        from ..core.optimizers import AdamOptimizer
        if ex.comm.distributed or getattr(ex.comm, "force", False) or (dist.is_available() and dist.is_initialized()):
            return False  # any process group (a forced world-1 RCCL one included): update() stays eager
        return type(m.optimizer) is AdamOptimizer and os.environ.get("FF_GRAPH_UPDATE", "0") == "1"

    def step(self):
        m = self.model
        ex = m.executor
        ov = bool(getattr(m.config, "overlap_update", False))
        if not self.enabled():
            ex.zero_gradients()
            ex.forward()
            ex.backward(overlap_update=ov)
            ex.update(m.optimizer)
            return
        if self.warm < 3:
            self.warm += 1
            auto = m.config.hip_graphs == "auto"
            # the first step pays autotuning, the second can still pay MIOpen's first-use kernel
            # compiles: time steps 2 and 3 and decide on the faster (AlexNet's step 2 landed on
            # either side of the threshold from box to box: 7.0 vs 13.4 ms steady state)
            if auto and self.warm >= 2:
                torch.cuda.synchronize()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
            ex.zero_gradients()
            ex.forward()
            ex.backward(overlap_update=ov)
            ex.update(m.optimizer)
            if auto and self.warm >= 2:
                en.record()
                en.synchronize()
                import torch.distributed as dist
                ms = _agree(ex, st.elapsed_time(en), dist.ReduceOp.MAX)
                self.eager_ms.append(ms)
                best = min(self.eager_ms)
                if best < float(m.config.graph_min_step_ms):
                    self.decision = True
                elif best < float(getattr(m.config, "graph_trial_max_ms", 30.0)):
                    self.decision = "trial"
                else:
                    self.decision = False
            return
        full = self._full_step(m, ex)
        just_captured = False
        if self.graph is None:
            import torch.distributed as dist
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            err = None
            step_idx = ex.step_idx
            if full:
                m.optimizer.use_device_alpha(ex.device)  # allocated outside the capture
            try:
                with torch.cuda.graph(g):
                    ex.zero_gradients()
                    ex.forward()
                    if full:
                        # the whole step: the overlapped per-bucket update and the rest of update();
                        # next() runs on the host before every replay (alpha_dev), not in the graph
                        ex.backward(overlap_update=ov)
                        ex._opt_next_done = m.optimizer
                        ex.update(m.optimizer)
                    else:
                        ex.backward()
                        if ex.comm.distributed:
                            # every bucket all-reduce is issued and joined back into the captured
                            # stream, so update() after a replay finds final gradients and no handle
                            ex.bucketer.flush()
            except Exception as e:  # noqa: BLE001 - any capture error falls back to eager
                err = e
                ex.step_idx = step_idx
                ex._opt_next_done = None
                ex._overlap_active = False
                ex._upd_done = set()
            # capture success is agreed over the world: a rank replaying its graph while a peer
            # runs eagerly would issue its collectives in a different order
            ok = _agree(ex, 0.0 if err is not None else 1.0, dist.ReduceOp.MIN) > 0.5
            if not ok:
                self.failed = True
                why = err if err is not None else "a peer rank's capture failed"
                print(f"[flexflow_amd] hipGraph capture failed ({why}); running eagerly", flush=True)
                del g
                torch.cuda.synchronize()
                ex.zero_gradients()
                ex.forward()
                ex.backward(overlap_update=ov)
                ex.update(m.optimizer)
                return
            self.graph = g
            just_captured = True
        timed = self.decision == "trial" and self.trial >= 1  # the first replay pays first-use costs
        if timed:
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
        if full:
            m.optimizer.next()  # alpha_t of this step into the device scalar the graph reads
            self.graph.replay()
            if not just_captured:  # the captured update() already counted the capturing step
                ex.step_idx += 1
        else:
            self.graph.replay()
            ex.update(m.optimizer)
        if self.decision == "trial":
            self.trial += 1
            if timed:
                en.record()
                en.synchronize()
                self.graph_ms.append(st.elapsed_time(en))
            if len(self.graph_ms) >= 2:
                import torch.distributed as dist
                keep = _agree(ex, float(min(self.graph_ms) < 0.98 * min(self.eager_ms)), dist.ReduceOp.MIN) > 0.5
                self.decision = keep
                if not keep:
                    self.graph = None  # releases the graph's memory pool


def run_train_step(model):
    sg = model._step_graph
    if sg is None:
        sg = model._step_graph = StepGraph(model)
    sg.step()
