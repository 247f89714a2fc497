"""hipGraph capture of the training step (replaces the reference's Legion tracing,
`begin_trace/end_trace` around forward/backward, examples/cpp/*).

A BERT-Large step is ~1.5k kernel launches; eager Python dispatch would dominate the GPU time.
After three eager warm-up steps (so every buffer of the torch caching allocator exists), the
zero-grad + forward + backward of one step is captured once into a hipGraph and replayed; the
optimizer update (one fused kernel per arena, with host-side bias-corrected scalars) and the
bucket all-reduces that belong to it run after the replay. Multi-rank steps with in-step
collectives are captured too when FF_GRAPH_COLLECTIVES=1 (RCCL supports stream capture);
otherwise they run eagerly with backward-overlapped bucketed all-reduce.

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


def capturable(model) -> bool:
    """Whether the model's iteration can be captured into a hipGraph at all (shared by the
    train_step graph below and begin_trace / end_trace, runtime/trace.py)."""
    ex = model.executor
    if getattr(ex, "zero", False) or ex.hooks:
        return False
    if not (model.config.hip_graphs and torch.cuda.is_available() and ex.device.type == "cuda"):
        return False
    if ex.comm.distributed and os.environ.get("FF_GRAPH_COLLECTIVES", "0") != "1":
        return False
    return True


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
        if ex.comm.distributed and os.environ.get("FF_GRAPH_COLLECTIVES", "0") != "1":
            return False
        return True

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
                ms = st.elapsed_time(en)
                self.eager_ms.append(ms)
                best = min(self.eager_ms)
                if best < float(m.config.graph_min_step_ms):
                    self.decision = True
                elif best < float(getattr(m.config, "graph_trial_max_ms", 30.0)):
                    self.decision = "trial"
                else:
                    self.decision = False
            return
        if self.graph is None:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    ex.zero_gradients()
                    ex.forward()
                    ex.backward()
            except Exception as e:  # fall back to eager, loudly
                self.failed = True
                print(f"[flexflow_amd] hipGraph capture failed ({e}); running eagerly", flush=True)
                torch.cuda.synchronize()
                ex.zero_gradients()
                ex.forward()
                ex.backward()
                ex.update(m.optimizer)
                return
            self.graph = g
        timed = self.decision == "trial" and self.trial >= 1  # the first replay pays first-use costs
        if timed:
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
        self.graph.replay()
        ex.update(m.optimizer)
        if self.decision == "trial":
            self.trial += 1
            if timed:
                en.record()
                en.synchronize()
                self.graph_ms.append(st.elapsed_time(en))
            if len(self.graph_ms) >= 2:
                keep = min(self.graph_ms) < 0.98 * min(self.eager_ms)
                self.decision = keep
                if not keep:
                    self.graph = None  # releases the graph's memory pool


def run_train_step(model):
    sg = model._step_graph
    if sg is None:
        sg = model._step_graph = StepGraph(model)
    sg.step()
