"""hipGraph capture of the training step (replaces the reference's Legion tracing,
`begin_trace/end_trace` around forward/backward, examples/cpp/*).

A BERT-Large step is ~1.5k kernel launches; eager Python dispatch would dominate the GPU time.
After two eager warm-up steps (so every buffer of the torch caching allocator exists), the
zero-grad + forward + backward of one step is captured once into a hipGraph and replayed; the
optimizer update (one fused kernel per arena, with host-side bias-corrected scalars) and the
bucket all-reduces that belong to it run after the replay. Multi-rank steps with in-step
collectives are captured too when FF_GRAPH_COLLECTIVES=1 (RCCL supports stream capture);
otherwise they run eagerly with backward-overlapped bucketed all-reduce.
"""
from __future__ import annotations

import os

import torch


class StepGraph:
    def __init__(self, model):
        self.model = model
        self.graph = None
        self.warm = 0
        self.failed = False

    def enabled(self) -> bool:
        m = self.model
        ex = m.executor
        if not (m.config.hip_graphs and torch.cuda.is_available() and ex.device.type == "cuda"):
            return False
        if self.failed or ex.hooks:  # per-op hooks time / inspect individual ops: run eagerly
            return False
        if ex.comm.distributed and os.environ.get("FF_GRAPH_COLLECTIVES", "0") != "1":
            return False
        return True

    def step(self):
        m = self.model
        ex = m.executor
        if not self.enabled():
            ex.zero_gradients()
            ex.forward()
            ex.backward()
            ex.update(m.optimizer)
            return
        if self.warm < 2:
            self.warm += 1
            ex.zero_gradients()
            ex.forward()
            ex.backward()
            ex.update(m.optimizer)
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
        self.graph.replay()
        ex.update(m.optimizer)


def run_train_step(model):
    sg = model._step_graph
    if sg is None:
        sg = model._step_graph = StepGraph(model)
    sg.step()
