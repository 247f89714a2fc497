"""Per-operator profiling and trace export (reference --profiling: every op's forward/backward task
prints its kernel time, src/ops/*.cc `if (m->profiling)` blocks; Legion Prof timelines).

Enabled by `--profiling` (prints a per-op table) and/or `--trace-dir DIR` (writes a Chrome trace
JSON per rank, loadable in chrome://tracing / Perfetto). On the GPU each op is bracketed by HIP
events on the compute stream, so the numbers are device time, not launch time; the events are read
once per report, never inside the step. HIP-graph capture is bypassed while a profiler is attached
(events inside a captured graph cannot be timed from the host).
"""
from __future__ import annotations

import json
import os
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List

import torch


class OpProfiler:
    def __init__(self, executor, rank: int = 0):
        self.ex = executor
        self.rank = rank
        self.cuda = executor.device.type == "cuda"
        self.records: List[tuple] = []  # (step, layer name, op type, phase, start, end)
        self.comm: List[tuple] = []     # (step, kind, edge, issue mark, wait mark)
        self._issued: Dict[tuple, tuple] = {}
        self.step = 0
        self._t0 = None

    def _mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    @contextmanager
    def op(self, layer, phase: str):
        if self._t0 is None:
            self._t0 = self._mark()
        s = self._mark()
        yield
        e = self._mark()
        self.records.append((self.step, layer.name, layer.op_type.name, phase, s, e))

    def comm_event(self, event, kind, edge):
        """Executor hook: an asynchronous transfer was issued / waited for. Each becomes a span on
        the trace's communication track (tid 2), beside the op spans of the compute stream."""
        if self._t0 is None:
            self._t0 = self._mark()
        if event == "issue":
            self._issued[edge] = (kind, self._mark())
        elif edge in self._issued:
            k, s = self._issued.pop(edge)
            self.comm.append((self.step, k, edge, s, self._mark()))

    def next_step(self):
        self.step += 1

    def _ms(self, a, b):
        if self.cuda:
            return a.elapsed_time(b)
        return (b - a) * 1e3

    def summary(self) -> Dict[str, Dict[str, float]]:
        """{layer: {fwd_ms, bwd_ms, calls}} averaged over the recorded steps."""
        if self.cuda:
            torch.cuda.synchronize()
        acc = defaultdict(lambda: {"fwd_ms": 0.0, "bwd_ms": 0.0, "op": "", "steps": set()})
        for step, name, op, phase, s, e in self.records:
            r = acc[name]
            r[f"{phase}_ms"] += self._ms(s, e)
            r["op"] = op
            r["steps"].add(step)
        out = {}
        for name, r in acc.items():
            n = max(1, len(r["steps"]))
            out[name] = {"op": r["op"], "fwd_ms": r["fwd_ms"] / n, "bwd_ms": r["bwd_ms"] / n}
        return out

    def report(self, top: int = 40) -> str:
        s = self.summary()
        rows = sorted(s.items(), key=lambda kv: -(kv[1]["fwd_ms"] + kv[1]["bwd_ms"]))
        tot_f = sum(r["fwd_ms"] for r in s.values())
        tot_b = sum(r["bwd_ms"] for r in s.values())
        lines = [f"[profile rank {self.rank}] forward {tot_f:.3f} ms  backward {tot_b:.3f} ms per step",
                 f"{'layer':40s} {'op':24s} {'fwd ms':>9s} {'bwd ms':>9s}"]
        for name, r in rows[:top]:
            lines.append(f"{name[:40]:40s} {r['op'][:24]:24s} {r['fwd_ms']:9.4f} {r['bwd_ms']:9.4f}")
        return "\n".join(lines)

    def chrome_trace(self, path: str):
        """Write a Chrome trace (complete 'X' events, microseconds) of the recorded ops."""
        if self.cuda:
            torch.cuda.synchronize()
        ev = []
        for step, name, op, phase, s, e in self.records:
            ts = self._ms(self._t0, s) * 1e3
            dur = self._ms(s, e) * 1e3
            ev.append({"name": f"{name} {phase}", "cat": op, "ph": "X", "ts": ts, "dur": max(dur, 0.001),
                       "pid": self.rank, "tid": 0 if phase == "fwd" else 1, "args": {"step": step}})
        for step, kind, edge, s, e in self.comm:
            ev.append({"name": f"{kind} {'/'.join(str(x) for x in edge)}", "cat": "comm", "ph": "X",
                       "ts": self._ms(self._t0, s) * 1e3, "dur": max(self._ms(s, e) * 1e3, 0.001),
                       "pid": self.rank, "tid": 2, "args": {"step": step, "stream": "process-group"}})
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
        return path
