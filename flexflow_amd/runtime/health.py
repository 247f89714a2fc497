"""Failure detection for long training jobs (the reference relies on Legion's runtime checks; an
SPMD job needs its own):

* NonFiniteGuard — `--check-nan N`: every N steps the loss is checked on the device; with
  FF_DEBUG_NAN=1 every op's outputs are checked in the forward pass and the first op producing a
  NaN/Inf is named (the data-dependent debugging mode of the reference's `--profiling` checks).
* Watchdog — `--watchdog SECONDS`: if one training step takes longer (a hung collective, a
  stuck kernel), every thread's Python stack is dumped to stderr (faulthandler) so the hang is
  attributable; torch.distributed's own collective timeout (`--dist-timeout`) then aborts.
* determinism_check — the race detector for kernels and schedules: runs the same step twice from
  the same state and compares every weight bit for bit (our kernels avoid atomics on every
  reduction path that feeds weights, so any difference is a race or an uninitialised read).
"""
from __future__ import annotations

import faulthandler
import os
import sys
from contextlib import contextmanager

import torch


class NonFiniteError(RuntimeError):
    pass


class NonFiniteGuard:
    def __init__(self, executor, every: int = 1, per_op: bool = False):
        self.ex = executor
        self.every = max(1, int(every))
        self.per_op = per_op
        self.steps = 0

    @contextmanager
    def op(self, layer, phase: str):
        yield
        if not self.per_op or phase != "fwd":
            return
        for o in layer.outputs:
            v = self.ex.values.get(o.guid)
            if v is not None and v.is_floating_point() and not bool(torch.isfinite(v).all()):
                raise NonFiniteError(f"non-finite values in the output of {layer.name} ({layer.op_type.name})")

    def after_step(self, loss_sum: torch.Tensor):
        self.steps += 1
        if self.steps % self.every == 0 and loss_sum is not None and not bool(torch.isfinite(loss_sum).all()):
            raise NonFiniteError(f"loss became non-finite at step {self.steps}")


class Watchdog:
    def __init__(self, seconds: float):
        self.seconds = float(seconds)

    def arm(self):
        faulthandler.dump_traceback_later(self.seconds, repeat=False, file=sys.stderr, exit=False)

    def disarm(self):
        faulthandler.cancel_dump_traceback_later()


def _snapshot(ex):
    return [ar.master.detach().clone() for ar in ex.arenas.values() if ar.size]


def determinism_check(model, steps: int = 1) -> bool:
    """Run `steps` training steps twice from the same weights/optimizer state and inputs and compare
    the resulting fp32 master weights bit for bit. Restores the starting state afterwards."""
    ex = model.executor
    opt = model.optimizer
    w0 = _snapshot(ex)
    st0 = {k: tuple(t.clone() for t in v) for k, v in getattr(opt, "state", {}).items()}
    bt = (getattr(opt, "beta1_t", None), getattr(opt, "beta2_t", None))

    def restore():
        for ar, w in zip([a for a in ex.arenas.values() if a.size], w0):
            ar.master.copy_(w)
            if ar.lowp is not None:
                ar.lowp.copy_(w.to(ar.lowp.dtype))
        for k, v in st0.items():
            for dst, src in zip(opt.state[k], v):
                dst.copy_(src)
        if bt[0] is not None:
            opt.beta1_t, opt.beta2_t = bt

    results = []
    for _ in range(2):
        restore()
        for _ in range(steps):
            ex.zero_gradients()
            ex.forward()
            ex.backward()
            ex.update(opt)
        results.append(_snapshot(ex))
    restore()
    return all(torch.equal(a, b) for a, b in zip(*results))
