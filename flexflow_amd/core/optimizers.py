"""SGD and Adam (reference include/flexflow/optimizer.h:15-120, src/runtime/optimizer.cc:23-610,
optimizer_kernel.cu).

The reference launches one update task per weight (with a NCCL all-reduce inside each). Here
every weight shard of a replica group lives in one flat fp32 arena, so an update is ONE fused HIP
kernel per arena (multi-tensor apply) that also refreshes the bf16 compute copy.
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K


class Optimizer:
    def __init__(self, ffmodel=None, lr=0.01):
        self.lr = lr
        self.ffmodel = ffmodel
        self.state = {}

    def set_learning_rate(self, learning_rate):
        self.lr = learning_rate

    def init_state(self, arena):
        pass

    def next(self):
        pass

    def step(self, arena):
        raise NotImplementedError

    def step_range(self, arena, lo, hi, max_blocks=0):
        """Update elements [lo, hi) of the arena only (sharded optimizer: this rank's chunk; the
        overlapped update: one gradient bucket, launched with at most max_blocks workgroups)."""
        raise NotImplementedError


class SGDOptimizer(Optimizer):
    def __init__(self, ffmodel=None, lr=0.01, momentum=0.0, nesterov=False, weight_decay=0.0):
        super().__init__(ffmodel, lr)
        self.momentum = momentum
        self.nesterov = nesterov
        self.weight_decay = weight_decay

    def init_state(self, arena):
        if self.momentum > 0:
            self.state[id(arena)] = torch.zeros_like(arena.master)

    def step(self, arena):
        K.sgd_update(arena.master, arena.grad, self.state.get(id(arena)), arena.lowp, self.lr, self.momentum,
                     self.nesterov, self.weight_decay)

    def step_range(self, arena, lo, hi, max_blocks=0):
        mom = self.state.get(id(arena))
        K.sgd_update(arena.master[lo:hi], arena.grad[lo:hi], mom[lo:hi] if mom is not None else None,
                     arena.lowp[lo:hi] if arena.lowp is not None else None, self.lr, self.momentum, self.nesterov,
                     self.weight_decay, max_blocks=max_blocks)


class AdamOptimizer(Optimizer):
    def __init__(self, ffmodel=None, alpha=0.001, beta1=0.9, beta2=0.999, weight_decay=0.0, epsilon=1e-8):
        super().__init__(ffmodel, alpha)
        self.alpha = alpha
        self.beta1, self.beta2 = beta1, beta2
        self.weight_decay = weight_decay
        self.epsilon = epsilon
        self.beta1_t = 1.0
        self.beta2_t = 1.0
        self.alpha_t = alpha
        # device copy of alpha_t, set up by a captured whole-step hipGraph (runtime/graph.py): the
        # replayed Adam launches read the step size from it, next() refreshes it before each step
        self.alpha_dev = None

    def use_device_alpha(self, device):
        if self.alpha_dev is None:
            self.alpha_dev = torch.full((1,), float(self.alpha_t), device=device, dtype=torch.float32)

    def set_learning_rate(self, learning_rate):
        self.alpha = learning_rate
        self.lr = learning_rate

    def init_state(self, arena):
        self.state[id(arena)] = (torch.zeros_like(arena.master), torch.zeros_like(arena.master))

    def next(self):
        # reference optimizer.cc:371-376
        self.beta1_t *= self.beta1
        self.beta2_t *= self.beta2
        self.alpha_t = self.alpha * math.sqrt(1 - self.beta2_t) / (1 - self.beta1_t)
        if self.alpha_dev is not None:
            self.alpha_dev.fill_(self.alpha_t)

    def step(self, arena):
        m, v = self.state[id(arena)]
        K.adam_update(arena.master, arena.grad, m, v, arena.lowp, self.alpha_t, self.beta1, self.beta2,
                      self.weight_decay, self.epsilon, alpha_dev=self.alpha_dev)

    def step_range(self, arena, lo, hi, max_blocks=0):
        m, v = self.state[id(arena)]
        K.adam_update(arena.master[lo:hi], arena.grad[lo:hi], m[lo:hi], v[lo:hi],
                      arena.lowp[lo:hi] if arena.lowp is not None else None, self.alpha_t, self.beta1, self.beta2,
                      self.weight_decay, self.epsilon, max_blocks=max_blocks, alpha_dev=self.alpha_dev)
