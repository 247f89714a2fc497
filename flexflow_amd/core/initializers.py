"""Weight initializers (reference include/flexflow/initializer.h:24-122, src/runtime/initializer.cc,
initializer_kernel.cu with curand).

Values are a pure function of (seed, global element index) — the counter-based generator of
csrc/kernels/init.hip — so a sharded weight is initialised to exactly the slice the unsharded
weight would have, independent of the parallelization chosen by the search.
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K


def _fans(shape):
    """fan_in / fan_out for [out, in, *receptive] weights (Linear: [out, in], Conv: [out, in, kh, kw]).
    Multi-head weights [.., H, d, E] are treated as [H*d (out), E (in)]."""
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[1], shape[0]
    if len(shape) == 4 and shape[0] > 1 and shape[0] != 3:  # conv kernel
        rf = shape[2] * shape[3]
        return shape[1] * rf, shape[0] * rf
    return shape[-1], int(math.prod(shape[:-1]))


class Initializer:
    seed = 0

    def fill_full(self, t: torch.Tensor, shape):
        raise NotImplementedError

    def __call__(self, t, shape):
        self.fill_full(t, shape)


class GlorotUniformInitializer(Initializer):
    def __init__(self, seed=0, fans=None):
        self.seed = seed  # None: the model-local default seed of the weight (Executor.init_weights)
        self.fans = fans  # (fan_in, fan_out) override, e.g. a padded weight's logical shape

    def fill_full(self, t, shape):
        fin, fout = self.fans if self.fans is not None else _fans(shape)
        sc = math.sqrt(6.0 / (fin + fout))
        K.init_uniform(t, -sc, sc, self.seed)


class ZeroInitializer(Initializer):
    def fill_full(self, t, shape):
        K.fill(t, 0.0)


class MaskedTailInitializer(Initializer):
    """Zeros for the first `valid` entries of a 1-D weight and `fill` after them: the bias of an
    output projection padded past its logical width (BERT's MLM decoder, vocab 30522 padded to a
    multiple of 64 so that every GEMM of the vocab projection runs on aligned tiles). A large
    negative fill makes the padded logits vanish under the softmax (probability 0, gradient 0),
    so the loss, accuracy and every real gradient equal the unpadded model's."""

    def __init__(self, valid, fill=-1e9):
        self.valid = int(valid)
        self.fill = float(fill)

    def fill_full(self, t, shape):
        K.fill(t, 0.0)
        if t.numel() > self.valid:
            t.view(-1)[self.valid:].fill_(self.fill)


class ConstantInitializer(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def fill_full(self, t, shape):
        K.fill(t, self.value)


class UniformInitializer(Initializer):
    def __init__(self, seed=0, min_val=0.0, max_val=1.0):
        self.seed, self.min_val, self.max_val = seed, min_val, max_val

    def fill_full(self, t, shape):
        K.init_uniform(t, self.min_val, self.max_val, self.seed)


class NormInitializer(Initializer):
    def __init__(self, seed=0, mean=0.0, stddev=1.0):
        self.seed, self.mean, self.stddev = seed, mean, stddev

    def fill_full(self, t, shape):
        K.init_normal(t, self.mean, self.stddev, self.seed)


def default_initializer(weight_name: str, seed: int) -> Initializer:
    if "bias" in weight_name or weight_name in ("beta",):
        return ZeroInitializer()
    if weight_name in ("gamma", "scale"):
        return ConstantInitializer(1.0)
    return GlorotUniformInitializer(seed)


class BlockInitializer(Initializer):
    """Initializer of a weight that a graph rewrite built by stacking other weights along axis 0
    (pcg/joint.py MergeSiblings). Each row block is filled exactly as its original weight would
    have been (its own initializer, fans and seed), so a rewritten graph starts from the same
    values as the graph the user wrote. `parts` = [(original Parameter, first row, rows)];
    `resolve(param) -> Initializer` supplies the default initializer of an original weight."""

    def __init__(self, parts):
        self.parts = list(parts)
        self.resolve = None

    def fill_full(self, t, shape):
        for w, start, size in self.parts:
            init = self.resolve(w) if self.resolve is not None else w.initializer
            blk = torch.empty(tuple(w.dims), dtype=t.dtype, device=t.device)
            init.fill_full(blk, tuple(w.dims))
            t[start:start + size].copy_(blk)
