"""Explicit parallel ops (reference src/parallel_ops/{partition,combine,replicate,reduction,
fused_parallel_op}.cc + allreduce).

In the reference these are PCG nodes whose task bodies are local copies while Legion moves the
data implicitly between region partitions. Here the data movement is the runtime's Transfer
(RCCL collective or batched P2P) between the producer's and the consumer's layouts, so a parallel
op is an identity whose *output layout is pinned*:

  Repartition(dim, degree)  output partitioned `degree` ways along `dim`
  Combine(dim)              output gathered along `dim` (degree 1), replicated on all devices
  Replicate(degree)         output replicated on `degree` devices
  Reduction / AllReduce     output = the sum of a partial-sum input, replicated (all-reduce) or,
                            for Reduction(dim, degree), reduce-scattered along `dim`
  FusedParallel(ops)        the composition of the above: the last op's layout

A user inserts them to force a layout (FFModel.repartition/combine/replicate/reduction/allreduce)
and the search keeps them fixed (pinned_config) while it chooses everything around them.
"""
from __future__ import annotations

from ..pcg.strategy import OpConfig
from ..type import OperatorType
from .base import OpImpl, register


class _ParallelOp(OpImpl):
    def forward(self, ctx, xs, ws):
        return [xs[0]]

    def backward(self, ctx, douts):
        return [douts[0]]

    def flops(self, *a):
        return 0.0

    def pinned_config(self, num_devices: int) -> OpConfig:
        raise NotImplementedError

    def _cfg(self, degrees, ndev):
        return OpConfig(tuple(degrees), tuple(range(ndev)))


def _dims(self):
    return len(self.layer.outputs[0].dims)


@register(OperatorType.OP_REPARTITION)
class Repartition(_ParallelOp):
    op_type = OperatorType.OP_REPARTITION

    def pinned_config(self, num_devices):
        n = _dims(self)
        dim = self.attrs["dim"] % n
        deg = min(int(self.attrs["degree"]), num_devices)
        degs = [1] * n
        degs[dim] = deg
        return self._cfg(degs, deg)


@register(OperatorType.OP_COMBINE)
class Combine(_ParallelOp):
    op_type = OperatorType.OP_COMBINE

    def pinned_config(self, num_devices):
        return self._cfg([1] * _dims(self), num_devices)


@register(OperatorType.OP_REPLICATE)
class Replicate(_ParallelOp):
    op_type = OperatorType.OP_REPLICATE

    def pinned_config(self, num_devices):
        return self._cfg([1] * _dims(self), min(int(self.attrs.get("degree", num_devices)), num_devices))


@register(OperatorType.OP_REDUCTION)
class Reduction(_ParallelOp):
    op_type = OperatorType.OP_REDUCTION

    def pinned_config(self, num_devices):
        n = _dims(self)
        degs = [1] * n
        deg = min(int(self.attrs.get("degree", 1)), num_devices)
        if deg > 1:
            degs[self.attrs.get("dim", 0) % n] = deg
            return self._cfg(degs, deg)
        return self._cfg(degs, num_devices)


@register(OperatorType.OP_ALLREDUCE)
class AllReduce(_ParallelOp):
    op_type = OperatorType.OP_ALLREDUCE

    def pinned_config(self, num_devices):
        return self._cfg([1] * _dims(self), num_devices)


@register(OperatorType.OP_FUSED_PARALLEL)
class FusedParallel(_ParallelOp):
    op_type = OperatorType.OP_FUSED_PARALLEL

    def pinned_config(self, num_devices):
        n = _dims(self)
        degs, ndev = [1] * n, num_devices
        for kind, dim, deg in self.attrs["ops"]:
            if kind == "repartition":
                degs[dim % n] *= deg
                ndev = 1
                for d in degs:
                    ndev *= d
            elif kind in ("combine", "allreduce"):
                degs[dim % n] = 1 if kind == "combine" else degs[dim % n]
                ndev = num_devices if kind == "allreduce" else ndev
            elif kind == "replicate":
                ndev = deg
        return self._cfg(degs, min(max(ndev, 1), num_devices))
