"""Operator contract.

Split of responsibilities (reference include/flexflow/operator.h:18-277 mixes all of these into
one Legion-task class with init/forward/backward task launchers):

  * graph level   – `infer` (output shapes/dtypes + weight specs) at layer-build time;
  * parallelization – the op's *parallel axes* (its output dims plus op-specific reduction axes)
    and, for every input / weight / output, which axis each tensor dim is partitioned along.
    This is the reference's ParallelDimMappingRecord machinery (model.cc:594-852) in
    declarative form; replica dims follow from the axes a tensor does NOT map;
  * execution     – `forward` / `backward` on the rank-local shards (HIP kernels via
    flexflow_amd.kernels), with activations saved in a per-op context;
  * cost          – analytic FLOP / byte counts for the simulator (measured costs override).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from ..type import DataType, OperatorType

OPS: Dict[OperatorType, type] = {}


def register(*types):
    def deco(cls):
        for t in types:
            OPS[t] = cls
        return cls
    return deco


@dataclass
class WeightSpec:
    name: str
    dims: Tuple[int, ...]
    dtype: DataType
    init: Any = None          # Initializer (None -> op default)
    trainable: bool = True


TORCH_DT = {DataType.DT_FLOAT: torch.float32, DataType.DT_BF16: torch.bfloat16, DataType.DT_HALF: torch.float16,
            DataType.DT_DOUBLE: torch.float64, DataType.DT_INT32: torch.int32, DataType.DT_INT64: torch.int64,
            DataType.DT_BOOLEAN: torch.bool}


def torch_dtype(dt: DataType):
    return TORCH_DT[dt]


@dataclass
class OpCtx:
    """Per-(op, rank) execution context."""
    layer: Any
    part_coords: Tuple[int, ...]            # this rank's coordinates along every parallel axis
    degrees: Tuple[int, ...]
    compute_dtype: DataType = DataType.DT_FLOAT
    training: bool = True
    saved: Dict[str, Any] = field(default_factory=dict)
    wgrads: List[Optional[torch.Tensor]] = field(default_factory=list)   # fp32 accumulators (+=)
    step: int = 0
    seed: int = 0
    extra: Dict[str, Any] = field(default_factory=dict)

    def coord(self, axis: int) -> int:
        return self.part_coords[axis]

    def degree(self, axis: int) -> int:
        return self.degrees[axis]


class OpImpl:
    op_type: OperatorType = OperatorType.OP_INVALID
    # extra (non-output) parallel axes: list of (name, kind) ; kinds: 'reduce', 'parameter'
    extra_axes: Tuple[str, ...] = ()

    def __init__(self, layer):
        self.layer = layer
        self.attrs = layer.attrs

    # ---------------------------------------------------------------- graph level
    @classmethod
    def infer(cls, attrs, in_dims: List[Tuple[int, ...]], in_dtypes: List[DataType]):
        """-> (out_dims list, out_dtypes list, weight specs list)."""
        return [in_dims[0]], [in_dtypes[0]], []

    # ---------------------------------------------------------------- parallelization
    def axis_sizes(self) -> List[int]:
        return list(self.layer.outputs[0].dims) + self.extra_axis_sizes()

    def extra_axis_sizes(self) -> List[int]:
        return []

    def axis_kinds(self) -> List[str]:
        """'sample' (dim 0), 'attribute' (spatial/sequence), 'parameter' (channel / heads /
        reduction), 'none' (must stay 1). Used to honour --only-data-parallel and the reference's
        enable_{sample,parameter,attribute}_parallel switches."""
        n = len(self.layer.outputs[0].dims)
        kinds = ["sample"] + ["attribute"] * (n - 1)
        return kinds + ["parameter"] * len(self.extra_axis_sizes())

    def input_maps(self) -> List[Tuple[Optional[int], ...]]:
        """For each input, the parallel axis each dim is partitioned along (None = full)."""
        n = len(self.layer.outputs[0].dims)
        return [tuple(range(n)) if len(t.dims) == n else tuple([None] * len(t.dims)) for t in self.layer.inputs]

    def weight_maps(self) -> List[Tuple[Optional[int], ...]]:
        return [tuple([None] * len(w.dims)) for w in self.layer.weights]

    def output_maps(self) -> List[Tuple[Optional[int], ...]]:
        return [tuple(range(len(o.dims))) if i == 0 else tuple([None] * len(o.dims))
                for i, o in enumerate(self.layer.outputs)]

    def partial_axes(self) -> List[int]:
        """Axes over which outputs are partial sums (must be reduced by the consumer edge)."""
        return list(range(len(self.layer.outputs[0].dims), len(self.axis_sizes())))

    def input_halo(self, idx: int, degrees) -> Optional[Tuple[int, ...]]:
        return None

    def supports_axis(self, axis: int) -> bool:
        """Whether the op implementation can run with this axis partitioned."""
        return True

    # ---------------------------------------------------------------- execution
    def forward(self, ctx: OpCtx, xs: List[torch.Tensor], ws: List[torch.Tensor]) -> List[torch.Tensor]:
        raise NotImplementedError(type(self).__name__)

    def backward(self, ctx: OpCtx, douts: List[Optional[torch.Tensor]]) -> List[Optional[torch.Tensor]]:
        raise NotImplementedError(type(self).__name__)

    def needs_input_grad(self, i: int) -> bool:
        return True

    def overwrites_wgrad(self, i: int) -> bool:
        """True if, when this layer is its weights' only user (ctx.extra['wgrad_overwrite']), the
        backward WRITES weight i's whole gradient (beta = 0) instead of adding to it: the executor
        then skips zeroing that gradient between steps. Conservative default."""
        return False

    # ---------------------------------------------------------------- cost model
    def flops(self, in_shapes, out_shapes, w_shapes) -> float:
        return float(sum(math.prod(s) for s in out_shapes))

    def mem_bytes(self, in_shapes, out_shapes, w_shapes, elem=2) -> float:
        return float(elem * (sum(math.prod(s) for s in in_shapes) + sum(math.prod(s) for s in out_shapes)
                             + sum(math.prod(s) for s in w_shapes)))

    def can_inplace(self) -> bool:
        """True if forward may write its (single) output into its first input's buffer."""
        return False

    def saves_output(self) -> bool:
        """True if backward reads this op's own output tensor (then a consumer must not overwrite
        it in place). Conservative default."""
        return True

    def accumulates_dx(self) -> bool:
        """True if backward honours ctx.extra['dx_accum'] = {input slot: tensor}: it then ADDS the
        input gradient into that tensor (same shape/dtype) and returns it for that slot."""
        return False

    def accum_target_ok(self, t) -> bool:
        """May t (an existing input gradient) be this op's dx_accum target? Default: row-major
        contiguous (GEMM outputs are written through a 2-D view)."""
        return t.is_contiguous()

    def accum_may_alias_douts(self) -> bool:
        """True if every read of the output gradients is issued before the first write into a
        dx_accum target, so that target may share storage with an output gradient."""
        return False

    def uses_mfma(self) -> bool:
        return False

    # ---------------------------------------------------------------- serialization
    def params_key(self) -> tuple:
        return tuple(sorted((k, repr(v)) for k, v in self.attrs.items()))
