"""Host side of csrc/kernels/transfer.hip: lists of rectangular regions ("boxes") copied or added
between two tensors in ONE kernel launch — the pack / unpack / local re-layout of an activation
transfer (parallel/comm.py exchange and generic P2P transfers) instead of one ATen slice copy per
overlap region.

A plan is built once per (transfer side, tensor geometry): each box is coalesced to the fewest
dimensions contiguous on both sides, the widest vector (16 / 8 / 4 / 2 / 1 bytes) dividing every
inner run, stride and offset is chosen, every reachable offset is checked against both tensors'
extents on the host, and the descriptors are uploaded to the device once (replays under a hipGraph
need no host work).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

_DIMS = 6
_WORDS = 3 + 3 * _DIMS
_MAX_BOXES = 65535


def available(t: Optional[torch.Tensor]) -> bool:
    """Device tensors always take the box kernels. FF_BOXCOPY_EMULATE=1 runs the same plans on CPU
    tensors through strided views (the gloo multi-rank tests exercise every plan that way)."""
    if t is None:
        return False
    if not t.is_cuda:
        return os.environ.get("FF_BOXCOPY_EMULATE") == "1"
    from .. import kernels as K
    K.ext()  # a GPU run without the extension fails loudly instead of silently using ATen copies
    return True


def region_box(t: torch.Tensor, rel: Sequence[Tuple[int, int]]):
    """(element offset, strides, extents) of the sub-region `rel` ([lo, hi) per dim) of tensor t."""
    st = t.stride()
    off = sum(lo * s for (lo, _), s in zip(rel, st))
    return off, tuple(st), tuple(hi - lo for lo, hi in rel)


def flat_box(off: int, extents: Sequence[int]):
    """A region stored contiguously at element offset `off` of a flat buffer."""
    st, acc = [], 1
    for e in reversed(extents):
        st.append(acc)
        acc *= e
    return off, tuple(reversed(st)), tuple(extents)


def _coalesce(ext, ss, ds):
    out: List[List[int]] = []
    for e, a, b in zip(ext, ss, ds):
        if e == 1:
            continue
        if out and out[-1][1] == a * e and out[-1][2] == b * e:
            out[-1] = [out[-1][0] * e, a, b]
        else:
            out.append([e, a, b])
    return out or [[1, 1, 1]]


def _span(t: torch.Tensor) -> int:
    return 1 + sum((n - 1) * s for n, s in zip(t.shape, t.stride()) if n > 0)


class BoxPlan:
    """boxes: [(src_off, src_strides, dst_off, dst_strides, extents)] in elements."""

    def __init__(self, boxes, src: torch.Tensor, dst: torch.Tensor):
        self.elem = src.element_size()
        self.n = len(boxes)
        self.dims = []
        sspan, dspan = _span(src), _span(dst)
        for so, ss, do, ds, ext in boxes:
            if any(e <= 0 for e in ext):
                continue
            # iterate dims in the source's memory order (outermost stride first), so a box of a
            # channel-last tensor walks its channels innermost: contiguous runs, 16-B vectors
            order = sorted(range(len(ext)), key=lambda k: (-ss[k], -ds[k]))
            dims = _coalesce([ext[k] for k in order], [ss[k] for k in order], [ds[k] for k in order])
            if len(dims) > _DIMS:
                raise ValueError("box_copy: more than 6 non-contiguous dimensions")
            hi_s = so + sum((e - 1) * a for e, a, _ in dims)
            hi_d = do + sum((e - 1) * b for e, _, b in dims)
            if so < 0 or do < 0 or hi_s >= sspan or hi_d >= dspan:
                raise ValueError(f"box_copy: box {so}/{do} {ext} outside its tensors ({sspan}, {dspan})")
            self.dims.append((so, do, dims))
        if len(self.dims) > _MAX_BOXES:
            raise ValueError("box_copy: too many boxes for one launch")
        self.vec = 1
        for vb in (16, 8, 4, 2):
            v = vb // self.elem
            if v < 1 or vb % self.elem:
                continue
            if all(so % v == 0 and do % v == 0 and d[-1][1] == 1 and d[-1][2] == 1 and d[-1][0] % v == 0
                   and all(a % v == 0 and b % v == 0 for _, a, b in d[:-1]) for so, do, d in self.dims):
                self.vec = v
                break
        self._desc: Dict[tuple, torch.Tensor] = {}
        self.device = src.device

    def _descriptors(self, v: int):
        key = (v,)
        if key not in self._desc:
            rows, mx = [], 0
            for so, do, dims in self.dims:
                ext = [e for e, _, _ in dims]
                ss = [a for _, a, _ in dims]
                ds = [b for _, _, b in dims]
                if v > 1:  # inner run contiguous on both sides: vectors of v elements
                    ext[-1] //= v
                    ss = [s // v for s in ss[:-1]] + [1]
                    ds = [s // v for s in ds[:-1]] + [1]
                pad = _DIMS - len(ext)
                n = math.prod(ext)
                mx = max(mx, n)
                rows.append([so // v, do // v, n] + [1] * pad + ext + [0] * pad + ss + [0] * pad + ds)
            t = torch.tensor(rows if rows else [[0] * _WORDS], dtype=torch.int64).to(self.device)
            self._desc[key] = (t, mx)
        return self._desc[key]

    def emulate(self, src: torch.Tensor, dst: torch.Tensor, add: bool = False):
        """The plan through strided views (CPU tensors; the GPU tests' reference)."""
        for so, do, dims in self.dims:
            ext = [e for e, _, _ in dims]
            a = src.as_strided(ext, [x for _, x, _ in dims], src.storage_offset() + so)
            b = dst.as_strided(ext, [x for _, _, x in dims], dst.storage_offset() + do)
            if add:
                b.add_(a)
            else:
                b.copy_(a)
        return dst

    def run(self, src: torch.Tensor, dst: torch.Tensor, add: bool = False):
        if not self.dims:
            return dst
        if not src.is_cuda:
            return self.emulate(src, dst, add)
        from .. import kernels as K
        v = 1 if add else self.vec
        vb = v * self.elem
        if not add and (src.data_ptr() % vb or dst.data_ptr() % vb):
            v, vb = 1, self.elem
        desc, mx = self._descriptors(v)
        K.ext().box_copy(src, dst, desc, len(self.dims), mx, vb, add)
        return dst


def plan_key(role, *tensors) -> tuple:
    return (role,) + tuple((tuple(t.shape), tuple(t.stride()), t.dtype, str(t.device)) for t in tensors)
