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
_WORDS = 4 + 3 * _DIMS
_MAX_BOXES = 65535
_MAX_SRCS = 16


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
    """Merge each dim into the next (inner) one where both sides are contiguous across it."""
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
    """boxes: [(src_off, src_strides, dst_off, dst_strides, extents[, src_index])] in elements;
    srcs: one tensor or a list of up to 16 (a box reads srcs[src_index]); a source stride may be
    negative (Reverse: the box walks that dim backwards from src_off)."""

    def __init__(self, boxes, srcs, dst: torch.Tensor, disjoint_dst: bool = False):
        srcs = list(srcs) if isinstance(srcs, (list, tuple)) else [srcs]
        if not 1 <= len(srcs) <= _MAX_SRCS:
            raise ValueError("box_copy: 1..16 source tensors")
        self.nsrc = len(srcs)
        self.elem = dst.element_size()
        self.dims = []
        spans = [_span(t) for t in srcs]
        dspan = _span(dst)
        dspans = []
        for bx in boxes:
            so, ss, do, ds, ext = bx[:5]
            si = bx[5] if len(bx) > 5 else 0
            if not 0 <= si < len(srcs):
                raise ValueError("box_copy: source index out of range")
            if any(e <= 0 for e in ext):
                continue
            # iterate dims in the source's memory order (largest stride first), so a box of a
            # channel-last tensor walks its channels innermost: contiguous runs, 16-B vectors
            order = sorted(range(len(ext)), key=lambda k: (-abs(ss[k]), -abs(ds[k])))
            dims = _coalesce([ext[k] for k in order], [ss[k] for k in order], [ds[k] for k in order])
            if len(dims) > _DIMS:
                raise ValueError("box_copy: more than 6 non-contiguous dimensions")
            lo_s = so + sum((e - 1) * a for e, a, _ in dims if a < 0)
            hi_s = so + sum((e - 1) * a for e, a, _ in dims if a > 0)
            lo_d = do + sum((e - 1) * b for e, _, b in dims if b < 0)
            hi_d = do + sum((e - 1) * b for e, _, b in dims if b > 0)
            if lo_s < 0 or lo_d < 0 or hi_s >= spans[si] or hi_d >= dspan:
                raise ValueError(f"box_copy: box {so}/{do} {ext} outside its tensors ({spans[si]}, {dspan})")
            self.dims.append((si, so, do, dims))
            dspans.append((lo_d, hi_d))
        if len(self.dims) > _MAX_BOXES:
            raise ValueError("box_copy: too many boxes for one launch")
        self.vec = 1
        for vb in (16, 8, 4, 2):
            v = vb // self.elem
            if v < 1 or vb % self.elem:
                continue
            if all(so % v == 0 and do % v == 0 and d[-1][1] == 1 and d[-1][2] == 1 and d[-1][0] % v == 0
                   and all(a % v == 0 and b % v == 0 for _, a, b in d[:-1]) for _, so, do, d in self.dims):
                self.vec = v
                break
        self._desc: Dict[tuple, torch.Tensor] = {}
        self.device = dst.device
        # Add mode read-modify-writes dst without atomics (one workgroup row per box), so boxes whose
        # destinations may overlap go to different launches: layers of boxes with pairwise-disjoint
        # destination element spans (first fit). disjoint_dst=True: the caller guarantees disjoint
        # destination regions (comm.py layers by exact region test), one launch.
        if disjoint_dst:
            self.add_layers = [list(range(len(self.dims)))]
        else:
            self.add_layers, ends = [], []
            for i in sorted(range(len(dspans)), key=lambda i: dspans[i]):
                lo, hi = dspans[i]
                for li, end in enumerate(ends):
                    if lo > end:
                        self.add_layers[li].append(i)
                        ends[li] = hi
                        break
                else:
                    self.add_layers.append([i])
                    ends.append(hi)

    def _descriptors(self, v: int, layer=None):
        key = (v, layer)
        if key not in self._desc:
            rows, mx = [], 0
            sel = self.dims if layer is None else [self.dims[i] for i in self.add_layers[layer]]
            for si, so, do, dims in sel:
                ext = [e for e, _, _ in dims]
                ss = [a for _, a, _ in dims]
                ds = [b for _, _, b in dims]
                if v > 1:  # inner run contiguous on both sides: vectors of v elements
                    ext[-1] //= v
                    ss = [x // v for x in ss[:-1]] + [1]
                    ds = [x // v for x in ds[:-1]] + [1]
                pad = _DIMS - len(ext)
                n = math.prod(ext)
                mx = max(mx, n)
                rows.append([si, so // v, do // v, n] + [1] * pad + ext + [0] * pad + ss + [0] * pad + ds)
            t = torch.tensor(rows if rows else [[0] * _WORDS], dtype=torch.int64).to(self.device)
            # 32-bit index math in the kernel when every reachable offset and box size fits
            lim = (1 << 31) - 1
            # (the kernel's grid-stride counter also stays below 2^31: max box + one whole grid,
            # at most 8192 blocks x 256 threads, box_copy in transfer.hip)
            idx32 = mx + 8192 * 256 < lim and all(abs(x) < lim for r in rows for x in r) and all(
                max(r[1], r[2]) + sum((r[4 + k] - 1) * max(abs(r[4 + _DIMS + k]), abs(r[4 + 2 * _DIMS + k]))
                                      for k in range(_DIMS)) < lim for r in rows)
            self._desc[key] = (t, mx, idx32)
        return self._desc[key]

    def emulate(self, srcs, dst: torch.Tensor, add: bool = False):
        """The plan through strided views (CPU tensors; the GPU tests' reference)."""
        srcs = list(srcs) if isinstance(srcs, (list, tuple)) else [srcs]
        for si, so, do, dims in self.dims:
            src = srcs[si]
            ext = [e for e, _, _ in dims]
            neg = [k for k, (_, x, _) in enumerate(dims) if x < 0]
            base = so + sum((dims[k][0] - 1) * dims[k][1] for k in neg)  # the lowest element
            a = src.as_strided(ext, [abs(x) for _, x, _ in dims], src.storage_offset() + base)
            if neg:
                a = a.flip(neg)
            b = dst.as_strided(ext, [x for _, _, x in dims], dst.storage_offset() + do)
            if add:
                b.add_(a)
            else:
                b.copy_(a)
        return dst

    def run(self, srcs, dst: torch.Tensor, add: bool = False):
        if not self.dims:
            return dst
        srcs = list(srcs) if isinstance(srcs, (list, tuple)) else [srcs]
        if len(srcs) != self.nsrc:
            raise ValueError("box_copy: wrong number of sources for this plan")
        if not dst.is_cuda:
            return self.emulate(srcs, dst, add)
        from .. import kernels as K
        v = 1 if add else self.vec
        vb = v * self.elem
        if not add and (dst.data_ptr() % vb or any(t.data_ptr() % vb for t in srcs)):
            v, vb = 1, self.elem
        if add:
            for li, lay in enumerate(self.add_layers):
                desc, mx, idx32 = self._descriptors(v, li)
                K.ext().box_copy(srcs, dst, desc, len(lay), mx, vb, True, False)
            return dst
        desc, mx, idx32 = self._descriptors(v)
        K.ext().box_copy(srcs, dst, desc, len(self.dims), mx, vb, add, idx32)
        return dst


def plan_key(role, *tensors) -> tuple:
    return (role,) + tuple((tuple(t.shape), tuple(t.stride()), t.dtype, str(t.device)) for t in tensors)


# ------------------------------------------------------------------ shape ops on box plans
def _dense_like(shape, like: torch.Tensor, device=None, dtype=None):
    """An uninitialised tensor of `shape` in like's memory format (channel-last 4-D stays so)."""
    cl = like.dim() == 4 and not like.is_contiguous() and like.is_contiguous(memory_format=torch.channels_last)
    # allocated in the target format directly (empty(...).contiguous(channels_last) launched a full
    # copy kernel per call: the r5 box-kernel concat A/B paid it, profiles/concat_box_ab_r5.txt)
    fmt = torch.channels_last if cl and len(shape) == 4 else torch.contiguous_format
    return torch.empty(shape, dtype=dtype or like.dtype, device=device or like.device, memory_format=fmt)


def _cached(cache: dict, key, build):
    p = cache.get(key)
    if p is None:
        p = cache[key] = build()
    return p


def concat(cache: dict, xs, ax: int):
    """torch.cat(xs, ax) as one launch (reference concat_kernels.cu: one copy per input); the
    output keeps the first input's memory format. Up to 16 inputs per launch, more in groups.
    None when a group's boxes would not move at least 8 B per element step (the caller falls back)."""
    shp = list(xs[0].shape)
    shp[ax] = sum(x.shape[ax] for x in xs)
    out = _dense_like(shp, xs[0])
    lo = 0
    for g0 in range(0, len(xs), _MAX_SRCS):
        grp = xs[g0:g0 + _MAX_SRCS]

        def build(grp=grp, lo=lo):
            boxes, c = [], lo
            for i, x in enumerate(grp):
                rel = [(0, e) for e in out.shape]
                rel[ax] = (c, c + x.shape[ax])
                do, ds, ext = region_box(out, rel)
                boxes.append((0, tuple(x.stride()), do, ds, ext, i))
                c += x.shape[ax]
            return BoxPlan(boxes, list(grp), out)
        key = ("cat", ax, lo) + plan_key("", out, *grp)
        plan = _cached(cache, key, build)
        if plan.vec * plan.elem < 8:  # element-wise boxes (mixed layouts, odd widths): the ATen cat
            return None
        plan.run(list(grp), out)
        lo += sum(x.shape[ax] for x in grp)
    return out


def split_dense(cache: dict, x: torch.Tensor, sizes, ax: int):
    """torch.split(x, sizes, ax) into DENSE parts (x's memory format, side by side in one buffer)
    by one launch; None when x is neither contiguous nor channel-last dense."""
    cl = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
    if not (cl or x.is_contiguous()):
        return None
    flat = torch.empty(x.numel(), dtype=x.dtype, device=x.device)
    outs, boxes, off, lo = [], [], 0, 0
    for n in sizes:
        shp = list(x.shape)
        shp[ax] = n
        if cl:  # NHWC strides of an [N, C, H, W] tensor
            _, C_, H_, W_ = shp
            st = (H_ * W_ * C_, 1, W_ * C_, C_)
        else:
            st, acc = [], 1
            for e in reversed(shp):
                st.append(acc)
                acc *= e
            st = tuple(reversed(st))
        outs.append(flat.as_strided(shp, st, off))
        rel = [(0, e) for e in x.shape]
        rel[ax] = (lo, lo + n)
        so, ss, ext = region_box(x, rel)
        boxes.append((so, ss, off, st, ext))
        off += math.prod(shp)
        lo += n
    key = ("split", tuple(sizes), ax) + plan_key("", x, flat)
    _cached(cache, key, lambda: BoxPlan(boxes, x, flat)).run(x, flat)
    return outs


def reverse(cache: dict, x: torch.Tensor, ax: int) -> torch.Tensor:
    """torch.flip(x, [ax]) as one launch (the source walked backwards along ax)."""
    out = _dense_like(list(x.shape), x)

    def build():
        st = list(x.stride())
        so = (x.shape[ax] - 1) * st[ax] if x.shape[ax] > 0 else 0
        st[ax] = -st[ax]
        return BoxPlan([(so, tuple(st), 0, tuple(out.stride()), tuple(x.shape))], x, out)
    _cached(cache, ("rev", ax) + plan_key("", x, out), build).run(x, out)
    return out
