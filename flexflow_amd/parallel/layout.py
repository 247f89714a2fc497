"""Sharded tensor layouts (the runtime form of the reference's ParallelTensorShape + MachineView).

A `Layout` says how a logical (global-shape) tensor is split over devices:

  * `degrees[i]`   – number of blocks along dim i (reference ParallelDim.degree),
  * `replicas`     – number of copies of every block (reference's trailing replica dim),
  * `partial`      – replicas hold partial SUMS that must be reduced (output of a Linear whose
                     input-channel dim is partitioned; reference Reduction parallel op),
  * `devices`      – the device (= rank) of every part; part index is row-major over
                     (block coords..., replica coord) with the replica coordinate fastest,
  * `halo[i]`      – optional overlap (in elements) on dim i, used by spatially partitioned
                     Conv2D/Pool2D (attribute parallelism) whose parts need neighbour rows.

Reference: include/flexflow/parallel_tensor.h:36-203 (ParallelDim/ParallelTensorShape),
include/flexflow/machine_view.h:14-96 (MachineView::device_ids). Unlike the reference, a layout
maps parts straight to ranks of the SPMD job; data movement between layouts is explicit
(flexflow_amd.parallel.comm) instead of implicit Realm copies between logical-region partitions.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence, Tuple

Region = Tuple[Tuple[int, int], ...]


@dataclass(frozen=True)
class Layout:
    shape: Tuple[int, ...]
    degrees: Tuple[int, ...]
    replicas: int = 1
    devices: Tuple[int, ...] = (0,)
    partial: bool = False
    halo: Optional[Tuple[int, ...]] = None

    def __post_init__(self):
        assert len(self.shape) == len(self.degrees), (self.shape, self.degrees)
        assert len(self.devices) == self.num_parts, (self.devices, self.degrees, self.replicas)
        for s, d in zip(self.shape, self.degrees):
            assert d >= 1 and s % d == 0, f"dim {s} not divisible by degree {d}"

    # ---------------------------------------------------------------- basics
    @property
    def ndim(self) -> int:
        return len(self.shape)

    @property
    def num_blocks(self) -> int:
        return int(math.prod(self.degrees))

    @property
    def num_parts(self) -> int:
        return self.num_blocks * self.replicas

    def block_shape(self) -> Tuple[int, ...]:
        return tuple(s // d for s, d in zip(self.shape, self.degrees))

    def coords(self, p: int) -> Tuple[Tuple[int, ...], int]:
        rep = p % self.replicas
        b = p // self.replicas
        cs = []
        for d in reversed(self.degrees):
            cs.append(b % d)
            b //= d
        return tuple(reversed(cs)), rep

    def part_index(self, block: Sequence[int], rep: int = 0) -> int:
        b = 0
        for c, d in zip(block, self.degrees):
            b = b * d + c
        return b * self.replicas + rep

    def block_region(self, block: Sequence[int]) -> Region:
        bs = self.block_shape()
        return tuple((c * s, (c + 1) * s) for c, s in zip(block, bs))

    def region(self, p: int) -> Region:
        """Region held by part p, including halo (clipped to the tensor)."""
        block, _ = self.coords(p)
        reg = self.block_region(block)
        if self.halo:
            reg = tuple((max(0, lo - h), min(s, hi + h)) for (lo, hi), h, s in zip(reg, self.halo, self.shape))
        return reg

    def local_shape(self, p: int) -> Tuple[int, ...]:
        return tuple(hi - lo for lo, hi in self.region(p))

    def parts_on(self, rank: int) -> list[int]:
        return [p for p, d in enumerate(self.devices) if d == rank]

    def replica_group(self, block: Sequence[int]) -> Tuple[int, ...]:
        return tuple(self.devices[self.part_index(block, r)] for r in range(self.replicas))

    def blocks(self):
        return itertools.product(*[range(d) for d in self.degrees])

    def device_set(self) -> Tuple[int, ...]:
        return tuple(sorted(set(self.devices)))

    def with_(self, **kw) -> "Layout":
        d = dict(shape=self.shape, degrees=self.degrees, replicas=self.replicas, devices=self.devices,
                 partial=self.partial, halo=self.halo)
        d.update(kw)
        return Layout(**d)

    def key(self):
        return (self.shape, self.degrees, self.replicas, self.devices, self.partial, self.halo)

    def __repr__(self):
        h = f", halo={self.halo}" if self.halo else ""
        p = ", partial" if self.partial else ""
        return f"Layout({list(self.shape)} deg={list(self.degrees)} rep={self.replicas}{p}{h} dev={list(self.devices)})"


def replicated(shape, devices: Sequence[int]) -> Layout:
    return Layout(tuple(shape), tuple(1 for _ in shape), len(devices), tuple(devices))


def single(shape, device: int = 0) -> Layout:
    return Layout(tuple(shape), tuple(1 for _ in shape), 1, (device,))


def intersect(a: Region, b: Region) -> Optional[Region]:
    out = []
    for (al, ah), (bl, bh) in zip(a, b):
        lo, hi = max(al, bl), min(ah, bh)
        if lo >= hi:
            return None
        out.append((lo, hi))
    return tuple(out)


def region_numel(r: Region) -> int:
    return int(math.prod(hi - lo for lo, hi in r))


def rel_slices(region: Region, within: Region):
    """Python slices selecting `region` inside a buffer that holds `within`."""
    return tuple(slice(lo - wl, hi - wl) for (lo, hi), (wl, _) in zip(region, within))


@dataclass
class TransferItem:
    src_part: int
    dst_part: int
    region: Region
    reduce: bool  # True: dst accumulates (sum); False: plain copy


def plan_transfer(src: Layout, dst: Layout, src_partial: bool) -> list[TransferItem]:
    """Generic block-to-block plan moving data from `src` parts to every `dst` part.

    Every dst part receives its full region. For a non-partial source, each element is read from
    exactly one owner replica (preferring a replica already on the destination device, otherwise
    spreading destinations over replicas). For a partial source every replica contributes and the
    destination sums. Sources are read from their owned (non-halo) block regions so that halo
    overlap never double counts.
    """
    assert src.shape == dst.shape, (src.shape, dst.shape)
    items: list[TransferItem] = []
    if src.halo and src_partial:
        # gradients of halo'd parts: every part's full (overlapping) region contributes
        for q in range(dst.num_parts):
            rq = dst.region(q)
            for p in range(src.num_parts):
                o = intersect(src.region(p), rq)
                if o is not None:
                    items.append(TransferItem(p, q, o, True))
        return items
    for q in range(dst.num_parts):
        rq = dst.region(q)
        dq_dev = dst.devices[q]
        # src blocks overlapping rq
        ranges = []
        bs = src.block_shape()
        for (lo, hi), s in zip(rq, bs):
            ranges.append(range(lo // s, (hi - 1) // s + 1))
        for blk in itertools.product(*ranges):
            o = intersect(src.block_region(blk), rq)
            if o is None:
                continue
            reps = [src.part_index(blk, r) for r in range(src.replicas)]
            if src_partial:
                for ps in reps:
                    items.append(TransferItem(ps, q, o, True))
            else:
                local = [ps for ps in reps if src.devices[ps] == dq_dev]
                ps = local[0] if local else reps[q % len(reps)]
                items.append(TransferItem(ps, q, o, False))
    return items


def transfer_bytes(src: Layout, dst: Layout, src_partial: bool, elem_bytes: int) -> dict:
    """Per (src_dev, dst_dev) byte counts of the generic plan (used by the cost model)."""
    out: dict = {}
    for it in plan_transfer(src, dst, src_partial):
        a, b = src.devices[it.src_part], dst.devices[it.dst_part]
        if a == b:
            continue
        out[(a, b)] = out.get((a, b), 0) + region_numel(it.region) * elem_bytes
    return out
