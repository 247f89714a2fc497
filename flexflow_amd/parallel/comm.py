"""Explicit data movement between sharded layouts over RCCL (torch.distributed 'nccl'; the CPU
multi-rank tests run the same calls on gloo — no backend-specific branches).

This replaces the reference's implicit Legion/Realm DMA between logical-region partitions and its
parallel-op kernels (src/parallel_ops/{partition,combine,replicate,reduction}.cc,
src/parallel_ops/kernels/*.cu) with explicit collectives chosen per edge:

    identity          same layout                                    (no-op)
    local slice       replicated -> partitioned on the same devices  (Repartition, no comm)
    all_gather        partitioned -> replicated                      (Combine / Replicate)
    reduce_scatter    partial    -> partitioned                      (Reduction + Repartition)
    all_reduce        partial    -> replicated                       (Reduction + Replicate)
    all_to_all        partitioned along a -> partitioned along b     (Combine(a) + Repartition(b)
                      on the same devices: every rank sends 1/k of its shard to each peer,
                      one link per peer on the fully connected xGMI node)
    exchange          any other re-partition among ONE device set (uneven splits, several dims
                      at once, permuted placement, no replicas / partial sums): one
                      all_to_all_single with per-peer split sizes over the packed overlaps
    generic P2P       anything else (placement changes between device groups, halos, partial
                      sums onto a different layout): batched isend/irecv of exactly the
                      overlapping blocks (no zero fill unless partial sums are added).

and the weight-gradient synchronisation (reference: one ncclAllReduce per weight followed by an
execution fence, src/runtime/optimizer_kernel.cu:88-94 / optimizer.cc:193) with bucketed
all-reduces over flat fp32 gradient arenas, issued asynchronously as soon as a bucket's last
gradient is produced so they overlap the rest of the backward pass (optionally in bf16, halving
the bytes: --grad-comm-dtype bf16).

Every transfer can be started asynchronously (`Transfer.start` -> `Pending`): with RCCL the
collective is enqueued on the process group's own stream behind an event on the compute stream,
and `Pending.wait()` makes the compute stream (not the host) wait for it, so the executor issues
activation collectives as soon as their producer has run and waits only where the consumer needs
the value (runtime/executor.py).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence

import math

import torch
import torch.distributed as dist

from . import boxcopy
from .layout import Layout, TransferItem, plan_transfer, rel_slices


def _slices(region, within):
    return rel_slices(region, within)


class Communicator:
    """Owns the SPMD process-group registry. Groups are created collectively (every rank calls
    `ensure_groups` with the same ordered list) as required by torch.distributed.new_group."""

    def __init__(self, rank: int = 0, world: int = 1):
        self.rank = rank
        self.world = world
        self.groups: Dict[tuple, object] = {}
        self.backend = dist.get_backend() if (dist.is_available() and dist.is_initialized()) else None
        # FF_FORCE_COLLECTIVES=1 (tests): a world-1 process group still takes the distributed path —
        # every gradient bucket is all-reduced (over one rank) and the step graph captures the
        # collectives — so the RCCL capture path runs on a one-GPU box
        self.force = os.environ.get("FF_FORCE_COLLECTIVES") == "1" and self.backend is not None

    @property
    def distributed(self) -> bool:
        return (self.world > 1 or self.force) and self.backend is not None

    def ensure_groups(self, rank_sets: Sequence[Sequence[int]]):
        for rs in rank_sets:
            key = tuple(sorted(set(rs)))
            if len(key) <= 1 or key in self.groups:
                continue
            if len(key) == self.world:
                self.groups[key] = dist.group.WORLD
            else:
                self.groups[key] = dist.new_group(list(key))

    def group(self, ranks) -> object:
        key = tuple(sorted(set(ranks)))
        if len(key) == self.world:
            return dist.group.WORLD
        g = self.groups.get(key)
        if g is None:
            raise RuntimeError(f"process group {key} was not created at compile time")
        return g

    @property
    def is_nccl(self):
        return self.backend == "nccl"


def _find_split_dim(a: Layout, b: Layout, factor: int) -> Optional[int]:
    """dim d where b.degrees[d] == a.degrees[d]*factor and all other degrees equal."""
    cand = None
    for d, (x, y) in enumerate(zip(a.degrees, b.degrees)):
        if x == y:
            continue
        if y == x * factor and cand is None:
            cand = d
        else:
            return None
    return cand


class Pending:
    """An in-flight transfer: wait() returns this rank's destination part (or None)."""

    def __init__(self, handles=(), finish=None, value=None, kind="identity", nbytes=0):
        self.handles = [h for h in handles if h is not None]
        self.finish = finish
        self.value = value
        self.kind = kind
        self.nbytes = nbytes
        self.done = not self.handles and finish is None

    def wait(self):
        if not self.done:
            for h in self.handles:
                h.wait()
            if self.finish is not None:
                self.value = self.finish()
            self.done = True
            self.handles = []
            self.finish = None
        return self.value


def _a2a_dims(S: Layout, D: Layout):
    """(a, b, k) when D re-partitions S from dim a to dim b k ways on the same devices, no replicas."""
    if S.replicas != 1 or D.replicas != 1 or S.halo or D.halo or len(S.degrees) != len(D.degrees):
        return None
    diff = [d for d in range(len(S.degrees)) if S.degrees[d] != D.degrees[d]]
    if len(diff) != 2:
        return None
    a = [d for d in diff if S.degrees[d] > 1 and D.degrees[d] == 1]
    b = [d for d in diff if D.degrees[d] > 1 and S.degrees[d] == 1]
    if len(a) != 1 or len(b) != 1 or S.degrees[a[0]] != D.degrees[b[0]]:
        return None
    a, b = a[0], b[0]
    k = S.degrees[a]
    if S.shape[a] % k or S.shape[b] % k:  # equal chunks only (chunk + stack in _all_to_all)
        return None
    for blk in S.blocks():
        if blk[a] != 0:
            continue
        sd, dd = _a2a_devices(S, D, blk, a, b, k)
        if len(set(sd)) != k or set(sd) != set(dd):
            return None
    return a, b, k


def _a2a_devices(S, D, blk, a, b, k):
    sd, dd = [], []
    for i in range(k):
        o = list(blk)
        o[a] = i
        sd.append(S.devices[S.part_index(o, 0)])
        o = list(blk)
        o[a] = 0
        o[b] = i
        dd.append(D.devices[D.part_index(o, 0)])
    return sd, dd


class Transfer:
    """A planned layout conversion for one tensor edge, executed by every rank (SPMD)."""

    def __init__(self, src: Layout, dst: Layout, src_partial: bool, rank: int, elem_dtype=None):
        self.src, self.dst, self.sp = src, dst, src_partial
        self.rank = rank
        self.kind = "generic"
        self.dim = None
        self.group_ranks: tuple = ()
        self._classify()
        self.items: Optional[list[TransferItem]] = None
        if self.kind in ("generic", "exchange"):
            self.items = plan_transfer(src, dst, src_partial)

    # ------------------------------------------------------------------ classification
    def _classify(self):
        S, D, sp = self.src, self.dst, self.sp
        same_blocks = S.degrees == D.degrees
        if not sp and same_blocks and S.replicas == D.replicas and S.devices == D.devices and S.halo == D.halo:
            self.kind = "identity"
            return
        if S.halo or D.halo:
            return
        if sp and same_blocks and S.replicas == D.replicas:
            ok = all(set(S.replica_group(b)) == set(D.replica_group(b)) for b in S.blocks())
            if ok:
                self.kind = "all_reduce"
                return
        if sp and D.replicas == 1 and S.replicas > 1:
            d = _find_split_dim(S, D, S.replicas)
            if d is not None and self._subblock_devices_match(S, D, d, S.replicas):
                self.kind, self.dim = "reduce_scatter", d
                return
        if not sp and S.replicas == 1 and D.replicas > 1:
            d = _find_split_dim(D, S, D.replicas)
            if d is not None and self._subblock_devices_match(D, S, d, D.replicas):
                self.kind, self.dim = "all_gather", d
                return
        if not sp and S.replicas > 1 and D.replicas == 1:
            d = _find_split_dim(S, D, S.replicas)
            if d is not None and self._subblock_devices_match(S, D, d, S.replicas, subset=True):
                self.kind, self.dim = "local_slice", d
                return
        if not sp:
            a2a = _a2a_dims(S, D)
            if a2a is not None:
                self.kind, self.dim = "all_to_all", a2a
                return
            # any other re-partition among one device set (uneven splits, several dims at once,
            # permuted placement): one all_to_all_single with per-peer split sizes
            if (S.replicas == 1 and D.replicas == 1 and set(S.devices) == set(D.devices)
                    and len(set(S.devices)) == len(S.devices) and len(set(D.devices)) == len(D.devices)
                    and len(S.devices) > 1):
                self.kind = "exchange"
                self.group_ranks = tuple(sorted(set(S.devices)))

    @staticmethod
    def _subblock_devices_match(coarse: Layout, fine: Layout, d: int, k: int, subset=False) -> bool:
        """Each coarse block's replica devices == devices of its k fine sub-blocks along dim d."""
        for blk in coarse.blocks():
            rep_devs = set(coarse.replica_group(blk))
            sub = []
            for j in range(k):
                fb = list(blk)
                fb[d] = blk[d] * k + j
                sub.append(fine.devices[fine.part_index(fb, 0)])
            if subset:
                if not set(sub) <= rep_devs or len(set(sub)) != k:
                    return False
            elif set(sub) != rep_devs or len(rep_devs) != k:
                return False
        return True

    def rank_sets(self) -> list[tuple]:
        """Process groups this transfer needs (for collective creation at compile time)."""
        out = []
        if self.kind == "all_reduce":
            for b in self.src.blocks():
                out.append(tuple(sorted(self.src.replica_group(b))))
        elif self.kind == "reduce_scatter":
            for b in self.src.blocks():
                out.append(tuple(sorted(self.src.replica_group(b))))
        elif self.kind == "all_gather":
            for b in self.dst.blocks():
                out.append(tuple(sorted(self.dst.replica_group(b))))
        elif self.kind == "all_to_all":
            a, b, k = self.dim
            for blk in self.src.blocks():
                if blk[a] == 0:
                    out.append(tuple(sorted(_a2a_devices(self.src, self.dst, blk, a, b, k)[0])))
        elif self.kind == "exchange":
            out.append(self.group_ranks)
        return out

    def bytes_moved(self, elem_bytes: int) -> int:
        """Bytes sent by this rank (cost accounting / tracing)."""
        S = self.src
        loc = S.parts_on(self.rank)
        if not loc:
            return 0
        n = 1
        for s in S.local_shape(loc[0]):
            n *= s
        if self.kind in ("identity", "local_slice"):
            return 0
        if self.kind == "all_reduce":
            r = S.replicas
            return int(2 * (r - 1) / r * n * elem_bytes)
        if self.kind == "reduce_scatter":
            r = S.replicas
            return int((r - 1) / r * n * elem_bytes)
        if self.kind == "all_gather":
            return int((self.dst.replicas - 1) * n * elem_bytes)
        if self.kind == "all_to_all":
            k = self.dim[2]
            return int((k - 1) / k * n * elem_bytes)
        tot = 0
        for it in self.items or []:
            if S.devices[it.src_part] == self.rank and self.dst.devices[it.dst_part] != self.rank:
                m = 1
                for lo, hi in it.region:
                    m *= hi - lo
                tot += m * elem_bytes
        return tot

    # ------------------------------------------------------------------ execution
    def run(self, comm: Communicator, x: Optional[torch.Tensor], like: Optional[torch.Tensor] = None):
        """x: this rank's src part (or None). Returns this rank's dst part (or None)."""
        return self.start(comm, x, like).wait()

    def start(self, comm: Communicator, x: Optional[torch.Tensor], like: Optional[torch.Tensor] = None) -> Pending:
        """Issue the transfer without waiting for it (every rank, same order); see Pending."""
        S, D, r = self.src, self.dst, self.rank
        dparts = D.parts_on(r)
        sparts = S.parts_on(r)
        if self.kind == "identity":
            return Pending(value=x)
        if self.kind == "local_slice":
            if not dparts:
                return Pending(value=None)
            q = dparts[0]
            return Pending(value=x[_slices(D.region(q), S.region(sparts[0]))].contiguous(), kind=self.kind)
        nb = self.bytes_moved(x.element_size() if x is not None else 2)
        if self.kind == "all_reduce":
            if x is None:
                return Pending(value=None)
            grp = tuple(sorted(S.replica_group(S.coords(sparts[0])[0])))
            y = x.contiguous().clone() if not x.is_contiguous() else x
            if len(grp) <= 1:
                return Pending(value=y)
            h = dist.all_reduce(y, group=comm.group(grp), async_op=True)
            return Pending([h], lambda: y, kind=self.kind, nbytes=nb)
        if self.kind == "reduce_scatter":
            if x is None:
                return Pending(value=None)
            return self._reduce_scatter(comm, x)
        if self.kind == "all_gather":
            if x is None and not dparts:
                return Pending(value=None)
            return self._all_gather(comm, x)
        if self.kind == "all_to_all":
            if x is None:
                return Pending(value=None)
            return self._all_to_all(comm, x)
        if self.kind == "exchange":
            if x is None:
                return Pending(value=None)
            return self._exchange(comm, x)
        return self._generic(comm, x, like)

    def _exchange(self, comm, x):
        """Every rank of the device set sends each peer the overlap of its source block with the
        peer's destination block, packed into one buffer in group-rank order, through ONE
        all_to_all_single with per-peer split sizes (the overlaps are listed in the same order on
        every rank: plan_transfer is deterministic)."""
        S, D, r = self.src, self.dst, self.rank
        grp = list(self.group_ranks)
        send = {p: [] for p in grp}
        recv = {p: [] for p in grp}
        for it in self.items:
            sd, dd = S.devices[it.src_part], D.devices[it.dst_part]
            if sd == r:
                send[dd].append(it)
            if dd == r:
                recv[sd].append(it)
        in_splits = [sum(_numel(it.region) for it in send[p]) for p in grp]
        out_splits = [sum(_numel(it.region) for it in recv[p]) for p in grp]
        q = D.parts_on(r)[0]
        boxes = boxcopy.available(x)
        if boxes:  # one pack launch over every region this rank sends
            inp = torch.empty(sum(in_splits), dtype=x.dtype, device=x.device)
            pack = [it for p in grp for it in send[p]]
            self._box_plan("xpack", x, inp, lambda: _pack_boxes(x, pack, S)).run(x, inp)
        else:
            chunks = [x[_slices(it.region, S.region(it.src_part))].reshape(-1) for p in grp for it in send[p]]
            inp = torch.cat(chunks) if chunks else x.new_empty(0)
        flat = torch.empty(sum(out_splits), dtype=x.dtype, device=x.device)
        h = dist.all_to_all_single(flat, inp.contiguous(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                                   group=comm.group(grp), async_op=True)

        def finish():
            out = torch.empty(D.local_shape(q), dtype=x.dtype, device=x.device)  # the overlaps tile it
            unpack = [it for p in grp for it in recv[p]]
            if boxes:  # one unpack launch
                self._box_plan("xunpack", flat, out, lambda: _unpack_boxes(out, unpack, D)).run(flat, out)
                return out
            off = 0
            for it in unpack:
                shp = tuple(hi - lo for lo, hi in it.region)
                n = math.prod(shp)
                out[_slices(it.region, D.region(it.dst_part))].copy_(flat[off:off + n].view(shp))
                off += n
            return out
        sent = sum(n for p, n in zip(grp, in_splits) if p != r) * x.element_size()
        return Pending([h], finish, kind="exchange", nbytes=sent)

    def _all_to_all(self, comm, x):
        S, D, r = self.src, self.dst, self.rank
        a, b, k = self.dim
        blk = list(S.coords(S.parts_on(r)[0])[0])
        me = blk[a]
        blk[a] = 0
        sdev, ddev = _a2a_devices(S, D, blk, a, b, k)
        grp = sorted(sdev)
        chunks = x.chunk(k, dim=b)  # chunk j belongs to the rank holding dst block j along b
        boxes = boxcopy.available(x)
        if boxes:  # one launch: every chunk into its group-rank slot of the send buffer
            inp = torch.empty((k,) + tuple(chunks[0].shape), dtype=x.dtype, device=x.device)
            self._box_plan("a2a_pack", x, inp, lambda: _view_boxes(
                [(chunks[ddev.index(g)], inp[i]) for i, g in enumerate(grp)], x, inp)).run(x, inp)
        else:
            inp = torch.stack([chunks[ddev.index(g)] for g in grp], 0).contiguous()
        out = torch.empty_like(inp)
        h = dist.all_to_all_single(out, inp, group=comm.group(grp), async_op=True)

        def finish():
            # out[q] came from group rank q, which holds src block sdev.index(grp[q]) along a
            if boxes:  # one launch: each received block into its slice along a
                shp = list(out.shape[1:])
                shp[a] *= k
                res = torch.empty(shp, dtype=out.dtype, device=out.device)
                ca = out.shape[1 + a]
                self._box_plan("a2a_unpack", out, res, lambda: _view_boxes(
                    [(out[grp.index(sdev[i])], res.narrow(a, i * ca, ca)) for i in range(k)], out, res)).run(out, res)
                return res
            return torch.cat([out[grp.index(sdev[i])] for i in range(k)], dim=a).contiguous()
        del me
        return Pending([h], finish, kind="all_to_all", nbytes=self.bytes_moved(x.element_size()))

    def _reduce_scatter(self, comm, x):
        S, D, d, r = self.src, self.dst, self.dim, self.rank
        blk, _ = S.coords(S.parts_on(r)[0])
        k = S.replicas
        grp = sorted(S.replica_group(blk))
        # order of fine sub-blocks by group rank
        sub_dev = []
        for j in range(k):
            fb = list(blk)
            fb[d] = blk[d] * k + j
            sub_dev.append(D.devices[D.part_index(fb, 0)])
        xm = x.movedim(d, 0)
        chunks = list(xm.chunk(k, 0))
        order = [sub_dev.index(g) for g in grp]  # chunk for group-rank i
        boxes = boxcopy.available(x)
        if order == list(range(k)) and xm.is_contiguous():
            inp = xm
        elif boxes:  # one launch: the chunks, dim d first, in group-rank order
            inp = torch.empty(tuple(xm.shape), dtype=x.dtype, device=x.device)
            m0 = chunks[0].shape[0]
            self._box_plan("rs_pack", x, inp, lambda: _view_boxes(
                [(chunks[j], inp.narrow(0, i * m0, m0)) for i, j in enumerate(order)], x, inp)).run(x, inp)
        else:
            inp = torch.cat([chunks[j] for j in order], 0).contiguous() if order != list(range(k)) else xm.contiguous()
        out_shape = list(inp.shape)
        out_shape[0] //= k
        out = torch.empty(out_shape, dtype=x.dtype, device=x.device)
        g = comm.group(grp)
        nb = self.bytes_moved(x.element_size())
        # one code path for every backend: RCCL on the GPU, gloo in the CPU multi-rank tests
        h = dist.reduce_scatter_tensor(out, inp, group=g, async_op=True)

        def finish():
            if d == 0:
                return out
            if boxes:  # one launch: dim d back in place
                res = torch.empty(tuple(out.movedim(0, d).shape), dtype=out.dtype, device=out.device)
                self._box_plan("rs_unpack", out, res, lambda: _view_boxes([(out.movedim(0, d), res)], out, res)
                               ).run(out, res)
                return res
            return out.movedim(0, d).contiguous()
        return Pending([h], finish, kind="reduce_scatter", nbytes=nb)

    def _all_gather(self, comm, x):
        S, D, d, r = self.src, self.dst, self.dim, self.rank
        k = D.replicas
        qblk, _ = D.coords(D.parts_on(r)[0])
        grp = sorted(D.replica_group(qblk))
        sub_dev = []
        for j in range(k):
            fb = list(qblk)
            fb[d] = qblk[d] * k + j
            sub_dev.append(S.devices[S.part_index(fb, 0)])
        boxes = boxcopy.available(x)
        xv = x.movedim(d, 0)
        if xv.is_contiguous():
            xm = xv
        elif boxes:  # one launch: dim d first (the collective's contiguous send buffer)
            xm = torch.empty(tuple(xv.shape), dtype=x.dtype, device=x.device)
            self._box_plan("ag_pack", x, xm, lambda: _view_boxes([(xv, xm)], x, xm)).run(x, xm)
        else:
            xm = xv.contiguous()
        g = comm.group(grp)
        nb = self.bytes_moved(x.element_size())
        out = torch.empty((k * xm.shape[0],) + tuple(xm.shape[1:]), dtype=x.dtype, device=x.device)
        h = dist.all_gather_into_tensor(out, xm, group=g, async_op=True)
        chunks = list(out.chunk(k, 0))

        def finish():
            # chunks[i] came from group-rank i == device grp[i]; reorder to dim order
            order = [grp.index(dev) for dev in sub_dev]
            if d == 0 and order == list(range(k)):
                return out
            if boxes:  # one launch: every block into its slice along d, in dim order
                shp = list(x.shape)
                shp[d] *= k
                res = torch.empty(shp, dtype=out.dtype, device=out.device)
                m0 = xv.shape[0]
                self._box_plan("ag_unpack", out, res, lambda: _view_boxes(
                    [(chunks[c].movedim(0, d), res.narrow(d, j * m0, m0)) for j, c in enumerate(order)], out, res)
                ).run(out, res)
                return res
            ordered = [chunks[c] for c in order]
            return torch.cat(ordered, 0).movedim(0, d).contiguous()
        return Pending([h], finish, kind="all_gather", nbytes=nb)

    def _generic(self, comm, x, like):
        S, D, r = self.src, self.dst, self.rank
        dparts = D.parts_on(r)
        sparts = S.parts_on(r)
        ref = x if x is not None else like
        out = None
        if dparts:
            q = dparts[0]
            # without partial sums or halos the overlaps tile the destination block: no zero fill
            # (a halo'd block reaching past the tensor's edge keeps zeros there)
            alloc = torch.zeros if (self.sp or D.halo or S.halo) else torch.empty
            out = alloc(D.local_shape(q), dtype=ref.dtype, device=ref.device)
        if boxcopy.available(ref):
            return self._generic_boxes(comm, x, out, ref)
        ops = []
        pending = []
        for it in self.items:
            sd, dd = S.devices[it.src_part], D.devices[it.dst_part]
            if sd != r and dd != r:
                continue
            if sd == r and dd == r:
                src_view = x[_slices(it.region, S.region(it.src_part))]
                dst_view = out[_slices(it.region, D.region(it.dst_part))]
                if it.reduce:
                    dst_view.add_(src_view)
                else:
                    dst_view.copy_(src_view)
            elif sd == r:
                buf = x[_slices(it.region, S.region(it.src_part))].contiguous()
                ops.append(dist.P2POp(dist.isend, buf, dd))
                pending.append(("send", buf, None, None))
            else:
                shp = tuple(hi - lo for lo, hi in it.region)
                buf = torch.empty(shp, dtype=ref.dtype, device=ref.device)
                ops.append(dist.P2POp(dist.irecv, buf, sd))
                pending.append(("recv", buf, it, None))
        reqs = dist.batch_isend_irecv(ops) if ops else []

        def finish():
            for kind, buf, it, _ in pending:
                if kind == "recv":
                    dst_view = out[_slices(it.region, D.region(it.dst_part))]
                    if it.reduce:
                        dst_view.add_(buf)
                    else:
                        dst_view.copy_(buf)
            return out
        return Pending(reqs, finish, kind="generic", nbytes=sum(b.numel() * b.element_size()
                                                               for k_, b, _, _ in pending if k_ == "send"))


    # ------------------------------------------------------------------ box-copy kernels (GPU)
    def _box_plan(self, role, src, dst, build, disjoint_dst=False):
        """The cached BoxPlan of one side of this transfer for these tensor geometries."""
        plans = self.__dict__.setdefault("_plans", {})
        key = boxcopy.plan_key(role, src, dst)
        if key not in plans:
            plans[key] = boxcopy.BoxPlan(build(), src, dst, disjoint_dst=disjoint_dst)
        return plans[key]

    def _generic_boxes(self, comm, x, out, ref):
        """_generic with every send packed by one launch into one buffer (the isend buffers are its
        slices), every receive landing in one buffer unpacked by one launch per mode (copy / add),
        and the local overlaps moved by one launch per mode."""
        S, D, r = self.src, self.dst, self.rank
        sends, recvs, local = [], [], []
        for it in self.items:
            sd, dd = S.devices[it.src_part], D.devices[it.dst_part]
            if sd == r and dd == r:
                local.append(it)
            elif sd == r:
                sends.append(it)
            elif dd == r:
                recvs.append(it)
        for mode in (False, True):
            loc = [it for it in local if bool(it.reduce) == mode]
            # add mode: one launch per layer of pairwise-disjoint destination regions (the add kernel
            # read-modify-writes dst with no atomics, so two boxes on one region would race)
            for li, lay in enumerate(_disjoint_layers(loc) if mode else ([loc] if loc else [])):
                self._box_plan(f"local{int(mode)}.{li}", x, out, lambda lay=lay: [
                    boxcopy.region_box(x, rel_slices_lohi(it.region, S.region(it.src_part)))[:2]
                    + boxcopy.region_box(out, rel_slices_lohi(it.region, D.region(it.dst_part))) for it in lay
                ], disjoint_dst=True).run(x, out, add=mode)
        ops = []
        sbuf = None
        if sends:
            sbuf = torch.empty(sum(_numel(it.region) for it in sends), dtype=x.dtype, device=x.device)
            self._box_plan("gpack", x, sbuf, lambda: _pack_boxes(x, sends, S)).run(x, sbuf)
            off = 0
            for it in sends:
                n = _numel(it.region)
                ops.append(dist.P2POp(dist.isend, sbuf[off:off + n], D.devices[it.dst_part]))
                off += n
        rbuf = None
        if recvs:
            rbuf = torch.empty(sum(_numel(it.region) for it in recvs), dtype=ref.dtype, device=ref.device)
            off = 0
            for it in recvs:
                n = _numel(it.region)
                ops.append(dist.P2POp(dist.irecv, rbuf[off:off + n], S.devices[it.src_part]))
                off += n
        reqs = dist.batch_isend_irecv(ops) if ops else []

        def finish(_sent=sbuf):  # the send buffer lives until the transfer is waited for
            if recvs:
                offs, off = [], 0
                for it in recvs:
                    offs.append(off)
                    off += _numel(it.region)
                for mode in (False, True):
                    sel = [(o, it) for o, it in zip(offs, recvs) if bool(it.reduce) == mode]
                    lays = _disjoint_layers(sel, key=lambda oi: oi[1]) if mode else ([sel] if sel else [])
                    for li, lay in enumerate(lays):
                        self._box_plan(f"gunpack{int(mode)}.{li}", rbuf, out, lambda lay=lay: [
                            boxcopy.flat_box(o, [hi - lo for lo, hi in it.region])[:2]
                            + boxcopy.region_box(out, rel_slices_lohi(it.region, D.region(it.dst_part)))
                            for o, it in lay], disjoint_dst=True).run(rbuf, out, add=mode)
            return out
        return Pending(reqs, finish, kind="generic", nbytes=(sbuf.numel() * sbuf.element_size()) if sbuf is not None
                       else 0)


def _view_boxes(pairs, src, dst):
    """Boxes moving each (source view, destination view) pair of equal shape: views of `src` /
    `dst` built with ordinary view ops (movedim / narrow / chunk / index), their storage offsets
    and strides taken relative to the base tensors the plan is run on — the collective reorders
    (one launch each instead of ATen cat / stack / movedim copies)."""
    boxes = []
    for sv, dv in pairs:
        assert tuple(sv.shape) == tuple(dv.shape), (sv.shape, dv.shape)
        boxes.append((sv.storage_offset() - src.storage_offset(), tuple(sv.stride()),
                      dv.storage_offset() - dst.storage_offset(), tuple(dv.stride()), tuple(sv.shape)))
    return boxes


def _regions_overlap(a, b) -> bool:
    return all(lo1 < hi2 and lo2 < hi1 for (lo1, hi1), (lo2, hi2) in zip(a, b))


def _disjoint_layers(items, key=lambda it: it):
    """Greedy first-fit split of transfer items into layers whose destination regions are pairwise
    disjoint (same destination part): each layer can be one add-mode box launch without a race.
    Partial-sum replicas all target one region and 2-D halo gradients overlap at the corners, so
    these plans do produce overlapping adds (layout.plan_transfer)."""
    layers = []
    for e in items:
        it = key(e)
        for lay in layers:
            if not any(key(o).dst_part == it.dst_part and _regions_overlap(key(o).region, it.region) for o in lay):
                lay.append(e)
                break
        else:
            layers.append([e])
    return layers


def _numel(region) -> int:
    return int(math.prod(hi - lo for lo, hi in region))


def rel_slices_lohi(region, within):
    return [(lo - wl, hi - wl) for (lo, hi), (wl, _) in zip(region, within)]


def _pack_boxes(x, items, S):
    """Boxes moving each item's region of the local source block into consecutive slots of a flat
    buffer (item order)."""
    boxes, off = [], 0
    for it in items:
        so, ss, ext = boxcopy.region_box(x, rel_slices_lohi(it.region, S.region(it.src_part)))
        boxes.append((so, ss) + boxcopy.flat_box(off, ext))
        off += _numel(it.region)
    return boxes


def _unpack_boxes(out, items, D):
    boxes, off = [], 0
    for it in items:
        ext = [hi - lo for lo, hi in it.region]
        boxes.append(boxcopy.flat_box(off, ext)[:2] + boxcopy.region_box(out, rel_slices_lohi(it.region, D.region(it.dst_part))))
        off += _numel(it.region)
    return boxes


class _WidenBack:
    """Handle of a bf16 gradient collective: wait() waits for it, then widens the summed bf16
    bucket back into its fp32 arena slice (on the waiting stream)."""

    def __init__(self, handle, low, dst, keep=None):
        self.handle, self.low, self.dst, self.keep = handle, low, dst, keep
        self.done = False

    def wait(self):
        if not self.done:
            self.handle.wait()
            self.dst.copy_(self.low)
            self.done = True
            self.low = self.keep = None
        return True


class GradBucketer:
    """Bucketed, backward-overlapped gradient all-reduce over flat fp32 arenas.

    Each arena holds the gradients of all weight shards that share one replica group (e.g. every
    data-parallel weight); buckets are contiguous slices in reverse forward order so the first
    bucket completes early in the backward pass. Bucket size is chosen for xGMI ring all-reduce
    (config.grad_bucket_mb, default 64 MiB: few, large collectives).
    """

    def __init__(self, comm: Communicator, bucket_bytes: int, comm_dtype: Optional[torch.dtype] = None):
        self.comm = comm
        self.bucket_bytes = bucket_bytes
        # bf16 gradient collectives (--grad-comm-dtype bf16): the bucket travels as bf16 (half the
        # xGMI bytes) and is widened back into the fp32 arena, where the optimizer accumulates
        self.comm_dtype = comm_dtype if comm_dtype not in (None, torch.float32) else None
        self.arenas = []  # (group_ranks, flat_grad, [buckets]) ; bucket = dict(lo, hi, params:set, ready:set)
        self.param_bucket = {}
        self.param_buckets = {}  # sharded arenas: a parameter may straddle bucket boundaries
        self.handles = []
        self.on_ready = None  # callback(bucket, async handle or None) once a bucket's grads are final
        # callback() right before a completed bucket is reduced / handed to on_ready: the executor
        # launches the parameter-gradient folds it queued (kernels.fold_flush), which finish those grads
        self.before_launch = None

    def add_sharded_arena(self, group_ranks, flat, segments, rank):
        """ZeRO-1 arena (flexflow_amd/runtime/executor.py 'sharded optimizer'): buckets are fixed
        element ranges whose length is a multiple of R x 16 (R = replicas), each reduce-SCATTERED
        so rank r keeps the summed gradient of chunk r of every bucket. Returns the buckets."""
        R = len(group_ranks)
        unit = 16 * R
        n = flat.numel()
        assert n % unit == 0, (n, unit)
        be = max(unit, (self.bucket_bytes // 4 + unit - 1) // unit * unit)
        me = list(group_ranks).index(rank)
        buckets = []
        for lo in range(0, n, be):
            hi = min(n, lo + be)
            c = (hi - lo) // R
            b = dict(lo=lo, hi=hi, params=set(), ready=set(), flat=flat, group=group_ranks, sharded=True,
                     own=(lo + me * c, lo + (me + 1) * c))
            buckets.append(b)
        for key, lo, hi in segments:
            for b in buckets:
                if lo < b["hi"] and hi > b["lo"]:
                    b["params"].add(key)
                    self.param_buckets.setdefault(key, []).append(b)
        for b in buckets:
            if not b["params"]:  # padding only: nothing to wait for
                b["params"] = {("pad", b["lo"])}
                b["ready"] = set(b["params"])
        self.arenas.append((group_ranks, flat, buckets))
        return buckets

    def add_arena(self, group_ranks, flat, segments):
        """segments: list of (param_key, lo, hi) in gradient-completion order."""
        buckets = []
        cur = None
        for key, lo, hi in segments:
            if cur is None or (cur["hi"] - cur["lo"]) * 4 >= self.bucket_bytes:
                cur = dict(lo=lo, hi=hi, params=set(), ready=set(), flat=flat, group=group_ranks)
                buckets.append(cur)
            cur["lo"] = min(cur["lo"], lo)
            cur["hi"] = max(cur["hi"], hi)
            cur["params"].add(key)
            self.param_bucket[key] = cur
        self.arenas.append((group_ranks, flat, buckets))

    def reset(self):
        for _, _, buckets in self.arenas:
            for b in buckets:
                b["ready"] = {k for k in b["params"] if isinstance(k, tuple) and k[:1] == ("pad",)}
        self.handles = []

    def mark_ready(self, key):
        bs = self.param_buckets.get(key)
        if bs is None:
            b = self.param_bucket.get(key)
            bs = [b] if b is not None else []
        for b in bs:
            b["ready"].add(key)
            if len(b["ready"]) == len(b["params"]):
                if self.before_launch is not None:
                    self.before_launch()
                h = self._launch(b)
                if self.on_ready is not None:
                    self.on_ready(b, h)

    def _launch(self, b):
        if (len(b["group"]) <= 1 and not getattr(self.comm, "force", False)) or not self.comm.distributed:
            return None
        view = b["flat"][b["lo"]:b["hi"]]
        g = self.comm.group(b["group"])
        if self.comm_dtype is not None:
            low = view.to(self.comm_dtype)
            if b.get("sharded"):
                lo, hi = b["own"]
                out_low = torch.empty(hi - lo, dtype=self.comm_dtype, device=view.device)
                h = _WidenBack(dist.reduce_scatter_tensor(out_low, low, group=g, async_op=True), out_low,
                               b["flat"][lo:hi], keep=low)
            else:
                h = _WidenBack(dist.all_reduce(low, group=g, async_op=True), low, view)
        elif b.get("sharded"):  # in-place reduce-scatter: this rank's chunk of the bucket gets the sum
            out = b["flat"][b["own"][0]:b["own"][1]]
            h = dist.reduce_scatter_tensor(out, view, group=g, async_op=True)
        else:
            h = dist.all_reduce(view, group=g, async_op=True)
        self.handles.append(h)
        return h

    def flush(self):
        if self.before_launch is not None:
            self.before_launch()
        for _, _, buckets in self.arenas:
            for b in buckets:
                if len(b["ready"]) != len(b["params"]):
                    self._launch(b)
                    b["ready"] = set(b["params"])
        for h in self.handles:
            h.wait()
        self.handles = []
