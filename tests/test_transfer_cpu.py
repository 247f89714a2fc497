"""Layout transfers executed over gloo by 4 processes (flexflow_amd/parallel/comm.py), each rank's
result against slicing the global tensor: the one-collective exchange (a split moved between dims
in halves, two dims at once, permuted placement), the generic P2P path (device-group changes, partial sums), and the
collective kinds. Reference counterpart: src/parallel_ops (Repartition / Combine / Replicate /
Reduction) over Legion region copies."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from flexflow_amd.parallel.comm import Transfer
from flexflow_amd.parallel.layout import Layout

W = 4
# (src layout, dst layout, src_partial, expected kind)
CASES = [
    (Layout((8, 12), (4, 1), 1, (0, 1, 2, 3)), Layout((8, 12), (2, 2), 1, (0, 1, 2, 3)), False, "exchange"),
    (Layout((8, 12), (2, 2), 1, (0, 1, 2, 3)), Layout((8, 12), (1, 4), 1, (3, 2, 1, 0)), False, "exchange"),
    (Layout((12, 5), (4, 1), 1, (1, 3, 0, 2)), Layout((12, 5), (4, 1), 1, (0, 1, 2, 3)), False, "exchange"),
    (Layout((4, 6, 8), (2, 1, 2), 1, (0, 1, 2, 3)), Layout((4, 6, 8), (1, 2, 2), 1, (1, 0, 3, 2)), False, "exchange"),
    (Layout((8, 16), (4, 1), 1, (0, 1, 2, 3)), Layout((8, 16), (1, 4), 1, (2, 0, 3, 1)), False, "all_to_all"),
    (Layout((8, 6), (2, 1), 1, (0, 1)), Layout((8, 6), (1, 2), 1, (2, 3)), False, "generic"),
    (Layout((8, 6), (1, 1), 4, (0, 1, 2, 3)), Layout((8, 6), (2, 2), 1, (3, 1, 2, 0)), True, "generic"),
    (Layout((8, 6), (1, 1), 4, (0, 1, 2, 3)), Layout((8, 6), (4, 1), 1, (0, 1, 2, 3)), True, "reduce_scatter"),
    (Layout((8, 6), (4, 1), 1, (0, 1, 2, 3)), Layout((8, 6), (1, 1), 4, (0, 1, 2, 3)), False, "all_gather"),
    # the reorders around the collectives: split dim != 0 (dim moved first and back) and permuted
    # device order (chunks out of group-rank order)
    (Layout((6, 8), (1, 1), 4, (0, 1, 2, 3)), Layout((6, 8), (1, 4), 1, (3, 1, 2, 0)), True, "reduce_scatter"),
    (Layout((6, 8), (1, 4), 1, (2, 0, 3, 1)), Layout((6, 8), (1, 1), 4, (0, 1, 2, 3)), False, "all_gather"),
    (Layout((4, 6, 8), (1, 1, 4), 1, (0, 1, 2, 3)), Layout((4, 6, 8), (1, 1, 1), 4, (0, 1, 2, 3)), False,
     "all_gather"),
]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _part(L, p, g):
    return g[tuple(slice(lo, hi) for lo, hi in L.region(p))]


def _worker(rank, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=W)
    from flexflow_amd.parallel.comm import Communicator
    comm = Communicator(rank, W)
    res = {}
    for i, (S, D, sp, kind) in enumerate(CASES):
        t = Transfer(S, D, sp, rank)
        comm.ensure_groups(t.rank_sets())
        g = torch.arange(int(np.prod(S.shape)), dtype=torch.float32).reshape(S.shape)
        sp_parts = S.parts_on(rank)
        x = None
        if sp_parts:
            x = _part(S, sp_parts[0], g).clone()
            if sp:
                x = x * (1 + rank)  # partial sums: rank r holds (1 + r) g
        y = t.run(comm, x, like=g)
        res[f"kind{i}"] = np.array([t.kind == kind])
        res[f"plans{i}"] = np.array([bool(t.__dict__.get("_plans"))])
        dp = D.parts_on(rank)
        if dp:
            ref = _part(D, dp[0], g) * (sum(1 + q for q in range(W)) if sp else 1)
            res[f"ok{i}"] = np.array([y is not None and tuple(y.shape) == tuple(ref.shape) and torch.equal(y, ref)])
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("boxes", [False, True])
def test_transfers_over_gloo(tmp_path, monkeypatch, boxes):
    """boxes: the exchange / generic packs, unpacks and local moves run as box-copy plans
    (parallel/boxcopy.py; on the GPU one transfer.hip launch each), emulated here on CPU tensors."""
    monkeypatch.setenv("FF_BOXCOPY_EMULATE", "1" if boxes else "0")
    mp.start_processes(_worker, args=(_port(), str(tmp_path)), nprocs=W, join=True, start_method="spawn")
    for r in range(W):
        d = dict(np.load(tmp_path / f"r{r}.npz"))
        for i in range(len(CASES)):
            assert bool(d[f"kind{i}"][0]), (r, i, "kind")
            if CASES[i][3] in ("exchange", "all_to_all") or i >= 9:
                # every rank packs / unpacks (exchange) or reorders around the collective (all-to-
                # all; reduce-scatter / all-gather along dim != 0 or out of group-rank order)
                # through box plans, not ATen cat / stack / movedim copies
                assert bool(d[f"plans{i}"][0]) == boxes, (r, i, "box plans")
            if f"ok{i}" in d:
                assert bool(d[f"ok{i}"][0]), (r, i, "value")


@pytest.mark.parametrize("cl", [False, True])
def test_concat_backward_dense_split(monkeypatch, cl):
    """Concat's backward splits its gradient into dense parts in dy's memory format with one box
    plan (ops/shape.py _split_dense; one transfer.hip launch on the GPU), equal to torch.split."""
    monkeypatch.setenv("FF_BOXCOPY_EMULATE", "1")
    from flexflow_amd.ops.shape import _split_dense

    class _Op:
        pass
    dy = torch.randn(2, 10, 3, 4)
    if cl:
        dy = dy.contiguous(memory_format=torch.channels_last)
    outs = _split_dense(_Op(), dy, [3, 5, 2], 1)
    for a, b in zip(outs, torch.split(dy, [3, 5, 2], 1)):
        assert torch.equal(a, b)
        assert a.is_contiguous(memory_format=torch.channels_last) if cl else a.is_contiguous()


def test_add_boxes_are_layered_by_disjoint_destinations():
    """overlapping add boxes must not share one launch. comm._disjoint_layers
    splits transfer items by exact region test; BoxPlan layers any add plan by destination spans."""
    from types import SimpleNamespace as NS

    from flexflow_amd.parallel import boxcopy
    from flexflow_amd.parallel.comm import _disjoint_layers
    it = lambda r, q=0: NS(region=r, dst_part=q)  # noqa: E731
    same = [it([(0, 4), (0, 6)]) for _ in range(3)]
    lays = _disjoint_layers(same)
    assert [len(l) for l in lays] == [1, 1, 1]
    corners = [it([(0, 5), (0, 5)]), it([(3, 8), (0, 5)]), it([(0, 5), (3, 8)]), it([(5, 8), (5, 8)])]
    lays = _disjoint_layers(corners)
    for lay in lays:
        for a in lay:
            for b in lay:
                assert a is b or not all(l1 < h2 and l2 < h1 for (l1, h1), (l2, h2) in zip(a.region, b.region))
    assert sum(len(l) for l in lays) == 4 and len(lays) >= 2
    assert len(_disjoint_layers([it([(0, 4)], 0), it([(0, 4)], 1)])) == 1  # different parts never clash
    # BoxPlan: the same overlapping boxes, emulated on CPU, give the sequential sum; spans layered
    x = torch.zeros(8, 8)
    flat = torch.ones(4 * 25)
    boxes = [boxcopy.flat_box(25 * i, (5, 5))[:2] + boxcopy.region_box(x, [(lo, lo + 5), (lo, lo + 5)])
             for i, lo in enumerate((0, 3, 0, 3))]
    plan = boxcopy.BoxPlan(boxes, flat, x)
    assert len(plan.add_layers) >= 2 and sorted(i for l in plan.add_layers for i in l) == [0, 1, 2, 3]
    plan.run(flat, x, add=True)
    ref = torch.zeros(8, 8)
    for lo in (0, 3, 0, 3):
        ref[lo:lo + 5, lo:lo + 5] += 1
    assert torch.equal(x, ref)
