"""ZeRO-1 sharded optimizer (--zero): data-parallel gradient buckets are reduce-scattered, each rank
updates its 1/R chunk of every bucket with Adam, and the compute copy is all-gathered back while
the next forward runs. Over gloo with 2 ranks the trained weights must match the all-reduce data
parallel run and a single-process run, and a checkpoint must hold the full (gathered) master."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
B = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(flags, steps=3, ckpt=None, resume=None):
    from flexflow_amd.core import (ActiMode, AdamOptimizer, DataType, FFConfig, FFModel, LossType,
                                   MetricsType)
    cfg = FFConfig(["--search", "dp", "--grad-bucket-mb", "0.02"] + flags)  # many small buckets
    cfg.batch_size = B
    ff = FFModel(cfg)
    x = ff.create_tensor([B, 40], DataType.DT_FLOAT)
    t = ff.dense(x, 64, ActiMode.AC_MODE_RELU, name="d1")
    t = ff.dense(t, 48, ActiMode.AC_MODE_RELU, name="d2")  # odd sizes: params straddle buckets
    ff.softmax(ff.dense(t, 10, name="d3"))
    ff.optimizer = AdamOptimizer(ff, 1e-2)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(0)
    x.set_tensor(ff, rng.standard_normal((B, 40)).astype(np.float32))
    ff.label_tensor.set_tensor(ff, rng.integers(0, 10, (B, 1)).astype(np.int32))
    if resume:
        ff.load_checkpoint(resume)
    for _ in range(steps):
        ff.train_step()
    res = {}
    for L in ff.layers:
        for i, w in enumerate(L.weights):
            res[f"{L.name}.{i}"] = np.asarray(w.get_weights(ff), dtype=np.float32)
    if ckpt:
        ff.save_checkpoint(ckpt)
    res["zero"] = np.array([int(bool(getattr(ff.executor, "zero", False)))])
    return res


def _worker(rank, world, port, flags, out_file, ckpt, steps=3, resume=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), FF_DIST_BACKEND="gloo")
    os.environ["CUDA_VISIBLE_DEVICES"] = ""
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    torch.set_num_threads(1)
    res = _train(flags, steps=steps, ckpt=ckpt, resume=resume)
    np.savez(out_file.replace(".npz", f"{rank}.npz"), **res)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _run(flags, world=2, ckpt=None, steps=3, resume=None):
    tmp = tempfile.mkdtemp()
    out = os.path.join(tmp, "out.npz")
    mp.start_processes(_worker, args=(world, _free_port(), flags, out, ckpt, steps, resume), nprocs=world, join=True,
                       start_method="spawn")
    return [dict(np.load(out.replace(".npz", f"{r}.npz"))) for r in range(world)]


def test_zero_matches_allreduce_dp_and_single(tmp_path):
    single = _train([])
    ar = _run([])
    zr = _run(["--zero"], ckpt=str(tmp_path / "ck"))
    assert zr[0]["zero"][0] == 1 and ar[0]["zero"][0] == 0
    for k, v in single.items():
        if k == "zero":
            continue
        for r in range(2):
            np.testing.assert_allclose(ar[r][k], v, rtol=1e-4, atol=1e-5, err_msg=f"dp rank{r} {k}")
            np.testing.assert_allclose(zr[r][k], v, rtol=1e-4, atol=1e-5, err_msg=f"zero rank{r} {k}")
    # each rank's checkpoint carries the full master, identical across ranks
    from safetensors.numpy import load_file
    a = load_file(str(tmp_path / "ck" / "rank0.safetensors"))
    b = load_file(str(tmp_path / "ck" / "rank1.safetensors"))
    for key in a:
        if key.endswith(".master"):
            np.testing.assert_array_equal(a[key], b[key])


@pytest.mark.parametrize("R,n", [(2, 1000), (4, 77)])
def test_sharded_bucket_geometry(R, n):
    """Bucket ranges tile the padded arena in multiples of 16 R, own chunks partition each bucket,
    and every parameter is registered with every bucket it overlaps."""
    import torch
    from flexflow_amd.parallel.comm import GradBucketer

    class _Comm:
        distributed = False
    unit = 16 * R
    size = (n * 3 + unit - 1) // unit * unit
    flat = torch.zeros(size)
    segs = [("a", 0, n), ("b", n, 2 * n), ("c", 2 * n, 3 * n)]
    bk = GradBucketer(_Comm(), bucket_bytes=4 * 3 * unit)
    bs = bk.add_sharded_arena(tuple(range(R)), flat, segs, rank=R - 1)
    assert bs[0]["lo"] == 0 and bs[-1]["hi"] == size
    for b0, b1 in zip(bs, bs[1:]):
        assert b0["hi"] == b1["lo"]
    for b in bs:
        c = (b["hi"] - b["lo"]) // R
        assert (b["hi"] - b["lo"]) % unit == 0 and b["own"] == (b["lo"] + (R - 1) * c, b["lo"] + R * c)
    for key, lo, hi in segs:
        touched = [b for b in bs if lo < b["hi"] and hi > b["lo"]]
        assert bk.param_buckets[key] == touched


def test_zero_checkpoint_resume_under_other_sharding(tmp_path):
    """A --zero checkpoint holds the gathered Adam state, so resuming it under a different bucket
    size, or without --zero, continues exactly like an uninterrupted run (advisor finding: the
    per-rank m/v used to be valid only on that rank's chunk of each bucket)."""
    ck = str(tmp_path / "ck")
    straight = _train([], steps=5)
    _run(["--zero"], ckpt=ck, steps=3)
    other_buckets = _run(["--zero", "--grad-bucket-mb", "0.005"], steps=2, resume=ck)
    no_zero = _run([], steps=2, resume=ck)
    for k, v in straight.items():
        if k == "zero":
            continue
        for r in range(2):
            np.testing.assert_allclose(other_buckets[r][k], v, rtol=1e-4, atol=1e-5, err_msg=f"zero->zero' rank{r} {k}")
            np.testing.assert_allclose(no_zero[r][k], v, rtol=1e-4, atol=1e-5, err_msg=f"zero->dp rank{r} {k}")


def test_zero_never_captured_in_hip_graph(monkeypatch):
    """--zero with FF_GRAPH_COLLECTIVES=1 must run eagerly: the per-layer all-gather waits live in
    Python and a replayed graph would read half-gathered weights."""
    from types import SimpleNamespace
    from flexflow_amd.runtime.graph import StepGraph
    monkeypatch.setenv("FF_GRAPH_COLLECTIVES", "1")
    ex = SimpleNamespace(zero=True, hooks=[], comm=SimpleNamespace(distributed=True),
                         device=SimpleNamespace(type="cuda"))
    m = SimpleNamespace(executor=ex, config=SimpleNamespace(hip_graphs=True))
    assert StepGraph(m).enabled() is False


def test_bucket_ready_callback_once_per_bucket_in_completion_order():
    """GradBucketer.on_ready (the overlapped optimizer update's trigger, Executor._on_bucket_ready)
    fires exactly once per bucket, when its last parameter is marked ready, in completion order;
    reset() re-arms every bucket for the next step; flush() never fires it."""
    import torch
    from flexflow_amd.parallel.comm import GradBucketer

    class _Comm:
        distributed = False
    flat = torch.zeros(64)
    segs = [("w3", 0, 8), ("w2", 8, 24), ("w1", 24, 40), ("w0", 40, 64)]  # backward-completion order
    bk = GradBucketer(_Comm(), bucket_bytes=4 * 20)  # a bucket closes once it holds >= 20 floats
    bk.add_arena((0,), flat, segs)
    assert [(b["lo"], b["hi"]) for b in bk.arenas[0][2]] == [(0, 24), (24, 64)]  # {w3, w2} {w1, w0}
    fired = []
    bk.on_ready = lambda b, h: fired.append((b["lo"], b["hi"], h))
    for step in range(2):
        bk.reset()
        fired.clear()
        bk.mark_ready("w3")
        assert fired == []  # w2 still pending in the first bucket
        bk.mark_ready("w2")
        bk.mark_ready("w1")
        assert fired == [(0, 24, None)]
        if step == 0:
            bk.mark_ready("w0")
            assert fired == [(0, 24, None), (24, 64, None)]
        bk.flush()  # step 1: w0 never marked (a frozen layer) -> update() updates that bucket itself
        assert len(fired) == (2 if step == 0 else 1)
