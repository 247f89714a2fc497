"""Multi-process (gloo, world_size 2) parallelism tests on CPU.

Each case trains a tiny model for two SGD steps under a parallel strategy (data, tensor/operator,
attribute, vocab/parameter, placement, hybrid) and compares the resulting weights and outputs
with a single-process run — the strategy must not change the math (reference test strategy:
tests/multi_gpu_tests.sh runs the same models at 1..N GPUs).
"""
import json
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, strat_file, out_file):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    os.environ["CUDA_VISIBLE_DEVICES"] = ""
    import torch
    torch.set_num_threads(1)
    import dist_models
    res = dist_models.run(name, world, strat_file)
    if rank == 0:
        np.savez(out_file, **res)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _run_parallel(name, world=2):
    import dist_models
    from flexflow_amd.core import FFConfig, FFModel
    from flexflow_amd.pcg.strategy import save_strategy
    tmp = tempfile.mkdtemp()
    strat_file = None
    ff = FFModel(FFConfig([]))
    ff.config.batch_size = dist_models.B
    dist_models.build(name, ff)
    s = dist_models.strategy(name, ff, world)
    if s is not None:
        strat_file = os.path.join(tmp, "s.json")
        save_strategy(strat_file, s, world)
    out = os.path.join(tmp, "out.npz")
    mp.start_processes(_worker, args=(world, _free_port(), name, strat_file, out), nprocs=world, join=True,
                       start_method="spawn")
    return dict(np.load(out))


def _run_single(name):
    import dist_models
    old = {k: os.environ.pop(k, None) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    try:
        return dist_models.run(name, 1)
    finally:
        for k, v in old.items():
            if v is not None:
                os.environ[k] = v


@pytest.mark.parametrize("name", ["mlp", "mlp_tp", "mlp_place", "mlp_hybrid", "parops", "attn", "attn_tp", "cnn",
                                  "cnn_attr", "emb", "emb_vocab"])
def test_parallel_matches_single(name):
    base = name.split("_")[0]
    ref = _run_single(base)
    par = _run_parallel(name)
    for k, v in ref.items():
        assert k in par, k
        np.testing.assert_allclose(par[k], v, rtol=2e-4, atol=2e-5, err_msg=f"{name}: {k}")


def test_bf16_placement_get_weights(monkeypatch):
    """bf16 model whose ops all sit on rank 0 (a placement the search picks for tiny models): rank 1
    holds no shard, yet get_weights() must post the same (fp32 master) message sizes on both ranks."""
    monkeypatch.setenv("FF_TEST_DTYPE", "bf16")
    ref = _run_single("mlp")
    par = _run_parallel("mlp_place")
    for k, v in ref.items():
        np.testing.assert_allclose(par[k], v, rtol=2e-2, atol=2e-3, err_msg=k)
