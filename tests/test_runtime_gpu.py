"""Runtime pieces that only exist on the device path: the data loader's pinned-slot ring + H2D
prefetch on the context's h2d stream (reference SingleDataLoader, src/dataloader/dataloader.cc:
every batch must reach the GPU shard in order, across epoch boundaries), and the device context's
workspace arena."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_prefetching_loader_feeds_batches_in_order():
    import torch
    from flexflow_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    cfg = FFConfig(["--no-hip-graphs"])
    B = 16
    cfg.batch_size = B
    ff = FFModel(cfg)
    x = ff.create_tensor([B, 32], DataType.DT_FLOAT, name="x")
    t = ff.dense(x, 10, ActiMode.AC_MODE_NONE, name="d")
    ff.softmax(t, name="sm")
    ff.optimizer = SGDOptimizer(ff, 0.0)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    n = 5 * B + 7  # ragged tail: the epoch wraps before the partial batch
    data = np.arange(n * 32, dtype=np.float32).reshape(n, 32)
    dl = ff.create_data_loader(x, data)
    assert dl._ring is not None and dl._pinned is not None and dl._pinned[0].is_pinned()
    seen = []
    for _ in range(12):
        dl.next_batch(ff)
        ff.forward()  # the consumer runs on the compute stream after the staged copy
        torch.cuda.synchronize()
        got = ff.executor.inputs[x.guid].float().cpu().numpy()
        seen.append(int(got[0, 0]) // 32)
    starts = [(i % 5) * B for i in range(12)]
    assert seen == starts, (seen, starts)


def test_device_context_workspace_reused():
    import torch
    from flexflow_amd.runtime.device import DeviceContext
    ctx = DeviceContext.get(torch.device("cuda", 0))
    a = ctx.workspace("t", 1000)
    b = ctx.workspace("t", 500)
    assert b.data_ptr() == a.data_ptr()
    c = ctx.workspace("t", 4000)
    assert c.numel() == 4000 and ctx.workspace_bytes() >= 16000
    assert ctx.h2d is not None and ctx.side is not None


@pytest.mark.parametrize("bucket_mb", [64.0, 0.25])
def test_overlapped_update_matches_serial(bucket_mb):
    """--overlap-update (each gradient bucket's Adam slice on a side stream during the backward,
    runtime/executor.py _on_bucket_ready) trains bitwise like the single update after backward,
    with one bucket or many (0.25 MiB)."""
    import torch
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(overlap):
        flags = ["--dtype", "bf16", "--no-hip-graphs", "--grad-bucket-mb", str(bucket_mb),
                 "--overlap-update" if overlap else "--no-overlap-update"]
        cfg = FFConfig(flags)
        bc = BertConfig(hidden=128, heads=2, layers=2, ffn=512, vocab=500, max_pos=64, seq=64)
        cfg.batch_size = 4
        ff = FFModel(cfg)
        ids, pos, _ = build_bert(ff, 4, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (4, 64), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(64, dtype=np.int32), (4, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (4, 64, 1), dtype=np.int32))
        for _ in range(3):
            ff.train_step()
        torch.cuda.synchronize()
        ws = {f"{L.name}.{i}": np.asarray(w.get_weights(ff)) for L in ff.layers for i, w in enumerate(L.weights)}
        nb = sum(len(bs) for _, _, bs in ff.executor.bucketer.arenas)
        return ws, nb, ff.executor._upd_stream is not None

    a, nb, used = run(True)
    b, _, unused = run(False)
    assert used and not unused
    if bucket_mb < 1:
        assert nb > 4
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_sparse_embedding_sgd_matches_dense_gpu(monkeypatch):
    """Row-sparse SGD of the embedding tables (HIP sgd_sparse_rows: mark pass + owner update that
    clears the gradient rows; zero_gradients then skips the tables) matches the dense update,
    eagerly and under hipGraph replay (6 steps: 3 eager warm-up, capture, replays)."""
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    from flexflow_amd.models import build

    def run(sparse):
        if sparse:
            monkeypatch.delenv("FF_SPARSE_EMB", raising=False)
        else:
            monkeypatch.setenv("FF_SPARSE_EMB", "0")
        cfg = FFConfig(["--dtype", "bf16", "--hip-graphs"])
        cfg.batch_size = 64
        ff = FFModel(cfg)
        inputs, out, loss, mets, make_batch = build("dlrm", ff, 64, small=True)
        ff.optimizer = SGDOptimizer(ff, 0.05)
        ff.compile(loss_type=loss, metrics=mets)
        n = sum(len(v) for v in ff.executor._sparse_plan(ff.optimizer).values())
        rng = np.random.default_rng(0)
        for _ in range(6):
            arrs, lab = make_batch(rng)
            for t, a in zip(inputs, arrs):
                t.set_tensor(ff, a)
            ff.label_tensor.set_tensor(ff, lab)
            ff.train_step()
        return n, [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]

    n1, a = run(True)
    n0, b = run(False)
    assert n1 > 0 and n0 == 0
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6, err_msg=str(k))


def test_graph_trial_policy_matches_eager():
    """'auto' hipGraph policy for mid-length steps: capture on trial, time two replays, keep the
    graph only if it beats the eager step. Whatever it decides, the weights after 8 steps match an
    eager run, and the trial ends in a definite decision."""
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    from flexflow_amd.models import build

    def run(flags, trial):
        cfg = FFConfig(["--dtype", "bf16"] + flags)
        if trial:
            cfg.graph_min_step_ms, cfg.graph_trial_max_ms = 0.0, 1e9  # every step length is a trial
        cfg.batch_size = 64
        ff = FFModel(cfg)
        inputs, out, loss, mets, make_batch = build("dlrm", ff, 64, small=True)
        ff.optimizer = SGDOptimizer(ff, 0.05)
        ff.compile(loss_type=loss, metrics=mets)
        rng = np.random.default_rng(0)
        for _ in range(8):
            arrs, lab = make_batch(rng)
            for t, a in zip(inputs, arrs):
                t.set_tensor(ff, a)
            ff.label_tensor.set_tensor(ff, lab)
            ff.train_step()
        return ff, [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]

    ff, a = run([], True)
    sg = ff._step_graph
    assert sg.decision in (True, False) and len(sg.graph_ms) == 2, (sg.decision, sg.graph_ms)
    assert (sg.graph is not None) == sg.decision
    _, b = run(["--no-hip-graphs"], False)
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5, err_msg=str(k))


@pytest.mark.parametrize("model", ["mlp_unify", "candle_uno"])
def test_graph_captures_adam_update(model, monkeypatch):
    """The whole training step, Adam's overlapped per-bucket update included, captured into one
    hipGraph (the launches read the per-step alpha_t from a device scalar refreshed before each
    replay): after 8 steps the weights and the optimizer's step count match an eager run."""
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel
    from flexflow_amd.models import build
    monkeypatch.setenv("FF_GRAPH_UPDATE", "1")

    def run(flags):
        cfg = FFConfig(["--dtype", "bf16"] + flags)
        cfg.graph_min_step_ms = 1e9  # capture whatever the step length
        cfg.batch_size = 64
        ff = FFModel(cfg)
        inputs, out, loss, mets, make_batch = build(model, ff, 64, small=True)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=loss, metrics=mets)
        rng = np.random.default_rng(0)
        for _ in range(8):
            arrs, lab = make_batch(rng)
            for t, a in zip(inputs, arrs):
                t.set_tensor(ff, a)
            ff.label_tensor.set_tensor(ff, lab)
            ff.train_step()
        torch.cuda.synchronize()
        return ff, [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]

    ff, a = run(["--hip-graphs"])
    sg = ff._step_graph
    assert sg.graph is not None and not sg.failed
    assert ff.optimizer.alpha_dev is not None
    ffe, b = run(["--no-hip-graphs"])
    assert ff.optimizer.beta1_t == ffe.optimizer.beta1_t and ff.executor.step_idx == ffe.executor.step_idx
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6, err_msg=str(k))


@pytest.mark.parametrize("model", ["candle_uno", "dlrm"])
def test_begin_end_trace_replays_hipgraph(model):
    """FFConfig.begin_trace / end_trace (reference: Legion tracing): from the fourth iteration the
    recorded forward / zero_gradients / backward sequence replays as one hipGraph (captured in the
    fourth iteration, after two timed eager ones); weights after 6
    iterations match an untraced eager run. DLRM under SGD takes the row-sparse embedding update,
    whose host bookkeeping a replay would skip: its trace runs eagerly (same weights)."""
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    from flexflow_amd.models import build

    def run(trace):
        cfg = FFConfig(["--dtype", "bf16"] + ([] if trace else ["--no-hip-graphs"]))
        cfg.batch_size = 64
        ff = FFModel(cfg)
        inputs, out, loss, mets, make_batch = build(model, ff, 64, small=True)
        ff.optimizer = SGDOptimizer(ff, 0.05)
        ff.compile(loss_type=loss, metrics=mets)
        rng = np.random.default_rng(0)
        for _ in range(6):
            arrs, lab = make_batch(rng)
            for t, a in zip(inputs, arrs):
                t.set_tensor(ff, a)
            ff.label_tensor.set_tensor(ff, lab)
            if trace:
                cfg.begin_trace(111)
            ff.forward()
            ff.zero_gradients()
            ff.backward()
            ff.update()
            if trace:
                cfg.end_trace(111)
        return cfg, [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]

    cfg, a = run(True)
    st = cfg._trace_state[111]
    assert st.seq == ["forward", "zero_gradients", "backward"]
    if model == "dlrm":
        assert st.graph is None and st.off
    else:
        assert st.graph is not None and not st.off
    _, b = run(False)
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5, err_msg=str(k))


def test_deferred_gradient_folds_match_inline(monkeypatch):
    """FF_DEFER_FOLDS=1: the bias / LayerNorm column folds and split-K slab sums of the backward
    run on the overlapped update's side stream (executor.backward). Weights after 4 train steps of
    a small BERT equal the inline-fold run's (same kernels, same order per gradient)."""
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(defer):
        monkeypatch.setenv("FF_DEFER_FOLDS", "1" if defer else "0")
        cfg = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
        cfg.batch_size = 4
        ff = FFModel(cfg)
        bc = BertConfig(vocab=512, hidden=128, layers=2, heads=2, ffn=512, seq=64)
        ids, pos, _ = build_bert(ff, 4, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (4, bc.seq), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (4, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (4, bc.seq, 1), dtype=np.int32))
        for _ in range(4):
            ff.train_step()
        torch.cuda.synchronize()
        return ff, [np.asarray(w.get_weights(ff), dtype=np.float32) for L in ff.layers for w in L.weights]

    from flexflow_amd import kernels as K
    n0 = K.reductions_deferred()
    _, a = run(True)
    assert K.reductions_deferred() > n0  # the folds did go to the side stream
    _, b = run(False)
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6, err_msg=str(k))


_RCCL_CHILD = r'''
import json, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.getcwd())
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
from flexflow_amd.models.bert import BertConfig, build_bert
cfg = FFConfig(["--dtype", "bf16", "--grad-bucket-mb", "1"])
B = 4
cfg.batch_size = B
ff = FFModel(cfg)
bc = BertConfig(hidden=128, heads=4, layers=2, ffn=512, vocab=256, max_pos=64, seq=64)
ids, pos, _ = build_bert(ff, B, bc)
ff.optimizer = AdamOptimizer(ff, 1e-3)
ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
ex = ff.executor
rng = np.random.default_rng(0)
ids.set_tensor(ff, rng.integers(0, bc.vocab, (B, bc.seq), dtype=np.int32))
pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (B, 1)))
ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (B, bc.seq, 1), dtype=np.int32))
calls = {"n": 0}
orig = dist.all_reduce
def counting(*a, **k):
    calls["n"] += 1
    return orig(*a, **k)
dist.all_reduce = counting
for _ in range(8):
    ff.train_step()
torch.cuda.synchronize()
sg = ff._step_graph
w = np.concatenate([np.asarray(x.get_weights(ff), dtype=np.float32).ravel() for L in ff.layers for x in L.weights])
print("RESULT " + json.dumps({"distributed": ex.comm.distributed, "backend": ex.comm.backend,
                              "captured": sg is not None and sg.graph is not None, "failed": bool(sg and sg.failed),
                              "buckets": sum(len(b) for _, _, b in ex.bucketer.arenas), "all_reduce_calls": calls["n"],
                              "wsum": float(np.abs(w).sum()), "w0": w[:64].tolist()}), flush=True)
dist.destroy_process_group()
'''


def _rccl_child(graph_collectives):
    import json
    import os
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               FF_FORCE_COLLECTIVES="1", FF_GRAPH_COLLECTIVES=graph_collectives, HSA_ENABLE_IPC_MODE_LEGACY="0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _RCCL_CHILD], cwd=root, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = r.stdout + r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[7:]), out


def test_world1_rccl_step_graph_captures_collectives():
    """the multi-rank hipGraph path (bucket all-reduces issued inside the capture and
    joined by bucketer.flush, capture success agreed with _agree) on a world-1 RCCL process group
    in a fresh process: the step is captured (no fallback), every replay still all-reduces, and
    8 steps train like the eager distributed step (FF_GRAPH_COLLECTIVES=0)."""
    g, out_g = _rccl_child("1")
    e, _ = _rccl_child("0")
    assert g["distributed"] and g["backend"] == "nccl", g
    assert g["captured"] and not g["failed"], out_g[-2000:]
    assert "capture failed" not in out_g
    assert g["buckets"] >= 2 and g["all_reduce_calls"] >= g["buckets"], g
    assert not e["captured"] and e["all_reduce_calls"] >= 8 * e["buckets"], e
    np.testing.assert_allclose(g["w0"], e["w0"], rtol=2e-2, atol=2e-4)
    assert abs(g["wsum"] - e["wsum"]) <= 1e-3 * abs(e["wsum"])


def _conv_chain_train(monkeypatch, fuse):
    import numpy as np
    from flexflow_amd.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    monkeypatch.setenv("FF_CONV_DACT_FUSION", "1" if fuse else "0")
    cfg = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
    B = 8
    cfg.batch_size = B
    ff = FFModel(cfg)
    x = ff.create_tensor([B, 16, 20, 20], DataType.DT_FLOAT, name="x")
    t = ff.conv2d(x, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    t = ff.conv2d(t, 48, 3, 3, 2, 2, 1, 1, ActiMode.AC_MODE_RELU, name="c2")   # stride-phase dgrad
    t = ff.conv2d(t, 64, 1, 7, 1, 1, 0, 3, ActiMode.AC_MODE_RELU, name="c3")
    t = ff.conv2d(t, 32, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_NONE, name="c4")
    t = ff.flat(t, name="f")
    t = ff.dense(t, 10, name="d")
    ff.softmax(t, name="sm")
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(0)
    x.set_tensor(ff, rng.standard_normal((B, 16, 20, 20)).astype(np.float32))
    ff.label_tensor.set_tensor(ff, rng.integers(0, 10, (B, 1)).astype(np.int32))
    fused = sum(1 for c in ff.executor.ctx.values() if c.extra.get("dact_fused"))
    for _ in range(4):  # the first backward tunes each site (unfused), later ones take the fused dgrad
        ff.train_step()
    torch.cuda.synchronize()
    w = {L.name: [np.asarray(p.get_weights(ff), dtype=np.float32) for p in L.weights] for L in ff.layers if L.weights}
    return fused, w


def test_conv_dact_fusion_matches_unfused(monkeypatch):
    """Conv -> Conv (Executor._plan_dact_fusion): the consumer's dgrad epilogue applies the
    producer's ReLU and sums its bias gradient (conv.hip IGemmArgs.dmask / dpart) — four SGD steps
    land where the separate mask + channel-sum pass does."""
    nf, wf = _conv_chain_train(monkeypatch, True)
    nu, wu = _conv_chain_train(monkeypatch, False)
    assert nf == 3 and nu == 0, (nf, nu)
    for name in wu:
        for a, b in zip(wf[name], wu[name]):
            np.testing.assert_allclose(a, b, rtol=2e-2, atol=2e-3, err_msg=name)


def test_batched_gradient_folds_match_inline_folds(monkeypatch):
    """FF_FOLD_BATCH (default on): the LayerNorm / bias gradient folds of a training backward are
    queued and launched a few per kernel (kernels.fold_flush, before each gradient bucket and at the
    end of the backward). Same per-fold arithmetic as the inline fold: every weight gradient of a
    small BERT bitwise equal with batching on and off (same forward, same tuned kernels); and the
    overlapped train_step path (bucket-ready flushes) gives the same losses."""
    from flexflow_amd import kernels as Kn
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def make():
        torch.manual_seed(0)
        cfg = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
        bc = BertConfig(hidden=256, heads=4, layers=2, ffn=1024, vocab=1024, max_pos=128, seq=128)
        cfg.batch_size = 4
        ff = FFModel(cfg)
        ids, pos, _ = build_bert(ff, 4, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (4, bc.seq), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (4, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (4, bc.seq, 1), dtype=np.int32))
        return ff

    ff = make()
    grads = []
    for on in ("1", "0"):
        monkeypatch.setenv("FF_FOLD_BATCH", on)
        ff.forward()
        ff.zero_gradients()
        ff.backward()
        torch.cuda.synchronize()
        assert Kn._FOLDQ["keep"] == [] and not Kn._FOLDQ["on"]
        grads.append({(li, i): ff.executor.get_weight_grad(w).detach().clone()
                      for li, L in enumerate(ff.layers) for i, w in enumerate(L.weights)})
    n_fold = 0
    for k, g in grads[0].items():
        if g.dim() == 1:
            n_fold += 1
        if "embed" in type(ff.layers[k[0]].impl).__name__.lower():
            continue  # the embedding backward adds with float atomics: order varies run to run
        assert torch.equal(g, grads[1][k]), k
    assert n_fold >= 8  # LayerNorm gammas / betas and biases took the batched path

    losses = []
    for on in ("1", "0"):
        monkeypatch.setenv("FF_FOLD_BATCH", on)
        f2 = make()
        ls = []
        for _ in range(3):
            f2.reset_metrics()
            f2.train_step()
            ls.append(f2.get_perf_metrics().get_loss())
        torch.cuda.synchronize()
        losses.append(np.array(ls))
    assert np.allclose(losses[0], losses[1], rtol=1e-3), losses


def test_batched_conv_bias_folds_match_inline(monkeypatch):
    """The channel-last conv bias-gradient fold (the [S][C] partials of nhwc_colred) joins the
    batched folds (fold_queue) instead of its finalize launch. A pool-free conv net (every reduction
    in its backward fixed-order): after an autotuning pass, two backward passes with batching on and
    off give bitwise-equal weight gradients and bias gradients equal up to fp32 summation order."""
    from flexflow_amd.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType,
                                   SGDOptimizer)
    from flexflow_amd import kernels as Kn
    torch.manual_seed(0)
    cfg = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
    B = 8
    cfg.batch_size = B
    ff = FFModel(cfg)
    x = ff.create_tensor([B, 64, 32, 32], DataType.DT_FLOAT, name="x")
    t = ff.conv2d(x, 64, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
    t = ff.conv2d(t, 128, 3, 3, 2, 2, 1, 1, ActiMode.AC_MODE_RELU, name="c2")
    t = ff.conv2d(t, 128, 1, 1, 1, 1, 0, 0, ActiMode.AC_MODE_RELU, name="c3")
    t = ff.flat(t, name="fl")
    t = ff.dense(t, 10, ActiMode.AC_MODE_NONE, name="fc")
    ff.softmax(t, name="sm")
    ff.optimizer = SGDOptimizer(ff, 0.0)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(1)
    x.set_tensor(ff, rng.standard_normal((B, 64, 32, 32)).astype(np.float32))
    ff.label_tensor.set_tensor(ff, rng.integers(0, 10, (B, 1), dtype=np.int32))
    grads = []
    for on in ("0", "1", "0"):  # the first pass autotunes the kernels (its outputs come from trials)
        monkeypatch.setenv("FF_FOLD_BATCH", on)
        ff.forward()
        ff.zero_gradients()
        ff.backward()
        torch.cuda.synchronize()
        assert Kn._FOLDQ["keep"] == []
        grads.append({(L.name, i): ff.executor.get_weight_grad(w).detach().float().clone()
                      for L in ff.layers for i, w in enumerate(L.weights)})
    assert torch.equal(grads[0][("c1", 0)], grads[2][("c1", 0)])  # the backward is deterministic
    nb = 0
    for k, g in grads[1].items():
        ref = grads[2][k]
        if g.dim() == 1:
            nb += 1
            assert torch.allclose(g, ref, rtol=1e-5, atol=1e-6 * max(1e-3, ref.abs().max().item())), k
        else:
            assert torch.equal(g, ref), k
    assert nb >= 3
