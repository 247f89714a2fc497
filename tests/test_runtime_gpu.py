"""Runtime pieces that only exist on the device path: the data loader's pinned-slot ring + H2D
prefetch on the context's h2d stream (reference SingleDataLoader, src/dataloader/dataloader.cc:
every batch must reach the GPU shard in order, across epoch boundaries), and the device context's
workspace arena."""
import numpy as np
import pytest

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
