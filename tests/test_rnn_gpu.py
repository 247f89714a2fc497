"""LSTM step kernels (csrc/kernels/rnn.hip) and the LSTM op on the GPU against torch.nn.LSTM in fp32
(fp32 and bf16 compute), and the NMT zoo model stepping on cuda:0."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,L,E,H", [(4, 6, 32, 64), (16, 10, 128, 256)])
def test_lstm_op_gpu(ffC, dtype, B, L, E, H):
    from flexflow_amd.ops.base import OpCtx
    from flexflow_amd.ops.rnn import LSTM
    torch.manual_seed(0)
    x, hx, cx = torch.randn(B, L, E), torch.randn(B, H), torch.randn(B, H)
    wih, whh, b = torch.randn(4 * H, E) / E ** 0.5, torch.randn(4 * H, H) / H ** 0.5, torch.randn(4 * H) * 0.1
    op = LSTM.__new__(LSTM)
    ctx = OpCtx(layer=None, part_coords=(0, 0, 0), degrees=(1, 1, 1))
    dW = [torch.zeros(4 * H, E, device=DEV), torch.zeros(4 * H, H, device=DEV), torch.zeros(4 * H, device=DEV)]
    ctx.wgrads = dW
    d = lambda t: t.to(DEV, dtype)  # noqa: E731
    y, hy, cy = op.forward(ctx, [d(x), d(hx), d(cx)], [d(wih), d(whh), d(b)])
    m = torch.nn.LSTM(E, H, batch_first=True)
    with torch.no_grad():
        m.weight_ih_l0.copy_(wih)
        m.weight_hh_l0.copy_(whh)
        m.bias_ih_l0.copy_(b)
        m.bias_hh_l0.zero_()
    xt, h0, c0 = x.clone().requires_grad_(), hx[None].clone().requires_grad_(), cx[None].clone().requires_grad_()
    yt, (hn, cn) = m(xt, (h0, c0))
    tol = 1e-4 if dtype == torch.float32 else 5e-2
    rel = lambda a, r: ((a.float().cpu() - r).norm() / (r.norm() + 1e-12)).item()  # noqa: E731
    assert rel(y, yt.detach()) < tol and rel(hy, hn[0].detach()) < tol and rel(cy, cn[0].detach()) < tol
    gy, ghy, gcy = torch.randn(B, L, H), torch.randn(B, H), torch.randn(B, H)
    torch.autograd.backward([yt, hn[0], cn[0]], [gy, ghy, gcy])
    dx, dhx, dcx = op.backward(ctx, [d(gy), d(ghy), d(gcy)])
    gt = 1e-4 if dtype == torch.float32 else 6e-2
    assert rel(dx, xt.grad) < gt and rel(dhx, h0.grad[0]) < gt and rel(dcx, c0.grad[0]) < gt
    for g, r in zip(dW, (m.weight_ih_l0.grad, m.weight_hh_l0.grad, m.bias_ih_l0.grad)):
        assert rel(g, r) < gt


def test_nmt_steps_on_gpu(ffC):
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    from flexflow_amd.models import build
    cfg = FFConfig(["--dtype", "bf16"])
    cfg.batch_size = 16
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build("nmt", ff, 16, small=True)
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=loss, metrics=mets)
    assert ff.executor.device.type == "cuda"
    arrs, lab = make_batch(np.random.default_rng(0))
    for t, a in zip(inputs, arrs):
        t.set_tensor(ff, a)
    ff.label_tensor.set_tensor(ff, lab)
    for _ in range(3):
        ff.reset_metrics()
        ff.train_step()
    torch.cuda.synchronize()
    assert np.isfinite(ff.get_perf_metrics().get_loss())
