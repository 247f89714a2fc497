"""LSTM op (flexflow_amd/ops/rnn.py; the reference's LSTM is its legacy nmt/ application): forward
and backward of the op against torch.nn.LSTM autograd, gradients flowing from all three outputs,
and the NMT seq2seq model training through FFModel."""
import numpy as np
import pytest
import torch

from flexflow_amd.ops.base import OpCtx
from flexflow_amd.ops.rnn import LSTM


@pytest.mark.parametrize("B,L,E,H", [(3, 5, 4, 6), (2, 1, 8, 8), (4, 7, 16, 5)])
def test_lstm_op_matches_torch(B, L, E, H):
    torch.manual_seed(0)
    x, hx, cx = torch.randn(B, L, E), torch.randn(B, H), torch.randn(B, H)
    wih, whh, b = torch.randn(4 * H, E) * 0.3, torch.randn(4 * H, H) * 0.3, torch.randn(4 * H) * 0.1
    op = LSTM.__new__(LSTM)
    ctx = OpCtx(layer=None, part_coords=(0, 0, 0), degrees=(1, 1, 1))
    dW = [torch.zeros(4 * H, E), torch.zeros(4 * H, H), torch.zeros(4 * H)]
    ctx.wgrads = dW
    y, hy, cy = op.forward(ctx, [x, hx, cx], [wih, whh, b])
    m = torch.nn.LSTM(E, H, batch_first=True)
    with torch.no_grad():
        m.weight_ih_l0.copy_(wih)
        m.weight_hh_l0.copy_(whh)
        m.bias_ih_l0.copy_(b)
        m.bias_hh_l0.zero_()
    xt, h0, c0 = x.clone().requires_grad_(), hx[None].clone().requires_grad_(), cx[None].clone().requires_grad_()
    yt, (hn, cn) = m(xt, (h0, c0))
    torch.testing.assert_close(y, yt.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(hy, hn[0].detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(cy, cn[0].detach(), rtol=1e-5, atol=1e-6)
    gy, ghy, gcy = torch.randn(B, L, H), torch.randn(B, H), torch.randn(B, H)
    torch.autograd.backward([yt, hn[0], cn[0]], [gy, ghy, gcy])
    dx, dhx, dcx = op.backward(ctx, [gy, ghy, gcy])
    torch.testing.assert_close(dx, xt.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dhx, h0.grad[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dcx, c0.grad[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dW[0], m.weight_ih_l0.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dW[1], m.weight_hh_l0.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dW[2], m.bias_ih_l0.grad, rtol=1e-4, atol=1e-5)


def test_lstm_no_output_grads():
    """Only hy used downstream: dy = None / dcy = None paths."""
    torch.manual_seed(1)
    B, L, E, H = 2, 4, 3, 5
    op = LSTM.__new__(LSTM)
    ctx = OpCtx(layer=None, part_coords=(0, 0, 0), degrees=(1, 1, 1))
    ctx.wgrads = [torch.zeros(4 * H, E), torch.zeros(4 * H, H), torch.zeros(4 * H)]
    x, hx, cx = torch.randn(B, L, E), torch.zeros(B, H), torch.zeros(B, H)
    w = [torch.randn(4 * H, E) * 0.3, torch.randn(4 * H, H) * 0.3, torch.zeros(4 * H)]
    op.forward(ctx, [x, hx, cx], w)
    m = torch.nn.LSTM(E, H, batch_first=True, bias=False)
    with torch.no_grad():
        m.weight_ih_l0.copy_(w[0])
        m.weight_hh_l0.copy_(w[1])
    xt = x.clone().requires_grad_()
    _, (hn, _) = m(xt)
    g = torch.randn(B, H)
    hn[0].backward(g)
    dx, _, _ = op.backward(ctx, [None, g, None])
    torch.testing.assert_close(dx, xt.grad, rtol=1e-4, atol=1e-5)


def test_nmt_seq2seq_trains():
    from flexflow_amd.core import FFConfig, FFModel
    from flexflow_amd.models.rnn import NMTConfig, build_nmt, nmt_batch
    cfg = FFConfig(["--device", "cpu"])
    nc = NMTConfig(vocab=50, embed=16, hidden=16, layers=2, src_len=6, dst_len=5)
    cfg.batch_size = 8
    ff = FFModel(cfg)
    src, dst, _ = build_nmt(ff, 8, nc)
    from flexflow_amd.core import AdamOptimizer, LossType, MetricsType
    ff.optimizer = AdamOptimizer(ff, 0.01)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    s, d, lab = nmt_batch(8, nc, np.random.default_rng(0))  # target = source reversed (learnable copy task)
    src.set_tensor(ff, s)
    dst.set_tensor(ff, d)
    ff.label_tensor.set_tensor(ff, lab)
    losses = []
    for _ in range(30):
        ff.reset_metrics()
        ff.train_step()
        losses.append(ff.get_perf_metrics().get_loss())
    assert losses[-1] < 0.7 * losses[0], losses
