"""CPU reference paths of the NCHW batch-norm / pooling kernels (flexflow_amd.kernels; the HIP
kernels are checked against the same torch references in tests/test_kernels_gpu.py)."""
import itertools

import numpy as np
import pytest
import torch

from flexflow_amd import kernels as K


@pytest.mark.parametrize("relu", [True, False])
def test_batchnorm_reference_matches_torch(relu):
    torch.manual_seed(0)
    x = torch.randn(4, 3, 5, 6) * 2 + 1
    g, b = torch.rand(3) + 0.5, torch.randn(3)
    rm, rv = torch.zeros(3), torch.ones(3)
    y, mean, rstd = K.batchnorm_fwd(x, g, b, rm, rv, True, relu)
    xr, gr, br = (t.clone().requires_grad_() for t in (x, g, b))
    rm2, rv2 = torch.zeros(3), torch.ones(3)
    ref = torch.nn.functional.batch_norm(xr, rm2, rv2, gr, br, training=True, momentum=0.1, eps=1e-5)
    ref = torch.relu(ref) if relu else ref
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rm, rm2)
    torch.testing.assert_close(rv, rv2)
    dy = torch.randn_like(x)
    ref.backward(dy)
    dg, db = torch.zeros(3), torch.zeros(3)
    dx = K.batchnorm_bwd(x, dy, g, b, mean, rstd, dg, db, relu)
    torch.testing.assert_close(dx, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-5)


def _naive_pool(x, k, s, pads, is_max, include_pad):
    """Direct loops over windows with torch's divisor rules (count_include_pad)."""
    N, C, H, W = x.shape
    pt, pb, pl, pr = pads
    OH, OW = K.pool_out_size(H, k, s, pt, pb), K.pool_out_size(W, k, s, pl, pr)
    y = np.zeros((N, C, OH, OW), np.float64)
    xn = x.double().numpy()
    for oh, ow in itertools.product(range(OH), range(OW)):
        h0, w0 = oh * s - pt, ow * s - pl
        rows = [h for h in range(h0, h0 + k) if 0 <= h < H]
        cols = [w for w in range(w0, w0 + k) if 0 <= w < W]
        win = xn[:, :, rows][:, :, :, cols]
        if is_max:
            y[:, :, oh, ow] = win.max((2, 3))
        else:
            h1, w1 = min(h0 + k, H + pb), min(w0 + k, W + pr)
            div = (h1 - h0) * (w1 - w0) if include_pad else len(rows) * len(cols)
            y[:, :, oh, ow] = win.sum((2, 3)) / div
    return torch.from_numpy(y).float()


@pytest.mark.parametrize("pads", [(1, 1, 1, 1), (1, 0, 0, 1), (0, 0, 0, 0), (2, 1, 0, 2)])
@pytest.mark.parametrize("is_max,inc", [(True, True), (False, True), (False, False)])
def test_pool_reference_asymmetric_pads(pads, is_max, inc):
    torch.manual_seed(1)
    x = torch.randn(2, 3, 9, 8)
    y, _ = K.pool2d_fwd(x, 3, 3, 2, 2, pads, is_max, inc, False, False)
    torch.testing.assert_close(y, _naive_pool(x, 3, 2, pads, is_max, inc), rtol=1e-5, atol=1e-6)
    dy = torch.randn_like(y)
    dx = K.pool2d_bwd(x, y, dy, None, 3, 3, 2, 2, pads, is_max, inc, False)
    assert dx.shape == x.shape
    # adjoint check: <dy, pool(x)> is linear in x for average pooling
    if not is_max:
        x2 = torch.randn_like(x)
        y2, _ = K.pool2d_fwd(x2, 3, 3, 2, 2, pads, is_max, inc, False, False)
        assert abs((dy * y2).sum().item() - (dx * x2).sum().item()) < 1e-4
