"""Channel-last vs NCHW pooling backward on one input: per-config error and where it sits."""
import sys
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import torch
from flexflow_amd import kernels as K

torch.manual_seed(0)
for (k, s, p, is_max, inc, relu) in [(3, 1, 1, False, True, False), (3, 2, 1, False, True, False),
                                     (2, 2, 0, False, True, False), (3, 1, 1, True, True, False),
                                     (1, 1, 0, False, True, False), (3, 1, 0, False, True, False)]:
    x = torch.randn(2, 16, 9, 7, device="cuda").bfloat16()
    xc = x.contiguous(memory_format=torch.channels_last)
    K.CHANNELS_LAST = False
    y0, i0 = K.pool2d_fwd(x, k, k, s, s, (p,) * 4, is_max, inc, relu, True)
    dy = torch.randn_like(y0)
    dx0 = K.pool2d_bwd(x, y0, dy, i0, k, k, s, s, (p,) * 4, is_max, inc, relu)
    K.CHANNELS_LAST = True
    y1, i1 = K.pool2d_fwd(xc, k, k, s, s, (p,) * 4, is_max, inc, relu, True)
    dx1 = K.pool2d_bwd(xc, y1, dy, i1, k, k, s, s, (p,) * 4, is_max, inc, relu)
    torch.cuda.synchronize()
    e = (dx1.float() - dx0.float()).abs()
    bad = (e > 1e-2).nonzero()
    print(k, s, p, is_max, "fwd", (y1.float() - y0.float()).abs().max().item(), "bwd", e.max().item(),
          "nbad", bad.shape[0], "first", bad[:6].tolist(), flush=True)
    if bad.shape[0]:
        n, c, h, w = bad[0].tolist()
        print("   dx0", dx0[n, c, h, :].float().tolist())
        print("   dx1", dx1[n, c, h, :].float().tolist())
