"""Multi-head attention two ways (reference examples/python/native/multi_head_attention.py):
`--explicit` builds it from dense / reshape / transpose / batch_matmul layers as the reference
script does; the default uses the fused multihead_attention op (flash attention on the device).
MSE regression to a synthetic target.

    python examples/python/native/multi_head_attention.py -b 8 --seq-length 256 --hidden-size 512
"""
import argparse
import sys

import _args  # noqa: F401  (puts the repo root on sys.path)
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def top_level_task(argv=None):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--seq-length", type=int, default=256)
    ap.add_argument("--num-heads", type=int, default=16)
    ap.add_argument("--hidden-size", type=int, default=512)
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--explicit", action="store_true")
    args, rest = ap.parse_known_args(sys.argv[1:] if argv is None else argv)
    ffconfig = FFConfig(rest)
    ffmodel = FFModel(ffconfig)
    b, s, h, nh = ffconfig.batch_size, args.seq_length, args.hidden_size, args.num_heads
    x = ffmodel.create_tensor([b, s, h], DataType.DT_FLOAT)
    if args.explicit:
        q, k, v = (ffmodel.dense(x, h) for _ in range(3))
        q = ffmodel.transpose(ffmodel.reshape(q, (b, s, nh, h // nh)), (0, 2, 1, 3))
        k = ffmodel.transpose(ffmodel.reshape(k, (b, s, nh, h // nh)), (0, 2, 3, 1))
        v = ffmodel.transpose(ffmodel.reshape(v, (b, s, nh, h // nh)), (0, 2, 1, 3))
        logits = ffmodel.softmax(ffmodel.batch_matmul(q, k))
        t = ffmodel.batch_matmul(logits, v)
        t = ffmodel.reshape(ffmodel.transpose(t, (0, 2, 1, 3)), (b, s, h))
    else:
        t = ffmodel.multihead_attention(x, x, x, h, nh, h // nh, h // nh)
    t = ffmodel.dense(t, h, ActiMode.AC_MODE_RELU)
    t = ffmodel.dense(t, h)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
                    metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    rng = np.random.default_rng(0)
    x.set_tensor(ffmodel, rng.standard_normal((b, s, h)).astype(np.float32))
    ffmodel.label_tensor.set_tensor(ffmodel, rng.standard_normal((b, s, h)).astype(np.float32) * 0.1)
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    for _ in range(args.iterations):
        ffmodel.train_step()
    pm = ffmodel.get_perf_metrics()
    run_time = 1e-6 * (ffconfig.get_current_time() - ts)
    print("attention: %d iterations, %.4fs, THROUGHPUT = %.2f samples/s, loss %.4f" %
          (args.iterations, run_time, b * args.iterations / run_time, pm.get_loss()))
    return pm


if __name__ == "__main__":
    top_level_task()
