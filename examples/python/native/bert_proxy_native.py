"""BERT proxy (reference examples/python/native/bert_proxy_native.py + bert_proxy_run_script.sh):
a stack of encoder-shaped layers (Q/K/V dense -> reshape/transpose -> batch_matmul attention ->
dense, residual adds, a wide intermediate dense) ending in a single-neuron dense, timed forward
passes in inference mode; `--train` also runs backward and the optimizer. The full BERT model
(embeddings, LayerNorm, fused attention, MLM head) is flexflow_amd.models.bert / bench.py.

    python examples/python/native/bert_proxy_native.py -b 8 --seq-length 128 --hidden-size 1024 \
        --num-heads 16 --num_layers 4 --iterations 10 [--search unity --enable-parameter-parallel]
"""
import argparse
import sys

import _args  # noqa: F401  (puts the repo root on sys.path)
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def mha(model, x, b, s, h, nh):
    kd = h // nh
    q = model.transpose(model.reshape(model.dense(x, h), (b, s, nh, kd)), (0, 2, 1, 3))
    k = model.transpose(model.reshape(model.dense(x, h), (b, s, nh, kd)), (0, 2, 3, 1))
    v = model.transpose(model.reshape(model.dense(x, h), (b, s, nh, kd)), (0, 2, 1, 3))
    logits = model.batch_matmul(q, k, a_seq_length_dim=2, b_seq_length_dim=3)
    out = model.batch_matmul(logits, v, a_seq_length_dim=3, b_seq_length_dim=2)
    out = model.reshape(model.transpose(out, (0, 2, 1, 3)), (b, s, h))
    return model.dense(out, h, ActiMode.AC_MODE_GELU)


def bert_layer(model, x, b, s, h, nh):
    t = mha(model, x, b, s, h, nh)
    t = model.add(model.dense(t, h, ActiMode.AC_MODE_GELU), x)
    inter = model.dense(t, h, ActiMode.AC_MODE_GELU)
    return model.add(model.dense(inter, h, ActiMode.AC_MODE_GELU), inter)


def top_level_task(argv=None):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--seq-length", type=int, default=512)
    ap.add_argument("--num-heads", type=int, default=16)
    ap.add_argument("--hidden-size", type=int, default=1024)
    ap.add_argument("--num_layers", type=int, default=24)
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--train", action="store_true")
    args, rest = ap.parse_known_args(sys.argv[1:] if argv is None else argv)
    ffconfig = FFConfig(rest)
    ffmodel = FFModel(ffconfig)
    b, s, h = ffconfig.batch_size, args.seq_length, args.hidden_size
    print(f"Model config: seq_length {s} hidden_size {h} num_heads {args.num_heads} layers {args.num_layers}")
    x = ffmodel.create_tensor([b, s, h], DataType.DT_FLOAT)
    t = x
    for _ in range(args.num_layers):
        t = bert_layer(ffmodel, t, b, s, h, args.num_heads)
    t = ffmodel.dense(t, 1)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 1e-3)
    ffmodel.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE,
                    metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR],
                    comp_mode=CompMode.TRAINING if args.train else CompMode.INFERENCE)
    rng = np.random.default_rng(0)
    x.set_tensor(ffmodel, rng.standard_normal((b, s, h)).astype(np.float32) * 0.1)
    ffmodel.label_tensor.set_tensor(ffmodel, np.zeros((b, s, 1), np.float32))
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    for it in range(args.iterations):
        ffconfig.begin_trace(111)
        if args.train:
            ffmodel.train_step()
        else:
            ffmodel.forward(seq_length=it)
        ffconfig.end_trace(111)
    out = np.asarray(t.get_tensor(ffmodel))  # host read-back: waits for the device
    elapsed = 1e-6 * (ffconfig.get_current_time() - ts)
    print(f" Time per iteration: {elapsed / args.iterations * 1e3:.3f} ms (output {out.shape})")
    return out


if __name__ == "__main__":
    top_level_task()
