"""Transformer encoder stack (reference examples/cpp/Transformer/transformer.cc): each layer is
self-attention followed by a bias-free dense ReLU and dense, and a final dense regresses one value per
position (MSE). Defaults: 12 layers, hidden 1024, 16 heads, sequence 512. Attention runs on the
flash-attention kernel. --small: 2 layers, hidden 64, 4 heads, sequence 16.

    python examples/python/native/transformer.py -b 8 --iterations 20
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403


def encoder(ff, x, layers, heads):
    h = x.dims[-1]
    t = x
    for _ in range(layers):
        t = ff.multihead_attention(t, t, t, h, heads, h // heads, h // heads)
        t = ff.dense(t, h, ActiMode.AC_MODE_RELU, use_bias=False)
        t = ff.dense(t, h, ActiMode.AC_MODE_NONE, use_bias=False)
    return ff.dense(t, 1, ActiMode.AC_MODE_NONE, use_bias=False)


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    seq, hidden, layers, heads = (16, 64, 2, 4) if small else (512, 1024, 12, 16)
    x = ffmodel.create_tensor([ffconfig.batch_size, seq, hidden], DataType.DT_FLOAT)
    out = encoder(ffmodel, x, layers, heads)
    zoo.train("transformer", ffconfig, ffmodel, [x], out, zoo.MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR],
              iterations)
