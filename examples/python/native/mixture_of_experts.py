"""Mixture of experts (reference examples/cpp/mixture_of_experts/moe.cc,
examples/python/native/mixture_of_experts.py) with the routing spelled out op by op: a ReLU gate
scores the experts, top_k picks `k` of them per sample (softmax-normalised weights), group_by scatters the samples to per-expert
batches (capacity alpha * k / n of the batch), each expert is a dense layer, and aggregate combines
the expert outputs with the gate weights and adds the load-balance loss (lambda_bal). MNIST-sized
inputs (784), 5 experts, top-2. --small: 64-wide inputs, 32-wide experts.

    python examples/python/native/mixture_of_experts.py -b 64 --iterations 20
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403


def moe_layer(ff, x, experts, k, hidden, alpha=2.0, lambda_bal=0.04):
    gate = ff.dense(x, experts, ActiMode.AC_MODE_RELU)
    weights, assign = ff.top_k(gate, k, False)
    groups = ff.group_by(x, assign, experts, alpha)
    outs = [ff.softmax(ff.dense(g, hidden, ActiMode.AC_MODE_RELU)) for g in groups]
    return ff.aggregate([ff.softmax(weights), assign, assign, gate] + outs, experts, lambda_bal)


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    d, hidden = (64, 32) if small else (784, 784)
    x = ffmodel.create_tensor([ffconfig.batch_size, d], DataType.DT_FLOAT)
    t = moe_layer(ffmodel, x, experts=5, k=2, hidden=hidden)
    out = ffmodel.softmax(ffmodel.dense(t, 10, ActiMode.AC_MODE_RELU))
    zoo.train("mixture_of_experts", ffconfig, ffmodel, [x], out, zoo.SCCE, zoo.ACC, iterations)
