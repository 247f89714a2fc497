"""MLP_Unify (reference examples/cpp/MLP_Unify/mlp.cc): two independent 8-deep, 8192-wide bias-free
dense towers over two 1024-wide inputs, summed and passed through softmax. The two towers are the
branch-parallel case the search can place on disjoint GPU subsets. The reference times forward only;
this example trains. --small: 64-wide inputs, 3-deep 128-wide towers.

    python examples/python/native/mlp_unify.py -b 64 --iterations 20
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403


def towers(ff, x1, x2, widths):
    for i, w in enumerate(widths):
        act = ActiMode.AC_MODE_NONE if i + 1 == len(widths) else ActiMode.AC_MODE_RELU
        x1 = ff.dense(x1, w, act, use_bias=False)
        x2 = ff.dense(x2, w, act, use_bias=False)
    return ff.softmax(ff.add(x1, x2))


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    d = 64 if small else 1024
    x1 = ffmodel.create_tensor([ffconfig.batch_size, d], DataType.DT_FLOAT)
    x2 = ffmodel.create_tensor([ffconfig.batch_size, d], DataType.DT_FLOAT)
    out = towers(ffmodel, x1, x2, [128] * 3 if small else [8192] * 8)
    zoo.train("mlp_unify", ffconfig, ffmodel, [x1, x2], out, zoo.SCCE, zoo.ACC, iterations)
