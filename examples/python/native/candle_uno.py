"""CANDLE Uno (reference examples/cpp/candle_uno/candle_uno.cc): drug-response regression. The two
dose scalars pass straight through; the cell RNA-seq profile and each drug's descriptors and
fingerprints go through their own 8-deep dense encoder (4192 wide); everything is concatenated and
a 4-deep dense head regresses one value (MSE). --small: 64-wide, 2-deep encoders and head.

    python examples/python/native/candle_uno.py -b 256 --iterations 20
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403

FEATURES = [("cell.rnaseq", 942), ("dose1", 1), ("dose2", 1),
            ("drug1.descriptors", 5270), ("drug1.fingerprints", 2048),
            ("drug2.descriptors", 5270), ("drug2.fingerprints", 2048)]


def dense_stack(ff, t, widths):
    for w in widths:
        t = ff.dense(t, w, ActiMode.AC_MODE_RELU, use_bias=False)
    return t


def candle_uno(ff, inputs, encoder, head):
    parts = [x if name.startswith("dose") else dense_stack(ff, x, encoder)
             for (name, _), x in zip(FEATURES, inputs)]
    t = dense_stack(ff, ff.concat(parts, -1), head)
    return ff.dense(t, 1, ActiMode.AC_MODE_NONE, use_bias=False)


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    inputs = [ffmodel.create_tensor([ffconfig.batch_size, n], DataType.DT_FLOAT, name=name)
              for name, n in FEATURES]
    out = candle_uno(ffmodel, inputs, [64] * 2 if small else [4192] * 8, [64] * 2 if small else [4192] * 4)
    zoo.train("candle_uno", ffconfig, ffmodel, inputs, out, zoo.MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR],
              iterations)
