"""ResNeXt-50 (reference examples/cpp/resnext50/resnext.cc): stages of grouped-convolution blocks
(1x1 -> grouped 3x3 carrying the stride -> 1x1 expanding to twice the width), 32 groups, 1000 classes
on 224 x 224 synthetic images (64 x 64, 4 groups, 10 classes with --small). As in the reference
example the blocks carry no shortcut.

    python examples/python/native/resnext50.py -b 64 --iterations 20
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403

R, NONE = ActiMode.AC_MODE_RELU, ActiMode.AC_MODE_NONE


def block(ff, x, width, stride, groups):
    t = ff.conv2d(x, width, 1, 1, 1, 1, 0, 0, R)
    t = ff.conv2d(t, width, 3, 3, stride, stride, 1, 1, R, groups)
    return ff.conv2d(t, 2 * width, 1, 1, 1, 1, 0, 0, NONE)


def resnext50(ff, x, groups=32, classes=1000):
    t = ff.conv2d(x, 64, 7, 7, 2, 2, 3, 3, R)
    t = ff.pool2d(t, 3, 3, 2, 2, 1, 1)
    for width, blocks, stride in ((128, 3, 1), (256, 4, 2), (512, 6, 2), (1024, 3, 2)):
        for b in range(blocks):
            t = block(ff, t, width, stride if b == 0 else 1, groups)
    t = ff.relu(t, False)
    t = ff.pool2d(t, t.dims[2], t.dims[3], 1, 1, 0, 0, PoolType.POOL_AVG)
    return ff.softmax(ff.dense(ff.flat(t), classes))


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    side = 64 if small else 224
    x = ffmodel.create_tensor([ffconfig.batch_size, 3, side, side], DataType.DT_FLOAT)
    out = resnext50(ffmodel, x, groups=4 if small else 32, classes=10 if small else 1000)
    zoo.train("resnext50", ffconfig, ffmodel, [x], out, zoo.SCCE, zoo.ACC, iterations)
