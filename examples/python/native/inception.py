"""Inception-v3 (reference examples/cpp/InceptionV3/inception.cc, examples/python/native/inception.py)
written as tables of towers: every inception module is a list of towers, each tower a list of convs
(out_channels, kernel_h, kernel_w, stride, pad_h, pad_w), optionally preceded by a pool; the towers'
outputs are concatenated on channels. Synthetic 299 x 299 images (139 with --small).

    python examples/python/native/inception.py -b 64 --iterations 20
    python -m flexflow_amd.run --nproc 8 examples/python/native/inception.py -b 512 --search unity
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403

R = ActiMode.AC_MODE_RELU
AVG3 = ("avg", 3, 1, 1)   # 3x3 average pool, stride 1, pad 1
MAX3 = ("max", 3, 2, 0)   # 3x3 max pool, stride 2, no pad


def A(pool_ch):
    return [[(64, 1, 1, 1, 0, 0)],
            [(48, 1, 1, 1, 0, 0), (64, 5, 5, 1, 2, 2)],
            [(64, 1, 1, 1, 0, 0), (96, 3, 3, 1, 1, 1), (96, 3, 3, 1, 1, 1)],
            [AVG3, (pool_ch, 1, 1, 1, 0, 0)]]


B = [[(384, 3, 3, 2, 0, 0)],
     [(64, 1, 1, 1, 0, 0), (96, 3, 3, 1, 1, 1), (96, 3, 3, 2, 0, 0)],
     [MAX3]]


def C(c):
    row, col = (c, 1, 7, 1, 0, 3), (c, 7, 1, 1, 3, 0)
    return [[(192, 1, 1, 1, 0, 0)],
            [(c, 1, 1, 1, 0, 0), row, (192, 7, 1, 1, 3, 0)],
            [(c, 1, 1, 1, 0, 0), col, row, col, (192, 1, 7, 1, 0, 3)],
            [AVG3, (192, 1, 1, 1, 0, 0)]]


D = [[(192, 1, 1, 1, 0, 0), (320, 3, 3, 2, 0, 0)],
     [(192, 1, 1, 1, 0, 0), (192, 1, 7, 1, 0, 3), (192, 7, 1, 1, 3, 0), (192, 3, 3, 2, 0, 0)],
     [MAX3]]


def tower(ff, x, layers):
    for l in layers:
        if isinstance(l[0], str):
            kind, k, s, p = l
            x = ff.pool2d(x, k, k, s, s, p, p, PoolType.POOL_AVG if kind == "avg" else PoolType.POOL_MAX)
        else:
            c, kh, kw, s, ph, pw = l
            x = ff.conv2d(x, c, kh, kw, s, s, ph, pw, R)
    return x


def module(ff, x, towers):
    return ff.concat([tower(ff, x, t) for t in towers], 1)


def module_e(ff, x):
    """The E module forks twice: a 1x3 / 3x1 pair after the 1x1 and after the 3x3 tower."""
    a = tower(ff, x, [(384, 1, 1, 1, 0, 0)])
    b = tower(ff, x, [(448, 1, 1, 1, 0, 0), (384, 3, 3, 1, 1, 1)])
    fork = lambda t: [tower(ff, t, [(384, 1, 3, 1, 0, 1)]), tower(ff, t, [(384, 3, 1, 1, 1, 0)])]  # noqa: E731
    return ff.concat([tower(ff, x, [(320, 1, 1, 1, 0, 0)])] + fork(a) + fork(b) +
                     [tower(ff, x, [AVG3, (192, 1, 1, 1, 0, 0)])], 1)


def inception_v3(ff, x, classes=10):
    t = tower(ff, x, [(32, 3, 3, 2, 0, 0), (32, 3, 3, 1, 0, 0), (64, 3, 3, 1, 1, 1), MAX3,
                      (80, 1, 1, 1, 0, 0), (192, 3, 3, 1, 1, 1), MAX3])
    for towers in (A(32), A(64), A(64), B, C(128), C(160), C(160), C(192), D):
        t = module(ff, t, towers)
    t = module_e(ff, module_e(ff, t))
    side = t.dims[2]
    t = ff.pool2d(t, side, side, 1, 1, 0, 0, PoolType.POOL_AVG)
    return ff.softmax(ff.dense(ff.flat(t), classes))


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    side = 139 if small else 299
    x = ffmodel.create_tensor([ffconfig.batch_size, 3, side, side], DataType.DT_FLOAT)
    out = inception_v3(ffmodel, x)
    zoo.train("inception", ffconfig, ffmodel, [x], out, zoo.SCCE, zoo.ACC, iterations)
