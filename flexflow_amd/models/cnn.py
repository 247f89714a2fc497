"""Convolutional model zoo built on the FFModel API: AlexNet, ResNet-50, ResNeXt-50 (32x4d-style
grouped bottlenecks) and Inception-v3 — the reference's examples/cpp/{AlexNet,ResNet,resnext50,
InceptionV3} and examples/python/native/{alexnet,resnet,inception}.py.

Differences from the reference, on purpose:
  * ResNet: the reference comments every batch_norm out (examples/cpp/ResNet/resnet.cc:41-55) because
    OP_BATCHNORM has no case in its create_operator_from_layer (model.cc:2605-2783). Ours has
    BatchNorm, so `batch_norm=True` builds the standard network; the default (False) mirrors the
    reference graph exactly.
  * Every builder takes the input dims, so CIFAR-sized smoke variants reuse the same code.
"""
from __future__ import annotations

from ..type import ActiMode, DataType, PoolType

RELU = ActiMode.AC_MODE_RELU
NONE = ActiMode.AC_MODE_NONE


def build_alexnet(ff, batch: int, image_hw: int = 229, num_classes: int = 10, dtype=DataType.DT_FLOAT):
    """examples/cpp/AlexNet/alexnet.cc:61-79 (input 3x229x229, 10 classes)."""
    x = ff.create_tensor([batch, 3, image_hw, image_hw], dtype)
    t = ff.conv2d(x, 64, 11, 11, 4, 4, 2, 2, RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = ff.conv2d(t, 192, 5, 5, 1, 1, 2, 2, RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = ff.conv2d(t, 384, 3, 3, 1, 1, 1, 1, RELU)
    t = ff.conv2d(t, 256, 3, 3, 1, 1, 1, 1, RELU)
    t = ff.conv2d(t, 256, 3, 3, 1, 1, 1, 1, RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = ff.flat(t)
    t = ff.dense(t, 4096, RELU)
    t = ff.dense(t, 4096, RELU)
    t = ff.dense(t, num_classes)
    t = ff.softmax(t)
    return x, t


def _bottleneck(ff, x, out_channels, stride, batch_norm):
    """examples/cpp/ResNet/resnet.cc:39-59."""
    t = ff.conv2d(x, out_channels, 1, 1, 1, 1, 0, 0, NONE)
    if batch_norm:
        t = ff.batch_norm(t)
    t = ff.conv2d(t, out_channels, 3, 3, stride, stride, 1, 1, NONE)
    if batch_norm:
        t = ff.batch_norm(t)
    t = ff.conv2d(t, 4 * out_channels, 1, 1, 1, 1, 0, 0)
    if batch_norm:
        t = ff.batch_norm(t, relu=False)
    if stride > 1 or x.dims[1] != out_channels * 4:
        x = ff.conv2d(x, 4 * out_channels, 1, 1, stride, stride, 0, 0, NONE)
        if batch_norm:
            x = ff.batch_norm(x, relu=False)
    return ff.relu(ff.add(x, t), False)


def build_resnet50(ff, batch: int, image_hw: int = 224, num_classes: int = 10, batch_norm: bool = False,
                   dtype=DataType.DT_FLOAT):
    """examples/cpp/ResNet/resnet.cc:90-113 (3-4-6-3 bottlenecks)."""
    x = ff.create_tensor([batch, 3, image_hw, image_hw], dtype)
    t = ff.conv2d(x, 64, 7, 7, 2, 2, 3, 3)
    if batch_norm:
        t = ff.batch_norm(t)
    t = ff.pool2d(t, 3, 3, 2, 2, 1, 1)
    for stage, (ch, n) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3))):
        for i in range(n):
            t = _bottleneck(ff, t, ch, 2 if (i == 0 and stage > 0) else 1, batch_norm)
    hw = t.dims[2]
    t = ff.pool2d(t, hw, hw, 1, 1, 0, 0, PoolType.POOL_AVG)
    t = ff.flat(t)
    t = ff.dense(t, num_classes)
    t = ff.softmax(t)
    return x, t


def _resnext_block(ff, x, stride, out_channels, groups, has_residual=False):
    """examples/cpp/resnext50/resnext.cc:12-32."""
    t = ff.conv2d(x, out_channels, 1, 1, 1, 1, 0, 0, RELU)
    t = ff.conv2d(t, out_channels, 3, 3, stride, stride, 1, 1, RELU, groups)
    t = ff.conv2d(t, 2 * out_channels, 1, 1, 1, 1, 0, 0, NONE)
    if (stride > 1 or x.dims[1] != out_channels * 2) and has_residual:
        x = ff.conv2d(x, 2 * out_channels, 1, 1, stride, stride, 0, 0, RELU)
        t = ff.relu(ff.add(x, t), False)
    return t


def build_resnext50(ff, batch: int, image_hw: int = 224, num_classes: int = 1000, groups: int = 32,
                    dtype=DataType.DT_FLOAT):
    """examples/cpp/resnext50/resnext.cc:57-87."""
    x = ff.create_tensor([batch, 3, image_hw, image_hw], dtype)
    t = ff.conv2d(x, 64, 7, 7, 2, 2, 3, 3, RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 1, 1, PoolType.POOL_MAX)
    for ch, n, s0 in ((128, 3, 1), (256, 4, 2), (512, 6, 2), (1024, 3, 2)):
        for i in range(n):
            t = _resnext_block(ff, t, s0 if i == 0 else 1, ch, groups)
    t = ff.relu(t, False)
    t = ff.pool2d(t, t.dims[2], t.dims[3], 1, 1, 0, 0, PoolType.POOL_AVG)
    t = ff.flat(t)
    t = ff.dense(t, num_classes)
    t = ff.softmax(t)
    return x, t


# ------------------------------------------------------------------ Inception-v3
def _inception_a(ff, x, pool_features):
    t1 = ff.conv2d(x, 64, 1, 1, 1, 1, 0, 0, RELU)
    t2 = ff.conv2d(x, 48, 1, 1, 1, 1, 0, 0, RELU)
    t2 = ff.conv2d(t2, 64, 5, 5, 1, 1, 2, 2, RELU)
    t3 = ff.conv2d(x, 64, 1, 1, 1, 1, 0, 0, RELU)
    t3 = ff.conv2d(t3, 96, 3, 3, 1, 1, 1, 1, RELU)
    t3 = ff.conv2d(t3, 96, 3, 3, 1, 1, 1, 1, RELU)
    t4 = ff.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG)
    t4 = ff.conv2d(t4, pool_features, 1, 1, 1, 1, 0, 0, RELU)
    return ff.concat([t1, t2, t3, t4], 1)


def _inception_b(ff, x):
    t1 = ff.conv2d(x, 384, 3, 3, 2, 2, 0, 0)
    t2 = ff.conv2d(x, 64, 1, 1, 1, 1, 0, 0)
    t2 = ff.conv2d(t2, 96, 3, 3, 1, 1, 1, 1)
    t2 = ff.conv2d(t2, 96, 3, 3, 2, 2, 0, 0)
    t3 = ff.pool2d(x, 3, 3, 2, 2, 0, 0)
    return ff.concat([t1, t2, t3], 1)


def _inception_c(ff, x, ch):
    t1 = ff.conv2d(x, 192, 1, 1, 1, 1, 0, 0)
    t2 = ff.conv2d(x, ch, 1, 1, 1, 1, 0, 0)
    t2 = ff.conv2d(t2, ch, 1, 7, 1, 1, 0, 3)
    t2 = ff.conv2d(t2, 192, 7, 1, 1, 1, 3, 0)
    t3 = ff.conv2d(x, ch, 1, 1, 1, 1, 0, 0)
    t3 = ff.conv2d(t3, ch, 7, 1, 1, 1, 3, 0)
    t3 = ff.conv2d(t3, ch, 1, 7, 1, 1, 0, 3)
    t3 = ff.conv2d(t3, ch, 7, 1, 1, 1, 3, 0)
    t3 = ff.conv2d(t3, 192, 1, 7, 1, 1, 0, 3)
    t4 = ff.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG)
    t4 = ff.conv2d(t4, 192, 1, 1, 1, 1, 0, 0)
    return ff.concat([t1, t2, t3, t4], 1)


def _inception_d(ff, x):
    t1 = ff.conv2d(x, 192, 1, 1, 1, 1, 0, 0)
    t1 = ff.conv2d(t1, 320, 3, 3, 2, 2, 0, 0)
    t2 = ff.conv2d(x, 192, 1, 1, 1, 1, 0, 0)
    t2 = ff.conv2d(t2, 192, 1, 7, 1, 1, 0, 3)
    t2 = ff.conv2d(t2, 192, 7, 1, 1, 1, 3, 0)
    t2 = ff.conv2d(t2, 192, 3, 3, 2, 2, 0, 0)
    t3 = ff.pool2d(x, 3, 3, 2, 2, 0, 0)
    return ff.concat([t1, t2, t3], 1)


def _inception_e(ff, x):
    t1 = ff.conv2d(x, 320, 1, 1, 1, 1, 0, 0)
    t2i = ff.conv2d(x, 384, 1, 1, 1, 1, 0, 0)
    t2 = ff.conv2d(t2i, 384, 1, 3, 1, 1, 0, 1)
    t3 = ff.conv2d(t2i, 384, 3, 1, 1, 1, 1, 0)
    t3i = ff.conv2d(x, 448, 1, 1, 1, 1, 0, 0)
    t3i = ff.conv2d(t3i, 384, 3, 3, 1, 1, 1, 1)
    t4 = ff.conv2d(t3i, 384, 1, 3, 1, 1, 0, 1)
    t5 = ff.conv2d(t3i, 384, 3, 1, 1, 1, 1, 0)
    t6 = ff.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG)
    t6 = ff.conv2d(t6, 192, 1, 1, 1, 1, 0, 0)
    return ff.concat([t1, t2, t3, t4, t5, t6], 1)


def build_inception_v3(ff, batch: int, image_hw: int = 299, num_classes: int = 10, dtype=DataType.DT_FLOAT):
    """examples/cpp/InceptionV3/inception.cc:26-174 (3xA, B, 4xC, D, 2xE)."""
    x = ff.create_tensor([batch, 3, image_hw, image_hw], dtype)
    t = ff.conv2d(x, 32, 3, 3, 2, 2, 0, 0, RELU)
    t = ff.conv2d(t, 32, 3, 3, 1, 1, 0, 0, RELU)
    t = ff.conv2d(t, 64, 3, 3, 1, 1, 1, 1, RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = ff.conv2d(t, 80, 1, 1, 1, 1, 0, 0, RELU)
    t = ff.conv2d(t, 192, 3, 3, 1, 1, 1, 1, RELU)
    t = ff.pool2d(t, 3, 3, 2, 2, 0, 0)
    t = _inception_a(ff, t, 32)
    t = _inception_a(ff, t, 64)
    t = _inception_a(ff, t, 64)
    t = _inception_b(ff, t)
    for ch in (128, 160, 160, 192):
        t = _inception_c(ff, t, ch)
    t = _inception_d(ff, t)
    t = _inception_e(ff, t)
    t = _inception_e(ff, t)
    hw = t.dims[2]
    t = ff.pool2d(t, hw, hw, 1, 1, 0, 0, PoolType.POOL_AVG)
    t = ff.flat(t)
    t = ff.dense(t, num_classes)
    t = ff.softmax(t)
    return x, t
