"""ResNet-18 from resnet18.ff evaluated on CIFAR-10 at 224x224 (reference
examples/python/pytorch/resnet.py; --small: 64x64, quarter width)."""
import os
import sys

from _args import parse  # noqa: I001
from _vision import run

if __name__ == "__main__":
    args, rest = parse(10000)
    small = "--small" in rest
    rest = [a for a in rest if a != "--small"]
    path = "resnet18_small.ff" if small else "resnet18.ff"
    if not os.path.exists(path):
        import resnet_torch
        resnet_torch.export(path, 16 if small else 64)
    run(path, rest, args.samples, 64 if small else 224, train="--train" in sys.argv)
