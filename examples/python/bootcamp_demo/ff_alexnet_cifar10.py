"""Bootcamp step 2: load alexnet.ff into an FFModel and train it on CIFAR-10 upscaled to 229x229
(synthetic stand-in data, no network) through data loaders and `fit` (reference
bootcamp_demo/ff_alexnet_cifar10.py; its softmax is part of the exported module).

    python examples/python/bootcamp_demo/ff_alexnet_cifar10.py -b 64 -e 1 [--samples N] [--ff alexnet.ff]
"""
import argparse
import os
import sys

import _path  # noqa: F401,I001
from _vision import run
from torch_alexnet_cifar10 import export

if __name__ == "__main__":
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--ff", default="alexnet.ff")
    args, rest = ap.parse_known_args(sys.argv[1:])
    if not os.path.exists(args.ff):
        export(args.ff)
    print("cifar10 alexnet")
    run(args.ff, rest, args.samples, 229, softmax=False)
