"""Train SqueezeNet loaded from squeezenet.ff on CIFAR-10 at 229x229 (reference
examples/python/pytorch/torch_vision.py; --small: 67x67)."""
import os

from _args import parse  # noqa: I001
from _vision import run

if __name__ == "__main__":
    args, rest = parse(10000)
    small = "--small" in rest
    rest = [a for a in rest if a != "--small"]
    if not os.path.exists("squeezenet.ff"):
        import torch_vision_torch
        torch_vision_torch.export()
    run("squeezenet.ff", rest, args.samples, 67 if small else 229)
