"""Train the RegNetX loaded from regnetX.ff on CIFAR-10 at 229x229 (reference
examples/python/pytorch/regnet.py; --small: 67x67, narrow widths)."""
import os

from _args import parse  # noqa: I001
from _vision import run

if __name__ == "__main__":
    args, rest = parse(10000)
    small = "--small" in rest
    rest = [a for a in rest if a != "--small"]
    path = "regnetX_small.ff" if small else "regnetX.ff"
    if not os.path.exists(path):
        import export_regnet_fx
        export_regnet_fx.export(path, small)
    run(path, rest, args.samples, 67 if small else 229)
