"""Export a RegNetX (grouped-convolution residual blocks) with a flatten + linear head to
regnetX.ff (reference examples/python/pytorch/export_regnet_fx.py, there classy_vision's
RegNetX32gf; --small: narrow widths)."""
import sys

import _args  # noqa: F401,I001
import torch.nn as nn
from models_torch import RegNetX

from flexflow_amd.torch import PyTorchModel


def export(path="regnetX.ff", small=False):
    m = RegNetX((1, 1, 2, 1), (32, 64, 96, 192), 16, 10) if small else RegNetX(num_classes=10)
    PyTorchModel(nn.Sequential(m, nn.Flatten())).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export(small="--small" in sys.argv))
