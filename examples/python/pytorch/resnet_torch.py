"""Export ResNet-18 (10 classes) to resnet18.ff (reference examples/python/pytorch/resnet_torch.py,
torchvision's resnet18; --small: quarter width)."""
import sys

import _args  # noqa: F401,I001
from models_torch import resnet18

from flexflow_amd.torch import PyTorchModel


def export(path="resnet18.ff", width=64):
    PyTorchModel(resnet18(10, width)).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export(width=16 if "--small" in sys.argv else 64))
