"""Export the two-input CIFAR-10 CNN to cnn.ff (reference examples/python/pytorch/cifar10_cnn_torch.py)."""
import sys

import _args  # noqa: F401,I001
from models_torch import CNN

from flexflow_amd.torch import PyTorchModel


def export(path="cnn.ff"):
    PyTorchModel(CNN()).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export(sys.argv[1] if len(sys.argv) > 1 else "cnn.ff"))
