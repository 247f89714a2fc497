"""Export the CIFAR-10 CNN from torch to cifar10_cnn_pt.onnx (reference examples/python/onnx/cifar10_cnn_pt.py)."""
import _args  # noqa: F401,I001
import torch
from models_pt import CNN

from flexflow_amd.onnx.export import export_torch


def export(path="cifar10_cnn_pt.onnx"):
    export_torch(CNN(), torch.randn(64, 3, 32, 32), path, export_params=False)
    return path


if __name__ == "__main__":
    print(export())
