"""Export AlexNet (10 classes) from torch to alexnet.onnx (reference examples/python/onnx/alexnet_pt.py)."""
import _args  # noqa: F401,I001
import torch
from models_pt import AlexNet

from flexflow_amd.onnx.export import export_torch


def export(path="alexnet.onnx", size=224):
    export_torch(AlexNet(num_classes=10, size=size), torch.randn(2, 3, size, size), path, export_params=False)
    return path


if __name__ == "__main__":
    print(export())
