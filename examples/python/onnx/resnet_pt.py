"""Export ResNet-18 from torch to resnet18.onnx (reference examples/python/onnx/resnet_pt.py)."""
import _args  # noqa: F401,I001
import torch
from models_pt import ResNet18

from flexflow_amd.onnx.export import export_torch


def export(path="resnet18.onnx", size=224, widths=(64, 128, 256, 512)):
    export_torch(ResNet18(10, widths).eval(), torch.randn(2, 3, size, size), path, export_params=False)
    return path


if __name__ == "__main__":
    print(export())
