"""Export the MNIST MLP from torch to mnist_mlp_pt.onnx (reference examples/python/onnx/mnist_mlp_pt.py,
there with torch.onnx.export; here with flexflow_amd.onnx.export_torch, the onnx package being absent)."""
import _args  # noqa: F401,I001  (repo root on sys.path)
import torch
from models_pt import MLP

from flexflow_amd.onnx.export import export_torch
from flexflow_amd.onnx.proto import load_model


def export(path="mnist_mlp_pt.onnx"):
    export_torch(MLP(), torch.randn(100, 784), path, export_params=False)
    return path


if __name__ == "__main__":
    for node in load_model(export()).graph.node:
        print(node.op_type, list(node.input), list(node.output))
