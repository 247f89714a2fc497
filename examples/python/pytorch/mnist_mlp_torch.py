"""Export a PyTorch MNIST MLP to the .ff IR file (reference examples/python/pytorch/mnist_mlp_torch.py):
torch.fx traces the module and PyTorchModel.torch_to_file writes one line per node; mnist_mlp.py
loads it into an FFModel."""
import sys

import _args  # noqa: F401  (puts the repo root on sys.path)
import torch.nn as nn

from flexflow_amd.torch import PyTorchModel


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(784, 512)
        self.linear2 = nn.Linear(512, 512)
        self.linear3 = nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x):
        y = self.relu(self.linear1(x))
        y = self.relu(self.linear2(y))
        return self.softmax(self.linear3(y))


def export(path="mnist_mlp.ff"):
    PyTorchModel(MLP()).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export(sys.argv[1] if len(sys.argv) > 1 else "mnist_mlp.ff"))
