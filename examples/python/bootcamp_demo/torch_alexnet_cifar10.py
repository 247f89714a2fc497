"""Bootcamp step 1: write a PyTorch AlexNet (10 classes) to alexnet.ff, the text IR that
ff_alexnet_cifar10.py loads (reference bootcamp_demo/torch_alexnet_cifar10.py).

    python examples/python/bootcamp_demo/torch_alexnet_cifar10.py [path]
"""
import sys

import _path  # noqa: F401,I001
import torch.nn as nn

from flexflow_amd.torch import PyTorchModel


class AlexNet(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, kernel_size=11, stride=4, padding=2), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2),
            nn.Conv2d(64, 192, kernel_size=5, padding=2), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2),
            nn.Conv2d(192, 384, kernel_size=3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(256, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2))
        self.classifier = nn.Sequential(
            nn.Linear(256 * 6 * 6, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes), nn.Softmax(dim=-1))

    def forward(self, x):
        return self.classifier(self.features(x).flatten(1))


def export(path="alexnet.ff"):
    PyTorchModel(AlexNet(10)).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export(*sys.argv[1:2]))
