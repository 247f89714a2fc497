"""Plain-PyTorch ResNet-152 training loop, the baseline the reference compares FlexFlow against
(examples/python/pytorch/resnet152_training.py; synthetic CIFAR-shaped batches upscaled to 224,
torchvision/datasets unavailable offline). --small: quarter width, 64 px, 2 steps."""
import sys
import time

import _args  # noqa: F401,I001
import torch
import torch.nn as nn
import torch.optim as optim
from models_torch import resnet152


def main(small=False, steps=20, batch_size=4):
    device = "cuda:0" if torch.cuda.is_available() else "cpu"
    size = 64 if small else 224
    model = resnet152(10, 16 if small else 64).to(device)
    criterion = nn.CrossEntropyLoss()
    optimizer = optim.SGD(model.parameters(), lr=0.001, momentum=0.9)
    g = torch.Generator().manual_seed(0)
    for i in range(steps):
        inputs = torch.rand(batch_size, 3, size, size, generator=g).to(device)
        labels = torch.randint(0, 10, (batch_size,), generator=g).to(device)
        start = time.time()
        optimizer.zero_grad()
        loss = criterion(model(inputs), labels)
        loss.backward()
        optimizer.step()
        if device.startswith("cuda"):
            torch.cuda.synchronize()
        print("Batch: %d Loss: %.3f Time per Image: %.5f" % (i, loss.item(), (time.time() - start) / batch_size))
    print("Finished Training")


if __name__ == "__main__":
    small = "--small" in sys.argv
    main(small, steps=2 if small else 20)
