"""Plain-PyTorch DistributedDataParallel ResNet-152 baseline (reference
examples/python/pytorch/resnet152_DDP_training.py), one process per GPU:
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 resnet152_DDP_training.py
Backend nccl (= RCCL on ROCm) on GPUs, gloo on CPU. --small: quarter width, 64 px, 2 steps."""
import os
import sys
import time

import _args  # noqa: F401,I001
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim
from models_torch import resnet152


def main(small=False, steps=20, batch_size=4):
    cuda = torch.cuda.is_available()
    dist.init_process_group("nccl" if cuda else "gloo")
    rank = dist.get_rank()
    local = int(os.environ.get("LOCAL_RANK", 0))
    device = torch.device("cuda", local) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    size = 64 if small else 224
    model = nn.parallel.DistributedDataParallel(resnet152(10, 16 if small else 64).to(device),
                                                device_ids=[local] if cuda else None)
    criterion = nn.CrossEntropyLoss()
    optimizer = optim.SGD(model.parameters(), lr=0.001, momentum=0.9)
    g = torch.Generator().manual_seed(rank)
    for i in range(steps):
        inputs = torch.rand(batch_size, 3, size, size, generator=g).to(device)
        labels = torch.randint(0, 10, (batch_size,), generator=g).to(device)
        start = time.time()
        optimizer.zero_grad()
        loss = criterion(model(inputs), labels)
        loss.backward()
        optimizer.step()
        if cuda:
            torch.cuda.synchronize()
        if rank == 0:
            print("Batch: %d Loss: %.3f Time per Image: %.5f" % (i, loss.item(), (time.time() - start) / batch_size))
    dist.destroy_process_group()


if __name__ == "__main__":
    small = "--small" in sys.argv
    main(small, steps=2 if small else 20)
