"""resnet (reference examples/cpp/resnet, examples/python/native): zoo model "resnet50" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("resnet50")
