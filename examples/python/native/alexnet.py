"""alexnet (reference examples/cpp/alexnet, examples/python/native): zoo model "alexnet" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("alexnet")
