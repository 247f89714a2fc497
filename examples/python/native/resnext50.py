"""resnext50 (reference examples/cpp/resnext50, examples/python/native): zoo model "resnext50" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("resnext50")
