"""transformer (reference examples/cpp/transformer, examples/python/native): zoo model "transformer" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("transformer")
