"""inception (reference examples/cpp/inception, examples/python/native): zoo model "inception_v3" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("inception_v3")
