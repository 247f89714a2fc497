"""xdl (reference examples/cpp/xdl, examples/python/native): zoo model "xdl" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("xdl")
