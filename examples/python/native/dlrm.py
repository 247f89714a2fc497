"""dlrm (reference examples/cpp/dlrm, examples/python/native): zoo model "dlrm" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("dlrm")
