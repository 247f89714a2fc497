"""mixture_of_experts (reference examples/cpp/mixture_of_experts, examples/python/native): zoo model "moe" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("moe")
