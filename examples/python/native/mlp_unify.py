"""mlp_unify (reference examples/cpp/mlp_unify, examples/python/native): zoo model "mlp_unify" trained on
synthetic batches through FFModel; flags in zoo.py."""
from zoo import run

if __name__ == "__main__":
    run("mlp_unify")
