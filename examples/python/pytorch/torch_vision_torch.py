"""Export SqueezeNet (10 classes) to squeezenet.ff (reference examples/python/pytorch/torch_vision_torch.py)."""
import _args  # noqa: F401,I001
from models_torch import SqueezeNet

from flexflow_amd.torch import PyTorchModel


def export(path="squeezenet.ff"):
    PyTorchModel(SqueezeNet(10)).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export())
