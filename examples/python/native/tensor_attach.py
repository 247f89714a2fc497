"""Attach a numpy array to an input tensor and read it back (reference
examples/python/native/tensor_attach.py)."""
from _args import parse  # noqa: I001
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def top_level_task(argv=None):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    inp = ffmodel.create_tensor([8, 3, 10, 10], DataType.DT_FLOAT)
    input_np = np.arange(8 * 3 * 10 * 10, dtype=np.float32).reshape(8, 3, 10, 10)
    inp.attach_numpy_array(ffconfig, input_np)
    assert inp.is_mapped()
    arr = inp.get_array(ffconfig, DataType.DT_FLOAT)
    assert np.array_equal(arr, input_np)
    print(arr.shape, arr.reshape(-1)[:8])
    inp.detach_numpy_array(ffconfig)
    assert not inp.is_mapped()


if __name__ == "__main__":
    args, rest = parse(0)
    top_level_task(rest)
