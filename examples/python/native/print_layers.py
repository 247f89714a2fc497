"""Layer / tensor / weight introspection (reference examples/python/native/print_layers.py,
print_weight.py, print_input.py, tensor_attach.py, split.py, demo_gather.py rolled into one):
walks the layers of a small CNN + MLP, reads and writes weights, attaches a numpy array to an input,
splits a tensor and gathers rows, then checks one forward pass against numpy."""
import _args  # noqa: F401  (puts the repo root on sys.path)
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403


def top_level_task(argv=None):
    ffconfig = FFConfig(argv or [])
    ffconfig.batch_size = 4
    ffmodel = FFModel(ffconfig)
    x = ffmodel.create_tensor([4, 3, 8, 8], DataType.DT_FLOAT)
    t = ffmodel.conv2d(x, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="conv1")
    t = ffmodel.flat(ffmodel.pool2d(t, 2, 2, 2, 2, 0, 0))
    a, c = ffmodel.split(t, [32, 32], 1)                      # split.py
    t = ffmodel.concat([c, a], 1)
    t = ffmodel.dense(t, 6, name="fc")
    idx = ffmodel.create_tensor([4, 6], DataType.DT_INT32, create_grad=False)
    g = ffmodel.gather(t, idx, 1)                              # demo_gather.py
    out = ffmodel.softmax(g)
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    ffmodel.print_layers()                                     # print_layers.py
    for i in range(len(ffmodel.get_layers())):
        layer = ffmodel.get_layer_by_id(i)
        print(i, layer.name, [tuple(w.dims) for w in layer.weights])
    fc = ffmodel.get_layer_by_name("fc")
    kernel = fc.get_weight_tensor()                            # print_weight.py
    w = kernel.get_weights(ffmodel)
    kernel.set_weights(ffmodel, np.full_like(w, 0.01))
    assert np.allclose(kernel.get_weights(ffmodel), 0.01)
    rng = np.random.default_rng(0)
    inp = rng.standard_normal((4, 3, 8, 8)).astype(np.float32)
    x.attach_numpy_array(ffmodel, inp)                         # tensor_attach.py
    x.detach_numpy_array(ffmodel)
    perm = np.tile(np.arange(6)[::-1], (4, 1)).astype(np.int32)
    idx.set_tensor(ffmodel, perm)
    ffmodel.forward()
    got = np.asarray(out.get_tensor(ffmodel))                  # print_input.py / get_tensor
    assert got.shape == (4, 6) and np.allclose(got.sum(1), 1.0, atol=1e-4)
    # every fc output is the same (uniform kernel), so the gathered softmax is uniform
    assert np.allclose(got, 1.0 / 6, atol=1e-3), got
    print("introspection ok:", got[0])
    return got


if __name__ == "__main__":
    top_level_task()
