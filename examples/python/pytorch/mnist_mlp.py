"""Train the exported .ff MLP on MNIST (reference examples/python/pytorch/mnist_mlp.py): the IR file
from mnist_mlp_torch.py is rebuilt layer by layer on an FFModel (PyTorchModel.file_to_ff), compiled
and trained through the FlexFlow API. `--copy-weights` instead builds straight from the nn.Module
(torch_to_ff) and loads its parameters (copy_weights)."""
import os
import sys

from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import mnist
from flexflow_amd.torch import PyTorchModel

from mnist_mlp_torch import MLP, export


def top_level_task(argv=None, num_samples=60000, copy_weights=False, ff_file="mnist_mlp.ff"):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    x = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    if copy_weights:
        pt = PyTorchModel(MLP())
        out = pt.torch_to_ff(ffmodel, [x])[0]
    else:
        if not os.path.exists(ff_file):
            export(ff_file)
        out = PyTorchModel.file_to_ff(ff_file, ffmodel, [x])[0]
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    if copy_weights:
        pt.copy_weights(ffmodel)
    (xt, yt), _ = mnist.load_data(num_train=num_samples, num_test=16)
    xt = xt.reshape(num_samples, 784).astype("float32") / 255
    yt = yt.astype("int32").reshape(num_samples, 1)
    dl_x = ffmodel.create_data_loader(x, xt)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, yt)
    ffmodel.init_layers()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    return ffmodel.get_perf_metrics()


if __name__ == "__main__":
    args, rest = parse(60000)
    cw = "--copy-weights" in rest
    rest = [a for a in rest if a != "--copy-weights"]
    pm = top_level_task(rest, args.samples, cw)
    if args.test_acc:
        assert pm.get_accuracy() >= ModelAccuracy.MNIST_MLP.value, pm.get_accuracy()
    sys.exit(0)
