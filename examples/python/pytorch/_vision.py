"""Shared driver of the image-model examples: CIFAR-10 nearest-upscaled to the model's input size
(the reference resizes with PIL, Image.NEAREST), loaded from a .ff file, trained or evaluated."""
import numpy as np

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.torch import PyTorchModel


def upscale(x, size):
    idx = (np.arange(size) * x.shape[-1] // size).astype(np.int64)
    return x[:, :, idx][:, :, :, idx]


def run(ff_file, argv, num_samples, size, softmax=True, train=True):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    inp = ffmodel.create_tensor([ffconfig.batch_size, 3, size, size], DataType.DT_FLOAT)
    out = PyTorchModel.file_to_ff(ff_file, ffmodel, [inp])
    if softmax:
        ffmodel.softmax(out[0])
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x = upscale(x_train[:num_samples], size).astype(np.float32) / 255
    y = y_train[:num_samples].astype("int32")
    dl_x = ffmodel.create_data_loader(inp, x)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y)
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    if train:
        ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    else:
        ffmodel.eval(x=dl_x, y=dl_y)
    run_s = 1e-6 * (ffconfig.get_current_time() - ts)
    print(f"epochs {ffconfig.epochs}, ELAPSED TIME = {run_s:.4f}s, THROUGHPUT = "
          f"{dl_x.num_samples * ffconfig.epochs / run_s:.2f} samples/s")
