"""Train the two-input CNN loaded from cnn.ff (reference examples/python/pytorch/cifar10_cnn.py):
both inputs are fed the same images; the first model output goes through softmax."""
import os

from _args import parse  # noqa: I001

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.keras.datasets import cifar10
from flexflow_amd.torch import PyTorchModel


def top_level_task(argv=None, num_samples=10000):
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    input_tensor = ffmodel.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    if not os.path.exists("cnn.ff"):
        import cifar10_cnn_torch
        cifar10_cnn_torch.export()
    output_tensors = PyTorchModel.file_to_ff("cnn.ff", ffmodel, [input_tensor, input_tensor])
    ffmodel.softmax(output_tensors[0])
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x_train, y_train), _ = cifar10.load_data(num_samples, num_test=16)
    x = x_train[:num_samples].astype("float32") / 255
    y = y_train[:num_samples].astype("int32")
    dl_x = ffmodel.create_data_loader(input_tensor, x)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y)
    ffmodel.init_layers()
    for name in [L.name for L in ffmodel.layers][:6]:
        print(name)
    ts = ffconfig.get_current_time()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    run = 1e-6 * (ffconfig.get_current_time() - ts)
    print(f"epochs {ffconfig.epochs}, ELAPSED TIME = {run:.4f}s, THROUGHPUT = "
          f"{dl_x.num_samples * ffconfig.epochs / run:.2f} samples/s")


if __name__ == "__main__":
    args, rest = parse(10000)
    top_level_task(rest, args.samples)
