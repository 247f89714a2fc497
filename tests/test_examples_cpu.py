"""The examples/ tree runs end to end on CPU at reduced sizes (reference test strategy: the
examples/python/* scripts are exercised by tests/python_interface_test.sh, and the
osdi22ae scripts by the artifact runs). Each script runs in its own process, as a user would."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "python")

CASES = [
    ("native/mnist_mlp.py", ["-b", "64", "-e", "2", "--samples", "2048", "-a"]),
    ("native/mnist_cnn.py", ["-b", "32", "--samples", "256"]),
    ("native/cifar10_cnn_concat.py", ["-b", "32", "--samples", "128"]),
    ("native/multi_head_attention.py", ["-b", "2", "--seq-length", "16", "--hidden-size", "32", "--num-heads", "4",
                                        "--iterations", "2", "--explicit"]),
    ("native/bert_proxy_native.py", ["-b", "2", "--seq-length", "16", "--hidden-size", "32", "--num-heads", "4",
                                     "--num_layers", "2", "--iterations", "2", "--train"]),
    ("native/print_layers.py", []),
    ("native/alexnet.py", ["-b", "4", "--iterations", "1", "--small"]),
    ("native/resnet.py", ["-b", "4", "--iterations", "2", "--small"]),
    ("native/dlrm.py", ["-b", "16", "--iterations", "2", "--small"]),
    ("native/transformer.py", ["-b", "2", "--iterations", "1", "--small"]),
    ("native/mixture_of_experts.py", ["-b", "16", "--iterations", "2", "--small"]),
    ("native/nmt.py", ["-b", "8", "--iterations", "2", "--small"]),
    ("native/inception.py", ["-b", "2", "--iterations", "1", "--small"]),
    ("native/resnext50.py", ["-b", "2", "--iterations", "1", "--small"]),
    ("native/xdl.py", ["-b", "16", "--iterations", "2", "--small"]),
    ("native/candle_uno.py", ["-b", "8", "--iterations", "2", "--small"]),
    ("native/mlp_unify.py", ["-b", "16", "--iterations", "2", "--small"]),
    ("native/tensor_attach.py", []),
    ("native/print_input.py", ["-b", "4"]),
    ("native/print_weight.py", ["-b", "16"]),
    ("native/split.py", ["-b", "32", "--samples", "64"]),
    ("native/demo_gather.py", ["-b", "4"]),
    ("native/mnist_mlp_attach.py", ["-b", "64", "--samples", "2048", "-e", "2", "-a"]),
    ("native/cifar10_cnn_attach.py", ["-b", "32", "--samples", "64"]),
    ("pytorch/cifar10_cnn.py", ["-b", "32", "--samples", "64"]),
    ("pytorch/resnet.py", ["--small", "-b", "8", "--samples", "16"]),
    ("pytorch/torch_vision.py", ["--small", "-b", "8", "--samples", "16"]),
    ("pytorch/regnet.py", ["--small", "-b", "8", "--samples", "16"]),
    ("pytorch/mnist_mlp_torch2.py", ["-b", "64", "--samples", "2048", "-e", "2", "-a"]),
    ("pytorch/mt5/mt5_ff.py", ["--tiny", "-b", "4", "-e", "1", "--samples", "16"]),
    ("pytorch/resnet152_training.py", ["--small"]),
    ("keras/seq_mnist_mlp.py", ["--samples", "1024", "-a"]),
    ("keras/func_mnist_mlp_concat.py", ["--samples", "512"]),
    ("keras/seq_reuters_mlp.py", ["--samples", "1024"]),
    ("keras/gather.py", []),
    ("keras/identity_loss.py", []),
    ("keras/reduce_sum.py", []),
    ("keras/rsqrt.py", []),
    ("keras/unary.py", []),
    ("keras/elementwise_mul_broadcast.py", []),
    ("keras/elementwise_max_min.py", []),
    ("keras/regularizer.py", []),
    ("keras/reshape.py", ["--samples", "256"]),
    ("keras/callback.py", ["--samples", "128"]),
    ("keras/func_mnist_mlp.py", ["--samples", "2048", "-a"]),
    ("keras/func_mnist_mlp_concat2.py", ["--samples", "128"]),
    ("keras/func_mnist_cnn.py", ["--samples", "128"]),
    ("keras/func_mnist_cnn_concat.py", ["--samples", "128"]),
    ("keras/seq_mnist_cnn.py", ["--samples", "128"]),
    ("keras/seq_mnist_cnn_nested.py", ["--samples", "128"]),
    ("keras/seq_cifar10_cnn.py", ["--samples", "128"]),
    ("keras/func_cifar10_cnn_nested.py", ["--samples", "128"]),
    ("keras/func_cifar10_cnn_concat.py", ["--samples", "128"]),
    ("keras/func_cifar10_cnn_concat_model.py", ["--samples", "128"]),
    ("keras/func_cifar10_cnn_concat_seq_model.py", ["--samples", "128"]),
    ("keras/func_cifar10_alexnet.py", ["--small", "--samples", "64"]),
    ("keras/func_mnist_mlp_net2net.py", ["--samples", "256"]),
    ("keras/seq_mnist_mlp_net2net.py", ["--samples", "256"]),
    ("keras/seq_mnist_cnn_net2net.py", ["--samples", "128"]),
    ("keras/func_cifar10_cnn_net2net.py", ["--samples", "128"]),
    ("keras/candle_uno/candle_uno.py", ["--small", "--samples", "256"]),
    ("pytorch/mnist_mlp.py", ["--samples", "1024", "-e", "2", "-a"]),
    ("keras_exp/func_mnist_mlp.py", ["--samples", "2048", "-a"]),
    ("onnx/mnist_mlp.py", ["--samples", "1024", "-e", "2", "-b", "64", "-a"]),
    ("onnx/mnist_mlp.py", ["--test_type", "0", "--samples", "1024", "-e", "2", "-b", "64", "-a"]),
    ("onnx/cifar10_cnn.py", ["--samples", "128", "-b", "32"]),
    ("onnx/cifar10_cnn.py", ["--test_type", "0", "--samples", "128", "-b", "32"]),
    ("onnx/alexnet.py", ["--small", "--samples", "32", "-b", "16"]),
    ("onnx/resnet.py", ["--small", "--samples", "32", "-b", "16"]),
    ("keras_exp/func_mnist_mlp_concat.py", ["--samples", "256"]),
    ("keras_exp/func_cifar10_cnn.py", ["--samples", "128"]),
    ("bootcamp_demo/keras_cnn_cifar10.py", ["--samples", "128", "--epochs", "1"]),
    ("bootcamp_demo/ff_alexnet_cifar10.py", ["--samples", "16", "-b", "8", "-e", "1"]),
    ("keras_exp/func_cifar10_cnn_concat.py", ["--samples", "128"]),
    ("keras_exp/func_cifar10_cnn_nested.py", ["--samples", "128"]),
]


@pytest.mark.parametrize("script,args", CASES, ids=[f"{c[0]}:{i}" for i, c in enumerate(CASES)])
def test_example_runs(script, args, tmp_path):
    env = dict(os.environ, FF_TUNABLEOP="off")
    r = subprocess.run([sys.executable, os.path.join(EX, script)] + args, cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


def test_osdi_scripts_parse():
    d = os.path.join(ROOT, "examples", "scripts", "osdi22ae")
    for f in sorted(os.listdir(d)):
        r = subprocess.run(["bash", "-n", os.path.join(d, f)], capture_output=True, text=True)
        assert r.returncode == 0, (f, r.stderr)
