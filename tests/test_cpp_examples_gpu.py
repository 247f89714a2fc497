"""C++ examples on cuda:0 (HIP kernels behind the C++ API): a CNN, a recommender, a transformer and
the MoE train one step each in --small mode."""
import pytest

from test_cpp_examples_cpu import build_examples, check, run_examples

pytestmark = pytest.mark.gpu


def test_cpp_examples_train_on_gpu():
    build_examples()
    check(run_examples(["AlexNet/alexnet", "DLRM/dlrm", "Transformer/transformer", "mixture_of_experts/moe"], {},
                       parallel=1, timeout=110))
