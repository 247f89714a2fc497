"""CIFAR-10 CNN with a concat branch (reference examples/python/native/cifar10_cnn_concat.py)."""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy
from cifar10_cnn import top_level_task

if __name__ == "__main__":
    args, rest = parse(50000)
    pm = top_level_task(rest, args.samples, concat=True)
    if args.test_acc:
        assert pm.get_accuracy() >= ModelAccuracy.CIFAR10_CNN.value, pm.get_accuracy()
