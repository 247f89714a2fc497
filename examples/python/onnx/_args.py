"""Shared CLI handling for the native examples: FlexFlow flags go to FFConfig (`-b`, `-e`,
`--search`, `--only-data-parallel`, ...), `--samples N` bounds the synthetic dataset, `-a/--test_acc`
asserts the accuracy floor (reference examples/python/native/*.py `__main__` blocks)."""
import argparse
import os
import sys

# run from a source checkout without installing: put the repo root on the path
_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)


def parse(default_samples):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--samples", type=int, default=default_samples)
    ap.add_argument("-a", "--test_acc", action="store_true")
    args, rest = ap.parse_known_args(sys.argv[1:])
    return args, rest
