"""Make the repo root and the pytorch / keras example helpers importable from this directory."""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(_HERE, "..", "..", ".."), os.path.join(_HERE, "..", "pytorch"), os.path.join(_HERE, "..", "keras")):
    p = os.path.abspath(p)
    if p not in sys.path:
        sys.path.insert(0, p)
