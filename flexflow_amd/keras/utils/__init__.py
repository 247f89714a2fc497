"""Keras utils (reference keras/utils/np_utils.py)."""
from .np_utils import normalize, to_categorical  # noqa: F401
