"""Keras preprocessing: sequence padding and the bag-of-words Tokenizer used by the Reuters MLP
example (reference keras/preprocessing)."""
from . import sequence, text  # noqa: F401
