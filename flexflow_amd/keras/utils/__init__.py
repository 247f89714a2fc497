"""Keras utils (reference keras/utils/{np_utils,generic_utils,data_utils}.py)."""
from . import data_utils, generic_utils  # noqa: F401
from .data_utils import GeneratorEnqueuer, OrderedEnqueuer, Sequence, get_file  # noqa: F401
from .generic_utils import CustomObjectScope, Progbar, custom_object_scope, get_custom_objects  # noqa: F401
from .np_utils import normalize, to_categorical  # noqa: F401
