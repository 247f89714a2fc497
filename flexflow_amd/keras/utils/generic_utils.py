"""Keras generic utilities (reference python/flexflow/keras/utils/generic_utils.py, which carries
upstream Keras's helpers): custom-object scopes and (de)serialization of named objects, a
progress bar, and small list / array helpers used by fit()."""
from __future__ import annotations

import inspect
import marshal
import sys
import time
import types

import numpy as np

_GLOBAL_CUSTOM_OBJECTS: dict = {}


class CustomObjectScope:
    """`with CustomObjectScope({"MyLayer": MyLayer}):` makes the names resolvable by
    deserialize_keras_object inside the block."""

    def __init__(self, *args):
        self.custom_objects = args
        self.backup = None

    def __enter__(self):
        self.backup = dict(_GLOBAL_CUSTOM_OBJECTS)
        for objs in self.custom_objects:
            _GLOBAL_CUSTOM_OBJECTS.update(objs)
        return self

    def __exit__(self, *exc):
        _GLOBAL_CUSTOM_OBJECTS.clear()
        _GLOBAL_CUSTOM_OBJECTS.update(self.backup)


def custom_object_scope(*args):
    return CustomObjectScope(*args)


def get_custom_objects():
    """The global name -> object registry (mutable)."""
    return _GLOBAL_CUSTOM_OBJECTS


def serialize_keras_object(instance):
    if instance is None:
        return None
    if hasattr(instance, "get_config"):
        return {"class_name": instance.__class__.__name__, "config": instance.get_config()}
    if hasattr(instance, "__name__"):
        return instance.__name__
    raise ValueError(f"cannot serialize {instance!r}")


def deserialize_keras_object(identifier, module_objects=None, custom_objects=None,
                             printable_module_name="object"):
    objects = dict(module_objects or {})
    objects.update(_GLOBAL_CUSTOM_OBJECTS)
    objects.update(custom_objects or {})
    if isinstance(identifier, dict):
        if "class_name" not in identifier or "config" not in identifier:
            raise ValueError(f"improper config format: {identifier}")
        cls = objects.get(identifier["class_name"])
        if cls is None:
            raise ValueError(f"unknown {printable_module_name}: {identifier['class_name']}")
        cfg = identifier["config"]
        if hasattr(cls, "from_config"):
            return cls.from_config(cfg)
        return cls(**cfg)
    if isinstance(identifier, str):
        obj = objects.get(identifier)
        if obj is None:
            raise ValueError(f"unknown {printable_module_name}: {identifier}")
        return obj() if inspect.isclass(obj) else obj
    raise ValueError(f"could not interpret serialized {printable_module_name}: {identifier!r}")


def func_dump(func):
    """(code, defaults, closure) of a Python function, code as marshalled bytes in latin-1."""
    code = marshal.dumps(func.__code__).decode("raw_unicode_escape")
    closure = tuple(c.cell_contents for c in func.__closure__) if func.__closure__ else None
    return code, func.__defaults__, closure


def func_load(code, defaults=None, closure=None, globs=None):
    if isinstance(code, (tuple, list)):
        code, defaults, closure = code
    raw = marshal.loads(code.encode("raw_unicode_escape"))
    cells = tuple(types.CellType(v) for v in closure) if closure is not None else None
    return types.FunctionType(raw, globs if globs is not None else globals(), name=raw.co_name,
                              argdefs=tuple(defaults) if defaults is not None else None, closure=cells)


def getargspec(fn):
    return inspect.getfullargspec(fn)


def has_arg(fn, name, accept_all=False):
    params = inspect.signature(fn).parameters
    if accept_all and any(p.kind == inspect.Parameter.VAR_KEYWORD for p in params.values()):
        return True
    p = params.get(name)
    return p is not None and p.kind in (inspect.Parameter.POSITIONAL_OR_KEYWORD, inspect.Parameter.KEYWORD_ONLY)


class Progbar:
    """Text progress bar: Progbar(target).update(current, values=[("loss", v), ...])."""

    def __init__(self, target, width=30, verbose=1, interval=0.05, stateful_metrics=None, unit_name="step"):
        self.target, self.width, self.verbose, self.interval = target, width, verbose, interval
        self.stateful_metrics = set(stateful_metrics or ())
        self.unit_name = unit_name
        self._values: dict = {}
        self._seen = 0
        self._start = time.time()
        self._last = 0.0

    def update(self, current, values=None):
        for k, v in values or []:
            if k in self.stateful_metrics:
                self._values[k] = [v, 1]
            else:
                s = self._values.setdefault(k, [0.0, 0])
                s[0] += v * (current - self._seen)
                s[1] += current - self._seen
        self._seen = current
        now = time.time()
        done = self.target is not None and current >= self.target
        if self.verbose != 1 or (now - self._last < self.interval and not done):
            return
        self._last = now
        if self.target:
            filled = int(self.width * current / self.target)
            bar = f"{current}/{self.target} [" + "=" * max(filled - 1, 0) + (">" if filled < self.width else "=") + \
                  "." * (self.width - filled) + "]"
        else:
            bar = f"{current}"
        info = " - ".join(f"{k}: {s[0] / max(s[1], 1):.4f}" for k, s in self._values.items())
        sys.stdout.write("\r" + bar + (" - " + info if info else "") + ("\n" if done else ""))
        sys.stdout.flush()

    def add(self, n, values=None):
        self.update(self._seen + n, values)


def to_list(x, allow_tuple=False):
    if isinstance(x, list):
        return x
    if allow_tuple and isinstance(x, tuple):
        return list(x)
    return [x]


def unpack_singleton(x):
    return x[0] if len(x) == 1 else x


def object_list_uid(object_list):
    return ", ".join(str(abs(id(x))) for x in to_list(object_list))


def is_all_none(iterable_or_element):
    return all(x is None for x in to_list(iterable_or_element, allow_tuple=True))


def slice_arrays(arrays, start=None, stop=None):
    """Slice an array or list of arrays by [start:stop] or by an index list in start."""
    if arrays is None:
        return [None]
    if isinstance(arrays, list):
        if hasattr(start, "__len__"):
            return [None if a is None else a[start] for a in arrays]
        return [None if a is None else a[start:stop] for a in arrays]
    if hasattr(start, "__len__"):
        return arrays[start]
    return arrays[start:stop]


def transpose_shape(shape, target_format, spatial_axes):
    """Shape given channels_last -> the same shape in target_format ('channels_first' moves the
    last axis in front of the spatial ones)."""
    if target_format == "channels_first":
        new = list(shape[:spatial_axes[0]]) + [shape[-1]] + [shape[a] for a in spatial_axes]
        return tuple(new) if isinstance(shape, tuple) else new
    if target_format == "channels_last":
        return shape
    raise ValueError(f"unknown data format {target_format}")


def check_for_unexpected_keys(name, input_dict, expected_values):
    unknown = set(input_dict.keys()) - set(expected_values)
    if unknown:
        raise ValueError(f"unknown entries in {name} dictionary: {sorted(unknown)}; only expected {expected_values}")


def to_array(x):
    return np.asarray(x)
