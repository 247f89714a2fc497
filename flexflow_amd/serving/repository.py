"""Model repository: `<root>/<model>/config.pbtxt` + `<root>/<model>/<version>/model.onnx`
(+ optional `model.strategy`), the layout Triton uses and the reference backend consumes
(triton/qa/L0_e2e/models/*). The newest version directory is served; models load at start-up
(or on `load`) and unload explicitly."""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional

from .config import ModelConfig
from .engine import ServedModel


class ModelRepository:
    def __init__(self, root: str, ff_flags: Optional[List[str]] = None):
        self.root = os.path.abspath(root)
        self.ff_flags = list(ff_flags or [])
        self.models: Dict[str, ServedModel] = {}
        self.errors: Dict[str, str] = {}
        self._mu = threading.Lock()

    def names(self) -> List[str]:
        if not os.path.isdir(self.root):
            return []
        return sorted(d for d in os.listdir(self.root)
                      if os.path.isfile(os.path.join(self.root, d, "config.pbtxt")))

    def versions(self, name: str) -> List[str]:
        d = os.path.join(self.root, name)
        return sorted((v for v in os.listdir(d) if v.isdigit() and os.path.isdir(os.path.join(d, v))), key=int)

    def load(self, name: str) -> ServedModel:
        # only names the repository lists (a plain directory under root): '..', absolute paths
        # and separators in a request path must never reach os.path.join
        if name not in self.names() or os.path.dirname(os.path.normpath(os.path.join(self.root, name))) != self.root:
            raise KeyError(f"no model {name!r} in {self.root}")
        cfg_path = os.path.join(self.root, name, "config.pbtxt")
        if not os.path.isfile(cfg_path):
            raise KeyError(f"no model {name!r} in {self.root}")
        with open(cfg_path) as f:
            cfg = ModelConfig.parse(f.read(), default_name=name)
        vs = self.versions(name)
        if not vs:
            raise FileNotFoundError(f"model {name!r} has no version directory")
        try:
            m = ServedModel(cfg, os.path.join(self.root, name, vs[-1]), self.ff_flags)
        except Exception as e:
            with self._mu:
                self.errors[name] = f"{type(e).__name__}: {e}"
            raise
        with self._mu:
            old = self.models.pop(name, None)
            self.models[name] = m
            self.errors.pop(name, None)
        if old is not None:
            old.close()
        return m

    def load_all(self, strict: bool = False) -> Dict[str, str]:
        """Loads every model; returns {name: error} for those that failed (raises if strict)."""
        for n in self.names():
            try:
                self.load(n)
            except Exception:  # noqa: BLE001 - recorded in self.errors, the rest still load
                if strict:
                    raise
        return dict(self.errors)

    def unload(self, name: str):
        with self._mu:
            m = self.models.pop(name, None)
        if m is not None:
            m.close()

    def get(self, name: str, version: Optional[str] = None) -> ServedModel:
        m = self.models.get(name)
        if m is None or (version not in (None, "") and version != m.version):
            raise KeyError(f"model {name!r}" + (f" version {version}" if version else "") + " is not ready")
        return m

    def index(self) -> List[dict]:
        out = []
        for n in self.names():
            m = self.models.get(n)
            e = {"name": n, "state": "READY" if m else ("UNAVAILABLE" if n in self.errors else "UNLOADED")}
            if m:
                e["version"] = m.version
            if n in self.errors:
                e["reason"] = self.errors[n]
            out.append(e)
        return out

    def close(self):
        for n in list(self.models):
            self.unload(n)
