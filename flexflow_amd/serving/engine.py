"""Model instances of the inference server.

Reference: the Triton "legion" backend (triton/src/model.cc `LegionModelState` loads
`<version>/model.onnx` with its ONNX parser (onnx_parser.cc) and partitions every layer by
`<version>/model.strategy` (strategy.cc); instance.cc runs requests through the Legion runtime).
Here a `ServedModel` builds the same ONNX graph through our ONNX frontend into an FFModel compiled
in INFERENCE mode (forward only, no optimizer state, weights from the initializers), imports the
`.strategy` file as the parallelization, and serves `infer()` calls. With `max_batch_size > 0`
requests are coalesced by the native dynamic batcher (`_core.RequestQueue`, C++) and run as one
padded batch of `max_batch_size` rows on the model's executor thread.
"""
from __future__ import annotations

import itertools
import os
import threading
from typing import Dict, List, Optional

import numpy as np

from .config import ModelConfig, TensorSpec, find_spec

_DT = {"TYPE_FP32": "DT_FLOAT", "TYPE_FP16": "DT_HALF", "TYPE_FP64": "DT_DOUBLE", "TYPE_INT32": "DT_INT32",
       "TYPE_INT64": "DT_INT64", "TYPE_BOOL": "DT_BOOLEAN"}


class InferError(ValueError):
    """A malformed request (bad name / shape / dtype): HTTP 400, the model keeps serving."""


class ServedModel:
    def __init__(self, config: ModelConfig, version_dir: str, ff_flags: Optional[List[str]] = None):
        from ..core import FFConfig, FFModel
        from ..onnx import ONNXModel
        from ..type import CompMode, DataType
        self.config = config
        self.version = os.path.basename(os.path.normpath(version_dir))
        onnx_path = os.path.join(version_dir, "model.onnx")
        if not os.path.exists(onnx_path):
            raise FileNotFoundError(f"{version_dir}: no model.onnx")
        flags = list(ff_flags or [])
        strat = os.path.join(version_dir, "model.strategy")
        if os.path.exists(strat) and "--import-strategy" not in flags:
            flags += ["--import-strategy", strat]
        if config.instance_kind == "KIND_CPU":
            flags += ["--device", "cpu"]
        cfg = FFConfig(flags)
        mbs = config.max_batch_size
        if not config.inputs:
            raise ValueError(f"model {config.name}: config.pbtxt declares no inputs")
        self.rows = mbs if mbs > 0 else int(config.inputs[0].dims[0]) if config.inputs[0].dims else 1
        cfg.batch_size = self.rows
        ff = FFModel(cfg)
        self.inputs = {}
        for s in config.inputs:
            dims = ([mbs] if mbs > 0 else []) + list(s.dims)
            self.inputs[s.name] = ff.create_tensor(dims, getattr(DataType, _DT.get(s.data_type, "DT_FLOAT")),
                                                   name=s.name)
        self.onnx = ONNXModel(onnx_path)
        self.onnx.apply(ff, dict(self.inputs))
        self.outputs = {}
        for s in config.outputs:
            t = self.onnx.symbol_table.get(s.name)
            if t is None:
                raise ValueError(f"model {config.name}: output {s.name!r} is not produced by the ONNX graph")
            self.outputs[s.name] = t
        ff.compile(comp_mode=CompMode.INFERENCE)
        self.onnx.load_initializers(ff)
        self.ff = ff
        self._lock = threading.Lock()
        self.n_inferences = 0
        self.n_executions = 0
        self.batcher = DynamicBatcher(self) if mbs > 0 else None

    # ------------------------------------------------------------------ request validation
    def _check(self, inputs: Dict[str, np.ndarray]) -> int:
        mbs = self.config.max_batch_size
        rows = None
        for s in self.config.inputs:
            if s.name not in inputs:
                raise InferError(f"model {self.config.name}: missing input {s.name!r}")
            a = inputs[s.name]
            want = list(s.dims)
            got = list(a.shape[1:] if mbs > 0 else a.shape)
            if got != want or (mbs > 0 and a.ndim != len(want) + 1):
                raise InferError(f"input {s.name!r}: shape {list(a.shape)} does not match "
                                 f"{([-1] if mbs > 0 else []) + want}")
            r = a.shape[0] if mbs > 0 else self.rows
            if rows is not None and r != rows:
                raise InferError("inputs disagree on the batch size")
            rows = r
        extra = set(inputs) - {s.name for s in self.config.inputs}
        if extra:
            raise InferError(f"unknown inputs {sorted(extra)}")
        if mbs > 0 and not (1 <= rows <= mbs):
            raise InferError(f"batch of {rows} rows exceeds max_batch_size {mbs}")
        return rows

    # ------------------------------------------------------------------ execution
    def execute(self, inputs: Dict[str, np.ndarray], rows: int) -> Dict[str, np.ndarray]:
        """One forward over `rows` valid rows (padded up to the compiled batch)."""
        with self._lock:
            for s in self.config.inputs:
                a = np.asarray(inputs[s.name], dtype=s.np_dtype if s.np_dtype != np.float64 else np.float32)
                if self.config.max_batch_size > 0 and rows < self.rows:
                    pad = np.zeros((self.rows - rows,) + a.shape[1:], dtype=a.dtype)
                    a = np.concatenate([a, pad], 0)
                self.inputs[s.name].set_tensor(self.ff, a)
            self.ff.executor.forward(training=False)
            out = {}
            for s in self.config.outputs:
                v = np.asarray(self.outputs[s.name].get_tensor(self.ff))
                if self.config.max_batch_size > 0:
                    v = v[:rows]
                out[s.name] = v.astype(s.np_dtype, copy=False)
            self.n_executions += 1
            return out

    def infer(self, inputs: Dict[str, np.ndarray], outputs: Optional[List[str]] = None) -> Dict[str, np.ndarray]:
        rows = self._check(inputs)
        for o in outputs or []:
            if find_spec(self.config.outputs, o) is None:
                raise InferError(f"model {self.config.name}: unknown output {o!r}")
        if self.batcher is not None:
            res = self.batcher.submit(inputs, rows)
        else:
            res = self.execute(inputs, rows)
        self.n_inferences += 1
        return {k: v for k, v in res.items() if not outputs or k in outputs}

    def stats(self) -> dict:
        st = {"inference_count": self.n_inferences, "execution_count": self.n_executions}
        if self.batcher is not None:
            b, r, rows = self.batcher.queue.stats()
            st["batcher"] = {"batches": b, "requests": r, "rows": rows}
        return st

    def close(self):
        if self.batcher is not None:
            self.batcher.close()


class _Pending:
    __slots__ = ("inputs", "rows", "event", "result", "error")

    def __init__(self, inputs, rows):
        self.inputs, self.rows = inputs, rows
        self.event = threading.Event()
        self.result = None
        self.error = None


class DynamicBatcher:
    """Coalesces concurrent requests of a `max_batch_size > 0` model into one padded forward.
    The queue and its batching policy are native (csrc/core/request_queue.cc); the request tensors
    stay here, keyed by id, and one executor thread per model pops batches."""

    def __init__(self, model: ServedModel):
        from .. import _core
        cfg = model.config
        delay = cfg.max_queue_delay_us if cfg.dynamic_batching else 0
        self.model = model
        self.queue = _core.RequestQueue(cfg.max_batch_size, delay, list(cfg.preferred_batch_size))
        self.pending: Dict[int, _Pending] = {}
        self.ids = itertools.count()
        self._mu = threading.Lock()
        self.thread = threading.Thread(target=self._loop, name=f"ff-serve-{cfg.name}", daemon=True)
        self.thread.start()

    def submit(self, inputs, rows):
        p = _Pending(inputs, rows)
        with self._mu:
            rid = next(self.ids)
            self.pending[rid] = p
        if not self.queue.push(rid, rows):
            with self._mu:
                self.pending.pop(rid, None)
            raise InferError("model is shutting down")
        p.event.wait()
        if p.error is not None:
            raise p.error
        return p.result

    def _loop(self):
        while True:
            ids = self.queue.pop(-1)
            if not ids:
                return  # closed and drained
            with self._mu:
                batch = [self.pending.pop(i) for i in ids]
            try:
                names = [s.name for s in self.model.config.inputs]
                merged = {n: np.concatenate([np.asarray(p.inputs[n]) for p in batch], 0) for n in names}
                rows = sum(p.rows for p in batch)
                out = self.model.execute(merged, rows)
                off = 0
                for p in batch:
                    p.result = {k: v[off:off + p.rows] for k, v in out.items()}
                    off += p.rows
            except Exception as e:  # noqa: BLE001 - delivered to every waiting request
                for p in batch:
                    p.error = e
            for p in batch:
                p.event.set()

    def close(self):
        self.queue.close()
        self.thread.join(timeout=5)
