"""SingleDataLoader (reference include/flexflow/dataloader.h:15-125, src/dataloader/dataloader.cc).

The reference attaches the whole dataset in zero-copy host memory and index-launches a copy
kernel per GPU shard each iteration. Here each rank keeps the dataset in host memory and, per
`next_batch`, stages ONLY its own shard of the batch (per the input tensor's layout) into a
persistent device buffer with an asynchronous pinned-memory H2D copy. When the native data-loader
ring (flexflow_amd._core.BatchRing) is available the next batch is pre-gathered into pinned memory
by a background C++ thread while the current step runs, and on a GPU its host->device copy is
issued on the device context's h2d stream right after the current batch is fed
(runtime/device.H2DPrefetcher: pinned host slots, two device staging buffers, the compute stream
waits on the copy's event only when the batch is consumed), so input staging never sits on the
step's critical path.
"""
from __future__ import annotations

import numpy as np
import torch

from ..type import DataType


class SingleDataLoader:
    def init_from_tensor(self, ffmodel, input, full_input, num_samples, data_type):
        """reference SingleDataLoader.init_from_tensor: the full dataset given as an FF tensor
        (attached array or set value)."""
        self.__init__(ffmodel, input, np.asarray(full_input.get_array(ffmodel)), num_samples, data_type)

    def init_from_ptr(self, ffmodel, input, full_input, num_samples, data_type):
        """reference SingleDataLoader.init_from_ptr: the full dataset given as host memory (any
        object with the buffer / array interface)."""
        self.__init__(ffmodel, input, np.asarray(full_input), num_samples, data_type)

    def __init__(self, ffmodel, input_tensor, full_input, num_samples=None, data_type=None):
        self.model = ffmodel
        self.tensor = input_tensor
        arr = full_input
        if not isinstance(arr, np.ndarray):
            arr = np.asarray(arr)
        if input_tensor.data_type == DataType.DT_INT32 and arr.dtype != np.int32:
            arr = arr.astype(np.int32)
        elif input_tensor.data_type == DataType.DT_INT64 and arr.dtype != np.int64:
            arr = arr.astype(np.int64)
        elif input_tensor.data_type == DataType.DT_FLOAT and arr.dtype != np.float32:
            arr = arr.astype(np.float32)
        bs = input_tensor.dims[0]
        if arr.ndim == len(input_tensor.dims) - 1:
            arr = arr.reshape(arr.shape + (1,))
        self.full = np.ascontiguousarray(arr)
        self._num_samples = int(num_samples if num_samples is not None else arr.shape[0])
        self.batch_size = bs
        self.idx = 0
        self._ring = None
        self._slot = None
        self._pf = None          # H2D prefetcher (GPU only)
        self._inflight = None    # host slot whose copy is in flight
        if self.full.shape[0] >= bs:
            try:
                from flexflow_amd import _core
                # 3 host staging slots filled by the native background thread (gather of the next
                # batch overlaps the current step); a slot is handed back once its batch was fed.
                # On a GPU the slots are pinned so their H2D copies are truly asynchronous.
                shape = (bs,) + self.full.shape[1:]
                if torch.cuda.is_available():
                    self._pinned = [torch.empty(shape, dtype=torch.from_numpy(self.full[:1]).dtype, pin_memory=True)
                                    for _ in range(3)]
                    self._bufs = [t.numpy() for t in self._pinned]
                else:
                    self._pinned = None
                    self._bufs = [np.empty(shape, dtype=self.full.dtype) for _ in range(3)]
                self._ring = _core.BatchRing(self.full, bs, self._bufs)
            except (ImportError, RuntimeError, TypeError):
                self._ring = None

    @property
    def num_samples(self):
        return self._num_samples

    @num_samples.setter
    def num_samples(self, v):
        self._num_samples = int(v)

    def reset(self):
        self.idx = 0
        self._drop_prefetch()
        if self._ring is not None:
            self._ring.reset(0)

    def _drop_prefetch(self):
        if self._pf is not None and self._pf.pending is not None:
            self._pf.take()
            self._release_inflight()

    def _release_inflight(self):
        if self._inflight is not None:
            ev = self._pf.events[self._pf.i] if self._pf is not None else None
            if ev is not None:
                ev.synchronize()
            self._ring.release(self._inflight)
            self._inflight = None

    def _prefetch(self, m):
        if self._pf is None:
            from ..runtime.device import DeviceContext, H2DPrefetcher
            self._pf = H2DPrefetcher(DeviceContext.get(m.executor.device))
        slot = self._ring.next()
        self._pf.stage(self._pinned[slot])
        self._inflight = slot

    def next_batch(self, ffmodel=None):
        m = ffmodel or self.model
        bs = self.batch_size
        if self.idx + bs > self._num_samples:
            self.idx = 0
            self._drop_prefetch()
            if self._ring is not None:
                self._ring.reset(0)
        if self._ring is not None and self._pinned is not None and m.executor.device.type == "cuda":
            if self._pf is None or self._pf.pending is None:
                self._prefetch(m)
            dev = self._pf.take()
            m.executor.feed(self.tensor, dev)  # device-to-device, ordered after the H2D event
            self._release_inflight()
            self.idx += bs
            if self.idx + bs <= self._num_samples:  # stage the next batch under the coming step
                self._prefetch(m)
            return
        if self._ring is not None:
            slot = self._ring.next()
            m.executor.feed(self.tensor, self._bufs[slot])  # pageable source: the copy is complete on return
            self._ring.release(slot)
        else:
            m.executor.feed(self.tensor, self.full[self.idx:self.idx + bs])
        self.idx += bs
