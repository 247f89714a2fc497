"""Per-rank device context (reference FFHandler, include/flexflow/config.h:63-77, created by
UtilityTasks::init_cuda_task, src/runtime/model.cu:77-125, once per GPU).

The reference keeps cuBLAS/cuDNN handles, a 1 GiB work area and an optional NCCL communicator per
GPU. Here one process drives one MI355X, so the context is per process and holds what the runtime
shares across ops:

  * streams: `compute` (the current stream: kernels, hipGraph replay), `h2d` (input staging —
    the next batch's host->device copy runs under the current step), `side` (auxiliary work that
    must not serialise with compute, e.g. host-visible metric snapshots);
  * a grow-only workspace arena keyed by purpose (kernel scratch such as the attention-backward
    dQ partial slabs), so steady-state steps allocate nothing;
  * the RCCL process groups live in parallel/comm.Communicator (one per replica set).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch


class DeviceContext:
    _by_device: Dict[str, "DeviceContext"] = {}

    def __init__(self, device: torch.device):
        self.device = device
        self.is_cuda = device.type == "cuda" and torch.cuda.is_available()
        if self.is_cuda:
            self.h2d = torch.cuda.Stream(device=device)
            self.side = torch.cuda.Stream(device=device)
        else:
            self.h2d = self.side = None
        self._ws: Dict[str, torch.Tensor] = {}

    @classmethod
    def get(cls, device: Optional[torch.device] = None) -> "DeviceContext":
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        key = str(device)
        ctx = cls._by_device.get(key)
        if ctx is None:
            ctx = cls._by_device[key] = DeviceContext(device)
        return ctx

    @property
    def compute(self):
        return torch.cuda.current_stream(self.device) if self.is_cuda else None

    def workspace(self, key: str, numel: int, dtype=torch.float32) -> torch.Tensor:
        """A buffer of at least `numel` elements reused across calls with the same key. Inside a
        hipGraph capture the buffer must already exist (it is part of the captured addresses)."""
        buf = self._ws.get(key)
        if buf is None or buf.numel() < numel or buf.dtype != dtype:
            if self.is_cuda and torch.cuda.is_current_stream_capturing():
                return torch.empty(numel, dtype=dtype, device=self.device)
            buf = torch.empty(max(numel, 1), dtype=dtype, device=self.device)
            self._ws[key] = buf
        return buf[:numel]

    def workspace_bytes(self) -> int:
        return sum(b.numel() * b.element_size() for b in self._ws.values())


class H2DPrefetcher:
    """Double-buffered host->device staging on the context's h2d stream: `stage(host_tensor)`
    starts the copy of the next batch (source must be pinned for the copy to be asynchronous) and
    returns immediately; `take()` makes the compute stream wait for it and returns the device
    tensor. The two device buffers alternate, so the batch being consumed is never overwritten by
    the one in flight."""

    def __init__(self, ctx: DeviceContext):
        self.ctx = ctx
        self.bufs = [None, None]
        self.events = [None, None]
        self.i = 0
        self.pending = None

    def stage(self, host: torch.Tensor):
        self.i ^= 1
        i = self.i
        b = self.bufs[i]
        if b is None or b.shape != host.shape or b.dtype != host.dtype:
            b = self.bufs[i] = torch.empty(host.shape, dtype=host.dtype, device=self.ctx.device)
        if not self.ctx.is_cuda:
            b.copy_(host)
            self.pending = i
            return
        st = self.ctx.h2d
        # the buffer's previous consumer (two batches ago) ran on the compute stream
        st.wait_stream(torch.cuda.current_stream(self.ctx.device))
        with torch.cuda.stream(st):
            b.copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        self.events[i] = ev
        self.pending = i

    def take(self) -> torch.Tensor:
        i = self.pending
        if i is None:
            raise RuntimeError("H2DPrefetcher.take() without a staged batch")
        self.pending = None
        if self.ctx.is_cuda and self.events[i] is not None:
            torch.cuda.current_stream(self.ctx.device).wait_event(self.events[i])
        return self.bufs[i]
