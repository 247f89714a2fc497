"""HTTP inference server speaking the KServe v2 / Triton HTTP protocol.

The reference serves its ONNX models through Triton (triton/src/backend.cc implements
TRITONBACKEND_ModelInstanceExecute; clients talk to Triton's HTTP endpoint, triton/qa/L0_e2e/
operator_test.py). This server is ours and speaks the same protocol, so the same requests work:

  GET  /v2  /v2/health/live  /v2/health/ready
  GET  /v2/models/<m>[/versions/<v>]            metadata       .../ready   .../config   .../stats
  POST /v2/models/<m>[/versions/<v>]/infer      inference (JSON tensors, or the binary tensor
                                                extension: Inference-Header-Content-Length)
  POST /v2/repository/index   /v2/repository/models/<m>/load   /v2/repository/models/<m>/unload

Each request is handled on its own thread; a model with max_batch_size > 0 coalesces concurrent
requests in the native dynamic batcher (engine.DynamicBatcher).
"""
from __future__ import annotations

import json
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import List, Optional, Tuple

import numpy as np

from .config import NP_TO_WIRE, WIRE_TO_NP
from .engine import InferError
from .repository import ModelRepository

VERSION = "0.2.0"
EXTENSIONS = ["binary_tensor_data", "model_repository", "statistics", "model_configuration"]
_MODEL = re.compile(r"^/v2/models/([^/]+)(?:/versions/([^/]+))?(/ready|/infer|/config|/stats)?/?$")
_REPO = re.compile(r"^/v2/repository/models/([^/]+)/(load|unload)/?$")


def decode_request(body: bytes, header_len: Optional[int]) -> Tuple[dict, dict]:
    """Returns (request json, {input name: ndarray})."""
    js = body[:header_len] if header_len is not None else body
    req = json.loads(js.decode() or "{}")
    tail = body[header_len:] if header_len is not None else b""
    off = 0
    arrays = {}
    for inp in req.get("inputs", []):
        name = inp["name"]
        dt = inp.get("datatype", "FP32")
        if dt not in WIRE_TO_NP:
            raise InferError(f"input {name!r}: unsupported datatype {dt}")
        shape = [int(d) for d in inp.get("shape", [])]
        nbytes = (inp.get("parameters") or {}).get("binary_data_size")
        if nbytes is not None:
            raw = tail[off:off + int(nbytes)]
            off += int(nbytes)
            a = np.frombuffer(raw, dtype=WIRE_TO_NP[dt])
        else:
            a = np.asarray(inp.get("data", []), dtype=WIRE_TO_NP[dt])
        if a.size != int(np.prod(shape)):
            raise InferError(f"input {name!r}: {a.size} elements for shape {shape}")
        arrays[name] = a.reshape(shape)
    return req, arrays


def encode_response(model_name: str, version: str, req: dict, outs: dict) -> Tuple[bytes, Optional[int]]:
    want = {o["name"]: o for o in req.get("outputs", [])}
    default_bin = bool((req.get("parameters") or {}).get("binary_data_output", False))
    items, blobs = [], []
    for name, v in outs.items():
        v = np.ascontiguousarray(v)
        o = {"name": name, "datatype": NP_TO_WIRE[v.dtype], "shape": list(v.shape)}
        binary = bool(((want.get(name) or {}).get("parameters") or {}).get("binary_data", default_bin))
        if binary:
            b = v.tobytes()
            o["parameters"] = {"binary_data_size": len(b)}
            blobs.append(b)
        else:
            o["data"] = v.reshape(-1).tolist()
        items.append(o)
    resp = {"model_name": model_name, "model_version": version, "outputs": items}
    if "id" in req:
        resp["id"] = req["id"]
    js = json.dumps(resp).encode()
    if blobs:
        return js + b"".join(blobs), len(js)
    return js, None


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server_version = "flexflow_amd/" + VERSION

    def log_message(self, fmt, *args):  # quiet by default
        if getattr(self.server, "verbose", False):
            super().log_message(fmt, *args)

    @property
    def repo(self) -> ModelRepository:
        return self.server.repo

    def _send(self, code: int, payload=None, raw: Optional[bytes] = None, header_len: Optional[int] = None):
        body = raw if raw is not None else (json.dumps(payload).encode() if payload is not None else b"")
        self.send_response(code)
        self.send_header("Content-Type", "application/octet-stream" if header_len is not None else "application/json")
        if header_len is not None:
            self.send_header("Inference-Header-Content-Length", str(header_len))
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _err(self, code: int, msg: str):
        self._send(code, {"error": msg})

    def do_GET(self):  # noqa: N802
        p = self.path.split("?")[0]
        if p in ("/v2", "/v2/"):
            return self._send(200, {"name": "flexflow_amd", "version": VERSION, "extensions": EXTENSIONS})
        if p == "/v2/health/live":
            return self._send(200)
        if p == "/v2/health/ready":
            return self._send(200 if self.server.ready.is_set() else 400)
        m = _MODEL.match(p)
        if not m:
            return self._err(404, f"no route {p}")
        name, ver, tail = m.group(1), m.group(2), m.group(3) or ""
        try:
            model = self.repo.get(name, ver)
        except KeyError as e:
            return self._err(400 if tail == "/ready" else 404, str(e))
        if tail == "/ready":
            return self._send(200)
        if tail == "/config":
            c = model.config
            return self._send(200, {"name": c.name, "backend": c.backend, "max_batch_size": c.max_batch_size,
                                    "input": [{"name": s.name, "data_type": s.data_type, "dims": s.dims}
                                              for s in c.inputs],
                                    "output": [{"name": s.name, "data_type": s.data_type, "dims": s.dims}
                                               for s in c.outputs],
                                    "dynamic_batching": {"preferred_batch_size": c.preferred_batch_size,
                                                         "max_queue_delay_microseconds": c.max_queue_delay_us}
                                    if c.dynamic_batching else None})
        if tail == "/stats":
            return self._send(200, {"model_stats": [dict(name=name, version=model.version, **model.stats())]})
        meta = model.config.to_json()
        meta["versions"] = [model.version]
        return self._send(200, meta)

    def do_POST(self):  # noqa: N802
        p = self.path.split("?")[0]
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n else b""
        if p == "/v2/repository/index":
            return self._send(200, self.repo.index())
        m = _REPO.match(p)
        if m:
            name, act = m.group(1), m.group(2)
            try:
                if act == "load":
                    self.repo.load(name)
                else:
                    self.repo.unload(name)
            except Exception as e:  # noqa: BLE001
                return self._err(400, f"{act} {name}: {e}")
            return self._send(200)
        m = _MODEL.match(p)
        if not m or m.group(3) != "/infer":
            return self._err(404, f"no route {p}")
        name, ver = m.group(1), m.group(2)
        try:
            model = self.repo.get(name, ver)
        except KeyError as e:
            return self._err(404, str(e))
        hl = self.headers.get("Inference-Header-Content-Length")
        try:
            req, arrays = decode_request(body, int(hl) if hl is not None else None)
            outs = model.infer(arrays, [o["name"] for o in req.get("outputs", [])] or None)
        except (InferError, KeyError, ValueError) as e:
            return self._err(400, str(e))
        except Exception as e:  # noqa: BLE001 - an execution failure is a 500, the server keeps serving
            return self._err(500, f"{type(e).__name__}: {e}")
        raw, header_len = encode_response(name, model.version, req, outs)
        return self._send(200, raw=raw, header_len=header_len)


class InferenceServer:
    """`InferenceServer(repo_root).start()` serves in a background thread; `serve_forever()` blocks."""

    def __init__(self, repo_root: str, host: str = "127.0.0.1", port: int = 8000, ff_flags: Optional[List[str]] = None,
                 verbose: bool = False, strict: bool = False):
        self.repo = ModelRepository(repo_root, ff_flags)
        self.strict = strict
        self.httpd = ThreadingHTTPServer((host, port), _Handler)
        self.httpd.daemon_threads = True
        self.httpd.repo = self.repo
        self.httpd.verbose = verbose
        self.httpd.ready = threading.Event()
        self._thread = None

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    @property
    def url(self) -> str:
        return f"{self.httpd.server_address[0]}:{self.port}"

    def load(self):
        errs = self.repo.load_all(strict=self.strict)
        self.httpd.ready.set()
        return errs

    def start(self):
        self.load()
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="ff-http", daemon=True)
        self._thread.start()
        return self

    def serve_forever(self):
        self.load()
        self.httpd.serve_forever()

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()
        self.repo.close()
