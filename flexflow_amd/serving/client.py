"""Minimal HTTP client for the server, mirroring tritonclient.http's surface
(InferenceServerClient / InferInput / InferRequestedOutput / InferResult), so the reference's
Triton tests (triton/qa/L0_e2e/operator_test.py) read the same against this server. Standard
library only (urllib); JSON tensors or the binary tensor extension."""
from __future__ import annotations

import json
import urllib.error
import urllib.request
from typing import List, Optional

import numpy as np

from .config import NP_TO_WIRE, WIRE_TO_NP


class InferenceServerException(Exception):
    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status

    def message(self):
        return str(self)


class InferInput:
    def __init__(self, name: str, shape: List[int], datatype: str):
        self._name, self._shape, self._datatype = name, list(shape), datatype
        self._data = None
        self._raw = None

    def name(self):
        return self._name

    def shape(self):
        return self._shape

    def datatype(self):
        return self._datatype

    def set_data_from_numpy(self, arr: np.ndarray, binary_data: bool = True):
        arr = np.ascontiguousarray(arr, dtype=WIRE_TO_NP[self._datatype])
        if list(arr.shape) != self._shape:
            raise InferenceServerException(f"{self._name}: array shape {list(arr.shape)} != {self._shape}")
        if binary_data:
            self._raw, self._data = arr.tobytes(), None
        else:
            self._raw, self._data = None, arr.reshape(-1).tolist()
        return self

    def _json(self):
        d = {"name": self._name, "shape": self._shape, "datatype": self._datatype}
        if self._raw is not None:
            d["parameters"] = {"binary_data_size": len(self._raw)}
        else:
            d["data"] = self._data
        return d


class InferRequestedOutput:
    def __init__(self, name: str, binary_data: bool = True):
        self._name, self._binary = name, binary_data

    def name(self):
        return self._name

    def _json(self):
        return {"name": self._name, "parameters": {"binary_data": self._binary}}


class InferResult:
    def __init__(self, resp: dict, tail: bytes):
        self._resp = resp
        self._arrays = {}
        off = 0
        for o in resp.get("outputs", []):
            dt = WIRE_TO_NP[o["datatype"]]
            n = (o.get("parameters") or {}).get("binary_data_size")
            if n is not None:
                a = np.frombuffer(tail[off:off + n], dtype=dt)
                off += n
            else:
                a = np.asarray(o.get("data", []), dtype=dt)
            self._arrays[o["name"]] = a.reshape(o["shape"])

    def as_numpy(self, name: str) -> Optional[np.ndarray]:
        return self._arrays.get(name)

    def get_response(self) -> dict:
        return self._resp


class InferenceServerClient:
    def __init__(self, url: str = "localhost:8000", timeout: float = 60.0):
        self.base = url if url.startswith("http") else "http://" + url
        self.timeout = timeout

    def _req(self, method, path, body=None, headers=None):
        r = urllib.request.Request(self.base + path, data=body, method=method, headers=headers or {})
        try:
            with urllib.request.urlopen(r, timeout=self.timeout) as f:
                return f.status, dict(f.headers), f.read()
        except urllib.error.HTTPError as e:
            data = e.read()
            try:
                msg = json.loads(data).get("error", data.decode())
            except Exception:  # noqa: BLE001
                msg = data.decode(errors="replace")
            raise InferenceServerException(msg, e.code) from None

    def _ok(self, path):
        try:
            return self._req("GET", path)[0] == 200
        except InferenceServerException:
            return False

    def is_server_live(self):
        return self._ok("/v2/health/live")

    def is_server_ready(self):
        return self._ok("/v2/health/ready")

    def is_model_ready(self, model_name, model_version=""):
        v = f"/versions/{model_version}" if model_version else ""
        return self._ok(f"/v2/models/{model_name}{v}/ready")

    def get_server_metadata(self):
        return json.loads(self._req("GET", "/v2")[2])

    def get_model_metadata(self, model_name, model_version=""):
        v = f"/versions/{model_version}" if model_version else ""
        return json.loads(self._req("GET", f"/v2/models/{model_name}{v}")[2])

    def get_model_config(self, model_name):
        return json.loads(self._req("GET", f"/v2/models/{model_name}/config")[2])

    def get_inference_statistics(self, model_name):
        return json.loads(self._req("GET", f"/v2/models/{model_name}/stats")[2])

    def get_model_repository_index(self):
        return json.loads(self._req("POST", "/v2/repository/index", b"")[2])

    def load_model(self, model_name):
        self._req("POST", f"/v2/repository/models/{model_name}/load", b"")

    def unload_model(self, model_name):
        self._req("POST", f"/v2/repository/models/{model_name}/unload", b"")

    def infer(self, model_name, inputs, model_version="", outputs=None, request_id=""):
        req = {"inputs": [i._json() for i in inputs]}
        if outputs:
            req["outputs"] = [o._json() for o in outputs]
        if request_id:
            req["id"] = request_id
        js = json.dumps(req).encode()
        blobs = b"".join(i._raw for i in inputs if i._raw is not None)
        headers = {"Content-Type": "application/octet-stream" if blobs else "application/json"}
        if blobs:
            headers["Inference-Header-Content-Length"] = str(len(js))
        v = f"/versions/{model_version}" if model_version else ""
        _, hdrs, body = self._req("POST", f"/v2/models/{model_name}{v}/infer", js + blobs, headers)
        hl = {k.lower(): v for k, v in hdrs.items()}.get("inference-header-content-length")
        if hl is not None:
            n = int(hl)
            return InferResult(json.loads(body[:n]), body[n:])
        return InferResult(json.loads(body), b"")


__all__ = ["InferenceServerClient", "InferInput", "InferRequestedOutput", "InferResult", "InferenceServerException",
           "NP_TO_WIRE"]
