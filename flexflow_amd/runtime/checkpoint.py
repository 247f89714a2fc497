"""Checkpoint / resume (the reference has only per-tensor host get/set, parallel_tensor.cc:650-748;
long runs need whole-job checkpoints).

Layout of a checkpoint directory:
    meta.json                 step, world size, strategy (per-op OpConfig JSON), optimizer hyper-
                              parameters and bias-correction state, arena layout
    rank{r}.safetensors       that rank's fp32 master weights and optimizer state, one tensor per
                              weight arena ("arena{i}.master", "arena{i}.m", "arena{i}.v", ...)
Every rank writes its own shard (no gather through rank 0: 288 GB HBM per GPU means shards can be
large), loading checks that the strategy and arena layout match the running job. Files are
safetensors — no pickle anywhere, so checkpoints from an untrusted source cannot execute code.
"""
from __future__ import annotations

import json
import os

import torch
from safetensors import safe_open
from safetensors.torch import load_file, save_file


def _weight_keys(model):
    """Sharding- and arena-order-independent identity of every weight: (layer position, slot)."""
    keys = {}
    for li, L in enumerate(model.layers):
        for i, w in enumerate(L.weights):
            keys.setdefault(w.guid, f"{li}:{i}")
    return keys


def _arenas(ex):
    return [(i, ar) for i, ar in enumerate(ex.arenas.values()) if ar.size]


def _used(ar) -> int:
    """Elements of the arena actually holding weights (the rest is alignment / ZeRO padding)."""
    return max((int(e[1]) + int(e[2]) for e in ar.entries), default=0)


def save_checkpoint(model, path: str):
    ex = model.executor
    opt = model.optimizer
    cfg = model.config
    if getattr(ex, "zero", False):
        # sharded optimizer: every rank saves the full master AND the full optimizer state, so
        # the checkpoint is independent of the sharding geometry it was written under
        ex.sync_master()
        ex.sync_optimizer_state(opt)
    os.makedirs(path, exist_ok=True)
    tensors = {}
    layout = []
    wkeys = _weight_keys(model)
    for i, ar in _arenas(ex):
        tensors[f"arena{i}.master"] = ar.master.detach().contiguous().cpu()
        st = getattr(opt, "state", {}).get(id(ar))
        if st is not None:
            for j, t in enumerate(st if isinstance(st, (tuple, list)) else (st,)):
                tensors[f"arena{i}.opt{j}"] = t.detach().contiguous().cpu()
        layout.append({"arena": i, "size": int(ar.size), "used": _used(ar),
                       "entries": [[wkeys.get(e[0].guid, getattr(e[0], "name", str(e[0]))), int(e[1]), int(e[2]),
                                    list(e[3])] for e in ar.entries]})
    # every rank's own arena layout travels inside its shard: arena order and offsets depend on
    # the rank's placement, self.training and weight sharing, so the loader maps entry by entry
    save_file(tensors, os.path.join(path, f"rank{cfg.rank}.safetensors"),
              metadata={"arenas": json.dumps(layout)})
    if cfg.rank == 0:
        meta = {
            "step": int(ex.step_idx),
            "world_size": int(cfg.world_size),
            # informational: the state above is gathered, so resuming under another sharding is fine
            "zero": bool(getattr(ex, "zero", False)),
            "grad_bucket_bytes": int(getattr(ex.bucketer, "bucket_bytes", 0) or 0),
            # positional (layer order), so a rebuilt model whose auto-generated names differ still matches
            "strategy": [[L.name, L.op_type.name, model.strategy[L.name].to_json()] for L in model.layers],
            "optimizer": {k: v for k, v in vars(opt).items() if isinstance(v, (int, float, bool, str))},
            "arenas": layout,
        }
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()
    return path


def load_checkpoint(model, path: str, strict: bool = True):
    ex = model.executor
    opt = model.optimizer
    cfg = model.config
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if strict and meta["world_size"] != cfg.world_size:
        raise ValueError(f"checkpoint was written by {meta['world_size']} ranks, job has {cfg.world_size}")
    if strict:
        cur = [[L.op_type.name, model.strategy[L.name].to_json()] for L in model.layers]
        if cur != [[op, c] for _, op, c in meta["strategy"]]:
            raise ValueError("checkpoint strategy differs from the compiled strategy (import it with "
                             "--import-strategy to resume)")
    fn = os.path.join(path, f"rank{cfg.rank}.safetensors")
    tensors = load_file(fn)
    with safe_open(fn, framework="pt") as f:
        md = f.metadata() or {}
    if "arenas" not in md:
        # written before per-entry layouts were stored: the old whole-arena copy is safe only when
        # this job has the writer's world size and strategy (checked above under strict=True) AND
        # its arenas have exactly the sizes the shard holds; equal sizes alone do not mean equal
        # contents (a permuted placement or bucket order gives equal sizes)
        if not strict:
            raise ValueError(f"{fn} has no per-entry arena layout (written by an older version); it can only be "
                             "loaded with strict=True (same world size and strategy)")
        arenas = _arenas(ex)
        if not all(f"arena{i}.master" in tensors and tensors[f"arena{i}.master"].numel() == ar.size
                   for i, ar in arenas):
            raise ValueError(f"{fn} has no per-entry arena layout (written by an older version) and its "
                             "arena sizes differ from this job's; it cannot be mapped safely")
        for i, ar in arenas:
            ar.master.copy_(tensors[f"arena{i}.master"].to(ar.master.device))
            st = getattr(opt, "state", {}).get(id(ar))
            for j, t in enumerate(list(st) if isinstance(st, (tuple, list)) else ([st] if st is not None else [])):
                if f"arena{i}.opt{j}" in tensors:
                    t.copy_(tensors[f"arena{i}.opt{j}"].to(t.device))
            if ar.lowp is not None:
                ar.lowp.copy_(ar.master.to(ar.lowp.dtype))
        md = None
    # saved weight key -> (arena index, offset, numel, shape)
    saved = {}
    for a in (json.loads(md["arenas"]) if md is not None else []):
        for key, off, n, shape in a["entries"]:
            saved[key] = (a["arena"], int(off), int(n), tuple(shape))
    wkeys = _weight_keys(model)
    for i, ar in (_arenas(ex) if md is not None else []):
        ar.master.zero_()
        st = getattr(opt, "state", {}).get(id(ar))
        st = list(st) if isinstance(st, (tuple, list)) else ([st] if st is not None else [])
        for t in st:
            t.zero_()
        for w, off, n, shape in ar.entries:
            key = wkeys.get(w.guid)
            if key not in saved:
                raise ValueError(f"weight {getattr(w, 'name', key)} ({key}) is not in checkpoint {fn}")
            si, soff, sn, sshape = saved[key]
            if sn != n or tuple(sshape) != tuple(shape):
                raise ValueError(f"weight {getattr(w, 'name', key)}: checkpoint shard {sshape} != job shard {tuple(shape)}")
            src = tensors[f"arena{si}.master"]
            ar.master[off:off + n].copy_(src[soff:soff + n].to(ar.master.device))
            for j, t in enumerate(st):
                sk = f"arena{si}.opt{j}"
                if sk in tensors:
                    t[off:off + n].copy_(tensors[sk][soff:soff + n].to(t.device))
        if ar.lowp is not None:
            ar.lowp.copy_(ar.master.to(ar.lowp.dtype))
    for k, v in meta.get("optimizer", {}).items():
        if hasattr(opt, k) and not callable(getattr(opt, k)):
            setattr(opt, k, v)
    ex._master_stale = False  # every rank now holds the full master
    ex.step_idx = int(meta["step"])
    return meta["step"]
