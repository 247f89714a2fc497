"""Strategy selection at compile time (reference FFModel::compile -> Graph::graph_optimize_task,
src/runtime/graph.cc:2047-2318, and the legacy FFModel::mcmc_optimize, model.cc:3286-3357).

Order of precedence:
  1. --import-strategy FILE          (JSON written by --export-strategy)
  2. --only-data-parallel / --search dp
  3. --search unity (default) | mcmc  — the native C++ search in flexflow_amd._core over the
     PCG with the MI355X cost model (pcg/costmodel.py); falls back to data parallel if the
     native core is unavailable.
All ranks compute the same strategy deterministically (the search is seeded); rank 0's choice is
broadcast anyway so that timing-dependent measured costs can never split the job.
"""
from __future__ import annotations

import json
import os

import torch
import torch.distributed as dist

from .strategy import (OpConfig, data_parallel_strategy, load_strategy, load_strategy_pb, load_strategy_text,
                       valid_config)


def _broadcast_strategy(model, strategy):
    if not (dist.is_available() and dist.is_initialized()) or model.config.world_size == 1:
        return strategy
    obj = [{k: v.to_json() for k, v in strategy.items()}]
    dist.broadcast_object_list(obj, src=0)
    return {k: OpConfig.from_json(v) for k, v in obj[0].items()}


def _file_rewrites(path):
    """Rewrite sequence stored in a strategy file's search report (joint search), or a bare list."""
    if not path or path.endswith((".pb", ".strategy")):
        return []
    with open(path) as f:
        doc = json.load(f)
    rw = doc if isinstance(doc, list) else ((doc.get("search") or {}).get("rewrites") or doc.get("rewrites") or [])
    return [(r["xfer"], r["match"]) if isinstance(r, dict) else tuple(r) for r in rw]


def choose_strategy(model):
    cfg = model.config
    n = cfg.num_devices
    report = {"algo": None}
    # a joint search's graph rewrites travel with its strategy file (or --import-rewrites): the
    # imported configs name the rewritten layers, so the graph is rebuilt first
    seq = _file_rewrites(cfg.import_rewrites_file) or _file_rewrites(cfg.import_strategy_file)
    if seq:
        from .joint import replay_broadcast
        replay_broadcast(model, seq)
        report["rewrites"] = [{"xfer": a, "match": b} for a, b in seq]
    layers = model.layers
    if cfg.import_strategy_file:
        if cfg.import_strategy_file.endswith(".pb"):  # the reference's protobuf strategy files
            strat = load_strategy_pb(cfg.import_strategy_file, layers, n)
        elif cfg.import_strategy_file.endswith(".strategy"):  # the reference Triton backend's text form
            strat = load_strategy_text(cfg.import_strategy_file, layers, n)
        else:
            strat, nd = load_strategy(cfg.import_strategy_file)
        missing = [L.name for L in layers if L.name not in strat]
        for L in layers:
            if L.name in strat and not valid_config(L, strat[L.name]):
                raise ValueError(f"imported config for {L.name} is invalid: {strat[L.name]}")
        if missing:
            dp = data_parallel_strategy([L for L in layers if L.name in missing], n)
            strat.update(dp)
        report["algo"] = "import"
        return _broadcast_strategy(model, strat), report
    algo = cfg.search_algo
    if algo in ("dp", "none") or n == 1:
        report["algo"] = "data_parallel"
        return data_parallel_strategy(layers, n), report
    try:
        from flexflow_amd import _core  # noqa: F401
        from .unity import search as native_search
    except ImportError:
        native_search = None
    if native_search is None:
        report["algo"] = "data_parallel(fallback: native core not built)"
        return data_parallel_strategy(layers, n), report
    distributed = dist.is_available() and dist.is_initialized() and cfg.world_size > 1
    # joint Unity search (graph rewrites x parallelization) by default at N > 1; --search mcmc and
    # FF_JOINT=0 search configs on the graph as written
    joint = algo == "unity" and os.environ.get("FF_JOINT", "1") != "0" and not seq
    if distributed and cfg.rank != 0:
        # rank 0 searches (its measured costs decide); everyone else receives the result and, for
        # the joint search, replays rank 0's rewrite sequence on its own copy of the graph
        obj = [None, None, None]
        dist.broadcast_object_list(obj, src=0)
        if obj[2]:
            from .joint import replay_broadcast
            replay_broadcast(model, obj[2])
        return {k: OpConfig.from_json(v) for k, v in obj[0].items()}, obj[1]
    seq = []
    import time
    t0 = time.perf_counter()
    if joint:
        from .joint import joint_search
        strat, report, seq = joint_search(model, algo)
    else:
        strat, report = native_search(model, algo)
    report = dict(report or {})
    report["search_wall_s"] = round(time.perf_counter() - t0, 2)  # measurement + search, rank 0
    from .costmodel import STATS
    report["cost_lookups"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in STATS.items()}
    from .costmodel import save_cost_table
    save_cost_table()
    if distributed:
        dist.broadcast_object_list([{k: v.to_json() for k, v in strat.items()}, report, seq], src=0)
    return strat, report
