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


def choose_strategy(model):
    cfg = model.config
    layers = model.layers
    n = cfg.num_devices
    report = {"algo": None}
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
    if distributed and cfg.rank != 0:
        # rank 0 searches (its measured costs decide); everyone else receives the result
        obj = [None, None]
        dist.broadcast_object_list(obj, src=0)
        return {k: OpConfig.from_json(v) for k, v in obj[0].items()}, obj[1]
    strat, report = native_search(model, algo)
    if distributed:
        dist.broadcast_object_list([{k: v.to_json() for k, v in strat.items()}, report], src=0)
    return strat, report
