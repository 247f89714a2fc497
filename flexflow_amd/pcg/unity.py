"""Search driver: lowers the layer graph to the native search problem (flexflow_amd._core) and maps
the chosen candidate indices back to per-op OpConfigs.

  unity : exact frontier-DP over per-op configs (additive cost) seeded into a simulator-driven
          MCMC refinement (overlap / inter-op concurrency) — reference GraphSearchHelper +
          SearchHelper (src/runtime/substitution.cc, graph.cc), with graph substitutions applied
          by pcg/substitutions.py before the search;
  mcmc  : the reference's MCMC (model.cc:3286-3357) from the data-parallel strategy, --budget
          iterations, --alpha temperature.
The parallelization axes explored follow the reference switches: sample (data) parallelism
always; parameter parallelism (channels / heads / reductions / vocab) unless
--only-data-parallel; attribute (spatial / sequence) parallelism with --enable-attribute-parallel.
"""
from __future__ import annotations

import os
import time

import torch

from ..parallel.layout import Layout
from ..type import DataType, OperatorType
from . import costmodel
from .strategy import OpConfig, data_parallel_config, enumerate_configs, op_layouts, valid_config


def _core():
    from flexflow_amd import _core
    return _core


def to_core_layout(l: Layout):
    c = _core().Layout()
    c.shape = list(l.shape)
    c.degrees = list(l.degrees)
    c.replicas = l.replicas
    c.devices = list(l.devices)
    c.partial = l.partial
    c.halo = list(l.halo) if l.halo else []
    return c


def machine_model(cfg):
    core = _core()
    mm = core.MachineModel()
    n = cfg.num_devices
    gpn = max(1, min(cfg.local_world_size if cfg.search_num_workers is None else cfg.search_num_workers, n))
    mm.gpus_per_node = gpn
    mm.num_nodes = max(1, n // gpn)
    if cfg.machine_model_file and os.path.exists(cfg.machine_model_file):
        import json
        with open(cfg.machine_model_file) as f:
            d = json.load(f)
        for k, v in d.items():
            if hasattr(mm, k):
                setattr(mm, k, v)
    return mm


def allowed_kinds(cfg):
    if cfg.only_data_parallel:
        return ("sample",)
    k = ["sample", "parameter"]
    if cfg.enable_attribute_parallel:
        k.append("attribute")
    return tuple(k)


def build_problem(model, n_devices: int, measure: bool):
    core = _core()
    cfg = model.config
    layers = model.layers
    idx = {L.name: i for i, L in enumerate(layers)}
    out_owner = {}
    for i, L in enumerate(layers):
        for j, o in enumerate(L.outputs):
            out_owner[o.guid] = (i, j)
    prob = core.Problem()
    prob.machine = machine_model(cfg)
    device = None
    if torch.cuda.is_available():
        device = torch.device("cuda", cfg.local_rank % torch.cuda.device_count())
    kinds = allowed_kinds(cfg)
    cdt = cfg.compute_dtype
    elem = 2 if cdt == DataType.DT_BF16 else 4
    all_cands = []
    nodes = []
    out_t = model.output_tensor()
    from .strategy import machine_device_sets
    dsets = machine_device_sets(n_devices, prob.machine.gpus_per_node)
    for i, L in enumerate(layers):
        cands = enumerate_configs(L, n_devices, kinds, max_configs=int(os.environ.get("FF_MAX_CANDS", "32")),
                                  device_sets=dsets)
        dp = data_parallel_config(L, n_devices)
        if dp not in cands:
            cands.append(dp)
        all_cands.append(cands)
        node = core.Node()
        node.name = L.name
        node.op_type = L.op_type.name
        node.inputs = [out_owner.get(t.guid, (-1, 0)) for t in L.inputs]
        node.input_needs_grad = [L.impl.needs_input_grad(j) and t.data_type == DataType.DT_FLOAT
                                 for j, t in enumerate(L.inputs)]
        node.elem_bytes = elem
        node.backward = L.op_type != OperatorType.OP_INPUT
        cc = []
        for c in cands:
            lo = op_layouts(L, c)
            oc = core.OpCandidate()
            oc.degrees = list(c.degrees)
            oc.devices = list(c.devices)
            f, b = costmodel.op_cost(L, c, cdt, measure, device)
            oc.fwd_ms, oc.bwd_ms = f, b
            oc.mem_bytes = costmodel.mem_bytes(L, c, cdt)
            oc.in_layouts = [to_core_layout(x) for x in lo.inputs]
            oc.out_layouts = [to_core_layout(x) for x in lo.outputs]
            oc.w_layouts = [to_core_layout(x) for x in lo.weights]
            cc.append(oc)
        node.cands = cc
        nodes.append(node)
    prob.nodes = nodes
    return prob, all_cands


def search(model, algo: str):
    cfg = model.config
    n = cfg.num_devices
    core = _core()
    t0 = time.perf_counter()
    measure = os.environ.get("FF_MEASURE_COSTS", "auto")
    do_measure = torch.cuda.is_available() if measure == "auto" else measure == "1"
    prob, cands = build_problem(model, n, do_measure)
    t_build = time.perf_counter() - t0
    dp_choice = [cands[i].index(data_parallel_config(L, n)) for i, L in enumerate(model.layers)]
    dp_sim = core.simulate(prob, dp_choice).makespan_ms
    budget = cfg.search_budget if cfg.search_budget and cfg.search_budget > 0 else None
    if algo == "mcmc":
        iters = budget or cfg.mcmc_iterations
        res = core.search_mcmc(prob, dp_choice, iters, cfg.search_alpha, cfg.seed)
    else:
        iters = budget if budget is not None else 300
        res = core.search_unity(prob, 4096, iters, cfg.search_alpha, cfg.seed)
    choice = list(res.choice)
    if res.cost_ms > dp_sim:  # never pick something the simulator thinks is worse than DP
        choice = dp_choice
    strat = {L.name: cands[i][choice[i]] for i, L in enumerate(model.layers)}
    report = {"algo": algo, "devices": n, "predicted_ms": round(min(res.cost_ms, dp_sim), 4),
              "predicted_dp_ms": round(dp_sim, 4), "predicted_speedup_vs_dp": round(dp_sim / max(min(res.cost_ms, dp_sim), 1e-9), 4),
              "dp_objective_ms": round(res.dp_cost_ms, 4), "states": int(res.states),
              "mcmc_iterations": int(res.iterations), "build_s": round(t_build, 3),
              "search_s": round(time.perf_counter() - t0 - t_build, 3), "measured_costs": bool(do_measure),
              "candidates": sum(len(c) for c in cands)}
    return strat, report
