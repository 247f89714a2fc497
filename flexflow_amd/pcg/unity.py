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
import sys
import time
from types import SimpleNamespace

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
    if cfg.device_mem and cfg.device_mem > 0:  # -ll:fsize, MiB of device memory per GPU
        mm.mem_capacity = float(cfg.device_mem) * (1 << 20)
    d = {}
    if cfg.machine_model_file and os.path.exists(cfg.machine_model_file):
        import json
        with open(cfg.machine_model_file) as f:
            d = json.load(f)
        for k, v in d.items():
            if hasattr(mm, k) and not callable(getattr(mm, k)) and k != "has_topology":
                setattr(mm, k, v)
    if cfg.machine_model_version == 1 or "links" in d or "topology" in d:
        mm.set_topology(network_topology(mm, d))
    return mm


def network_topology(mm, d: dict):
    """machine_model_version 1 (reference NetworkedMachineModel, src/runtime/network.cc): an explicit
    link graph with shortest-path routing and per-link contention. From the machine-model JSON either
    "links": [[a, b, GB/s], ...] over GPUs 0..N-1 plus "switches": K extra vertices N..N+K-1, or a
    generated MI355X cluster, "topology": "fat_tree" | "big_switch" (default fat_tree) with
    "oversub" (leaf-to-spine oversubscription), using link_gbps / inter_node_gbps of the model."""
    core = _core()
    if "links" in d:
        t = core.NetworkTopology()
        t.num_gpus = mm.num_devices()
        for _ in range(mm.num_devices() + int(d.get("switches", 0))):
            t.add_node()
        for a, b, g in d["links"]:
            t.add_link(int(a), int(b), float(g))
        t.build_routes()
        return t
    return core.make_mi355x_cluster(mm.num_nodes, mm.gpus_per_node, mm.link_gbps, mm.inter_node_gbps,
                                    d.get("topology", "fat_tree"), float(d.get("oversub", 1.0)))


def allowed_kinds(cfg):
    if cfg.only_data_parallel:
        return ("sample",)
    k = ["sample", "parameter"]
    if cfg.enable_attribute_parallel:
        k.append("attribute")
    return tuple(k)


_CAND_CACHE: dict = {}


def layer_signature(L) -> tuple:
    """Everything an op's candidate configs, layouts and costs depend on (not its name/position)."""
    return (L.op_type.value, tuple((tuple(t.dims), t.data_type.value) for t in L.inputs),
            tuple((tuple(w.dims), w.data_type.value) for w in L.weights),
            tuple((tuple(o.dims), o.data_type.value) for o in L.outputs),
            repr(sorted((k, repr(v)) for k, v in L.attrs.items() if k not in ("kernel_init", "bias_init", "name"))),
            tuple(L.impl.needs_input_grad(j) for j in range(len(L.inputs))))


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
    max_cands = int(os.environ.get("FF_MAX_CANDS", "32"))
    progress = os.environ.get("FF_SEARCH_PROGRESS") == "1"  # long measured searches: a line per 16 ops
    t_prog = time.perf_counter()
    for i, L in enumerate(layers):
        if progress and i % 16 == 0:
            print(f"[search] costing op {i}/{len(layers)} ({time.perf_counter() - t_prog:.1f} s)", file=sys.stderr,
                  flush=True)
        # candidates and their costs depend only on the op's signature: identical layers (BERT's 24
        # encoder layers) and the unchanged layers of a rewritten graph (joint search) reuse them
        key = (layer_signature(L), n_devices, kinds, cdt, bool(measure), prob.machine.gpus_per_node, max_cands,
               str(device))
        hit = _CAND_CACHE.get(key)
        if hit is None:
            cands = enumerate_configs(L, n_devices, kinds, max_configs=max_cands, device_sets=dsets)
            dp = data_parallel_config(L, n_devices)
            if dp not in cands:
                cands.append(dp)
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
            hit = _CAND_CACHE[key] = (cands, cc)
        cands, cc = hit
        all_cands.append(list(cands))
        node = core.Node()
        node.name = L.name
        node.op_type = L.op_type.name
        node.inputs = [out_owner.get(t.guid, (-1, 0)) for t in L.inputs]
        node.input_needs_grad = [L.impl.needs_input_grad(j) and t.data_type == DataType.DT_FLOAT
                                 for j, t in enumerate(L.inputs)]
        node.elem_bytes = elem
        node.backward = L.op_type != OperatorType.OP_INPUT
        node.cands = cc
        nodes.append(node)
    prob.nodes = nodes
    return prob, all_cands


def search(model, algo: str, quick: bool = False):
    """quick: the frontier DP only (no simulator-driven MCMC, no resource-split refinement) — how
    the joint search ranks candidate graphs before the full search of the best one."""
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

    def run_search():
        if quick:  # ranking rewritten graphs (joint search): a narrower frontier, no refinement
            return core.search_unity(prob, int(os.environ.get("FF_JOINT_BEAM", "512")), 0, cfg.search_alpha, cfg.seed)
        if algo == "mcmc":
            return core.search_mcmc(prob, dp_choice, budget or cfg.mcmc_iterations, cfg.search_alpha, cfg.seed)
        return core.search_unity(prob, 4096, budget if budget is not None else 300, cfg.search_alpha, cfg.seed)

    mem_report = None
    if cfg.perform_memory_search:
        res, mem_report = memory_search(prob, run_search)
    else:
        res = run_search()
    choice = list(res.choice)
    split_report = []
    if algo != "mcmc" and n > 1 and not quick and os.environ.get("FF_NONSEQ_SPLIT", "1") != "0":
        # resource-split refinement: parallel branches re-searched on disjoint device groups
        sr = core.search_split(prob, choice, 4096)
        for si in sr.splits:
            split_report.append({"fork": model.layers[si.start].name, "join": model.layers[si.end].name,
                                 "branches": si.components, "groups": si.groups,
                                 "whole_ms": round(si.whole_ms, 4), "split_ms": round(si.split_ms, 4),
                                 "sim_before_ms": round(si.sim_before_ms, 4), "sim_after_ms": round(si.sim_after_ms, 4),
                                 "accepted": bool(si.accepted)})
        if sr.cost_ms < res.cost_ms:
            choice = list(sr.choice)
            res = SimpleNamespace(choice=choice, cost_ms=sr.cost_ms, dp_cost_ms=res.dp_cost_ms, states=res.states,
                                  iterations=res.iterations)
    if res.cost_ms > dp_sim:  # never pick something the simulator thinks is worse than DP
        choice = dp_choice
    strat = {L.name: cands[i][choice[i]] for i, L in enumerate(model.layers)}
    report = {"algo": algo, "devices": n, "predicted_ms": round(min(res.cost_ms, dp_sim), 4),
              "predicted_dp_ms": round(dp_sim, 4), "predicted_speedup_vs_dp": round(dp_sim / max(min(res.cost_ms, dp_sim), 1e-9), 4),
              "dp_objective_ms": round(res.dp_cost_ms, 4), "states": int(res.states),
              "mcmc_iterations": int(res.iterations), "build_s": round(t_build, 3),
              "search_s": round(time.perf_counter() - t0 - t_build, 3), "measured_costs": bool(do_measure),
              "candidates": sum(len(c) for c in cands)}
    if mem_report is not None:
        report["memory_search"] = mem_report
    if split_report:
        report["nonsequence_splits"] = split_report
    return strat, report


def _set_lambda(prob, base, lam):
    """cost'(candidate) = fwd_ms + lam * GiB the candidate keeps on each of its devices."""
    nodes = prob.nodes
    for node, bs in zip(nodes, base):
        cc = node.cands
        for oc, (f, m) in zip(cc, bs):
            oc.fwd_ms = f + lam * m / float(1 << 30)
        node.cands = cc
    prob.nodes = nodes


def memory_search(prob, run_search, max_iters: int = 10):
    """Memory-aware search (reference src/runtime/memory_optimization.cc + graph.cc's
    lambda loop): minimise run time + lambda * per-device memory, with lambda (ms per GiB) raised
    by doubling and then bisected until the simulated peak per-device memory fits the machine's
    capacity (-ll:fsize MiB, or mem_capacity of --machine-model-file; 288 GB HBM3E by default).
    The smallest fitting lambda wins: the fastest strategy that fits. The search's own costs
    are restored before the final simulation, so reported times are real run-time predictions."""
    core = _core()
    cap = prob.machine.mem_capacity
    base = [[(oc.fwd_ms, oc.mem_bytes) for oc in node.cands] for node in prob.nodes]

    def attempt(lam):
        _set_lambda(prob, base, lam)
        r = run_search()
        _set_lambda(prob, base, 0.0)
        sim = core.simulate(prob, list(r.choice))
        return r, sim

    res, sim = attempt(0.0)
    tried = [(0.0, sim.max_mem)]
    best = (res, sim, 0.0) if sim.max_mem <= cap else None
    if best is None:
        lo, hi = 0.0, 1.0
        while len(tried) < max_iters:
            r, s = attempt(hi)
            tried.append((hi, s.max_mem))
            if s.max_mem <= cap:
                best = (r, s, hi)
                break
            lo, hi = hi, hi * 8
        while best is not None and len(tried) < max_iters and hi - lo > 1e-3 * hi:
            mid = 0.5 * (lo + hi)
            r, s = attempt(mid)
            tried.append((mid, s.max_mem))
            if s.max_mem <= cap:
                best, hi = (r, s, mid), mid
            else:
                lo = mid
    if best is None:  # nothing fits: keep the least-memory strategy found
        res, sim = attempt(tried[-1][0])
        best = (res, sim, tried[-1][0])
    r, sim, lam = best
    # the real (lambda-free) simulated time of the chosen strategy
    res = SimpleNamespace(choice=list(r.choice), cost_ms=sim.makespan_ms, dp_cost_ms=r.dp_cost_ms, states=r.states,
                          iterations=r.iterations)
    return res, {"lambda_ms_per_gib": lam, "capacity_gib": round(cap / (1 << 30), 3),
                 "max_mem_gib": round(sim.max_mem / (1 << 30), 4), "fits": bool(sim.max_mem <= cap),
                 "iterations": len(tried), "tried": [(round(a, 4), round(b / (1 << 30), 4)) for a, b in tried]}
