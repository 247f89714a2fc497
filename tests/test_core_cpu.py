"""Native core (flexflow_amd._core, csrc/core): data-loader ring, transfer classification parity with
the Python runtime, simulator, DP / MCMC / Unity search, substitution rule loading and matching
(reference test strategy: the C++ unit tests of the PCG/search utilities)."""
import itertools
import json
import os

import numpy as np
import pytest

from flexflow_amd import _core
from flexflow_amd.parallel.comm import Transfer
from flexflow_amd.parallel.layout import Layout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_batch_ring_order_and_wrap():
    data = np.arange(10 * 3, dtype=np.float32).reshape(10, 3)
    bufs = [np.empty((4, 3), np.float32) for _ in range(3)]
    ring = _core.BatchRing(data, 4, bufs)
    assert ring.depth() == 3
    got = []
    for _ in range(2):
        s = ring.next()
        got.append(bufs[s].copy())
        ring.release(s)
    np.testing.assert_array_equal(got[0], data[0:4])
    np.testing.assert_array_equal(got[1], data[4:8])
    ring.reset(0)
    s = ring.next()
    np.testing.assert_array_equal(bufs[s], data[0:4])
    ring.release(s)
    with pytest.raises(RuntimeError):
        _core.BatchRing(data, 4, [np.empty((2, 3), np.float32)])  # slot too small


def _core_layout(l: Layout):
    c = _core.Layout()
    c.shape, c.degrees, c.replicas, c.devices, c.partial = list(l.shape), list(l.degrees), l.replicas, \
        list(l.devices), l.partial
    c.halo = list(l.halo) if l.halo else []
    return c


KIND = {"identity": "IDENTITY", "local_slice": "LOCAL_SLICE", "all_reduce": "ALL_REDUCE",
        "reduce_scatter": "REDUCE_SCATTER", "all_gather": "ALL_GATHER", "all_to_all": "ALL_TO_ALL",
        "generic": "GENERIC"}


@pytest.mark.parametrize("src_deg,dst_deg,rep_s,rep_d,partial", [
    ((1, 1), (1, 1), 4, 4, False),     # replicated -> replicated: identity
    ((1, 1), (4, 1), 4, 1, False),     # replicated -> sharded: local slice
    ((4, 1), (1, 1), 1, 4, False),     # sharded -> replicated: all-gather
    ((1, 1), (1, 1), 4, 4, True),      # partial sums -> replicated: all-reduce
    ((1, 1), (4, 1), 4, 1, True),      # partial sums -> sharded: reduce-scatter
    ((4, 1), (1, 4), 1, 1, False),     # row -> column sharding on the same ranks: all-to-all
])
def test_transfer_classification_matches_runtime(src_deg, dst_deg, rep_s, rep_d, partial):
    shape = (16, 8)
    src = Layout(shape, src_deg, rep_s, tuple(range(4)), partial=partial)
    dst = Layout(shape, dst_deg, rep_d, tuple(range(4)))
    py = Transfer(src, dst, partial, 0).kind
    mm = _core.MachineModel()
    mm.gpus_per_node = 4
    c = _core.transfer_cost(_core_layout(src), _core_layout(dst), partial, 2, mm)
    assert c.kind.name == KIND[py], (py, c.kind)
    assert (c.ms < 1e-3) == (py in ("identity", "local_slice"))  # local copies cost only HBM time


def _chain_problem(n_ops=6, devices=4):
    """A chain of ops with two candidates each: data parallel (cheap compute, weight sync) and
    replicated-compute (no sync, 4x compute)."""
    p = _core.Problem()
    mm = _core.MachineModel()
    mm.gpus_per_node = devices
    p.machine = mm
    nodes = []
    for i in range(n_ops):
        n = _core.Node()
        n.name, n.op_type = f"op{i}", "OP_LINEAR"
        n.inputs = [(i - 1, 0)] if i else []
        n.input_needs_grad = [True] if i else []
        n.elem_bytes = 2
        n.backward = True
        cands = []
        for deg, ms in (((devices, 1), 1.0), ((1, 1), 4.0)):
            c = _core.OpCandidate()
            c.degrees = list(deg)
            c.devices = list(range(devices))
            c.fwd_ms, c.bwd_ms = ms, 2 * ms
            c.mem_bytes = 1 << 20
            lay = Layout((64, 64), deg, devices // deg[0], tuple(range(devices)))
            c.in_layouts = [_core_layout(lay)] if i else []
            c.out_layouts = [_core_layout(lay)]
            w = Layout((64, 64), (1, 1), devices, tuple(range(devices)))
            c.w_layouts = [_core_layout(w)]
            cands.append(c)
        n.cands = cands
        nodes.append(n)
    p.nodes = nodes
    return p


def test_simulator_and_searches_agree_on_chain():
    p = _chain_problem()
    n = len(p.nodes)
    dp = [0] * n
    rep = [1] * n
    sim_dp, sim_rep = _core.simulate(p, dp), _core.simulate(p, rep)
    assert sim_dp.makespan_ms < sim_rep.makespan_ms
    assert sim_dp.compute_ms > 0 and sim_dp.max_mem > 0
    # exhaustive optimum of the additive objective equals the DP search
    best = min(_core.simulate(p, list(c)).makespan_ms for c in itertools.product((0, 1), repeat=n))
    r = _core.search_dp(p, 4096)
    assert abs(_core.simulate(p, list(r.choice)).makespan_ms - best) < 1e-6 + 0.05 * best
    u = _core.search_unity(p, 4096, 200, 0.05, 1)
    m = _core.search_mcmc(p, rep, 500, 0.05, 1)
    assert u.cost_ms <= sim_rep.makespan_ms + 1e-9
    assert m.cost_ms <= sim_rep.makespan_ms + 1e-9
    assert len(u.choice) == n and u.states > 0


def test_rules_load_and_match():
    rules = _core.load_rules(os.path.join(ROOT, "substitutions", "flexflow_amd_rules.json"))
    names = {r.name for r in rules}
    assert "fuse_add_layernorm" in names and "fuse_linear_relu" in names
    r = next(r for r in rules if r.name == "fuse_linear_relu")
    g = []
    for typ, ins in (("OP_INPUT", []), ("OP_LINEAR", [(0, 0), (-1000001, 0), (-1000002, 0)]),
                     ("OP_RELU", [(1, 0)]), ("OP_SOFTMAX", [(2, 0)])):
        n = _core.GNode()
        n.type, n.inputs, n.num_outputs = typ, ins, 1
        n.params = {"PM_ACTI": 0} if typ == "OP_LINEAR" else {}
        g.append(n)
    ms = _core.match_rule(r, g, 8)
    assert len(ms) == 1 and sorted(ms[0].op_nodes) == [1, 2]
    g[1].params = {"PM_ACTI": 2}  # already fused -> no match
    assert len(_core.match_rule(r, g, 8)) == 0


def test_reference_rule_file_loads():
    """The reference's TASO-derived rule collection parses (JSON read with the safe json module)."""
    path = "/root/reference/substitutions/graph_subst_3_v2.json"
    if not os.path.exists(path):
        pytest.skip("reference rules not present")
    rules = _core.load_rules(path)
    assert len(rules) > 100
    with open(path) as f:
        assert len(json.load(f)["rule"]) == len(rules)


def test_reference_op_layer_classes():
    """get_layer_by_id returns the reference's per-op classes (flexflow_cffi.py Linear, Exp, ...)."""
    from flexflow_amd import core
    ff = core.FFModel(core.FFConfig([]))
    x = ff.create_tensor([4, 8], core.DataType.DT_FLOAT)
    t = ff.exp(ff.dense(x, 4))
    ff.add_layer(core.OpType.EXP if hasattr(core, "OpType") else None, "my_exp")
    l0, l1 = ff.get_layer_by_id(0), ff.get_layer_by_id(1)
    assert isinstance(l0, core.Linear) and isinstance(l0, core.Layer)
    assert isinstance(l1, core.Exp) and l1.name == "my_exp"
    assert l0.get_weight_tensor() is not None and t is l1.get_output_tensor()


def test_config_flag_values():
    """Our own flags raise on a malformed value; a foreign `-p no:plugin` (pytest) or a flag whose
    value is the next flag is ignored with a warning and the next flag is still parsed."""
    import pytest
    from flexflow_amd.config import FFConfig
    with pytest.raises(ValueError):
        FFConfig(["-b", "32x"])
    with pytest.raises(ValueError):
        FFConfig(["--lr", "1e-3,"])
    with pytest.warns(UserWarning):
        c = FFConfig(["-p", "no:cacheprovider", "-b", "48"])
    assert c.batch_size == 48
    with pytest.warns(UserWarning):
        c = FFConfig(["--lr", "--zero", "-b", "16"])
    assert c.batch_size == 16 and c.zero_optimizer


def test_op_forward_init_and_dataloader_helpers():
    """reference Op.forward / Op.init, SingleDataLoader.init_from_ptr / init_from_tensor and
    RegionNdarray (flexflow_cffi.py)."""
    import numpy as np
    from flexflow_amd.core import (DataType, FFConfig, FFModel, LossType, RegionNdarray, SGDOptimizer,
                                   SingleDataLoader)
    cfg = FFConfig(["--device", "cpu"])
    cfg.batch_size = 4
    ff = FFModel(cfg)
    x = ff.create_tensor([4, 8], DataType.DT_FLOAT)
    y = ff.dense(x, 3)
    ff.optimizer = SGDOptimizer(ff, 0.1)
    ff.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE)
    dense = ff.get_layer_by_id(0) if ff.get_layer_by_id(0).weights else ff.layers[-1]
    xv = np.arange(32, dtype=np.float32).reshape(4, 8) / 32
    x.set_tensor(ff, xv)
    dense._add_to_model(ff)
    dense.forward(ff)
    w = np.asarray(dense.get_parameter_by_id(0).get_weights(ff))
    b = np.asarray(dense.get_parameter_by_id(1).get_weights(ff))
    np.testing.assert_allclose(np.asarray(y.get_tensor(ff)), xv @ w.T + b, rtol=1e-5, atol=1e-6)
    dense.get_parameter_by_id(0).set_weights(ff, np.zeros_like(w))
    dense.init(ff)  # back to the deterministic initial values
    np.testing.assert_allclose(np.asarray(dense.get_parameter_by_id(0).get_weights(ff)), w)
    buf = np.arange(40, dtype=np.float32).reshape(5, 8)
    view = np.asarray(RegionNdarray(buf.shape, DataType.DT_FLOAT, buf.ctypes.data, buf.strides, True))
    np.testing.assert_array_equal(view, buf)
    dl = SingleDataLoader.__new__(SingleDataLoader)
    dl.init_from_ptr(ff, x, view, 5, DataType.DT_FLOAT)
    assert dl.num_samples == 5
