"""Search-space coverage: candidate quotas per part count and the non-sequence (resource-split)
refinement of the native search (reference SearchHelper::execute_nonsequence_split,
src/runtime/graph.cc:188-330)."""
import pytest

from flexflow_amd.core import FFConfig, FFModel
from flexflow_amd.pcg.strategy import enumerate_configs

core = pytest.importorskip("flexflow_amd._core")


def _layout(devs, shape=(8,)):
    lo = core.Layout()
    lo.shape = list(shape)
    lo.degrees = [1] * len(shape)
    lo.replicas = len(devs)
    lo.devices = list(devs)
    lo.partial = False
    lo.halo = []
    return lo


def _node(name, inputs, views, ms=1.0):
    n = core.Node()
    n.name = name
    n.op_type = "OP_LINEAR"
    n.inputs = inputs
    n.input_needs_grad = [False] * len(inputs)
    n.elem_bytes = 2
    n.backward = False
    cc = []
    for devs in views:
        c = core.OpCandidate()
        c.degrees = [1]
        c.devices = list(devs)
        c.fwd_ms, c.bwd_ms = ms, 0.0
        c.mem_bytes = 0.0
        c.in_layouts = [_layout(devs) for _ in inputs]
        c.out_layouts = [_layout(devs)]
        c.w_layouts = []
        cc.append(c)
    n.cands = cc
    return n


def _branchy_problem():
    """fork -> {a1 -> a2, b1 -> b2} -> join; every op takes 1 ms wherever it runs (latency-bound),
    so the two branches on disjoint halves of the machine run concurrently: 4 -> 2 ms."""
    full, lo, hi = tuple(range(8)), (0, 1, 2, 3), (4, 5, 6, 7)
    views = [full, lo, hi]
    nodes = [_node("fork", [], [full]),
             _node("a1", [(0, 0)], views), _node("b1", [(0, 0)], views),
             _node("a2", [(1, 0)], views), _node("b2", [(2, 0)], views),
             _node("join", [(3, 0), (4, 0)], [full])]
    p = core.Problem()
    p.machine = core.MachineModel()
    p.nodes = nodes
    return p


def test_sequence_bottlenecks():
    p = _branchy_problem()
    assert list(core.sequence_bottlenecks(p)) == [5]


def test_nonsequence_split_puts_branches_on_disjoint_devices():
    p = _branchy_problem()
    base = [0] * 6  # everything on all 8 devices
    before = core.simulate(p, base).makespan_ms
    r = core.search_split(p, base, 4096)
    after = core.simulate(p, list(r.choice)).makespan_ms
    assert len(r.splits) == 1 and r.splits[0].accepted and r.splits[0].groups == 2
    assert after < before - 1.5
    devs = [set(p.nodes[i].cands[r.choice[i]].devices) for i in (1, 3)], \
           [set(p.nodes[i].cands[r.choice[i]].devices) for i in (2, 4)]
    a = set.union(*devs[0])
    b = set.union(*devs[1])
    assert not (a & b)  # the two branches never share a device


def test_split_never_makes_the_simulation_worse():
    p = _branchy_problem()
    # make subset placements slow: the refinement must keep the whole-machine plan
    for n in p.nodes[1:5]:
        cc = n.cands
        for c in cc[1:]:
            c.fwd_ms = 10.0
        n.cands = cc
    base = [0] * 6
    r = core.search_split(p, base, 4096)
    assert list(r.choice) == base and not r.splits[0].accepted


def test_candidate_quota_keeps_small_placements():
    cfg = FFConfig([])
    cfg.batch_size = 64
    ff = FFModel(cfg)
    x = ff.create_tensor([64, 1024])
    ff.dense(x, 4096)
    lin = ff.layers[-1]
    cands = enumerate_configs(lin, 8, ("sample", "parameter"), max_configs=32)
    parts = {c.num_parts for c in cands}
    assert {1, 2, 4, 8} <= parts and len(cands) <= 32
    # both halves of the machine appear among the 4-device views
    starts = {c.devices[0] for c in cands if c.num_parts == 4}
    assert {0, 4} <= starts


def test_native_cost_model_classifies_all_to_all():
    def lay(degs, devs):
        lo = core.Layout()
        lo.shape = [64, 1024]
        lo.degrees = list(degs)
        lo.replicas = 1
        lo.devices = list(devs)
        lo.partial = False
        lo.halo = []
        return lo
    mm = core.MachineModel()
    x = core.transfer_cost(lay([8, 1], range(8)), lay([1, 8], [3, 1, 0, 2, 7, 5, 6, 4]), False, 2, mm)
    assert x.kind == core.XferKind.ALL_TO_ALL and x.ms > 0
    g = core.transfer_cost(lay([8, 1], range(8)), lay([1, 4], range(4)), False, 2, mm)
    assert g.kind == core.XferKind.GENERIC
