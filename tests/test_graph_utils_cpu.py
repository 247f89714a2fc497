"""Native graph / machine-view utilities (csrc/core/graph_utils.h) — the cases of the reference's
gtest unit tests (tests/unit/test_dominators.cc, test_machine_view.cc, test_disjoint_set.cc,
test_random_utils.cc) re-expressed against flexflow_amd._core. Node ids are dense ints here, so the
reference's 1-based example graphs are shifted down by one."""
import random

import pytest

_core = pytest.importorskip("flexflow_amd._core")


def _g(n, edges, base=0):
    return _core.Digraph(n, [(a - base, b - base) for a, b in edges])


DOM_EDGES = [(1, 2), (1, 7), (2, 3), (2, 4), (3, 6), (4, 5), (4, 6), (5, 6), (6, 8), (7, 8), (8, 9), (8, 10),
             (9, 11), (10, 11)]


def _shift(d):
    return {k - 1: sorted(x - 1 for x in v) for k, v in d.items()}


def test_pred_succ():
    g = _g(5, [(0, 2), (1, 2), (2, 3), (2, 4)])
    assert [g.predecessors(v) for v in range(5)] == [[], [], [0, 1], [2], [2]]
    assert [g.successors(v) for v in range(5)] == [[2], [2], [3, 4], [], []]


def test_topo_sort():
    g = _g(4, [(3, 1), (3, 0), (1, 0), (0, 2)])
    assert g.topo_order() == [3, 1, 0, 2]


def test_dominators():
    g = _g(11, DOM_EDGES, base=1)
    want = _shift({1: {1}, 2: {1, 2}, 3: {1, 2, 3}, 4: {1, 2, 4}, 5: {1, 2, 4, 5}, 6: {1, 2, 6}, 7: {1, 7},
                   8: {1, 8}, 9: {1, 8, 9}, 10: {1, 8, 10}, 11: {1, 8, 11}})
    assert {v: d for v, d in enumerate(g.dominators())} == want


def test_post_dominators():
    g = _g(11, DOM_EDGES, base=1)
    want = _shift({1: {1, 8, 11}, 2: {2, 6, 8, 11}, 3: {3, 6, 8, 11}, 4: {4, 6, 8, 11}, 5: {5, 6, 8, 11},
                   6: {6, 8, 11}, 7: {7, 8, 11}, 8: {8, 11}, 9: {9, 11}, 10: {10, 11}, 11: {11}})
    assert {v: d for v, d in enumerate(g.post_dominators())} == want


def test_imm_dominators():
    g = _g(11, DOM_EDGES, base=1)
    want = {1: 1, 2: 1, 3: 2, 4: 2, 5: 4, 6: 2, 7: 1, 8: 1, 9: 8, 10: 8, 11: 8}
    assert g.imm_dominators() == [want[v + 1] - 1 for v in range(11)]
    want_post = {1: 8, 2: 6, 3: 6, 4: 6, 5: 6, 6: 8, 7: 8, 8: 11, 9: 11, 10: 11, 11: 11}
    assert g.imm_post_dominators() == [want_post[v + 1] - 1 for v in range(11)]


def test_imm_post_dominators_multisource():
    g = _g(5, [(1, 3), (2, 3), (3, 4), (3, 5)], base=1)
    assert g.imm_post_dominators() == [2, 2, 2, 3, 4]  # 1->3, 2->3, 3->3, 4->4, 5->5 (1-based)


def test_bottlenecks_are_sequence_split_points():
    g = _g(11, DOM_EDGES, base=1)
    assert g.bottlenecks() == [0, 7, 10]  # nodes 1, 8, 11
    # two sources joining at a node: that node (and everything after on a chain) splits
    h = _g(5, [(1, 3), (2, 3), (3, 4), (4, 5)], base=1)
    assert h.bottlenecks() == [2, 3, 4]


@pytest.mark.parametrize("edges,want", [
    ([(1, 2), (2, 3), (1, 3)], [(1, 2), (2, 3)]),
    ([(1, 4), (1, 5), (2, 3), (2, 4), (2, 6), (3, 4), (4, 5), (4, 6), (5, 6)], [(1, 4), (2, 3), (3, 4), (4, 5), (5, 6)]),
])
def test_transitive_reduction(edges, want):
    n = max(max(e) for e in edges)
    r = _g(n, edges, base=1).transitive_reduction()
    assert sorted(r.edges()) == sorted((a - 1, b - 1) for a, b in want)


def test_roots_leaves_descendants_components():
    g = _g(6, [(1, 3), (2, 3), (3, 4), (3, 5), (3, 6)], base=1)
    assert g.roots() == [0, 1] and g.leaves() == [3, 4, 5]
    d = _g(6, [(1, 2), (2, 3), (2, 4), (3, 5), (4, 5)], base=1)
    assert d.descendants(1) == [1, 2, 3, 4]
    assert d.descendants(1, True) == [0, 1, 2, 3, 4]
    w = _g(6, [(1, 3), (2, 3), (4, 5)], base=1)
    comps = sorted(sorted(c) for c in w.weakly_connected_components())
    assert comps == [[0, 1, 2], [3, 4], [5]]


def test_cycle_detected():
    g = _g(3, [(0, 1), (1, 2), (2, 0)])
    with pytest.raises(RuntimeError):
        g.topo_order()


def test_disjoint_set():
    ds = _core.DisjointSet(6)
    assert ds.unite(0, 1) and ds.unite(2, 3) and not ds.unite(1, 0)
    ds.unite(1, 3)
    assert ds.same(0, 2) and not ds.same(0, 4)
    assert ds.find(3) == ds.find(0)


def test_select_random_distribution():
    w = [1.0, 0.0, 3.0]
    rng = random.Random(0)
    counts = [0, 0, 0]
    for _ in range(4000):
        counts[_core.select_random(w, rng.random())] += 1
    assert counts[1] == 0
    assert 0.2 < counts[0] / 4000 < 0.3
    with pytest.raises(ValueError):
        _core.select_random([0.0], 0.5)


def test_machine_view_device_ids():
    mv = _core.MachineView(2, [2], [1])  # reference test_machine_view.cc
    assert mv.device_id([0]) == 2 and mv.device_id([1]) == 3
    mv2 = _core.MachineView(1, [2, 3], [8, 1])  # 2 nodes x 3 GPUs starting at GPU 1
    assert mv2.device_ids() == [1, 2, 3, 9, 10, 11] and mv2.num_parts() == 6
    assert mv2 == _core.MachineView(1, [2, 3], [8, 1]) and mv2.hash() != mv.hash()


def test_machine_resource_views():
    r = _core.MachineResource(num_nodes=1, gpus_per_node=8)
    views = r.enumerate_views()
    sets = {tuple(v.device_ids()) for v in views}
    # every aligned contiguous block i | 8
    for p in (1, 2, 4, 8):
        for st in range(0, 8, p):
            assert tuple(range(st, st + p)) in sets
    assert all(r.is_valid_machine_view(v) for v in views)
    assert not r.is_valid_machine_view(_core.MachineView(6, [4], [1]))
    r2 = _core.MachineResource(num_nodes=2, gpus_per_node=8)
    sets2 = {tuple(v.device_ids()) for v in r2.enumerate_views()}
    assert tuple(range(16)) in sets2          # both nodes
    assert (3, 11) in sets2                   # one GPU per node (strided view)
    half = _core.MachineResource(num_nodes=1, gpus_per_node=8, available_gpus_per_node=4, start_gpu_id=4)
    assert all(min(v.device_ids()) >= 4 for v in half.enumerate_views())
