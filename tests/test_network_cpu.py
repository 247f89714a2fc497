"""Topology-aware network model (machine_model_version 1; reference src/runtime/network.cc:
NetworkedMachineModel, fat-tree / big-switch generators, shortest-path routing)."""
import json

import pytest

from flexflow_amd.core import ActiMode, DataType, FFConfig, FFModel

_core = pytest.importorskip("flexflow_amd._core")


def test_single_node_xgmi_uses_every_link():
    t = _core.make_mi355x_cluster(1, 8, 64.0, 50.0)
    assert t.num_links == 28 and t.hops(0, 5) == 1
    # an 8-rank all-reduce over r-1 rotated rings drives all 7 links of every GPU
    assert t.ring_busbw(list(range(8))) == pytest.approx(7 * 64.0, rel=1e-6)
    assert t.ring_busbw([0, 1]) == pytest.approx(64.0, rel=1e-6)
    # 1 GB all-gather over 4 ranks: each link carries (r-1) steps x (B/r)/(r-1)
    assert t.allgather_ms([0, 1, 2, 3], 1e9) == pytest.approx(3 * (1e9 / 4 / 3) / 64e6, rel=1e-6)


@pytest.mark.parametrize("kind,hops", [("big_switch", 2), ("fat_tree", 4)])
def test_multi_node_routes_and_nic_bottleneck(kind, hops):
    t = _core.make_mi355x_cluster(2, 8, 64.0, 50.0, kind)
    assert t.hops(0, 7) == 1 and t.hops(0, 8) == hops
    assert t.path_gbps(0, 8) == pytest.approx(50.0)
    intra = t.ring_busbw(list(range(8)))
    inter = t.ring_busbw(list(range(16)))
    assert inter < intra / 3  # the NIC uplinks, not xGMI, bound a 2-node ring
    # 8 concurrent node0 -> node1 transfers: one per NIC, no contention in a non-blocking fabric
    x = [(i, 8 + i, 1e9) for i in range(8)]
    assert t.transfers_ms(x) == pytest.approx(1e9 / 50e6, rel=1e-6)
    # all eight from ONE GPU share its NIC
    y = [(0, 8 + i, 1e9) for i in range(8)]
    assert t.transfers_ms(y) == pytest.approx(8 * 1e9 / 50e6, rel=1e-6)


def test_oversubscribed_fat_tree_is_slower():
    full = _core.make_mi355x_cluster(2, 8, 64.0, 50.0, "fat_tree", 1.0)
    over = _core.make_mi355x_cluster(2, 8, 64.0, 50.0, "fat_tree", 4.0)
    r = list(range(16))
    assert over.allreduce_ms(r, 1e9) > 2 * full.allreduce_ms(r, 1e9)


def test_custom_links_and_search_with_topology(tmp_path):
    # a 4-GPU ring (0-1-2-3-0) instead of all-to-all: 0 -> 2 takes two hops
    mf = tmp_path / "mm.json"
    mf.write_text(json.dumps({"links": [[0, 1, 64], [1, 2, 64], [2, 3, 64], [3, 0, 64]]}))
    cfg = FFConfig(["--search-num-workers", "4", "--machine-model-file", str(mf), "--machine-model-version", "1"])
    cfg.batch_size = 64
    ff = FFModel(cfg)
    x = ff.create_tensor([64, 512], DataType.DT_FLOAT)
    ff.softmax(ff.dense(ff.dense(x, 1024, ActiMode.AC_MODE_RELU), 16))
    from flexflow_amd.pcg import unity
    mm = unity.machine_model(cfg)
    assert mm.has_topology and mm.p2p_gbps(0, 2) == pytest.approx(64.0)
    ring4 = mm.ring_busbw([0, 1, 2, 3])
    mm2 = unity.machine_model(FFConfig(["--search-num-workers", "4"]))
    assert not mm2.has_topology and ring4 < mm2.ring_busbw([0, 1, 2, 3])  # fewer links than all-to-all
    strat, rep = unity.search(ff, "unity")
    assert rep["predicted_ms"] > 0 and set(strat) == {L.name for L in ff.layers}
