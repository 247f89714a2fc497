"""The reference's protobuf strategy files (examples/cpp/DLRM/strategies/*.pb, read as data) imported
with --import-strategy: per-table embedding placement + data-parallel MLPs (reference DLRM strategy
generator examples/cpp/DLRM/strategies/dlrm_strategy.py)."""
import os

import pytest

from flexflow_amd.core import FFConfig, FFModel
from flexflow_amd.models.recsys import DLRMConfig, build_dlrm
from flexflow_amd.pcg.search import choose_strategy
from flexflow_amd.pcg.strategy import load_strategy_pb
from flexflow_amd.type import OperatorType

PB = "/root/reference/examples/cpp/DLRM/strategies/dlrm_strategy_8embs_8gpus.pb"
pytestmark = pytest.mark.skipif(not os.path.exists(PB), reason="reference strategy files not mounted")


def test_dlrm_pb_strategy_places_tables_and_keeps_mlp_data_parallel():
    cfg = FFConfig(["--search-num-workers", "8", "--import-strategy", PB])
    cfg.batch_size = 64
    ff = FFModel(cfg)
    build_dlrm(ff, 64, DLRMConfig(embedding_size=[1000] * 8))
    strat, rep = choose_strategy(ff)
    assert rep["algo"] == "import"
    embs = [L for L in ff.layers if L.op_type == OperatorType.OP_EMBEDDING]
    assert len(embs) == 8
    for k, L in enumerate(embs):  # "embedding<k>": whole table on GPU k % 8
        c = strat[L.name]
        assert c.num_parts == 1 and c.devices == (k % 8,), (L.name, c)
    for L in ff.layers:
        if L.op_type in (OperatorType.OP_LINEAR, OperatorType.OP_CONCAT):  # "linear" / "concat": 8-way DP
            c = strat[L.name]
            assert c.degrees[0] == 8 and c.devices == tuple(range(8)), (L.name, c)


def test_pb_entries_that_do_not_fit_fall_back():
    # 16-table strategy on a 4-table model planning for 8 devices: only the first 4 names match
    cfg = FFConfig(["--search-num-workers", "8"])
    cfg.batch_size = 64
    ff = FFModel(cfg)
    build_dlrm(ff, 64, DLRMConfig(embedding_size=[1000] * 4))
    pb16 = PB.replace("8embs_8gpus", "16embs_8gpus")
    table = load_strategy_pb(pb16, ff.layers, 8)
    embs = [L.name for L in ff.layers if L.op_type == OperatorType.OP_EMBEDDING]
    assert all(e in table for e in embs)
