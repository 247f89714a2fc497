"""Memory-aware search (reference src/runtime/memory_optimization.cc and the lambda loop of
graph.cc): minimise time + lambda * per-device memory, raising lambda until the strategy fits."""
import pytest

from flexflow_amd.core import ActiMode, DataType, FFConfig, FFModel
from flexflow_amd.pcg import unity

_core = pytest.importorskip("flexflow_amd._core")


def _model(flags=(), b=4096, h=2048):
    cfg = FFConfig(["--search-num-workers", "4"] + list(flags))
    cfg.batch_size = b
    ff = FFModel(cfg)
    x = ff.create_tensor([b, 1024], DataType.DT_FLOAT)
    t = ff.dense(x, h, ActiMode.AC_MODE_RELU)
    t = ff.dense(t, h, ActiMode.AC_MODE_RELU)
    ff.softmax(ff.dense(t, 16))
    return ff


def _search(prob):
    return lambda: _core.search_unity(prob, 4096, 100, 1.2, 1)


def test_lambda_search_trades_time_for_memory():
    prob, _ = unity.build_problem(_model(), 4, False)
    free = _search(prob)()
    free_sim = _core.simulate(prob, list(free.choice))
    # the least-memory strategy the search can reach (a very large lambda)
    base = [[(oc.fwd_ms, oc.mem_bytes) for oc in node.cands] for node in prob.nodes]
    unity._set_lambda(prob, base, 1e9)
    frugal = _search(prob)()
    unity._set_lambda(prob, base, 0.0)
    frugal_sim = _core.simulate(prob, list(frugal.choice))
    assert frugal_sim.max_mem <= free_sim.max_mem

    # generous capacity: lambda stays 0 and the unconstrained optimum is kept
    res, rep = unity.memory_search(prob, _search(prob))
    assert rep["fits"] and rep["lambda_ms_per_gib"] == 0.0
    assert res.cost_ms == pytest.approx(free_sim.makespan_ms)

    assert frugal_sim.max_mem < 0.9 * free_sim.max_mem  # this model trades time for memory
    if True:
        # capacity between the two peaks: a fitting strategy, never faster than the unconstrained one
        # (the native search's OOM penalty may already get there at lambda = 0)
        prob.machine.mem_capacity = 0.5 * (frugal_sim.max_mem + free_sim.max_mem)
        prob2, _ = unity.build_problem(_model(), 4, False)
        prob2.machine.mem_capacity = prob.machine.mem_capacity
        res, rep = unity.memory_search(prob2, _search(prob2))
        assert rep["fits"]
        assert rep["max_mem_gib"] * (1 << 30) <= prob2.machine.mem_capacity
        assert res.cost_ms >= free_sim.makespan_ms - 1e-6

    # impossible capacity: reported as not fitting, least-memory strategy kept
    prob3, _ = unity.build_problem(_model(), 4, False)
    prob3.machine.mem_capacity = 1.0
    res, rep = unity.memory_search(prob3, _search(prob3))
    assert not rep["fits"]


def test_memory_search_flag_reports():
    ff = _model(["--memory-search", "-ll:fsize", "100000"])
    strat, rep = unity.search(ff, "unity")
    assert rep["memory_search"]["fits"]
    assert rep["memory_search"]["capacity_gib"] == pytest.approx(100000 / 1024, rel=1e-3)
    assert set(strat) == {L.name for L in ff.layers}
