"""Convolution implementation pick policy (kernels._conv_pick, CPU): the per-site timing keeps the
fastest of our implicit GEMM / the pointwise plain GEMM, and MIOpen only when it beats that by
_CONV_LIB_MARGIN; the 1 x 1 GEMM candidate's eligibility; when the forward packs the dgrad operand."""
import torch

from flexflow_amd import kernels as K


def _pick(monkeypatch, times, key):
    monkeypatch.setattr(K, "_TUNE", True)
    monkeypatch.setattr(K, "_CONV_IMPL", "")
    monkeypatch.setattr(K, "_TUNE_CACHE", "")
    monkeypatch.setattr(K, "_conv_tuned", {})
    monkeypatch.setattr(K, "TUNE_LOG", [])
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setattr(K, "_time_all", lambda cands, rounds=2: {k: times[k] for k in cands})
    cands = {k: (lambda: None) for k in times}
    return K._conv_pick("bwd", key, cands)


def test_lib_needs_margin(monkeypatch):
    m = K._CONV_LIB_MARGIN
    assert 0.0 < m < 1.0
    assert _pick(monkeypatch, {"ours": 1.0, "lib": 1.0 - m / 2}, ("a",)) == "ours"
    assert _pick(monkeypatch, {"ours": 1.0, "lib": 1.0 - 2 * m}, ("b",)) == "lib"


def test_gemm_candidate_competes(monkeypatch):
    assert _pick(monkeypatch, {"ours": 1.0, "lib": 0.95, "gemm": 0.9}, ("c",)) == "gemm"
    # the margin is taken against the best of our two candidates
    m = K._CONV_LIB_MARGIN
    assert _pick(monkeypatch, {"ours": 1.0, "lib": 0.9 * (1 - m) + 0.01, "gemm": 0.9}, ("d",)) == "gemm"
    assert _pick(monkeypatch, {"ours": 1.0, "lib": 0.9 * (1 - m) - 0.01, "gemm": 0.9}, ("e",)) == "lib"
    assert _pick(monkeypatch, {"ours": 0.8, "lib": 0.8 * (1 - m) + 0.01, "gemm": 0.9}, ("f",)) == "ours"


def test_pointwise_gemm_eligibility():
    x = torch.randn(2, 16, 5, 5).contiguous(memory_format=torch.channels_last)
    w1 = torch.randn(32, 16, 1, 1)
    w3 = torch.randn(32, 16, 3, 3)
    assert K._pointwise_gemm_ok(K.conv_geometry(x, w1, (1, 1), (0, 0), 1), x)
    assert not K._pointwise_gemm_ok(K.conv_geometry(x, w1, (2, 2), (0, 0), 1), x)  # strided
    assert not K._pointwise_gemm_ok(K.conv_geometry(x, w3, (1, 1), (1, 1), 1), x)  # 3 x 3
    assert not K._pointwise_gemm_ok(K.conv_geometry(x, torch.randn(32, 8, 1, 1), (1, 1), (0, 0), 2), x)  # grouped
    assert not K._pointwise_gemm_ok(K.conv_geometry(x, w1, (1, 1), (0, 0), 1), x.contiguous())  # NCHW memory
    # the row view of a channel-last tensor is a view (the GEMM writes through it)
    r = K._rows(x)
    assert r.shape == (2 * 5 * 5, 16) and r.data_ptr() == x.data_ptr()


def test_forward_packs_dgrad_operand_only_for_our_dgrad(monkeypatch):
    g = [2, 16, 5, 5, 32, 5, 5, 3, 3, 1, 1, 1, 1, 1]
    monkeypatch.setattr(K, "_CONV_IMPL", "")
    monkeypatch.setattr(K, "_conv_tuned", {})
    assert K._bwd_picks_ours(g, True)  # not tuned yet: pack (harmless if unused)
    monkeypatch.setattr(K, "_conv_tuned", {("bwd", tuple(g) + (True, True, True)): "lib"})
    assert not K._bwd_picks_ours(g, True)
    monkeypatch.setattr(K, "_conv_tuned", {("bwd", tuple(g) + (True, True, True)): "ours"})
    assert K._bwd_picks_ours(g, True)
    monkeypatch.setattr(K, "_CONV_IMPL", "lib")
    assert not K._bwd_picks_ours(g, True)
