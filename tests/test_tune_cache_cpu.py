"""Persistent autotune cache (FF_TUNE_CACHE): choices written by one run are found by the next."""
import json

import torch

from flexflow_amd import kernels as K


def test_tune_cache_round_trip(tmp_path, monkeypatch):
    path = str(tmp_path / "tune.json")
    gkey = (16384, 1024, 4096, True, False, 4096, 1024, 1024, 1, torch.bfloat16, False, False, 10, False, None)
    ckey = ("fwd", (64, 64, 56, 56, 64, 56, 56, 3, 3, 1, 1, 1, 1, 1))
    monkeypatch.setattr(K, "_tuned", {gkey: "pp_sk4", ("dact", 1, 2): "unfused", (1, 2, 3): ("lt", 7, 0)})
    monkeypatch.setattr(K, "_timed", {gkey, ("dact", 1, 2), (1, 2, 3), (9, 9)})
    monkeypatch.setattr(K, "_conv_tuned", {ckey: "ours"})
    monkeypatch.setattr(K, "_cached", {"gemm": {}, "conv": {}})
    assert K.tune_cache_save(path) == 3  # the process-local "lt" plan is not persisted
    saved = json.load(open(path))
    assert set(saved) == {"gemm", "conv", "stamp"} and len(saved["gemm"]) == 2
    monkeypatch.setattr(K, "_tuned", {})
    monkeypatch.setattr(K, "_conv_tuned", {})
    monkeypatch.setattr(K, "_TUNE_CACHE", path)
    assert K.tune_cache_load(path) == 3
    assert K._tune_cache_lookup("gemm", gkey) == "pp_sk4"
    assert K._tune_cache_lookup("gemm", ("dact", 1, 2)) == "unfused"
    assert K._tune_cache_lookup("conv", ckey) == "ours"
    assert K._tune_cache_lookup("gemm", (1, 2, 3)) is None
    # a later save keeps what the file held and adds the new choices
    monkeypatch.setattr(K, "_tuned", {(9, 9): "lib"})
    assert K.tune_cache_save(path) == 4


def test_tune_cache_absent_file(tmp_path):
    assert K.tune_cache_load(str(tmp_path / "missing.json")) == 0
    assert K.tune_cache_load("") == 0


def test_tune_cache_skips_untimed_and_foreign_files(tmp_path, monkeypatch):
    path = str(tmp_path / "tune.json")
    monkeypatch.setattr(K, "_cached", {"gemm": {}, "conv": {}})
    # a default picked without timing (FF_GEMM_TUNE=0, or first call during capture) is not saved
    monkeypatch.setattr(K, "_tuned", {(1, 1): "k256", (2, 2): "lib"})
    monkeypatch.setattr(K, "_timed", {(2, 2)})
    monkeypatch.setattr(K, "_conv_tuned", {})
    assert K.tune_cache_save(path) == 1
    saved = json.load(open(path))
    assert list(saved["gemm"].values()) == ["lib"]
    # a file written for another device / kernel build is ignored
    saved["stamp"] = {"device": "other", "build": "x"}
    json.dump(saved, open(path, "w"))
    monkeypatch.setattr(K, "_cached", {"gemm": {}, "conv": {}})
    assert K.tune_cache_load(path) == 0
