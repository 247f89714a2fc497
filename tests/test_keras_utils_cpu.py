"""Keras utils (reference keras/utils/{generic_utils,data_utils}.py): custom-object scopes and
(de)serialization, Progbar, list helpers, the Sequence protocol and its background enqueuers."""
import numpy as np
import pytest

from flexflow_amd.keras.utils import data_utils, generic_utils


class _Doubler:
    def __init__(self, k=2):
        self.k = k

    def get_config(self):
        return {"k": self.k}


def test_custom_objects_roundtrip():
    s = generic_utils.serialize_keras_object(_Doubler(3))
    assert s == {"class_name": "_Doubler", "config": {"k": 3}}
    with pytest.raises(ValueError):
        generic_utils.deserialize_keras_object(s)
    with generic_utils.custom_object_scope({"_Doubler": _Doubler}):
        assert generic_utils.deserialize_keras_object(s).k == 3
    assert "_Doubler" not in generic_utils.get_custom_objects()


def test_small_helpers(capsys):
    assert generic_utils.to_list(1) == [1] and generic_utils.unpack_singleton([5]) == 5
    assert generic_utils.is_all_none([None, None]) and not generic_utils.is_all_none([None, 1])
    a, b = np.arange(10), np.arange(10) * 2
    np.testing.assert_array_equal(generic_utils.slice_arrays([a, b], 2, 4)[1], [4, 6])
    assert generic_utils.transpose_shape((8, 32, 32, 3), "channels_first", (1, 2)) == (8, 3, 32, 32)
    assert generic_utils.has_arg(lambda x, y=1: 0, "y")
    f = generic_utils.func_load(generic_utils.func_dump(lambda x, k=3: x * k))
    assert f(2) == 6
    bar = generic_utils.Progbar(4)
    for i in range(1, 5):
        bar.update(i, [("loss", 1.0 / i)])
    assert "4/4" in capsys.readouterr().out


class _Seq(data_utils.Sequence):
    def __init__(self):
        self.epochs = 0

    def __len__(self):
        return 5

    def __getitem__(self, i):
        return np.full(3, i)

    def on_epoch_end(self):
        self.epochs += 1


def test_sequence_enqueuers():
    seq = _Seq()
    assert [int(b[0]) for b in seq] == [0, 1, 2, 3, 4]
    enq = data_utils.OrderedEnqueuer(seq)
    enq.start(workers=2, max_queue_size=3)
    gen = enq.get()
    got = [int(next(gen)[0]) for _ in range(7)]
    enq.stop()
    assert got == [0, 1, 2, 3, 4, 0, 1] and seq.epochs >= 1
    genq = data_utils.GeneratorEnqueuer(iter(range(6)))
    genq.start(workers=2)
    assert sorted(genq.get()) == list(range(6))
    genq.stop()
    with pytest.raises(FileNotFoundError):
        data_utils.get_file("definitely-not-cached.npz", origin="https://example.invalid/x.npz")
