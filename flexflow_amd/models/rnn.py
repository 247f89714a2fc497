"""Seq2seq NMT with stacked LSTMs (the reference's legacy nmt/ application: nmt/nmt.cc, rnn.cu —
source / target embeddings, an encoder and a decoder LSTM stack whose layers start from the
encoder's final states, a vocabulary projection and softmax; defaults there: 2 layers, hidden and
embedding 2048, vocabulary 20480, 64 sequences per GPU of 20 steps).

Built with the FFModel API (FFModel.lstm, ops/rnn.py). The reference placed each layer's time
chunks on GPUs by hand (nmt/rnn_mapper.cc, GlobalConfig); here the layers are ordinary ops, so the
strategy search (or an imported strategy) decides data parallelism and layer placement.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..type import AggrMode, DataType


@dataclass
class NMTConfig:
    vocab: int = 20 * 1024
    embed: int = 2048
    hidden: int = 2048
    layers: int = 2
    src_len: int = 20
    dst_len: int = 20

    @staticmethod
    def small():
        return NMTConfig(vocab=1000, embed=128, hidden=128, layers=2, src_len=10, dst_len=10)

    def params(self) -> int:
        e, h = self.embed, self.hidden
        lstm = sum(4 * h * ((e if i == 0 else h) + h + 1) for i in range(self.layers))
        return 2 * self.vocab * e + 2 * lstm + h * self.vocab + self.vocab

    def train_flops_per_seq(self) -> float:
        e, h = self.embed, self.hidden
        per_tok = sum(2 * 4 * h * ((e if i == 0 else h) + h) for i in range(self.layers))
        return 3.0 * (per_tok * (self.src_len + self.dst_len) + 2 * h * self.vocab * self.dst_len)


def build_nmt(ff, batch: int, cfg: NMTConfig):
    """Returns (src_ids, dst_ids, output probabilities [batch, dst_len, vocab])."""
    src = ff.create_tensor([batch, cfg.src_len], DataType.DT_INT32, name="src_ids")
    dst = ff.create_tensor([batch, cfg.dst_len], DataType.DT_INT32, name="dst_ids")
    x = ff.embedding(src, cfg.vocab, cfg.embed, AggrMode.AGGR_MODE_NONE, name="src_embed")
    states = []
    for i in range(cfg.layers):
        x, h, c = ff.lstm(x, cfg.hidden, name=f"encoder{i}")
        states.append((h, c))
    t = ff.embedding(dst, cfg.vocab, cfg.embed, AggrMode.AGGR_MODE_NONE, name="dst_embed")
    for i in range(cfg.layers):
        t, _, _ = ff.lstm(t, cfg.hidden, states[i][0], states[i][1], name=f"decoder{i}")
    logits = ff.dense(t, cfg.vocab, name="linear")
    return src, dst, ff.softmax(logits, name="softmax")


def nmt_batch(batch: int, cfg: NMTConfig, rng):
    """Synthetic copy task (no dataset offline): the target is the source reversed, teacher-forced
    (decoder input = target shifted right after a start token 0)."""
    s = rng.integers(1, cfg.vocab, (batch, cfg.src_len), dtype=np.int32)
    tgt = s[:, ::-1][:, :cfg.dst_len]
    if tgt.shape[1] < cfg.dst_len:
        tgt = np.pad(tgt, ((0, 0), (0, cfg.dst_len - tgt.shape[1])))
    d = np.concatenate([np.zeros((batch, 1), np.int32), tgt[:, :-1]], 1)
    return s, np.ascontiguousarray(d), np.ascontiguousarray(tgt.reshape(batch, cfg.dst_len, 1))
