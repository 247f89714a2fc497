"""BERT encoder (BERT-Large: 24 layers, hidden 1024, 16 heads, FFN 4096, seq 512, vocab 30522).

Built against the FFModel API exactly as a user would (reference examples:
examples/python/native/bert_proxy_native.py — a proxy without LayerNorm/softmax — and
examples/cpp/Transformer/transformer.cc). This is the full post-LN BERT encoder with token +
position embeddings and a masked-LM style head over every position (dense+GELU, LayerNorm,
vocab projection, softmax, sparse categorical cross-entropy).
"""
from __future__ import annotations

from dataclasses import dataclass

from ..type import ActiMode, AggrMode, DataType


@dataclass
class BertConfig:
    hidden: int = 1024
    heads: int = 16
    layers: int = 24
    ffn: int = 4096
    vocab: int = 30522
    # pad the MLM decoder's output width to a multiple of this (0: no padding); the padded logits
    # carry a -1e9 bias (MaskedTailInitializer), so the model computes exactly the unpadded loss
    pad_vocab_multiple: int = 0
    max_pos: int = 512
    seq: int = 512
    dropout: float = 0.0
    mlm_head: bool = True

    @staticmethod
    def large(seq=512):
        return BertConfig(seq=seq)

    @staticmethod
    def base(seq=512):
        return BertConfig(hidden=768, heads=12, layers=12, ffn=3072, seq=seq)

    @staticmethod
    def tiny(seq=64):
        return BertConfig(hidden=128, heads=2, layers=2, ffn=256, vocab=1000, max_pos=seq, seq=seq)

    def padded_vocab(self) -> int:
        m = int(self.pad_vocab_multiple or 0)
        return (self.vocab + m - 1) // m * m if m > 1 else self.vocab

    def params(self) -> int:
        h, f = self.hidden, self.ffn
        per_layer = 4 * h * h + 4 * h + 2 * h * f + f + h + 4 * h
        emb = (self.vocab + self.max_pos) * h + 2 * h
        head = h * h + h + 2 * h + h * self.vocab + self.vocab if self.mlm_head else h * 2 + 2
        return self.layers * per_layer + emb + head

    def train_flops_per_seq(self) -> float:
        """6 * matmul-params * tokens + attention (fwd 4*S^2*H, x3 for fwd+bwd)."""
        h, f, S = self.hidden, self.ffn, self.seq
        mm = self.layers * (4 * h * h + 2 * h * f) + (h * h + h * self.vocab if self.mlm_head else 0)
        att = self.layers * 4 * S * S * h
        return 6.0 * mm * S + 3.0 * att


def build_bert(ff, batch: int, cfg: BertConfig):
    """Returns (ids_tensor, pos_tensor, output). Output: [batch, seq, vocab] probabilities."""
    S, H = cfg.seq, cfg.hidden
    ids = ff.create_tensor([batch, S], DataType.DT_INT32, name="input_ids")
    pos = ff.create_tensor([batch, S], DataType.DT_INT32, name="position_ids")
    x = ff.embedding(ids, cfg.vocab, H, AggrMode.AGGR_MODE_NONE, name="tok_emb")
    p = ff.embedding(pos, cfg.max_pos, H, AggrMode.AGGR_MODE_NONE, name="pos_emb")
    x = ff.add(x, p, name="emb_add")
    x = ff.layer_norm(x, [-1], name="emb_ln")
    for l in range(cfg.layers):
        a = ff.multihead_attention(x, x, x, H, cfg.heads, name=f"l{l}_attn")
        if cfg.dropout > 0:
            a = ff.dropout(a, cfg.dropout, l, name=f"l{l}_attn_drop")
        x = ff.layer_norm(ff.add(a, x, name=f"l{l}_res1"), [-1], name=f"l{l}_ln1")
        h = ff.dense(x, cfg.ffn, ActiMode.AC_MODE_GELU, name=f"l{l}_ffn1")
        h = ff.dense(h, H, name=f"l{l}_ffn2")
        if cfg.dropout > 0:
            h = ff.dropout(h, cfg.dropout, 1000 + l, name=f"l{l}_ffn_drop")
        x = ff.layer_norm(ff.add(h, x, name=f"l{l}_res2"), [-1], name=f"l{l}_ln2")
    if cfg.mlm_head:
        t = ff.dense(x, H, ActiMode.AC_MODE_GELU, name="mlm_transform")
        t = ff.layer_norm(t, [-1], name="mlm_ln")
        vp = cfg.padded_vocab()
        if vp > cfg.vocab:
            from ..core.initializers import GlorotUniformInitializer, MaskedTailInitializer
            # the real rows are initialised as in the unpadded model (same values, same fans)
            t = ff.dense(t, vp, kernel_initializer=GlorotUniformInitializer(seed=None, fans=(H, cfg.vocab)),
                         bias_initializer=MaskedTailInitializer(cfg.vocab), name="mlm_decoder")
        else:
            t = ff.dense(t, cfg.vocab, name="mlm_decoder")
    else:
        t = ff.dense(x, 2, name="cls")
    out = ff.softmax(t, name="mlm_softmax")
    return ids, pos, out
