"""Seq2seq NMT with stacked LSTMs (reference nmt/nmt.cc, the legacy Legion RNN application: 2-layer
encoder/decoder, hidden = embedding = 2048, vocabulary 20480, 64 sequences per GPU of 20 steps).
The encoder LSTMs read the source embeddings; each decoder layer starts from the final (h, c) of the
matching encoder layer and reads the target embeddings; a vocabulary projection and softmax follow.
The reference placed each layer's time chunks on GPUs by hand (nmt/rnn_mapper.cc); here the layers
are ordinary ops and the strategy search decides. --small: vocabulary 1000, width 128, 10 steps.

    python -m flexflow_amd.run --nproc 8 examples/python/native/nmt.py -b 512 --search unity
"""
import zoo
from flexflow_amd.core import *  # noqa: F401,F403


def seq2seq(ff, src, dst, vocab, embed, hidden, layers):
    x = ff.embedding(src, vocab, embed, AggrMode.AGGR_MODE_NONE, name="src_embed")
    final = []
    for i in range(layers):
        x, h, c = ff.lstm(x, hidden, name=f"encoder{i}")
        final.append((h, c))
    t = ff.embedding(dst, vocab, embed, AggrMode.AGGR_MODE_NONE, name="dst_embed")
    for i, (h, c) in enumerate(final):
        t, _, _ = ff.lstm(t, hidden, h, c, name=f"decoder{i}")
    return ff.softmax(ff.dense(t, vocab, name="linear"), name="softmax")


if __name__ == "__main__":
    ffconfig, ffmodel, small, iterations = zoo.setup()
    vocab, width, steps = (1000, 128, 10) if small else (20 * 1024, 2048, 20)
    src = ffmodel.create_tensor([ffconfig.batch_size, steps], DataType.DT_INT32, name="src_ids")
    dst = ffmodel.create_tensor([ffconfig.batch_size, steps], DataType.DT_INT32, name="dst_ids")
    out = seq2seq(ffmodel, src, dst, vocab, width, width, 2)
    zoo.train("nmt", ffconfig, ffmodel, [src, dst], out, zoo.SCCE, zoo.ACC, iterations,
              index_range={src.guid: vocab, dst.guid: vocab})
