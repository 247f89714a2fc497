"""Seq2seq NMT with stacked LSTMs (reference nmt/nmt.cc, the legacy Legion RNN application: 2-layer
encoder/decoder, hidden = embedding = 2048, vocabulary 20480, 64 sequences per GPU): zoo model
"nmt" trained on synthetic batches through FFModel; `--small` shrinks it for CPU; flags in zoo.py.

    python -m flexflow_amd.run --nproc 8 examples/python/native/nmt.py -b 512 --search unity
"""
from zoo import run

if __name__ == "__main__":
    run("nmt")
