"""MT5 fine-tuning through the HuggingFace import path (reference
examples/python/pytorch/mt5/mt5_ff.py: MT5ForConditionalGeneration -> PyTorchModel(is_hf_model=True)
-> torch_to_ff -> SGD with sparse categorical cross-entropy).

No network here: the model is built from an MT5 config with random weights (google/mt5-small's
shape by default, `--tiny` for a seconds-long run) and the data is a synthetic copy task (target =
the source sequence) in place of the reference's tokenized translation pairs. Inputs are unpadded,
so attention_mask is all ones (the import folds it; flexflow_amd/torch/export.py).

    python examples/python/pytorch/mt5/mt5_ff.py [--tiny] [-b 8] [-e 1] [--samples 256]
"""
import argparse
import os
import sys

_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..", ".."))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

import numpy as np  # noqa: E402

from flexflow_amd.core import *  # noqa: E402,F401,F403
from flexflow_amd.torch.model import PyTorchModel  # noqa: E402


def mt5_config(tiny):
    from transformers import MT5Config
    if tiny:
        return MT5Config(vocab_size=512, d_model=64, d_kv=16, d_ff=128, num_layers=2, num_decoder_layers=2,
                         num_heads=4, relative_attention_num_buckets=8, dropout_rate=0.0)
    # google/mt5-small (vocabulary cut to 32k: the 250k-entry table is not what this example exercises)
    return MT5Config(vocab_size=32128, d_model=512, d_kv=64, d_ff=1024, num_layers=8, num_decoder_layers=8,
                     num_heads=6, relative_attention_num_buckets=32, dropout_rate=0.1,
                     feed_forward_proj="gated-gelu")


def synthetic_copy_task(n, src_len, tgt_len, vocab, seed=0):
    """(source ids, decoder input ids, labels): the target is the source; the decoder input is the
    target shifted right after the pad/start token 0 (reference preprocess_train)."""
    rng = np.random.default_rng(seed)
    src = rng.integers(1, vocab, (n, src_len)).astype(np.int64)
    tgt = src[:, :tgt_len]
    dec = np.concatenate([np.zeros((n, 1), np.int64), tgt[:, :-1]], 1)
    return src, dec, tgt.astype(np.int32).reshape(n, tgt_len, 1)


def top_level_task(argv, tiny, num_samples, src_len=48, tgt_len=48):
    from transformers import MT5ForConditionalGeneration
    ffconfig = FFConfig(argv)
    ffmodel = FFModel(ffconfig)
    cfg = mt5_config(tiny)
    model = MT5ForConditionalGeneration(cfg)
    if tiny:
        src_len, tgt_len = 16, 12
    batch_size = ffconfig.batch_size
    input_tensors = [
        ffmodel.create_tensor([batch_size, src_len], DataType.DT_INT64),  # input_ids
        ffmodel.create_tensor([batch_size, src_len], DataType.DT_INT64),  # attention_mask
        ffmodel.create_tensor([batch_size, tgt_len], DataType.DT_INT64),  # decoder_input_ids
    ]
    print("Tracing the model...")
    hf_model = PyTorchModel(model, is_hf_model=True,
                            input_names=["input_ids", "attention_mask", "decoder_input_ids"],
                            batch_size=batch_size, seq_length=(src_len, tgt_len))
    hf_model.torch_to_ff(ffmodel, input_tensors)
    ffoptimizer = SGDOptimizer(ffmodel, lr=0.01)
    print("Compiling the model...")
    ffmodel.compile(optimizer=ffoptimizer, loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    src, dec, labels = synthetic_copy_task(num_samples, src_len, tgt_len, cfg.vocab_size)
    dls = [ffmodel.create_data_loader(input_tensors[0], src),
           ffmodel.create_data_loader(input_tensors[1], np.ones_like(src)),
           ffmodel.create_data_loader(input_tensors[2], dec)]
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, labels)
    ffmodel.init_layers()
    print("Training...")
    ffmodel.fit(x=dls, y=dl_y, batch_size=batch_size, epochs=ffconfig.epochs)
    return ffmodel.get_perf_metrics().get_loss() if hasattr(ffmodel.get_perf_metrics(), "get_loss") else None


if __name__ == "__main__":
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--samples", type=int, default=256)
    args, rest = ap.parse_known_args(sys.argv[1:])
    top_level_task(rest, args.tiny, args.samples)
