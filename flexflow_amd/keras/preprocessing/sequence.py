import numpy as np


def pad_sequences(sequences, maxlen=None, dtype="int32", padding="pre", truncating="pre", value=0):
    maxlen = maxlen or max(len(s) for s in sequences)
    out = np.full((len(sequences), maxlen), value, dtype=dtype)
    for i, s in enumerate(sequences):
        s = list(s)
        s = s[-maxlen:] if truncating == "pre" else s[:maxlen]
        if padding == "pre":
            out[i, maxlen - len(s):] = s
        else:
            out[i, :len(s)] = s
    return out
