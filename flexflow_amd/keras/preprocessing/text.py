import numpy as np


class Tokenizer:
    def __init__(self, num_words=None, **kw):
        self.num_words = num_words

    def sequences_to_matrix(self, sequences, mode="binary"):
        n = self.num_words
        out = np.zeros((len(sequences), n), dtype=np.float32)
        for i, s in enumerate(sequences):
            for w in s:
                if w < n:
                    if mode == "count":
                        out[i, w] += 1
                    else:
                        out[i, w] = 1
        if mode == "freq":
            out /= np.maximum(out.sum(1, keepdims=True), 1)
        return out
