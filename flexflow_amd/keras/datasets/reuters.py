"""Reuters newswire topics: lists of word-index sequences + 46 topic labels (synthetic offline)."""
import numpy as np


def load_data(num_words=1000, test_split=0.2, seed=113, n=11228, num_classes=46, maxlen=200, **kw):
    rng = np.random.default_rng(seed)
    topic_words = rng.integers(1, num_words, (num_classes, 20))
    y = rng.integers(0, num_classes, n)
    xs = []
    for c in y:
        ln = int(rng.integers(20, maxlen))
        words = np.where(rng.random(ln) < 0.5, rng.choice(topic_words[c], ln), rng.integers(1, num_words, ln))
        xs.append(list(words.astype(np.int64)))
    x = np.empty(n, dtype=object)
    x[:] = xs
    cut = int(n * (1 - test_split))
    return (x[:cut], y[:cut]), (x[cut:], y[cut:])
