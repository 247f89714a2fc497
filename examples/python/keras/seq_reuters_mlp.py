"""Reuters topic MLP on bag-of-words features (reference examples/python/keras/seq_reuters_mlp.py)."""
from _args import parse  # noqa: I001  (puts the repo root on sys.path)
from accuracy import ModelAccuracy

from flexflow_amd.keras import layers, optimizers
from flexflow_amd.keras.datasets import reuters
from flexflow_amd.keras.models import Sequential
from flexflow_amd.keras.preprocessing.text import Tokenizer


def top_level_task(argv=None, num_samples=11228, epochs=4, max_words=1000):
    (xtr, ytr), _ = reuters.load_data(num_words=max_words, n=num_samples)
    x = Tokenizer(num_words=max_words).sequences_to_matrix(xtr, mode="binary").astype("float32")
    y = ytr.astype("int32").reshape(-1, 1)
    model = Sequential([layers.Dense(512, input_shape=(max_words,), activation="relu"),
                        layers.Dropout(0.2),
                        layers.Dense(46),
                        layers.Activation("softmax")])
    model.compile(optimizer=optimizers.Adam(learning_rate=0.001), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy"], batch_size=32)
    return model.fit(x, y, epochs=epochs)


if __name__ == "__main__":
    args, rest = parse(11228)
    hist = top_level_task(rest, args.samples)
    if args.test_acc:
        assert hist.history["accuracy"][-1] >= ModelAccuracy.REUTERS_MLP.value
