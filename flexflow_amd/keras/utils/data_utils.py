"""Keras data utilities (reference python/flexflow/keras/utils/data_utils.py): the Sequence
batch-provider protocol, background enqueuers that prefetch its batches (threads), and get_file /
validate_file over the local Keras cache (this build runs without network: get_file only resolves
files already in the cache)."""
from __future__ import annotations

import hashlib
import os
import queue
import random
import shutil
import threading


def cleanup_keras_folder(fpath=os.path.join("/tmp", ".keras")):
    if os.path.exists(fpath):
        shutil.rmtree(fpath)


def _hash_file(fpath, algorithm="sha256", chunk_size=65535):
    h = hashlib.sha256() if algorithm in ("sha256", "auto") else hashlib.md5()
    with open(fpath, "rb") as f:
        for chunk in iter(lambda: f.read(chunk_size), b""):
            h.update(chunk)
    return h.hexdigest()


def validate_file(fpath, file_hash, algorithm="auto", chunk_size=65535):
    if algorithm == "auto":
        algorithm = "sha256" if len(file_hash) == 64 else "md5"
    return _hash_file(fpath, algorithm, chunk_size) == str(file_hash)


def get_file(fname, origin=None, untar=False, md5_hash=None, file_hash=None, cache_subdir="datasets",
             hash_algorithm="auto", extract=False, archive_format="auto", cache_dir=None):
    """Path of fname in the Keras cache (~/.keras/<cache_subdir>, or /tmp/.keras when the home
    directory is not writable); the file must already be there (no downloads in this build)."""
    cache_dir = cache_dir or os.path.join(os.path.expanduser("~"), ".keras")
    candidates = [os.path.join(cache_dir, cache_subdir, fname), os.path.join("/tmp", ".keras", cache_subdir, fname)]
    for path in candidates:
        if os.path.exists(path):
            if (file_hash or md5_hash) and not validate_file(path, file_hash or md5_hash, hash_algorithm):
                raise ValueError(f"{path}: hash mismatch")
            if untar or extract:
                shutil.unpack_archive(path, os.path.dirname(path))
            return path
    raise FileNotFoundError(f"{fname} is not in the Keras cache ({candidates[0]}) and this build does not "
                            f"download (origin {origin})")


class Sequence:
    """Base class of a batch provider: implement __getitem__(index) -> batch and __len__()."""

    def __getitem__(self, index):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError

    def on_epoch_end(self):
        pass

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class SequenceEnqueuer:
    """Runs a producer in background threads, filling a bounded queue that get() drains."""

    def __init__(self, sequence, use_multiprocessing=False):
        self.sequence = sequence
        self.use_multiprocessing = use_multiprocessing  # threads only here
        self._queue = None
        self._stop = None
        self._threads = []

    def is_running(self):
        return self._stop is not None and not self._stop.is_set()

    def start(self, workers=1, max_queue_size=10):
        self._queue = queue.Queue(max_queue_size)
        self._stop = threading.Event()
        self._threads = [threading.Thread(target=self._run, daemon=True) for _ in range(max(1, workers))]
        for t in self._threads:
            t.start()

    def stop(self, timeout=None):
        if self._stop is None:
            return
        self._stop.set()
        while self._queue is not None and not self._queue.empty():
            self._queue.get_nowait()
        for t in self._threads:
            t.join(timeout)
        self._threads = []

    def _put(self, item):
        while not self._stop.is_set():
            try:
                self._queue.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _run(self):
        raise NotImplementedError

    def get(self):
        while self.is_running() or (self._queue is not None and not self._queue.empty()):
            try:
                item = self._queue.get(timeout=0.1)
            except queue.Empty:
                continue
            if isinstance(item, BaseException):
                raise item
            if item is _END:
                return
            yield item


_END = object()


class OrderedEnqueuer(SequenceEnqueuer):
    """Prefetches a Sequence's batches in order (optionally shuffled per epoch), epoch after epoch."""

    def __init__(self, sequence, use_multiprocessing=False, shuffle=False):
        super().__init__(sequence, use_multiprocessing)
        self.shuffle = shuffle
        self._lock = threading.Lock()

    def start(self, workers=1, max_queue_size=10):
        super().start(1, max_queue_size)  # one producer keeps the batches ordered

    def _run(self):
        try:
            while not self._stop.is_set():
                order = list(range(len(self.sequence)))
                if self.shuffle:
                    random.shuffle(order)
                for i in order:
                    if not self._put(self.sequence[i]):
                        return
                self.sequence.on_epoch_end()
        except BaseException as e:  # surfaced by get()
            self._put(e)


class GeneratorEnqueuer(SequenceEnqueuer):
    """Prefetches a Python generator's items in background threads."""

    def __init__(self, sequence, use_multiprocessing=False, wait_time=None, random_seed=None):
        super().__init__(sequence, use_multiprocessing)
        self._lock = threading.Lock()

    def _run(self):
        try:
            while not self._stop.is_set():
                with self._lock:
                    try:
                        item = next(self.sequence)
                    except StopIteration:
                        self._put(_END)
                        return
                if not self._put(item):
                    return
        except BaseException as e:
            self._put(e)
