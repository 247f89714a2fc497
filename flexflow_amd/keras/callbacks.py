"""Keras callbacks (reference keras/callbacks.py): hooks called by Model.fit."""
from __future__ import annotations


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        """Return True to stop training early."""
        return False

    def on_batch_begin(self, batch, logs=None):
        pass

    def on_batch_end(self, batch, logs=None):
        pass


class LearningRateScheduler(Callback):
    """schedule(epoch) -> learning rate, applied at the start of every epoch."""

    def __init__(self, schedule):
        super().__init__()
        self.schedule = schedule

    def on_epoch_begin(self, epoch, logs=None):
        lr = self.schedule(epoch)
        self.model.optimizer.set_learning_rate(lr)


class VerifyMetrics(Callback):
    """Assert at the end of training that accuracy (percent) reached `accuracy`."""

    def __init__(self, accuracy):
        super().__init__()
        self.accuracy = float(getattr(accuracy, "value", accuracy))

    def on_train_end(self, logs=None):
        acc = self.model.ffmodel.get_perf_metrics().get_accuracy()
        assert acc >= self.accuracy, f"accuracy {acc:.2f}% below {self.accuracy}%"


class EpochVerifyMetrics(Callback):
    """Stop training early once accuracy (percent) reaches `accuracy`."""

    def __init__(self, accuracy, early_stop=True):
        super().__init__()
        self.accuracy = float(getattr(accuracy, "value", accuracy))
        self.early_stop = early_stop

    def on_epoch_end(self, epoch, logs=None):
        acc = self.model.ffmodel.get_perf_metrics().get_accuracy()
        return bool(self.early_stop and acc >= self.accuracy)


class History(Callback):
    def __init__(self):
        super().__init__()
        self.history = {}
        self.epoch = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)
        return False
