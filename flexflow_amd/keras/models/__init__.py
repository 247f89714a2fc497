"""Keras Model / Sequential (reference python/flexflow/keras/models/{base_model,model,sequential}.py).

The symbolic graph recorded by layer calls is lowered onto an FFModel at compile(); the batch size
comes from compile(batch_size=...) or the FFConfig (-b), as in the reference where the batch is a
launch flag. A Model can be called on tensors like a layer (nested models are inlined into the
outer graph). fit/evaluate/predict stream numpy arrays through SingleDataLoader.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np

from ...core import FFConfig, FFModel
from ...core.dataloader import SingleDataLoader
from ...type import CompMode, DataType, LossType
from .. import callbacks as kcb
from .. import losses as klosses
from .. import metrics as kmetrics
from .. import optimizers as kopt
from ..layers import InputLayer, KTensor, Layer


class Model(Layer):
    def __init__(self, inputs=None, outputs=None, name=None):
        super().__init__(name=name or "model")
        self._inputs: List[KTensor] = list(inputs) if isinstance(inputs, (list, tuple)) else \
            ([inputs] if inputs is not None else [])
        self._outputs: List[KTensor] = list(outputs) if isinstance(outputs, (list, tuple)) else \
            ([outputs] if outputs is not None else [])
        self._ffconfig: Optional[FFConfig] = None
        self._ffmodel: Optional[FFModel] = None
        self._optimizer = None
        self._loss = None
        self._metrics = []
        self._ff_inputs = []
        self._ff_output = None
        self.stop_training = False

    # ---------------------------------------------------------------- properties
    @property
    def input(self):
        """The model's input tensors, always a list (reference keras/models/base_model.py:66)."""
        return list(self._inputs)

    @property
    def output(self):
        return self._outputs if len(self._outputs) != 1 else self._outputs[0]

    @property
    def ffmodel(self):
        return self._ffmodel

    @property
    def ffconfig(self):
        return self._ffconfig

    @property
    def optimizer(self):
        return self._optimizer

    @property
    def layers(self) -> List[Layer]:
        return [L for L in self._topo_layers() if not isinstance(L, InputLayer)]

    def get_layer(self, name=None, index=None):
        layers = self.layers
        if index is not None:
            if index >= len(layers):
                raise ValueError(f"layer index {index} out of range ({len(layers)} layers)")
            return layers[index]
        for L in layers:
            if L.name == name:
                return L
        raise ValueError(f"No such layer: {name}")

    def _all_layers(self):
        """Every layer of this model, nested models expanded."""
        out = []
        for L in self.layers:
            out.extend(L._all_layers() if isinstance(L, Model) else [L])
        return out

    def get_weights(self, ffmodel=None):
        m = ffmodel or (self._ffmodel if self._ffmodel is not None else self._model.ffmodel)
        return [w for L in self._all_layers() for w in L.get_weights(m)]

    def set_weights(self, weights, ffmodel=None):
        m = ffmodel or (self._ffmodel if self._ffmodel is not None else self._model.ffmodel)
        it = iter(weights)
        for L in self._all_layers():
            n = sum(len(fl.weights) for fl in L.ff_layers[:1])
            if n:
                L.set_weights([next(it) for _ in range(n)], m)

    # ---------------------------------------------------------------- graph
    def _topo_layers(self):
        """Layers reachable from the outputs, in dependency order (each once)."""
        order, seen = [], set()

        def visit(t: KTensor):
            L = t.layer
            if L is None or id(L) in seen:
                return
            for call in L.inbound:
                for x in call:
                    visit(x)
            seen.add(id(L))
            order.append(L)

        for o in self._outputs:
            visit(o)
        return order

    def compute_output_shape(self, in_shapes):
        return [o.shape for o in self._outputs]

    def output_dtypes(self, in_dtypes):
        return [o.dtype for o in self._outputs]

    def _lower(self, ff, xs):
        """Inline this model's graph with its inputs bound to xs (nested model)."""
        return self._lower_graph(ff, dict(zip([id(t) for t in self._inputs], xs)))

    def _lower_graph(self, ff, env: Dict[int, object]):
        def val(t):
            if id(t) in env:
                return env[id(t)]
            L = t.layer
            call = None
            for ci, outs in enumerate(L.outbound):
                if any(o is t for o in outs):
                    call = ci
                    break
            ins = [val(x) for x in L.inbound[call]]
            outs = L._lower(ff, ins)
            for o, v in zip(L.outbound[call], outs):
                env[id(o)] = v
            return env[id(t)]

        return [val(o) for o in self._outputs]

    # ---------------------------------------------------------------- compile / train
    def compile(self, optimizer, loss=None, metrics=None, loss_weights=None, weighted_metrics=None,
                run_eagerly=None, comp_mode=CompMode.TRAINING, batch_size=None, ffconfig=None, **kwargs):
        if loss is None:
            raise ValueError("loss is None")
        self._loss = klosses.get(loss)
        self._metrics = [kmetrics.get(m) for m in (metrics or [])]
        self._ffconfig = ffconfig or FFConfig()
        if batch_size is not None:
            self._ffconfig.batch_size = int(batch_size)
        bs = self._ffconfig.batch_size
        ff = FFModel(self._ffconfig)
        env = {}
        self._ff_inputs = []
        for t in self._inputs:
            ft = ff.create_tensor((bs,) + t.shape, t.dtype, name=t.name)
            env[id(t)] = ft
            self._ff_inputs.append(ft)
        outs = self._lower_graph(ff, env)
        stack = list(self.layers)
        while stack:  # every layer and nested model reads weights through this (root) model
            L = stack.pop()
            L._model = self
            if isinstance(L, Model):
                stack.extend(L.layers)
        if len(outs) != 1:
            raise NotImplementedError("one model output (as the reference)")
        self._ff_output = outs[0]
        self._optimizer = kopt.get(optimizer)
        ff.optimizer = self._optimizer.create_ffhandle(ff)
        ff.compile(loss_type=self._loss.type, metrics=[m.type for m in self._metrics], comp_mode=comp_mode)
        self._ffmodel = ff

    def _loaders(self, x, y):
        xs = x if isinstance(x, (list, tuple)) else [x]
        if len(xs) != len(self._ff_inputs):
            raise ValueError(f"expected {len(self._ff_inputs)} input arrays, got {len(xs)}")
        for a, t in zip(xs, self._ff_inputs):
            if tuple(a.shape[1:]) != tuple(t.dims[1:]):
                raise ValueError(f"input shape {a.shape[1:]} != model input {tuple(t.dims[1:])}")
        dls = [SingleDataLoader(self._ffmodel, t, a) for t, a in zip(self._ff_inputs, xs)]
        ydl = None
        if y is not None:
            lab = self._ffmodel.label_tensor
            y = np.asarray(y)
            if self._loss.type == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
                y = y.astype(np.int32).reshape((y.shape[0],) + tuple(lab.dims[1:]))
            else:
                y = y.astype(np.float32).reshape((y.shape[0],) + tuple(lab.dims[1:]))
            ydl = SingleDataLoader(self._ffmodel, lab, y)
        return dls, ydl

    def _logs(self):
        pm = self._ffmodel.get_perf_metrics()
        logs = {"loss": pm.get_loss()}
        if any(isinstance(m, kmetrics.Accuracy) for m in self._metrics):
            logs["accuracy"] = pm.get_accuracy()
        return logs

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose=1, callbacks=None, shuffle=True, **kwargs):
        if self._ffmodel is None:
            raise RuntimeError("compile() the model first")
        if batch_size is not None and batch_size != self._ffconfig.batch_size:
            raise ValueError(f"batch_size {batch_size} != compiled batch {self._ffconfig.batch_size}")
        dls, ydl = self._loaders(x, y)
        cbs = list(callbacks or [])
        hist = kcb.History()
        cbs.append(hist)
        for cb in cbs:
            cb.set_model(self)
            cb.set_params({"epochs": epochs})
            cb.on_train_begin()
        bs = self._ffconfig.batch_size
        iters = dls[0].num_samples // bs
        self.stop_training = False
        t0 = time.perf_counter()
        for ep in range(epochs):
            for cb in cbs:
                cb.on_epoch_begin(ep)
            for d in dls + ([ydl] if ydl else []):
                d.reset()
            self._ffmodel.reset_metrics()
            for it in range(iters):
                for cb in cbs:
                    cb.on_batch_begin(it)
                for d in dls + ([ydl] if ydl else []):
                    d.next_batch(self._ffmodel)
                self._ffmodel.train_step()
                for cb in cbs:
                    cb.on_batch_end(it)
            logs = self._logs()
            if verbose and self._ffconfig.rank == 0:
                print(f"epoch {ep + 1}/{epochs}: " + ", ".join(f"{k}={v:.4f}" for k, v in logs.items()), flush=True)
            stop = False
            for cb in cbs:
                stop = bool(cb.on_epoch_end(ep, logs)) or stop
            if stop or self.stop_training:
                break
        el = time.perf_counter() - t0
        if verbose and self._ffconfig.rank == 0:
            print(f"ELAPSED TIME = {el:.4f}s, THROUGHPUT = {iters * bs * (ep + 1) / max(el, 1e-9):.2f} samples/s")
        for cb in cbs:
            cb.on_train_end()
        return hist

    def evaluate(self, x=None, y=None, batch_size=None, verbose=1, **kwargs):
        dls, ydl = self._loaders(x, y)
        bs = self._ffconfig.batch_size
        for d in dls + ([ydl] if ydl else []):
            d.reset()
        self._ffmodel.reset_metrics()
        for _ in range(dls[0].num_samples // bs):
            for d in dls + ([ydl] if ydl else []):
                d.next_batch(self._ffmodel)
            self._ffmodel.executor.forward(training=False)
            self._ffmodel.executor.compute_loss_grad()
        logs = self._logs()
        if verbose and self._ffconfig.rank == 0:
            print("evaluate: " + ", ".join(f"{k}={v:.4f}" for k, v in logs.items()), flush=True)
        return logs

    def predict(self, x, batch_size=None, verbose=0, **kwargs):
        xs = x if isinstance(x, (list, tuple)) else [x]
        bs = self._ffconfig.batch_size
        n = xs[0].shape[0] // bs * bs
        outs = []
        for s in range(0, n, bs):
            for t, a in zip(self._ff_inputs, xs):
                t.set_tensor(self._ffmodel, a[s:s + bs])
            self._ffmodel.forward()
            outs.append(np.asarray(self._ff_output.get_tensor(self._ffmodel), dtype=np.float32))
        return np.concatenate(outs, 0) if outs else np.zeros((0,) + tuple(self._ff_output.dims[1:]), np.float32)

    def summary(self, line_length=None, positions=None, print_fn=None):
        s = "Layer (type)\t\tOutput Shape\t\tInput Shape\tConnected to\n"
        for t in self._inputs:
            s += f"{t.name} (InputLayer)\t\t[{t.batch_shape}]\n"
        for L in self.layers:
            s += L.get_summary()
        if print_fn:
            print_fn(s)
        return s


class Sequential(Model):
    def __init__(self, layers=None, name=None):
        super().__init__(name=name or "sequential")
        self._seq: List = []
        for L in layers or []:
            self.add(L)

    def add(self, layer):
        if isinstance(layer, KTensor):  # an Input(...) tensor
            if self._inputs:
                raise ValueError("Input must be the first element")
            self._inputs = [layer]
            self._outputs = [layer]
            return
        if not self._inputs:
            if layer.input_shape is None:
                raise ValueError("the first layer needs input_shape= (or start with Input)")
            t = InputLayer(layer.input_shape, dtype=layer.dtype or "float32").output_tensor
            self._inputs = [t]
            self._outputs = [t]
        self._seq.append(layer)
        self._outputs = [layer(self._outputs[0])]

    def pop(self):
        raise NotImplementedError("pop() is not supported (as the reference)")


__all__ = ["Model", "Sequential"]


# reference names: keras/models/base_model.py BaseModel (the common base of Model and Sequential)
# and keras/models/tensor.py Tensor (the symbolic tensor of layer calls)
BaseModel = Model
Tensor = KTensor
