"""DistriModel: the model contract the training roles talk to, and its implementations.

Reference contract ``DistributedModel`` (/root/reference/src/common/models.ts:7-72):
``fit(x, y) -> grads``, ``update(grads)``, ``predict(x)``, ``evaluate(x, y) -> number[]``, ``getVars()``,
``setVars(vals)``, ``inputShape`` / ``outputShape`` (no batch dim).  Server models add ``version``,
``setup()``, ``save()`` (save => new version) (/root/reference/src/server/models.ts:38-61); client
models add ``setup()`` (/root/reference/src/client/models.ts:7-34).

Implementations:
  * :class:`EngineModel` (reference ``DistributedTfModel``, models.ts:74-151) — wraps the MI355X engine
    (:class:`~distriflow_amd.models.net.Net`): HIP kernels, flat fp32 master + bf16 compute copies.
    Besides the list API it exposes the zero-copy flat API the roles use on the hot path
    (``fit_flat`` returns the live flat gradient buffer in HBM, ``update_flat`` is one fused SGD launch).
  * :class:`DynamicModel` (reference ``DistributedDynamicModel``, models.ts:153-208) — raw variables +
    predict/loss callables through torch autograd (any device).  Fixes the reference's
    ``-this.learningRate`` NaN.
  * Server models: :class:`InMemoryServerModel` (models.ts:63-75), :class:`CheckpointedServerModel`
    (tf.js LayersModel directories + ``current`` symlink, models.ts:86-151),
    :class:`DynamicServerModel` (flat meta.json/data.bin, models.ts:153-267).
  * :class:`ClientModel` (client/models.ts:18-24).
"""
from __future__ import annotations

import warnings

import os
import time
from abc import ABC, abstractmethod
from typing import Callable, Optional, Sequence, Union

import torch

from .. import ops
from ..checkpoint import VersionedStore, load_flat, load_layers_model_weights, save_flat, save_layers_model
from ..config import compile_args
from ..losses import accuracy, get_loss
from .net import Net


class DistriModel(ABC):
    is_distri_model = True

    @abstractmethod
    def fit(self, x, y) -> list[torch.Tensor]: ...

    @abstractmethod
    def update(self, grads: Sequence[torch.Tensor]) -> None: ...

    @abstractmethod
    def predict(self, x) -> torch.Tensor: ...

    @abstractmethod
    def evaluate(self, x, y) -> list[float]: ...

    @abstractmethod
    def get_vars(self) -> list[torch.Tensor]: ...

    @abstractmethod
    def set_vars(self, vals: Sequence[torch.Tensor]) -> None: ...

    @property
    @abstractmethod
    def input_shape(self) -> list: ...

    @property
    @abstractmethod
    def output_shape(self) -> list: ...

    # ---- flat API (default implementations via the list API) ----
    def get_flat(self) -> torch.Tensor:
        return torch.cat([v.detach().reshape(-1).float() for v in self.get_vars()])

    def set_flat(self, flat: torch.Tensor) -> None:
        vals, off = [], 0
        for v in self.get_vars():
            n = v.numel()
            vals.append(flat[off: off + n].reshape(v.shape))
            off += n
        self.set_vars(vals)

    def fit_flat(self, x, y) -> torch.Tensor:
        return torch.cat([g.reshape(-1).float() for g in self.fit(x, y)])

    def update_flat(self, flat_grad: torch.Tensor, scale: float = 1.0) -> None:
        grads, off = [], 0
        for v in self.get_vars():
            n = v.numel()
            grads.append(flat_grad[off: off + n].reshape(v.shape) * scale)
            off += n
        self.update(grads)

    # ---- README DistriModel fields: modelID + savedGradient (/root/reference/README.md:24-29) ----
    # The reference advertises ``modelID: UUID`` and ``savedGradient: tf.grads (aggregated gradients
    # local)`` but never implements them.  Here the saved gradient is a flat fp32
    # accumulator on the model's device: ``accumulate(x, y)`` / ``save_gradient(g)`` add into it,
    # ``apply_saved_gradient()`` applies the mean (or sum) with one ``update_flat`` and clears it.
    @property
    def model_id(self) -> str:
        mid = self.__dict__.get("_model_id")
        if mid is None:
            import uuid

            mid = self.__dict__["_model_id"] = str(uuid.uuid4())
        return mid

    @property
    def saved_gradient(self) -> Optional[torch.Tensor]:
        return self.__dict__.get("_saved_grad")

    @property
    def saved_count(self) -> int:
        return self.__dict__.get("_saved_count", 0)

    def save_gradient(self, grads) -> None:
        """Add one gradient (flat tensor or per-variable list) into the local saved gradient."""
        flat = grads if isinstance(grads, torch.Tensor) else torch.cat([g.reshape(-1).float() for g in grads])
        acc = self.saved_gradient
        if acc is None:
            self.__dict__["_saved_grad"] = flat.detach().float().clone()
        else:
            if acc.numel() != flat.numel():
                raise ValueError(f"saved gradient has {acc.numel()} elements, got {flat.numel()}")
            acc.add_(flat.to(acc.device, torch.float32))
        self.__dict__["_saved_count"] = self.saved_count + 1

    def accumulate(self, x, y) -> torch.Tensor:
        """``fit`` one microbatch and add its gradient into the saved gradient (copies out of the live
        engine buffer, which the next ``fit`` overwrites)."""
        self.save_gradient(self.fit_flat(x, y))
        return self.saved_gradient

    def clear_saved_gradient(self) -> None:
        self.__dict__["_saved_grad"] = None
        self.__dict__["_saved_count"] = 0

    def apply_saved_gradient(self, mean: bool = True) -> int:
        """Apply the saved gradient (averaged over the saved microbatches when ``mean``) and clear it.
        Returns how many microbatches it held (0: nothing applied)."""
        n, acc = self.saved_count, self.saved_gradient
        if n == 0 or acc is None:
            return 0
        self.update_flat(acc, 1.0 / n if mean else 1.0)
        self.clear_saved_gradient()
        return n

    # reference camelCase aliases
    @property
    def modelID(self):
        return self.model_id

    @property
    def savedGradient(self):
        return self.saved_gradient

    def getVars(self):
        return self.get_vars()

    def setVars(self, vals):
        return self.set_vars(vals)

    @property
    def inputShape(self):
        return self.input_shape

    @property
    def outputShape(self):
        return self.output_shape


ModelSource = Union[Net, str, Callable[[], Net]]


def fetch_model(src: ModelSource, device=None) -> Net:
    """Reference ``fetchModel`` (utils.ts:236-244): a Net, a callable returning one, a zoo name, or a
    tf.js model.json path (topology + weights)."""
    from .zoo import MODELS, build_model

    if isinstance(src, Net):
        return src
    if callable(src):
        return src()
    if isinstance(src, str):
        dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
        if src in MODELS:
            return build_model(src, device=dev)
        path = src[len("file://"):] if src.startswith("file://") else src
        if os.path.isdir(path):
            path = os.path.join(path, "model.json")
        if os.path.exists(path):
            from ..checkpoint.tfjs import load_topology
            from .keras import layers_from_keras

            topo = load_topology(path)
            layers, shape = layers_from_keras(topo)
            net = Net(layers, shape, device=dev, name=os.path.basename(os.path.dirname(path)) or "model")
            net.topology = topo
            try:
                load_layers_model_weights(net, path, strict=True)
            except (KeyError, FileNotFoundError):
                pass  # topology-only model.json (e.g. the reference's, whose shards are not shipped)
            return net
        raise FileNotFoundError(f"model source {src!r} is neither a zoo name nor a model.json")
    raise TypeError(f"cannot fetch a model from {type(src).__name__}")


_CE_LOSSES = {"softmaxCrossEntropy", "categorical_crossentropy", "categoricalCrossentropy"}
_WARNED_LOSSES: set = set()


class EngineModel(DistriModel):
    """The MI355X engine behind the DistriModel contract (reference DistributedTfModel)."""

    def __init__(self, model: ModelSource, compile_config: Optional[dict] = None, device=None,
                 strict_loss: bool = False):
        self._src = model
        self._device = device
        self.compile = compile_args(compile_config)
        self.learning_rate = float(self.compile["learningRate"])
        self.loss_fn = get_loss(self.compile["loss"])
        self.net: Optional[Net] = model if isinstance(model, Net) else None
        self.momentum = 0.0
        self.weight_decay = 0.0
        self._strict_loss = strict_loss
        # checked now when the output is known (or cannot matter); a sigmoidCrossEntropy compile loss on a
        # not-yet-fetched model is checked once fetch_initial() knows whether the model ends in sigmoid
        if self.net is not None or self.compile["loss"] != "sigmoidCrossEntropy":
            self._check_loss()

    def _check_loss(self):
        """the reference's fit() always optimises softmax cross-entropy and the
        compile loss (default meanSquaredError) only feeds evaluate().  The engine trains the cross-entropy
        that matches the model's output (softmax CE, or sigmoid CE for a model ending in sigmoid) and says
        so once when the compile loss differs, instead of silently training another loss."""
        loss = self.compile["loss"]
        trained = "sigmoidCrossEntropy" if getattr(self.net, "final_act", "") == "sigmoid" else "softmax cross-entropy"
        ok = loss == "sigmoidCrossEntropy" if trained == "sigmoidCrossEntropy" else loss in _CE_LOSSES
        if ok:
            return
        if self._strict_loss:
            raise ValueError(f"EngineModel trains {trained} on logits; compile loss {loss!r} "
                             "is not trainable by the engine")
        if (loss, trained) not in _WARNED_LOSSES:
            _WARNED_LOSSES.add((loss, trained))
            warnings.warn(f"EngineModel trains {trained} on logits; the compile loss {loss!r} is "
                          "used for evaluate() metrics only (reference fit(), models.ts:137-142)", stacklevel=3)

    def fetch_initial(self):
        if self.net is None:
            self.net = fetch_model(self._src, self._device)
            if self.compile["loss"] == "sigmoidCrossEntropy":
                self._check_loss()
        self._sync_hyper()
        return self.net

    fetchInitial = fetch_initial

    def _need(self) -> Net:
        if self.net is None:
            self.fetch_initial()
        return self.net

    def _sync_hyper(self, grad_scale: float = 1.0):
        self.net.store.set_hyper(self.learning_rate, self.momentum, self.weight_decay, grad_scale)

    @property
    def device(self):
        return self._need().device

    def _prep(self, x, y):
        net = self._need()
        if isinstance(x, ops.GatherRef):
            xx = x
        else:
            xx = x.to(net.device)
            if xx.dim() == len(net.input_shape):
                xx = xx.unsqueeze(0)
            xx = xx.reshape((xx.shape[0],) + tuple(net.input_shape))
        y = y.to(net.device)
        if y.dim() > 1:  # one-hot labels (reference convention) -> class indices
            y = y.argmax(dim=1)
        return xx, y.to(torch.int32)

    # ---- contract ----
    def fit_flat(self, x, y) -> torch.Tensor:
        """fwd + fused softmax-CE + bwd; returns the LIVE flat fp32 gradient buffer (mean over the batch)."""
        xx, yy = self._prep(x, y)
        self.last_stats = self.net.compute_gradients(xx, yy)
        return self.net.store.grad

    def fit(self, x, y) -> list[torch.Tensor]:
        self.fit_flat(x, y)
        st = self.net.store
        return [st.gradient(s.name).clone() for s in st.specs]

    def update_flat(self, flat_grad: torch.Tensor, scale: float = 1.0) -> None:
        """w -= lr * scale * g — ONE fused launch over every parameter."""
        st = self._need().store
        if flat_grad.data_ptr() != st.grad.data_ptr():
            st.grad[: flat_grad.numel()].copy_(flat_grad.reshape(-1))
        self._sync_hyper(scale)
        st.sgd_step()

    def update(self, grads: Sequence[torch.Tensor]) -> None:
        st = self._need().store
        for s, g in zip(st.specs, grads):
            st.gradient(s.name).copy_(torch.as_tensor(g).reshape(s.shape))
        self._sync_hyper(1.0)
        st.sgd_step()

    def predict(self, x) -> torch.Tensor:
        net = self._need()
        xx, _ = self._prep(x, torch.zeros(1))
        return net.predict(xx)

    def evaluate(self, x, y) -> list[float]:
        """[compiled loss, accuracy] on (x, y) — the reference's model.evaluate with the compile args.
        GPU: the engine's forward kernels + one metrics launch (csrc/metrics.hip), no framework ops."""
        net = self._need()
        xx, yy = self._prep(x, y)
        n = xx.shape[0]
        loss = self.compile["loss"]
        if net.is_gpu and loss in ops.METRIC_KINDS:
            z = net._forward_eval(xx.to(net.dtype) if not isinstance(xx, ops.GatherRef) else xx)
            if not hasattr(self, "_metric_buf") or self._metric_buf.device != z.device:
                self._metric_buf = torch.zeros(2, dtype=torch.float32, device=z.device)
            st = ops.classifier_metrics(z, yy, loss, net.final_act, self._metric_buf).tolist()
            out = [st[0] / max(n, 1)]
            if "accuracy" in self.compile["metrics"] or "acc" in self.compile["metrics"]:
                out.append(st[1] / max(n, 1))
            return out
        probs = net.predict(xx)
        labels = torch.nn.functional.one_hot(yy.long(), net.num_classes).float()
        out = [float(self.loss_fn(labels, probs).mean())]
        if "accuracy" in self.compile["metrics"] or "acc" in self.compile["metrics"]:
            out.append(float(accuracy(yy, probs).mean()))
        return out

    def get_vars(self) -> list[torch.Tensor]:
        return self._need().store.get_vars()

    def set_vars(self, vals) -> None:
        self._need().store.set_vars(vals)

    def get_flat(self) -> torch.Tensor:
        return self._need().store.master

    def set_flat(self, flat: torch.Tensor) -> None:
        self._need().store.set_flat(flat.to(self.net.store.master.device))

    @property
    def num_params(self) -> int:
        return self._need().store.total

    @property
    def input_shape(self) -> list:
        return list(self._need().input_shape)

    @property
    def output_shape(self) -> list:
        return [self._need().num_classes]


class DynamicModel(DistriModel):
    """Raw variables + ``predict(x)`` + ``loss(labels, preds) -> per-example`` (reference DistributedDynamicModel)."""

    def __init__(self, vars: Sequence[torch.Tensor], predict: Callable, loss: Callable, input_shape, output_shape,
                 learning_rate: float = 0.001):
        self.vars = [v.detach().clone().requires_grad_(True) for v in vars]
        self._predict = predict
        self._loss = loss
        self._in = list(input_shape)
        self._out = list(output_shape)
        self.learning_rate = learning_rate

    def fit(self, x, y):
        loss = self._loss(y, self._predict(x)).mean()
        return list(torch.autograd.grad(loss, self.vars))

    def update(self, grads):
        with torch.no_grad():
            for v, g in zip(self.vars, grads):
                v.sub_(self.learning_rate * torch.as_tensor(g, device=v.device))

    def predict(self, x):
        with torch.no_grad():
            return self._predict(x)

    def evaluate(self, x, y):
        with torch.no_grad():
            return self._loss(y, self._predict(x)).reshape(-1).tolist()

    def get_vars(self):
        return [v.detach() for v in self.vars]

    def set_vars(self, vals):
        with torch.no_grad():
            for v, n in zip(self.vars, vals):
                v.copy_(torch.as_tensor(n).reshape(v.shape))

    @property
    def input_shape(self):
        return self._in

    @property
    def output_shape(self):
        return self._out


# ------------------------------------------------------------------------------------------ server models
class ServerModelMixin:
    is_distri_server_model = True
    version: str = "0"

    def _bump_version(self) -> str:
        last = int(self.version) if str(self.version).isdigit() else 0
        self.version = str(max(int(time.time() * 1000), last + 1))
        return self.version


class InMemoryServerModel(ServerModelMixin, EngineModel):
    """setup = fetch_initial + save; save = new version (no disk I/O)."""

    def setup(self):
        self.fetch_initial()
        self.save()

    def save(self):
        return self._bump_version()


class CheckpointedServerModel(ServerModelMixin, EngineModel):
    """Versioned tf.js LayersModel checkpoints: ``<save_dir>/<version>/model.json`` + ``current`` link;
    ``setup`` resumes from the last version when one exists."""

    def __init__(self, save_dir: str, model: ModelSource, compile_config: Optional[dict] = None, device=None,
                 keep_last: Optional[int] = None, save_every: int = 1):
        super().__init__(model, compile_config, device)
        self.store_dir = VersionedStore(save_dir, keep_last)
        self.save_every = max(1, int(save_every))
        self._saves = 0

    def list(self):
        return self.store_dir.list()

    def last(self):
        return self.store_dir.last()

    def setup(self):
        self.store_dir.setup()
        last = self.last()
        self.fetch_initial()
        if last is not None:
            self.load(last)
        else:
            self.save()

    def save(self):
        self.version = self.store_dir.new_version()
        self._saves += 1
        if self._saves == 1 or self._saves % self.save_every == 0:
            save_layers_model(self.net, self.store_dir.path(self.version))
            self.store_dir.mark_current(self.version)
            self.store_dir.prune()
        return self.version

    def load(self, version: str):
        load_layers_model_weights(self._need(), os.path.join(self.store_dir.path(version), "model.json"))
        self.version = version
        self.store_dir.mark_current(version)


class DynamicServerModel(ServerModelMixin, DynamicModel):
    """Flat-variable checkpoints ``<save_dir>/<version>/{meta.json,data.bin}``."""

    def __init__(self, save_dir: str, *args, **kw):
        super().__init__(*args, **kw)
        self.store_dir = VersionedStore(save_dir)

    def setup(self):
        self.store_dir.setup()
        last = self.store_dir.last()
        if last is not None:
            self.load(last)
        else:
            self.save()

    def save(self):
        self.version = self.store_dir.new_version()
        save_flat(self.store_dir.path(self.version), self.get_vars())
        self.store_dir.mark_current(self.version)
        return self.version

    def load(self, version: str):
        self.set_vars(load_flat(self.store_dir.path(version)))  # the reference forgot to assign these
        self.version = version


class ClientModel(EngineModel):
    is_distri_client_model = True

    def setup(self):
        self.fetch_initial()


def is_server_model(m) -> bool:
    return bool(getattr(m, "is_distri_server_model", False))


def is_client_model(m) -> bool:
    return bool(getattr(m, "is_distri_client_model", False))


# reference names
DistributedModel = DistriModel
DistributedTfModel = EngineModel
DistributedDynamicModel = DynamicModel
DistributedServerInMemoryModel = InMemoryServerModel
DistributedServerTfModel = CheckpointedServerModel
DistributedServerDynamicModel = DynamicServerModel
DistributedClientTfModel = ClientModel
