"""Fully fledged depth models with the reference's API (mirrors pldepth/models/pl_hourglass.py).

``FullyFledgedModel`` keeps the surface the reference's drivers use on its keras.Model
(pldepth/PLDepth.py:115-181, run_scripts/*, hyperopt/*): ``compile(loss, optimizer)``,
``fit(x, epochs, steps_per_epoch, callbacks, validation_data, verbose)``, ``train_on_batch``,
``evaluate``, ``predict``, ``__call__``, ``get_weights``/``set_weights``,
``save_weights``/``load_weights`` and the ``asc_depth_order`` property. Underneath, every step is
the HIP engine (EffNetFF) driven by a graph-captured ReplicaTrainer; inputs are NHWC float32
arrays (numpy or device tensors), outputs device tensors [B,H,W,1].

``EffNetFullyFledged.get_model_and_normalization(input_shape, ranking_size, loss_type)`` returns
``(model, preprocess_fn)`` like pl_hourglass.py:45-100; EfficientNet's preprocess_input is the
identity (its Rescaling/Normalization live inside the model).
"""
import abc
import logging
import math

import numpy as np
import torch

from ..losses.losses_meta import DepthLossType

log = logging.getLogger(__name__)


def preprocess_input_effnet(x, data_format=None):
    """keras.applications.efficientnet.preprocess_input: a pass-through."""
    return x


class FullyFledgedModel(object):
    def __init__(self, engine, asc_depth_order=False, batch_size=None):
        self.engine = engine
        self.asc_depth_order = asc_depth_order
        self.batch_size = batch_size or engine.B
        self.loss = None
        self.optimizer = None
        self.trainer = None
        self.stop_training = False
        self.history = {}

    # ------------------------------------------------------------------ properties
    @property
    def asc_depth_order(self):
        """True when closer points have LOWER depth values (NYUDv2, Ibims, ...); HR-WSI is
        descending (pl_hourglass.py:22-35)."""
        return self._asc_depth_order

    @asc_depth_order.setter
    def asc_depth_order(self, value):
        self._asc_depth_order = value

    @staticmethod
    @abc.abstractmethod
    def get_model_and_normalization(input_shape, ranking_size, loss_type=DepthLossType.NLL):
        pass

    # ------------------------------------------------------------------ compile / train
    def compile(self, loss=None, optimizer=None, **kwargs):
        from ..optimizers import Adam
        from ..trainer import ReplicaTrainer
        self.loss = loss
        self.optimizer = optimizer if optimizer is not None else Adam(amsgrad=True)
        eng = self.engine
        self.trainer = ReplicaTrainer((eng.H, eng.W, 3), eng.B, loss.ranking_size, 1,
                                      engine=eng, gpu_sampler=False,
                                      beta_1=self.optimizer.beta_1, beta_2=self.optimizer.beta_2,
                                      epsilon=self.optimizer.epsilon)
        self._captured = False
        pending = getattr(self, "_pending_optimizer_state", None)
        if pending:  # a load_model()ed file: restore its Adam slots now that they exist
            from ..util import keras_h5
            keras_h5.load_optimizer_state(self, pending)
            self._pending_optimizer_state = None

    def train_on_batch(self, x, y, return_loss=True):
        """One optimizer step on (x [B,H,W,3], y [B,R,L,2]); returns the batch loss (float)."""
        if self.trainer is None:
            raise RuntimeError("compile() the model first")
        tr = self.trainer
        tr.set_batch(x, None, None)
        tr.set_rankings(y)
        if not self._captured:
            tr.step_eager(self.optimizer.lr)
            tr.capture()
            self._captured = True
        else:
            tr.step(self.optimizer.lr)
        self.optimizer.iterations += 1
        return tr.loss_value() if return_loss else None

    def fit(self, x=None, y=None, epochs=1, steps_per_epoch=None, callbacks=None,
            validation_data=None, verbose=1, initial_epoch=0, **kwargs):
        """Keras-style loop. ``x``: an iterable of (x_batch, y_batch) pairs (a provider dataset,
        repeated as needed), or an array with ``y`` given."""
        callbacks = list(callbacks or [])
        for cb in callbacks:
            if hasattr(cb, "set_model"):
                cb.set_model(self)
            else:
                cb.model = self
        if x is not None and y is not None:
            xs, ys = np.asarray(x), np.asarray(y)
            B = self.batch_size
            n = len(xs) // B
            data = [(xs[i * B:(i + 1) * B], ys[i * B:(i + 1) * B]) for i in range(n)]
            steps_per_epoch = steps_per_epoch or n
        else:
            data = x
        it = iter(data)

        def next_batch():
            nonlocal it
            try:
                return next(it)
            except StopIteration:
                it = iter(data)
                return next(it)

        self._cb("on_train_begin", callbacks)
        for epoch in range(initial_epoch, epochs):
            self._cb("on_epoch_begin", callbacks, epoch)
            losses = []
            for step in range(steps_per_epoch):
                self._cb("on_batch_begin", callbacks, step)
                xb, yb = next_batch()
                loss = self.train_on_batch(xb, yb)
                losses.append(loss)
                logs = {"loss": loss}
                self._cb("on_batch_end", callbacks, step, logs)
                if not math.isfinite(loss):
                    log.warning("Batch %d: invalid loss, terminating training", step)
                    self.stop_training = True
                if self.stop_training:
                    break
            logs = {"loss": float(np.mean(losses)) if losses else float("nan")}
            if validation_data is not None:
                logs["val_loss"] = self.evaluate(validation_data, verbose=0)
            for k, v in logs.items():
                self.history.setdefault(k, []).append(v)
            if verbose:
                print(f"Epoch {epoch + 1}/{epochs} - " +
                      " - ".join(f"{k}: {v:.4f}" for k, v in logs.items()), flush=True)
            self._cb("on_epoch_end", callbacks, epoch, logs)
            if self.stop_training:
                break
        self._cb("on_train_end", callbacks)
        return self

    @staticmethod
    def _cb(name, callbacks, *args):
        for cb in callbacks:
            fn = getattr(cb, name, None)
            if fn is not None:
                fn(*args)

    # ------------------------------------------------------------------ inference
    def __call__(self, x, training=False):
        eng = self.engine
        xb = torch.as_tensor(x, dtype=torch.float32)
        if xb.shape[0] != eng.B:
            raise ValueError(f"batch {xb.shape[0]} != compiled batch {eng.B}; use predict()")
        stream = self.trainer.stream if self.trainer is not None else torch.cuda.current_stream()
        with torch.cuda.stream(stream):
            eng.act["input"].copy_(xb.reshape(eng.act["input"].shape))
            out = eng.forward(training=training)
            res = out.clone()
        torch.cuda.current_stream().wait_stream(stream)
        return res

    def predict(self, x, batch_size=None, verbose=0):
        """Inference-mode forward (BN moving statistics) over any number of images."""
        x = np.asarray(x, np.float32) if not isinstance(x, torch.Tensor) else x
        n = x.shape[0]
        B = self.engine.B
        outs = []
        for i in range(0, n, B):
            xb = x[i:i + B]
            k = xb.shape[0]
            if k < B:  # pad the tail batch
                pad = (np.zeros((B - k,) + tuple(xb.shape[1:]), np.float32)
                       if not isinstance(xb, torch.Tensor) else
                       torch.zeros((B - k,) + tuple(xb.shape[1:]), device=xb.device))
                xb = np.concatenate([xb, pad]) if not isinstance(xb, torch.Tensor) \
                    else torch.cat([xb, pad])
            outs.append(self(xb, training=False)[:k].cpu().numpy())
        return np.concatenate(outs) if outs else np.zeros((0, self.engine.H, self.engine.W, 1))

    def evaluate(self, data, verbose=0):
        """Mean loss over (x, y) batches with BN in inference mode (Keras validation)."""
        losses = []
        for xb, yb in data:
            pred = self(xb, training=False)
            losses.append(float(self.loss(yb, pred).item()))
        return float(np.mean(losses)) if losses else float("nan")

    # ------------------------------------------------------------------ weights
    def get_weights(self):
        return self.engine.get_weights()

    def set_weights(self, weights):
        self.engine.set_weights(weights)

    def save_weights(self, path):
        """``.h5`` / ``.hdf5`` / ``.keras``: the Keras HDF5 weights format (util/keras_h5.py;
        what the reference's load_weights reads, PLDepth.py:136-137). Any other path: an .npz of
        Keras-named float32 arrays (HWIO kernels) plus the Adam slots, for exact resume (the
        reference writes a TF checkpoint there, a format this build does not implement)."""
        if path.endswith((".h5", ".hdf5", ".keras")):
            from ..util import keras_h5
            keras_h5.save_weights(self.engine, path)
            return
        w = self.get_weights()
        if self.trainer is not None:
            m, v, vh = self.engine.adam_state()
            for store, name in ((m, "m"), (v, "v"), (vh, "vhat")):
                w[f"__adam__/{name}"] = store.detach().cpu().numpy()
            w["__adam__/step"] = self.trainer.step_dev.cpu().numpy()
        np.savez(path if path.endswith(".npz") else path + ".npz", **w)

    def load_weights(self, path):
        """Keras HDF5 (weights or whole-model file; detected by signature) or this build's .npz."""
        from ..util import hdf5
        if hdf5.is_hdf5(path):
            from ..util import keras_h5
            return keras_h5.load_weights(self.engine, path)
        path = path if path.endswith(".npz") else path + ".npz"
        with np.load(path, allow_pickle=False) as z:
            w = {k: z[k] for k in z.files}
        self.set_weights({k: v for k, v in w.items() if not k.startswith("__adam__")})
        if self.trainer is not None and "__adam__/m" in w:
            m, v, vh = self.engine.adam_state()
            for store, name in ((m, "m"), (v, "v"), (vh, "vhat")):
                store.copy_(torch.from_numpy(w[f"__adam__/{name}"]))
            self.trainer.step_dev.copy_(torch.from_numpy(w["__adam__/step"]))

    def save(self, filepath, overwrite=True, include_optimizer=True, **kwargs):
        """keras.Model.save('... .h5') (PLDepth.py:181): model config, weights and the Adam
        slots in Keras' HDF5 model layout; ``load_model`` (models/__init__.py) reads it back."""
        import os
        from ..util import keras_h5
        if not overwrite and os.path.exists(filepath):
            raise FileExistsError(filepath)
        opt = self.optimizer
        if not include_optimizer:
            self.optimizer = None
        try:
            keras_h5.save_model(self, filepath)
        finally:
            self.optimizer = opt

    def count_params(self):
        return self.engine.count_trainable()


class EffNetFullyFledged(FullyFledgedModel):
    @staticmethod
    def get_model_and_normalization(input_shape, ranking_size, loss_type=DepthLossType.NLL,
                                    batch_size=4, seed=0):
        """pl_hourglass.py:45-100. ``batch_size`` fixes the per-GPU batch the device buffers are
        laid out for (Keras builds for a dynamic batch; the reference always trains with a
        fixed one, PLDepth.py:31,129)."""
        from .effnet_ff import EffNetFF
        if loss_type != DepthLossType.NLL:
            raise ValueError(f"unsupported loss type {loss_type}")
        eng = EffNetFF(tuple(input_shape), batch_size, seed=seed)
        return EffNetFullyFledged(eng, batch_size=batch_size), preprocess_input_effnet
