"""Learning-rate schedules and callbacks (mirrors pldepth/util/training_utils.py).

``SGDRScheduler`` (training_utils.py:20-97): per-batch cosine schedule set at on_batch_end, with
restarts at epoch ends; the reference constructs it with min_lr = initial_lr / lr_multi (> max_lr
at the default lr_multi = 0.25, PLDepth.py:121-126) so the LR rises over training — reproduced as
is. ``LearningRateScheduleProvider`` (:102-135) and ``LearningRateLoggingCallback`` (:7-17, which
logs to wandb in the reference; here to a list / the Python logger).
"""
import logging

import numpy as np


class Callback(object):
    def __init__(self):
        self.model = None

    def set_model(self, model):
        self.model = model


class LearningRateLoggingCallback(Callback):
    def __init__(self):
        super().__init__()
        self.lrs = []

    def on_batch_end(self, batch, logs=None):
        self.lrs.append(self.model.optimizer.lr)

    def on_epoch_end(self, epoch, logs=None):
        logging.info("epoch %d lr %g", epoch, self.model.optimizer.lr)


class SGDRScheduler(Callback):
    def __init__(self, min_lr, max_lr, steps_per_epoch, lr_decay=1, cycle_length=10,
                 mult_factor=2):
        super().__init__()
        self.min_lr = min_lr
        self.max_lr = max_lr
        self.lr_decay = lr_decay
        self.batch_since_restart = 0
        self.next_restart = cycle_length
        self.steps_per_epoch = steps_per_epoch
        self.cycle_length = cycle_length
        self.mult_factor = mult_factor
        self.history = {}

    def clr(self):
        fraction_to_restart = self.batch_since_restart / (self.steps_per_epoch * self.cycle_length)
        return self.min_lr + 0.5 * (self.max_lr - self.min_lr) * (
            1 + np.cos(fraction_to_restart * np.pi))

    def on_train_begin(self, logs=None):
        self.model.optimizer.lr = self.max_lr

    def on_batch_end(self, batch, logs=None):
        logs = logs or {}
        self.history.setdefault("lr", []).append(self.model.optimizer.lr)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(v)
        self.batch_since_restart += 1
        self.model.optimizer.lr = float(self.clr())

    def on_epoch_end(self, epoch, logs=None):
        if epoch + 1 == self.next_restart:
            self.batch_since_restart = 0
            self.cycle_length = np.ceil(self.cycle_length * self.mult_factor)
            self.next_restart += self.cycle_length
            self.max_lr *= self.lr_decay
            self.best_weights = self.model.get_weights()


class LearningRateScheduleProvider(object):
    def __init__(self, steps=None, init_lr=1e-3, multiplier=0.1, warmup=0):
        self.steps = [80, 120, 160, 180] if steps is None else steps
        self.init_lr = init_lr
        self.multiplier = multiplier
        self.warmup = warmup

    def get_lr_schedule(self, epoch):
        if self.warmup > 0 and epoch < self.warmup:
            return (epoch + 1) * self.init_lr / self.warmup
        lr = self.init_lr
        for loc_steps in self.steps:
            if epoch >= loc_steps:
                lr *= self.multiplier
            else:
                break
        return lr


class TerminateOnNaN(Callback):
    """keras.callbacks.TerminateOnNaN (PLDepth.py:163)."""

    def on_batch_end(self, batch, logs=None):
        loss = (logs or {}).get("loss")
        if loss is not None and not np.isfinite(loss):
            logging.warning("Batch %d: Invalid loss, terminating training", batch)
            self.model.stop_training = True


class ModelCheckpoint(Callback):
    """keras.callbacks.ModelCheckpoint as tracking_utils.py:21-30 builds it (monitor='val_loss',
    save_best_only=True): at each epoch end, save the model (``model.save``: Keras HDF5 model
    file, util/keras_h5.py) or only its weights, when ``monitor`` improved (mode 'auto': 'min'
    unless the name contains 'acc'). ``filepath`` may hold ``{epoch}`` / log-key format fields."""

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False,
                 save_weights_only=False, mode="auto", save_freq="epoch", **kwargs):
        super().__init__()
        if save_freq != "epoch":
            raise NotImplementedError("ModelCheckpoint: save_freq='epoch' only")
        self.filepath, self.monitor, self.verbose = filepath, monitor, verbose
        self.save_best_only, self.save_weights_only = save_best_only, save_weights_only
        if mode == "auto":
            mode = "max" if "acc" in monitor else "min"
        self.better = np.less if mode == "min" else np.greater
        self.best = np.inf if mode == "min" else -np.inf

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        path = self.filepath.format(epoch=epoch + 1, **logs)
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None:
                logging.warning("ModelCheckpoint: %s not available, skipping", self.monitor)
                return
            if not self.better(cur, self.best):
                if self.verbose:
                    logging.info("Epoch %d: %s did not improve from %.5f", epoch + 1,
                                 self.monitor, self.best)
                return
            if self.verbose:
                logging.info("Epoch %d: %s improved from %.5f to %.5f, saving model to %s",
                             epoch + 1, self.monitor, self.best, cur, path)
            self.best = cur
        if self.save_weights_only:
            self.model.save_weights(path)
        else:
            self.model.save(path)
