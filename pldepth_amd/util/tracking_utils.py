"""Checkpoint / logging callbacks (mirrors pldepth/util/tracking_utils.py).

``construct_model_checkpoint_callback`` is the reference's (tracking_utils.py:21-30): a
ModelCheckpoint on 'val_loss', save_best_only, writing ``pldepth_<model>_model.h5`` (Keras HDF5
model file) under ``<CACHE_PATH_PREFIX>/saved_models/<time>``. TensorBoard and mlflow are not
part of this build: ``construct_tensorboard_callback`` returns a callback that appends the same
per-epoch scalars to ``<log_dir>/scalars.jsonl``, and ``log_parameter_dict`` logs through the
Python logger.
"""
import json
import logging
import os
import time

from .training_utils import Callback, ModelCheckpoint


def get_time_str():
    """time_utils.py: current time in ms as a string."""
    return str(int(round(time.time() * 1000)))


def log_parameter_dict(param_dict):
    for key in param_dict:
        logging.info("param %s = %s", key, param_dict[key])


def get_model_checkpoint_path(config, use_mlflow=False):
    if use_mlflow:
        raise NotImplementedError("mlflow tracking is not part of this build")
    return os.path.join(config["DATA"]["CACHE_PATH_PREFIX"], "saved_models", get_time_str())


def construct_model_checkpoint_callback(config, model_type, verbosity):
    save_dir = get_model_checkpoint_path(config, use_mlflow=False)
    os.makedirs(save_dir, exist_ok=True)
    filepath = os.path.join(save_dir, "pldepth_%s_model.h5" % model_type)
    return ModelCheckpoint(filepath=filepath, monitor="val_loss", verbose=verbosity,
                           save_best_only=True)


class ScalarLogCallback(Callback):
    """Per-epoch scalars (loss, val_loss, lr) to ``<log_dir>/scalars.jsonl``."""

    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir

    def on_epoch_end(self, epoch, logs=None):
        os.makedirs(self.log_dir, exist_ok=True)
        rec = {"epoch": epoch, **{k: float(v) for k, v in (logs or {}).items()}}
        if self.model is not None and getattr(self.model, "optimizer", None) is not None:
            rec["lr"] = float(self.model.optimizer.lr)
        with open(os.path.join(self.log_dir, "scalars.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")


def construct_tensorboard_callback(config, dir_name):
    return ScalarLogCallback(os.path.join(config["LOGGING"]["TENSORBOARD_LOG_DIR"], dir_name))
