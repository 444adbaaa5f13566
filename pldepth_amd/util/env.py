"""Process setup (mirrors pldepth/util/env.py: get_config, init_tensorflow, init_env).

Same names and call shapes as the reference; what they set up is this build's host side:
``init_tensorflow(seed, num_threads=8)`` seeds torch / NumPy and fixes the host thread count
(the reference: tf.random.set_seed + 8 intra/inter-op threads, env.py:39-58); the ini config is
read from ``conf/run.ini`` (or $PLD_CONFIG) when present, with the [DATA] / [LOGGING] keys the
drivers read defaulted. Tracking services (wandb, mlflow: env.py:28-36,61-65) are out of scope:
``use_mlflow=True`` raises, and no credentials are set anywhere.
"""
import configparser
import logging
import os

import numpy as np

ROOT_DIR = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
CONFIG_FILE = "conf/run.ini"
CONFIG_FILE_ENCODING = "utf-8-sig"
_DEFAULTS = {
    "LOGGING": {"LOG_LEVEL": "INFO", "TENSORBOARD_LOG_DIR": os.path.join(ROOT_DIR, "logs")},
    "DATA": {"CACHE_PATH_PREFIX": os.path.join(ROOT_DIR, "cache")},
}


def get_config(path=None, config_file_name=None):
    config = configparser.ConfigParser()
    config.optionxform = str  # keep the upper-case keys the drivers index with
    for sec, kv in _DEFAULTS.items():
        config[sec] = dict(kv)
    if path is None:
        path = os.environ.get("PLD_CONFIG") or os.path.join(ROOT_DIR,
                                                           config_file_name or CONFIG_FILE)
    if os.path.exists(path):
        config.read(path, encoding=CONFIG_FILE_ENCODING)
    return config


def init_tensorflow(seed, use_float16=False, num_threads=8):
    """env.py:39-58. fp16 (Keras floatx) is never enabled by the reference's callers; the HIP
    path computes in fp32 (bf16x3 MFMA for convs), so it is rejected rather than ignored."""
    if use_float16:
        raise ValueError("use_float16: the PLDepth HIP path computes in fp32")
    import torch
    torch.manual_seed(seed)
    np.random.seed(seed)
    torch.set_num_threads(num_threads)


def init_env(tracking_uri=None, experiment_name=None, autolog_freq=100, seed=0,
             use_float16=False, use_mlflow=False):
    """env.py:68-98 without the tracking services; returns the config."""
    if use_mlflow:
        raise NotImplementedError("mlflow tracking is not part of this build")
    config = get_config()
    level = config["LOGGING"]["LOG_LEVEL"]
    if level not in ("DEBUG", "INFO", "WARNING", "ERROR"):
        raise ValueError(
            "Unknown log level provided in the configuration file: {}".format(level))
    logging.basicConfig(level=getattr(logging, level))
    init_tensorflow(seed, use_float16=use_float16)
    return config
