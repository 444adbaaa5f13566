"""Model identifiers and the parameter bag (mirrors pldepth/models/models_meta.py:8-70).

Same names and behaviour as the reference: ``StringEnum``, ``ModelType``,
``get_model_type_by_name`` ('ff_effnet' / 'ff_redweb', raising ValueError otherwise) and
``ModelParameters`` (set/get/duplicate/load_parameters_from_file). ``log_parameters`` writes to the
Python logger instead of mlflow (tracking services are out of scope).
"""
import copy
import json
import logging
from enum import Enum


class StringEnum(Enum):
    def __str__(self):
        return str(self.value)


class ModelType(StringEnum):
    FULLY_FLEDGED_REDWEB = "FFReDWeb"
    FULLY_FLEDGED_EFFNET = "FFEffNet"


def get_model_type_by_name(model_name):
    if model_name == "ff_redweb":
        return ModelType.FULLY_FLEDGED_REDWEB
    elif model_name == "ff_effnet":
        return ModelType.FULLY_FLEDGED_EFFNET
    else:
        raise ValueError("Unknown model name: {}".format(model_name))


class ModelParameters(object):
    def __init__(self):
        self.parameters = {}

    def set_parameter(self, name, value):
        self.parameters[name] = value

    def get_parameter(self, name, default=None):
        return self.parameters.get(name, default)

    def log_parameters(self):
        for k, v in self.parameters.items():
            logging.info("param %s = %s", k, v)

    def get_parameter_string(self):
        return "_".join(f"{k}_{v}" for k, v in self.parameters.items())

    def load_parameters_from_file(self, json_file_path, key, exclude_keys=None):
        with open(json_file_path) as f:
            ext = json.load(f)
        if key not in ext:
            raise ValueError("Could not find entry for key {} in external parameter file {}."
                             .format(key, json_file_path))
        for k, value in ext[key].items():
            if exclude_keys is not None and k in exclude_keys:
                continue
            if isinstance(value, str):
                value = value == "True" or value == "true"
            self.set_parameter(k, value)

    def duplicate(self):
        r = ModelParameters()
        r.parameters = copy.deepcopy(self.parameters)
        return r
