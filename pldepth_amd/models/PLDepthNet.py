"""Model factory (mirrors pldepth/models/PLDepthNet.py:6-21)."""
from .models_meta import ModelType
from .pl_hourglass import EffNetFullyFledged
from .redweb import ReDWebNetTFVersion


def get_pl_depth_net(model_params, input_shape):
    model_type = model_params.get_parameter("model_type")
    kw = {}
    if model_params.get_parameter("batch_size") is not None:
        kw["batch_size"] = model_params.get_parameter("batch_size")
    if model_params.get_parameter("seed") is not None:
        kw["seed"] = model_params.get_parameter("seed")
    if model_type == ModelType.FULLY_FLEDGED_EFFNET:
        return EffNetFullyFledged.get_model_and_normalization(
            input_shape, model_params.get_parameter("ranking_size"),
            model_params.get_parameter("loss_type"), **kw)
    elif model_type == ModelType.FULLY_FLEDGED_REDWEB:
        return ReDWebNetTFVersion.get_model_and_normalization(
            input_shape, model_params.get_parameter("ranking_size"),
            model_params.get_parameter("loss_type"), **kw)
    raise ValueError("Unknown model type: {}".format(model_params.get_parameter("model_type")))
