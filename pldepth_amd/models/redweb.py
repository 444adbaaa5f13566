"""ff_redweb (ResNet-50 encoder + ReDWeb feature-fusion decoder; pldepth/models/redweb.py:402-434).

``ReDWebNetTFVersion.get_model_and_normalization(input_shape, ranking_size, loss_type)`` returns
``(model, preprocess_fn)`` like the reference: the model is a FullyFledgedModel over the HIP
engine ``RedWebFF`` (pldepth_amd/models/redweb_ff.py); ``preprocess_fn`` is Keras' caffe-mode
ResNet50 preprocessing (RGB->BGR, minus ImageNet means), which the reference's pipeline applies
to its [0,1] images (PLDepth.py:169-173) — callers apply it, the model does not.
"""
from ..losses.losses_meta import DepthLossType
from .pl_hourglass import FullyFledgedModel
from .redweb_ff import CAFFE_MEAN_BGR, preprocess_input  # noqa: F401

preprocess_input_resnet = preprocess_input


class ReDWebNetTFVersion(FullyFledgedModel):
    @staticmethod
    def get_model_and_normalization(input_shape, ranking_size, loss_type=DepthLossType.NLL,
                                    batch_size=4, seed=0):
        from .redweb_ff import RedWebFF
        if loss_type != DepthLossType.NLL:
            raise ValueError(f"unsupported loss type {loss_type}")
        eng = RedWebFF(tuple(input_shape), batch_size, seed=seed)
        return ReDWebNetTFVersion(eng, batch_size=batch_size), preprocess_input
