"""ff_redweb (ResNet-50 encoder + ReDWeb feature-fusion decoder; pldepth/models/redweb.py:402-434).

The ResNet-50/ReDWeb HIP engine is not built yet (BASELINE cfg3): this
surface exists so callers get a clear error instead of an import failure. ``preprocess_input``
is Keras' caffe-mode ResNet50 preprocessing (RGB->BGR, minus ImageNet means), applied as the
reference does to [0,1] inputs.
"""
import numpy as np

from ..losses.losses_meta import DepthLossType
from .pl_hourglass import FullyFledgedModel

CAFFE_MEAN_BGR = np.array([103.939, 116.779, 123.68], np.float32)


def preprocess_input_resnet(x, data_format=None):
    x = np.asarray(x, np.float32)[..., ::-1]
    return x - CAFFE_MEAN_BGR


class ReDWebNetTFVersion(FullyFledgedModel):
    @staticmethod
    def get_model_and_normalization(input_shape, ranking_size, loss_type=DepthLossType.NLL,
                                    batch_size=4, seed=0):
        raise NotImplementedError(
            "ff_redweb (ResNet-50 + ReDWeb decoder) has no HIP engine yet; use ff_effnet")
