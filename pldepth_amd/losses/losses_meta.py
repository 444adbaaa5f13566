"""Loss identifiers (mirrors pldepth/losses/losses_meta.py:1-5)."""
from ..models.models_meta import StringEnum


class DepthLossType(StringEnum):
    NLL = "NLL"
