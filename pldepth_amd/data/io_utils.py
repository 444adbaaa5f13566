"""Dataset-name dispatch (mirrors pldepth/data/io_utils.py:4-25): the names the drivers accept.

Only HR-WSI has a data-access object in this build (pldepth_amd.data.dao.hr_wsi); the other
datasets are evaluation-only in the reference (out of scope) and resolve to their
enum value so that driver code parsing them runs unchanged.
"""
from ..models.models_meta import StringEnum


class Dataset(StringEnum):
    HR_WSI = "HR-WSI"
    IBIMS = "IBIMS"
    SINTEL = "SINTEL"
    DIODE = "DIODE"
    TUM = "TUM"


_ALIASES = {"hr_wsi": Dataset.HR_WSI}


def get_dataset_type_by_name(dataset_name):
    """io_utils.py:12-25: case-insensitive match on the enum values (plus 'hr_wsi')."""
    key = dataset_name.lower()
    for d in Dataset:
        if key == d.value.lower():
            return d
    if key in _ALIASES:
        return _ALIASES[key]
    raise ValueError("Unknown dataset name: {}".format(dataset_name))
