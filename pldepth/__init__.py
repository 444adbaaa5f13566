"""The reference's import paths, served by this implementation (SURVEY §8(b) boundary).

Every reference caller imports ``pldepth.<subpackage>.<module>`` (pldepth/PLDepth.py:4-21,
pldepth/models/PLDepthNet.py:1-3, run_scripts/*, hyperopt/*). This package holds no code of its
own: a meta-path finder resolves ``pldepth.X[.Y...]`` to the module object ``pldepth_amd.X[.Y...]``
(the same object, registered under both names), so ``from pldepth.models.PLDepthNet import
get_pl_depth_net`` returns this build's factory and a reference driver runs unchanged on the HIP
path. Names with no counterpart here (wandb/mlflow tracking, hyper-opt, active-learning drivers:
out of scope) raise the usual ModuleNotFoundError.
"""
import importlib
import importlib.abc
import importlib.util
import sys

_TARGET = "pldepth_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, real):
        self.real = real

    def create_module(self, spec):
        return importlib.import_module(self.real)

    def exec_module(self, module):
        pass  # the real module is already executed


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(__name__ + "."):
            return None
        real = _TARGET + fullname[len(__name__):]
        try:
            real_spec = importlib.util.find_spec(real)
        except ModuleNotFoundError:
            return None
        if real_spec is None:
            return None
        spec = importlib.util.spec_from_loader(
            fullname, _AliasLoader(real),
            is_package=real_spec.submodule_search_locations is not None)
        return spec


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())
