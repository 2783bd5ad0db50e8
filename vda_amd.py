"""Import shim: exposes the package directory ``video-depth-anything_amd/`` as ``vda_amd``.

The directory name carries a hyphen (not a valid Python identifier), so ``import vda_amd`` loads
it explicitly as a package; submodules (``vda_amd.model``, ``vda_amd.ops`` ...) resolve normally.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "video-depth-anything_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
