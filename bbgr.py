"""Import shim: exposes the package directory
``beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/``
(not a valid Python identifier) under the import name ``bbgr``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(
    _os.path.dirname(_os.path.abspath(__file__)),
    "beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd")
_spec = _ilu.spec_from_file_location("bbgr", _os.path.join(_DIR, "__init__.py"),
                                     submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["bbgr"] = _mod
_spec.loader.exec_module(_mod)
