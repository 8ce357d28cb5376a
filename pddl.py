"""Import shim: exposes the package directory `parallel-and-distributed-deep-learning_amd/`
(whose name is not a valid Python identifier) as the importable package `pddl`.

    import pddl
    from pddl.models.resnet50 import build_layout
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "parallel-and-distributed-deep-learning_amd")
_spec = _ilu.spec_from_file_location("pddl", _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["pddl"] = _mod
_spec.loader.exec_module(_mod)
