"""Import shim: ``import sat_amd`` loads the package in ./show-attend-and-tell_amd/.

The package directory name contains dashes (it is fixed by the build contract),
so it cannot be imported by name; this module replaces itself in sys.modules
with that package.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "show-attend-and-tell_amd")
_spec = importlib.util.spec_from_file_location("sat_amd", os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["sat_amd"] = _mod
_spec.loader.exec_module(_mod)
