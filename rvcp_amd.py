"""Import shim: loads the package directory ``rvcp-real-time-path-tracer_amd/`` (whose name
is not a valid Python identifier) as the module ``rvcp_amd``."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rvcp-real-time-path-tracer_amd")

if "rvcp_amd._pkg" not in sys.modules:
    _spec = importlib.util.spec_from_file_location(
        "rvcp_amd._pkg", os.path.join(_PKG_DIR, "__init__.py"),
        submodule_search_locations=[_PKG_DIR])
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules["rvcp_amd._pkg"] = _mod
    _spec.loader.exec_module(_mod)

_pkg = sys.modules["rvcp_amd._pkg"]
globals().update({k: getattr(_pkg, k) for k in _pkg.__all__})
PKG_DIR = _PKG_DIR
__all__ = list(_pkg.__all__) + ["PKG_DIR"]
