"""Import shim: registers the package directory ``audio-visual-tubes_amd/`` (not a valid
Python identifier) as the importable package ``avt_amd`` and re-exports its public API.

    import avtubes                       # once
    from avt_amd.model import AVENet     # drop-in for reference model.py:87
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "audio-visual-tubes_amd")


def _register():
    if "avt_amd" in sys.modules:
        return sys.modules["avt_amd"]
    spec = importlib.util.spec_from_file_location(
        "avt_amd", os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["avt_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


avt_amd = _register()
