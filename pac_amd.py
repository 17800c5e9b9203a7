"""Import shim: ``import pac_amd`` loads the package directory
``perceptual-audio-codec_amd/`` (whose name is not a Python identifier) and
registers it under the module name ``pac_amd``.  Nothing else lives here."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "perceptual-audio-codec_amd")


def _load():
    spec = importlib.util.spec_from_file_location(
        __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[__name__] = mod
    spec.loader.exec_module(mod)
    return mod


_load()
