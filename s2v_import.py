"""Import helper: the package directory is named ``speech-to-video-mpp_amd`` (hyphens are not
importable), so it is registered in ``sys.modules`` under the import name ``s2v_amd``.

    import s2v_import; s2v = s2v_import.load()      # then: import s2v_amd.models
"""
import importlib.util
import os
import sys

PKG_NAME = "s2v_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "speech-to-video-mpp_amd")


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod


load()
