"""Imports the `dlrm.jl_amd/` package under the module name `dlrm_jl_amd`.

The package directory is named after the reference (darchr/DLRM.jl), and a dot is not
legal in a Python import path, so it is loaded by file location once and registered in
sys.modules; afterwards `import dlrm_jl_amd` works anywhere in the process.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "dlrm.jl_amd")
NAME = "dlrm_jl_amd"


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[NAME]
        raise
    return mod
