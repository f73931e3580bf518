"""Registers the package directory ``onc-rpc_amd/`` as the module
``onc_rpc_amd`` (the directory name is not a valid identifier)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "onc-rpc_amd")


def load():
    if "onc_rpc_amd" in sys.modules:
        return sys.modules["onc_rpc_amd"]
    spec = importlib.util.spec_from_file_location(
        "onc_rpc_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["onc_rpc_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
