"""Import alias for the product package.

The package directory is ``pose-estimation-with-message-passing-networks_amd/`` (the name the
layout requires); a hyphenated directory is not importable by name, so ``import pemp_amd``
resolves here and replaces itself with that package.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                    "pose-estimation-with-message-passing-networks_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
