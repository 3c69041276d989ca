"""Import helper: the package directory is named ``euclidiannormalizingflows.jl_amd`` (the dot makes
it unimportable by a plain ``import``), so it is registered here under the module name
``euclidiannormalizingflows_jl_amd``.

    from enf_pkg import load
    enf = load()
    Y, ladj = enf.with_logabsdet_jacobian(enf.JohnsonTrafo(...) @ enf.HouseholderTrafo(...), X)
"""
from __future__ import annotations

import importlib.util
import os
import sys

NAME = "euclidiannormalizingflows_jl_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "euclidiannormalizingflows.jl_amd")


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
