"""Import helper: the package directory is named ``marl-traffic-intersection_amd``
(not a valid Python identifier), so it is registered as
``marl_traffic_intersection_amd`` from its path."""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_NAME = "marl_traffic_intersection_amd"
PKG_DIR = os.path.join(ROOT, "marl-traffic-intersection_amd")


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(PKG_NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod
