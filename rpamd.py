"""Import helper for the package directory ``repair-pipelining_amd/`` (its
name is not a Python identifier).  ``rpamd.load()`` returns it registered as
the module ``repair_pipelining_amd``."""
import importlib.util
import sys
from pathlib import Path

NAME = "repair_pipelining_amd"
PKG_DIR = Path(__file__).resolve().parent / "repair-pipelining_amd"


def load(shape_knobs: bool = False):
    """The package; with ``shape_knobs`` the process opts in to libecx's launch-shape knobs
    (ECX_SHAPE_KNOBS=1, include/ecx_tune.h), read by the library at its first ecx_tune call."""
    if shape_knobs:
        import os
        os.environ["ECX_SHAPE_KNOBS"] = "1"
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
