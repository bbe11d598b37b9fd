"""Load the product package from its (non-identifier) directory name as ``pgmg_amd``."""
import importlib.util
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent
PKG_DIR = ROOT / "parallel-geometric-multigrid-for-poisson-problem_amd"
NAME = "pgmg_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
