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


def source_hash():
    """The hash the Makefile stamps into libpgmg.so (pgmg_source_hash), computed over this
    tree: sha256 of csrc/<SRCS> and csrc/*.h and include/pgmg.h concatenated in path order
    (the Makefile's $(sort ...) of the same path strings), first 16 hex digits."""
    import hashlib
    import re
    here = str(PKG_DIR) + "/"
    mk = (PKG_DIR / "Makefile").read_text()
    srcs = re.search(r"^SRCS = (.*)$", mk, re.M).group(1).split()
    paths = [here + "csrc/" + x for x in srcs]
    paths += [str(p) for p in sorted((PKG_DIR / "csrc").glob("*.h"))]
    paths.append(here + "../include/pgmg.h")
    h = hashlib.sha256()
    for p in sorted(set(paths)):
        h.update(pathlib.Path(p).read_bytes())
    return h.hexdigest()[:16]

