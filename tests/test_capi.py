"""CPU: the C-ABI library builds, loads and exports every symbol include/pgmg.h declares.

No compute calls here (no GPU in the build container); the GPU parity tests live in
test_gpu_parity.py and call the same symbols.
"""
import ctypes as C
import re

import pytest

from conftest import ROOT

HEADER = ROOT / "include" / "pgmg.h"


def declared_symbols():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pgmg_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("pgmg_create", "pgmg_vcycle", "pgmg_jacobi", "pgmg_residual", "pgmg_restrict",
                 "pgmg_prolong", "pgmg_get_solution", "pgmg_set_problem"):
        assert must in syms


def test_library_exports_every_declared_symbol(pgmg):
    lib = pgmg.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_signatures_cover_header(pgmg):
    from importlib import import_module
    capi = import_module("pgmg_amd._capi")
    names = {n for n, _, _ in capi.SIGNATURES}
    assert set(declared_symbols()) <= names


def test_config_defaults_match_reference(pgmg):
    cfg = pgmg.default_config(513)
    assert (cfg.v1, cfg.v2, cfg.coarse_iter, cfg.n_coarse, cfg.alpha) == (1, 1, 10, 5, 3)
    assert cfg.eps == 1e-7 and (cfg.a, cfg.p, cfg.q) == (1.0, 1.0, 1.0)
    assert cfg.world == 1 and cfg.rank == 0


def test_config_struct_layout(pgmg, tmp_path):
    """The ctypes mirror agrees with the C struct: size and every field offset."""
    from importlib import import_module
    import subprocess
    capi = import_module("pgmg_amd._capi")
    fields = [f for f, _ in capi.PgmgConfig._fields_]
    src = tmp_path / "layout.c"
    body = "".join(f'printf("%zu ", offsetof(pgmg_config, {f}));' for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "pgmg.h"\n'
                   f'int main(void){{printf("%zu ", sizeof(pgmg_config));{body}return 0;}}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(capi.PgmgConfig)] + [getattr(capi.PgmgConfig, f).offset for f in fields]
    assert got == want


def test_create_fails_loudly_without_gpu(pgmg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pgmg.PgmgError):
        pgmg.Solver(33)


def test_bad_grid_size_rejected(pgmg):
    with pytest.raises(pgmg.PgmgError):
        pgmg.Solver(100)


def test_flag_constants_match_header(pgmg):
    """Every PGMG_FLAG_* the Python plumbing names has the header's value."""
    from importlib import import_module
    capi = import_module("pgmg_amd._capi")
    txt = HEADER.read_text()
    vals = {m.group(1): int(m.group(2)) for m in
            re.finditer(r"#define (PGMG_FLAG_[A-Z0-9_]+) (\d+)u", txt)}
    assert vals["PGMG_FLAG_NO_SPEC_FIRE"] == 32768
    for name, v in vals.items():
        if hasattr(capi, name):
            assert getattr(capi, name) == v, name


@pytest.mark.parametrize("bit", [8192, 16384])
def test_retired_flag_bits_rejected(pgmg, bit):
    """A flag bit that meant something else in an older header (8192: PGMG_FLAG_L1POST, then
    r03's PGMG_FLAG_NO_SPEC_FIRE; 16384) fails pgmg_create with PGMG_ERR_ARG before any device
    call, instead of silently selecting another option."""
    lib = pgmg.load()
    cfg = pgmg.default_config(129)
    cfg.flags = bit
    h = C.c_void_p()
    assert lib.pgmg_create(C.byref(h), C.byref(cfg)) == -1   # PGMG_ERR_ARG
    assert not h.value


def test_library_built_from_this_tree(pgmg):
    """libpgmg.so carries the hash of the sources it was built from (Makefile "srchash"); it
    must equal this tree's, so the library the GPU box loads is the one these sources make."""
    import _pkgload
    assert pgmg.load().pgmg_source_hash().decode() == _pkgload.source_hash()

