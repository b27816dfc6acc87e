"""CPU checks of the reference-side binding (integration/deig_backend.py): it imports
nothing but ctypes, numpy and the standard library (a maintainer drops it next to the
reference's distributed.py), and every libdeig symbol it binds is declared in
include/deig.h and exported by the built library."""
import ast
import ctypes
import os

import pytest

from distributed_eigenspaces_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "integration", "deig_backend.py")


def _tree():
    return ast.parse(open(STUB).read())


def test_stub_imports_only_ctypes_numpy():
    mods = set()
    for node in ast.walk(_tree()):
        if isinstance(node, ast.Import):
            mods |= {a.name.split(".")[0] for a in node.names}
        elif isinstance(node, ast.ImportFrom):
            mods.add((node.module or "").split(".")[0])
    assert mods <= {"ctypes", "numpy", "os", "warnings", "__future__"}, mods


def test_stub_binds_declared_exported_symbols():
    src = open(STUB).read()
    bound = sorted({n for n in _lib.header_symbols() if f"_L.{n}" in src})
    assert {"deig_syrk_shift", "deig_topk_sym_ex", "deig_projavg_topk_f32"} <= set(bound)
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdeig.so not built")
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in bound:
        assert hasattr(L, name), name
