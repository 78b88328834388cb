"""The C-ABI library loads, its struct layouts match the ctypes mirrors, every declared symbol exists."""
import ctypes
import os
import re

import pytest

from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "nmgp_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|int64_t|void)\s+(nmgp_\w+)\s*\(", src)))


def test_library_loads_and_abi_sizes_match():
    lib = L.lib()          # raises on a struct-size mismatch
    assert lib.nmgp_version() >= 1


def test_every_header_symbol_is_exported_and_bound():
    lib = L.lib()
    declared = _declared_symbols()
    assert len(declared) > 30
    for name in declared:
        assert hasattr(lib, name), name
        assert name in L.exported_symbols(), f"{name} has no ctypes signature"
