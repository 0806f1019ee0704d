"""libipo_hip.so loads on a machine without a GPU and exports every symbol
that include/ipo_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import ipo_amd
from conftest import REPO


def declared_functions():
    with open(os.path.join(REPO, "include", "ipo_hip.h")) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"typedef[^;]*;", "", text)          # function-pointer typedefs are not symbols
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", text)
    return sorted(set(n for n in names if n not in ("if", "while", "sizeof")))


def test_header_declares_reference_plugin_points():
    names = declared_functions()
    for n in ("solver", "ldltfac", "forwardbackward", "inv_clo"):
        assert n in names


def test_library_exports_all_declared_symbols():
    lib = ipo_amd.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(ipo_amd.EXPORTED) <= set(declared_functions())


def test_version_and_device_count_callable():
    assert ipo_amd.lib().ipo_hip_version().startswith(b"ipo-hip")
    assert ipo_amd.device_count() >= 0
