"""The C-ABI library loads on a CPU-only host and exports every symbol include/*.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.join(os.path.dirname(__file__), "..")


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(nhip_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_declares_entry_points():
    names = declared_symbols()
    for must in ("nhip_init", "nhip_destroy", "nhip_mtree_verify", "nhip_tip5_hash_pair", "nhip_tip5_hash_varlen"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import neptune_hip._lib as L
    lib = L.load()
    missing = [n for n in sorted(declared_symbols()) if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding types every declared symbol, and nothing else
    assert set(L.SIGNATURES) == declared_symbols()


def test_no_device_is_an_error_not_a_fallback():
    import neptune_hip as nh
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(nh.NhipError):
        nh.Context(0)
