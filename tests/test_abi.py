"""libnarde.so: loads, exports every symbol include/narde.h declares, and the
Python binding declares exactly those.  No compute calls (CPU-safe)."""
import ctypes
import os
import re

import pytest

from gym_narde import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "narde.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(narde_\w+)\s*\(", src)))


def test_library_is_built():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"


def test_exports_every_header_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/narde.h but not exported"


def test_binding_matches_header():
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_version_and_error_string():
    lib = _lib.load()
    assert lib.narde_version() == 1
    assert isinstance(lib.narde_last_error(), bytes)


def test_gpu_kernels_are_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_create_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.NardeLibraryError):
        _lib.Handle(0, 16)
