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
    assert lib.narde_version() == 2
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


def test_argument_errors_are_einval_before_any_device_call():
    """Every entry point validates its arguments first: NULL handles and
    pointers, bad sizes and counts return NARDE_EINVAL (-1) with a message,
    without touching a GPU (this runs on the CPU-only container)."""
    lib = _lib.load()
    N = None
    cases = [
        ("narde_step", (N, N, N, N, N, N, N, N, N, 1, N)),
        ("narde_step_full", (N, N, N, N, N, N, N, N, N, 1, N)),
        ("narde_rollout", (N, 10, N, N, N, N, N, N, N)),
        ("narde_reset", (N, N, N, 0, N)),
        ("narde_legal_full", (N, N, N, N)),
        ("narde_legal_mask576_move2", (N, N, N, N, N)),
        ("narde_dqn_transition", (N, N, N, N, N, N, N, N, N, 1, N, N, N, N, N, N, N, 16, N)),
        ("narde_policy_masked_argmax576", (0, N, 576, N, 16, 0.1, 0, 0, 0, N, N)),
        ("narde_policy_masked_argmax576_dev", (0, N, 576, N, 16, N, 0, N, 0, N, 0, N, N, N)),
        ("narde_violates_block_rule", (0, N, 4, N, N)),
        ("narde_per_sample", (0, N, N, 100, 64, 0, N, N, 0.001, N, N, N, N, N)),
        ("narde_per_prefix", (0, N, 100, 0.6, N, N, N, 1, N)),
        ("narde_gather_batch", (0, N, 64, 198, N, 64, 128, N, N, N, N, N, N, N, N, N)),
        ("narde_rowmax_addend", (0, N, 576, N, 576, N, 64, N, N)),
        ("narde_get_totals", (N, N, N)),
        ("narde_dqn_heads_forward", (0, N, 256, N, 256, N, N, 832, N, N, 64, N, N, N)),
        ("narde_dqn_heads_backward", (0, N, N, N, 256, N, 256, N, 832, N, 64, N, N, N, N, N, N)),
        ("narde_relu_bias_grad", (0, N, N, 64, 256, N, N, N, N)),
        ("narde_dqn_loss", (0, N, N, N, N, N, N, N, 64, 0.99, N, N, N, N, N, N)),
        ("narde_prio_update", (0, N, N, 64, 0.01, N, N, N, 0.01, 0.995, N, 0, 1, N, N)),
        ("narde_adam_clip", (0, 0, N, N, N, N, N, N, 1e-3, 0.9, 0.999, 1e-8, 10.0, N, N)),
        ("narde_per_sample_gather", (0, N, N, 100, 64, 0, N, N, N, N, 198, N, 64, 128, N, N, N, N, N, N, N, N, N)),
        ("narde_target_max2", (0, N, 576, N, 576, N, 576, 64, N, N, N, N)),
        ("narde_dqn_loss_prio", (0, N, N, N, N, N, N, N, 64, 0.99, N, N, N, N, N, N, 0.01, N, N, N, 0.01, 0.995,
                                 N, 0, 1, N, N, N, 0.001, N)),
    ]
    for name, args in cases:
        rc = getattr(lib, name)(*args)
        assert rc == -1, f"{name} returned {rc}"
        assert lib.narde_last_error(), name
