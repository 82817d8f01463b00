"""ctypes binding of libnarde.so (include/narde.h).

The product path has exactly one implementation: the HIP kernels in
libnarde.so.  There is no CPU fallback -- if the library or a GPU is missing,
every entry point raises NardeLibraryError.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NARDE_LIB", os.path.join(HERE, "libnarde.so"))

OK = 0
OFF = 24
MAX_MOVES = 64
TOTAL_ROWS = 64  # NARDE_TOTAL_ROWS


def wg_rows(num_envs):
    """NARDE_WG_ROWS: rows of narde_rollout_timed's per-workgroup totals."""
    return (int(num_envs) + 255) // 256
DICE_ALL36 = 0
DICE_NODOUBLES = 1

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64

# name -> (restype, argtypes); mirrors include/narde.h one to one
SIGNATURES = {
    "narde_version": (_i32, []),
    "narde_last_error": (ctypes.c_char_p, []),
    "narde_create": (_i32, [_i32, _i64, _i64, _u64, _i32, _i32, ctypes.POINTER(_vp)]),
    "narde_destroy": (_i32, [_vp]),
    "narde_num_envs": (_i64, [_vp]),
    "narde_get_ply": (_i32, [_vp, ctypes.POINTER(_u32)]),
    "narde_set_ply": (_i32, [_vp, _u32]),
    "narde_reset": (_i32, [_vp, _vp, _vp, _i32, _vp]),
    "narde_set_state": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_get_state": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_peek_dice": (_i32, [_vp, _vp, _vp]),
    "narde_legal_moves": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_step": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "narde_rollout": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_selfplay": (_i32, [_vp, _i32, _vp]),
    "narde_step_full": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "narde_rollout_full": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_selfplay_full": (_i32, [_vp, _i32, _vp]),
    "narde_rollout_timed": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_rollout_plan_create": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_rollout_plan_launch": (_i32, [_vp]),
    "narde_rollout_plan_destroy": (_i32, [_vp]),
    "narde_timing_event_create": (_i32, [_i32, ctypes.c_uint, ctypes.POINTER(_vp)]),
    "narde_timing_event_destroy": (_i32, [_vp]),
    "narde_timing_event_elapsed_ms": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_float)]),
    "narde_legal_full": (_i32, [_vp, _vp, _vp, _vp]),
    "narde_get_stats": (_i32, [_vp, _vp, _vp]),
    "narde_get_totals": (_i32, [_vp, _vp, _vp]),
    "narde_apply_moves": (_i32, [_vp, _vp, _vp, _vp]),
    "narde_observe": (_i32, [_vp, _vp, _vp, _vp]),
    "narde_legal_mask576": (_i32, [_vp, _vp, _vp]),
    "narde_legal_mask576_move2": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "narde_play_set": (_i32, [_vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "narde_act_masks": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "narde_explore_plays": (_i32, [_vp, _vp, _vp, _u64, _vp, _vp, _i64, _vp]),
    "narde_policy_masked_argmax576": (_i32, [_i32, _vp, _i64, _vp, _i64, ctypes.c_float, _u64, _u32,
                                             _i32, _vp, _vp]),
    "narde_policy_masked_argmax576_dev": (_i32, [_i32, _vp, _i64, _vp, _i64, _vp, _u64, _vp, _i32, _vp,
                                                 _i64, _vp, _vp, _vp]),
    "narde_head_policy576_dev": (_i32, [_i32, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _u64, _vp, _i32,
                                        _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp]),
    "narde_dqn_transition": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _i64, _vp]),
    "narde_per_sample": (_i32, [_i32, _vp, _vp, _i64, _i64, _u64, _vp, _vp, ctypes.c_double, _vp, _vp, _vp,
                                _vp, _vp]),
    "narde_per_prefix": (_i32, [_i32, _vp, _i64, ctypes.c_double, _vp, _vp, _vp, _i64, _vp]),
    "narde_gather_batch": (_i32, [_i32, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _vp]),
    "narde_rowmax_addend": (_i32, [_i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp]),
    "narde_dqn_heads_forward": (_i32, [_i32, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp,
                                       _vp]),
    "narde_dqn_heads_backward": (_i32, [_i32, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp,
                                        _vp, _vp, _vp, _vp]),
    "narde_relu_bias_grad": (_i32, [_i32, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "narde_dqn_loss": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, ctypes.c_float, _vp, _vp, _vp,
                              _vp, _vp, _vp]),
    "narde_prio_update": (_i32, [_i32, _vp, _vp, _i64, ctypes.c_float, _vp, _vp, _vp, ctypes.c_float,
                                 ctypes.c_float, _vp, _i64, _i64, _vp, _vp]),
    "narde_per_sample_gather": (_i32, [_i32, _vp, _vp, _i64, _i64, _u64, _vp, _vp, _vp, _vp, _i32, _vp, _i64, _i64,
                                       _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_target_max2": (_i32, [_i32, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "narde_dqn_loss_prio": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, ctypes.c_float, _vp, _vp, _vp,
                                   _vp, _vp, _vp, ctypes.c_float, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, _vp,
                                   _i64, _i64, _vp, _vp, _vp, ctypes.c_double, _vp]),
    "narde_learner_variant": (_i32, [_i32]),
    "narde_adam_clip": (_i32, [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float,
                               ctypes.c_float, ctypes.c_float, ctypes.c_float, _vp, _vp]),
    "narde_violates_block_rule": (_i32, [_i32, _vp, _i64, _vp, _vp]),
    "narde_host_legal_moves": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_host_step": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "narde_host_apply_moves": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "narde_host_violates_block_rule": (_i32, [_vp, _i64, _vp, _vp]),
}


class NardeLibraryError(RuntimeError):
    pass


class NardeValueError(NardeLibraryError, ValueError):
    """NARDE_EINVAL: an invalid argument or position."""


_lib = None


def load():
    """Load libnarde.so (raises NardeLibraryError if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NardeLibraryError(
            f"libnarde.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != OK:
        msg = load().narde_last_error().decode(errors="replace")
        cls = NardeValueError if rc == -1 else NardeLibraryError
        raise cls(f"{what} failed ({rc}): {msg}")


def ptr(a):
    """Raw pointer of a numpy array / torch tensor / None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


class Handle:
    """Owns one narde_env (B envs resident on one device)."""

    def __init__(self, device, num_envs, env_id_offset=0, seed=0, dice_mode=DICE_ALL36,
                 max_episode_steps=1000):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.narde_create(int(device), int(num_envs), int(env_id_offset),
                                    int(seed) & (2 ** 64 - 1), int(dice_mode),
                                    int(max_episode_steps), ctypes.byref(h)), "narde_create")
        self.h = h
        self.device = int(device)
        self.num_envs = int(num_envs)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.narde_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def call(self, name, *args):
        check(getattr(self.lib, name)(self.h, *args), name)

    @property
    def ply(self):
        t = _u32()
        check(self.lib.narde_get_ply(self.h, ctypes.byref(t)), "narde_get_ply")
        return t.value

    @ply.setter
    def ply(self, t):
        check(self.lib.narde_set_ply(self.h, int(t) & 0xFFFFFFFF), "narde_set_ply")


_host_handle = None


def host_handle():
    """Process-wide handle used by the scalar facade for its host calls."""
    global _host_handle
    if _host_handle is None:
        dev = int(os.environ.get("NARDE_DEVICE", "0"))
        _host_handle = Handle(dev, 1)
    return _host_handle
