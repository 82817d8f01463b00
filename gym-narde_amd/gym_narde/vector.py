"""VecNardeEnv -- B Narde envs stepped in lockstep on one GPU.

This is the batched hot path the scalar NardeEnv (narde_env.py:27-103 of the
reference) is replaced by: state stays resident in HBM (32 B/env), every call
is one stream-ordered kernel launch on the caller's current torch stream, and
outputs land in preallocated device tensors (valid until the next call of the
same kind -- clone them to keep them).

Dice of ply t for global env e are Philox4x32-10({t, e, 0, 0}, seed), so
`dice()` / `legal_moves()` / `legal_mask()` describe exactly the roll the next
`step()` will use (the reference's callers peek/roll their own dice instead,
train_deepq_pytorch.py:866).  Actions are the reference's codes
(from*24 + to, (from<=5, to==0) = bear-off).

rules="ref2" (default) is the reference's NardeEnv.step: at most two checker
moves per step, quirks included.  rules="full4" is the build's whole-turn
mode (include/narde.h): four sub-moves on doubles, max
dice used, the higher die when only one can be used.  Its actions are plays,
(B,4,2) int8 (from, die) sub-moves; info["legal"] is the first sub-move's
set with the max dice usable in bits 56-58, info["played"] the sub-moves
played (bytes 2k/2k+1 = from/die, 0xFF unused).
"""
import ctypes
import os
import weakref

import numpy as np

from . import _lib

DICE_MODES = {"all36": _lib.DICE_ALL36, "nodoubles": _lib.DICE_NODOUBLES}
RULES = ("ref2", "full4")


def decode_compact(compact):
    """Compact legal set(s) (u64, see include/narde.h) -> list(s) of (from, to)
    with to == 'off' for bear-off, in the reference's list order."""
    arr = np.atleast_1d(np.asarray(compact, dtype=np.uint64))
    out = []
    for c in arr.tolist():
        lh, ll = c & 0xFFFFFF, (c >> 24) & 0xFFFFFF
        dh, dl = (c >> 48) & 0xF, (c >> 52) & 0xF
        moves = []
        for L, d in ((lh, dh), (ll, dl)):
            if d == 0:
                continue
            for p in range(24):
                if (L >> p) & 1:
                    moves.append((p, "off" if p - d < 0 else p - d))
        out.append(moves)
    return out if np.ndim(compact) else out[0]


def decode_full_legal(word):
    """FULL4 legal word (u64) -> (max_dice, [(from, die), ...]) in list
    order (higher die first, ascending source)."""
    c = int(np.uint64(word))
    ch, cl = c & 0xFFFFFF, (c >> 24) & 0xFFFFFF
    dh, dl, m = (c >> 48) & 0xF, (c >> 52) & 0xF, (c >> 56) & 0x7
    opts = [(p, dh) for p in range(24) if (ch >> p) & 1]
    if dl != dh:
        opts += [(p, dl) for p in range(24) if (cl >> p) & 1]
    return m, opts


def decode_played(word):
    """FULL4 played word (u64) -> [(from, die), ...] sub-moves in order."""
    c = int(np.uint64(word))
    out = []
    for k in range(4):
        f, d = (c >> (16 * k)) & 0xFF, (c >> (16 * k + 8)) & 0xFF
        if f == 0xFF:
            break
        out.append((f, d))
    return out


PLAY_KINDS = {"act": 0, "step": 1}


def decode_play_set(legal, words, kind="act"):
    """One env's play set (VecNardeEnv.play_set: its compact list #1 and
    its (2, 24) entry words) in the reference's terms.
    kind "act": DQNAgent.act's valid_move_combinations
    (train_deepq_pytorch.py:430-507) -- a list of (move1_code, move2_code)
    in act()'s order, duplicates included ('off' coded as to = 0, no second
    move as 0).  kind "step": the set of plays NardeEnv.step carries out
    (narde_env.py:45-93) as move tuples ((m1, m2), or (m1,) alone), as
    Narde.get_valid_plays returns them."""
    c = int(np.uint64(np.int64(legal)))
    w = np.asarray(words).astype(np.int64).reshape(2, 24)
    masks = (c & 0xFFFFFF, (c >> 24) & 0xFFFFFF)
    dies = ((c >> 48) & 0xF, (c >> 52) & 0xF)
    entries = [(k, p, dies[k]) for k in range(2) if dies[k] for p in range(24) if (masks[k] >> p) & 1]
    out = [] if kind == "act" else set()
    for k, p, d in entries:
        wd = int(w[k, p])
        m2, rem = wd & 0xFFFFFF, (wd >> 24) & 7
        seconds = [(q, "off" if q < rem else q - rem) for q in range(24) if (m2 >> q) & 1]
        m1 = (p, "off" if p < d else p - d)
        if kind == "act":
            c1 = p * 24 + (0 if m1[1] == "off" else m1[1])
            if not seconds:
                out.append((c1, 0))
            for q, t in seconds:
                out.append((c1, q * 24 + (0 if t == "off" else t)))
        elif len(entries) == 1 or not seconds:
            out.add((m1,))
        else:
            out.update((m1, m2_) for m2_ in seconds)
    return out


class VecNardeEnv:
    def __init__(self, num_envs, device=None, seed=0, env_id_offset=0, dice_mode="all36",
                 max_episode_steps=1000, autoreset=True, rules="ref2"):
        import torch

        if rules not in RULES:
            raise ValueError(f"rules must be one of {RULES}")
        self.rules = rules
        self.full = rules == "full4"

        self.torch = torch
        dev = torch.device(device if device is not None else "cuda")
        if dev.type != "cuda":
            raise ValueError("VecNardeEnv runs on a GPU device only")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.num_envs = int(num_envs)
        self.autoreset = bool(autoreset)
        self.handle = _lib.Handle(dev.index, num_envs, env_id_offset, seed, DICE_MODES[dice_mode],
                                  max_episode_steps)
        B = self.num_envs
        z = dict(device=dev)
        self.obs = torch.zeros((B, 24), dtype=torch.int32, **z)
        self.reward = torch.zeros(B, dtype=torch.int32, **z)
        self.terminated = torch.zeros(B, dtype=torch.uint8, **z)
        self.truncated = torch.zeros(B, dtype=torch.uint8, **z)
        self.legal = torch.zeros(B, dtype=torch.int64, **z)
        self.actions_used = torch.zeros((B, 2), dtype=torch.int16, **z)
        self.played = torch.zeros(B, dtype=torch.int64, **z)
        # per-call plumbing of step(), resolved once: the bound entry point and
        # the output buffers' pointers (they never move)
        lib = self.handle.lib
        self._step_fn = lib.narde_step_full if self.full else lib.narde_step
        self._step_out = tuple(_lib.ptr(t) for t in (
            (self.obs, self.reward, self.terminated, self.truncated, self.legal, self.played) if self.full else
            (self.obs, self.reward, self.terminated, self.truncated, self.legal, self.actions_used)))

    # ------------------------------------------------------------ plumbing
    def _s(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _dev(self, x, dtype, shape):
        if (isinstance(x, self.torch.Tensor) and x.dtype == dtype and x.device == self.device
                and x.is_contiguous() and tuple(x.shape) == tuple(shape)):
            return x  # already a device tensor of the right layout
        t = self.torch.as_tensor(x, device=self.device).to(dtype).contiguous()
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    @property
    def ply(self):
        return self.handle.ply

    @ply.setter
    def ply(self, t):
        self.handle.ply = t

    # ------------------------------------------------------------ API
    def reset(self, mask=None, opening=None):
        """NardeEnv.reset (narde_env.py:105-120) for all (or the masked) envs;
        returns obs (B,24) int32.  opening: (B,K,2) uint8 opening draws
        (white roll, black roll) per env in the reference's draw order -- the
        first pair of different dice decides who moves first, pairs with a
        die outside 1..6 are padding -- or None for the device draw (also
        for an env whose row has no deciding pair)."""
        B = self.num_envs
        m = None if mask is None else self._dev(mask, self.torch.uint8, (B,))
        o, pairs = None, 0
        if opening is not None:
            o = self.torch.as_tensor(opening, device=self.device).to(self.torch.uint8).contiguous()
            if o.dim() == 2:
                o = o.reshape(B, 1, 2)
            if o.dim() != 3 or o.shape[0] != B or o.shape[2] != 2 or o.shape[1] < 1:
                raise ValueError(f"opening must be (B, K, 2) with B = {B}, got {tuple(o.shape)}")
            pairs = int(o.shape[1])
        self.handle.call("narde_reset", _lib.ptr(m), _lib.ptr(o), pairs, self._s())
        self._keep = (m, o)  # inputs alive until the kernel has read them
        return self.observe()

    def observe(self):
        self.handle.call("narde_observe", _lib.ptr(self.obs), None, self._s())
        return self.obs

    def tesauro198(self, out=None):
        """README.md:42-102 198-float observation, (B,198) float32."""
        if out is None:
            out = self.torch.empty((self.num_envs, 198), dtype=self.torch.float32, device=self.device)
        self.handle.call("narde_observe", None, _lib.ptr(out), self._s())
        return out

    def observe_host(self, kind="int24", out=None):
        """Observations for CPU-side agents:
        the observe kernel writes the device buffer and a non-blocking copy
        lands it in PINNED host memory on the same stream.  Returns (host
        tensor, event); read the host tensor after event.synchronize().
        kind: "int24" (the reference's int32[24] obs) or "tesauro198"."""
        t = self.torch
        if kind == "int24":
            dev, shape, dt = self.observe(), (self.num_envs, 24), t.int32
        elif kind == "tesauro198":
            dev, shape, dt = self.tesauro198(), (self.num_envs, 198), t.float32
        else:
            raise ValueError("kind must be 'int24' or 'tesauro198'")
        if out is None:
            out = t.empty(shape, dtype=dt, pin_memory=True)
        elif tuple(out.shape) != shape or out.dtype != dt or not out.is_pinned():
            raise ValueError(f"out must be a pinned {dt} tensor of shape {shape}")
        out.copy_(dev, non_blocking=True)
        ev = t.cuda.Event()
        ev.record(t.cuda.current_stream(self.device))
        self._keep_host = dev  # the source stays alive until the copy is done
        return out, ev

    def dice(self):
        """Dice of the next device-RNG step, (B,2) uint8 in roll order."""
        d = self.torch.empty((self.num_envs, 2), dtype=self.torch.uint8, device=self.device)
        self.handle.call("narde_peek_dice", _lib.ptr(d), self._s())
        return d

    def legal_moves(self, dice=None, expanded=True):
        """Narde.get_valid_moves per env.  dice: (B,k) k<=4 (0 = unused) or None
        for the next step's dice.  Returns (count (B,) int16, moves (B,64,2)
        int8 or None, compact (B,) int64 or None)."""
        B = self.num_envs
        d4 = None
        if dice is not None:
            d = self.torch.as_tensor(dice, device=self.device).to(self.torch.uint8)
            d4 = self.torch.zeros((B, 4), dtype=self.torch.uint8, device=self.device)
            d4[:, : d.shape[1]] = d
        count = self.torch.empty(B, dtype=self.torch.int16, device=self.device)
        moves = (self.torch.empty((B, _lib.MAX_MOVES, 2), dtype=self.torch.int8, device=self.device)
                 if expanded else None)
        # compact form is only defined for <= 2 dice (the kernel writes 0 otherwise)
        compact = self.torch.empty(B, dtype=self.torch.int64, device=self.device)
        self.handle.call("narde_legal_moves", _lib.ptr(d4), _lib.ptr(count), _lib.ptr(moves),
                         _lib.ptr(compact), self._s())
        return count, moves, compact

    def legal_mask(self, out=None):
        """(B,9) int64 = 576-bit mask of move1 codes the next step accepts."""
        if out is None:
            out = self.torch.empty((self.num_envs, 9), dtype=self.torch.int64, device=self.device)
        self.handle.call("narde_legal_mask576", _lib.ptr(out), self._s())
        return out

    def legal_mask_move2(self, move1, dice=None, out=None):
        """(B,9) int64 = 576-bit mask of move2 codes step() accepts after the
        move1 codes (B,), for dice (B,2) or the next step's device dice (all
        zero where move1 would not be played)."""
        B = self.num_envs
        m1 = self._dev(move1, self.torch.int16, (B,))
        d = None if dice is None else self._dev(dice, self.torch.uint8, (B, 2))
        if out is None:
            out = self.torch.empty((B, 9), dtype=self.torch.int64, device=self.device)
        self.handle.call("narde_legal_mask576_move2", _lib.ptr(m1), _lib.ptr(d), _lib.ptr(out),
                         self._s())
        self._keep = (m1, d)
        return out

    def play_set(self, dice=None, kind="act"):
        """The plays of each env's two-dice roll (narde_play_set; the
        README's get_valid_actions, README.md:156-165) for dice (B,2) in roll
        order or the next step's device dice.  Returns (legal (B,) int64
        compact list #1, words (B,2,24) int32 -- per list-#1 entry its
        second-move sources | rem << 24 | 1 << 27, count (B,) int32 plays).
        kind "act": DQNAgent.act's combinations, second moves on the
        PRE-move board (train_deepq_pytorch.py:430-507); "step": the plays
        NardeEnv.step carries out, second moves on the POST-move board
        (narde_env.py:45-93).  decode_play_set() turns one env's row into
        the reference's list / set."""
        if kind not in PLAY_KINDS:
            raise ValueError(f"kind must be one of {tuple(PLAY_KINDS)}")
        B, t = self.num_envs, self.torch
        d = None if dice is None else self._dev(dice, t.uint8, (B, 2))
        legal = t.empty(B, dtype=t.int64, device=self.device)
        words = t.empty((B, 2, 24), dtype=t.int32, device=self.device)
        count = t.empty(B, dtype=t.int32, device=self.device)
        self.handle.call("narde_play_set", _lib.ptr(d), PLAY_KINDS[kind], _lib.ptr(legal), _lib.ptr(words),
                         _lib.ptr(count), self._s())
        self._keep = (d,)
        return legal, words, count

    def act_masks(self, move1=None, dice=None, out=None):
        """DQNAgent.act's greedy candidate sets (narde_act_masks) as (B,9)
        int64 576-bit masks: move1 None -- the move-1 codes of list #1
        (valid_first_moves' keys); move1 (B,) int64 (any positive stride)
        -- the move-2 codes act() offers after it (the pre-move second list
        of the last list-#1 entry with that code; code 0 alone if empty)."""
        B, t = self.num_envs, self.torch
        d = None if dice is None else self._dev(dice, t.uint8, (B, 2))
        if move1 is not None and (move1.dtype != t.int64 or move1.dim() != 1 or move1.shape[0] != B
                                  or move1.device != self.device or move1.stride(0) < 1):
            raise ValueError(f"move1 must be ({B},) int64 on the env's device")
        if out is None:
            out = t.empty((B, 9), dtype=t.int64, device=self.device)
        self.handle.call("narde_act_masks", _lib.ptr(d), _lib.ptr(move1),
                         move1.stride(0) if move1 is not None else 1, _lib.ptr(out), self._s())
        self._keep = (d, move1)
        return out

    def explore_plays(self, actions, epsilon, seed, tag, dice=None):
        """The DQN driver's exploration (narde_explore_plays): rows whose
        explore draw ({tag, row, 0, 5}, seed) is below epsilon get a play
        drawn uniformly from act()'s combination list written into their
        (B, 2) int64 action row (in place); epsilon (f32) and tag (int64)
        are device scalars (graph-safe)."""
        B, t = self.num_envs, self.torch
        if (actions.dtype != t.int64 or tuple(actions.shape) != (B, 2) or actions.stride(1) != 1
                or actions.device != self.device):
            raise ValueError(f"actions must be ({B}, 2) int64 rows on the env's device")
        d = None if dice is None else self._dev(dice, t.uint8, (B, 2))
        self.handle.call("narde_explore_plays", _lib.ptr(d), _lib.ptr(epsilon), int(seed) & (2 ** 64 - 1),
                         _lib.ptr(tag), _lib.ptr(actions), actions.stride(0), self._s())
        self._keep = (d,)
        return actions

    def legal_full(self, dice=None):
        """FULL4: (B,) int64 legal words (first sub-move set | max dice << 56)
        for dice (B,2) or the next step's device dice."""
        B = self.num_envs
        d = None if dice is None else self._dev(dice, self.torch.uint8, (B, 2))
        out = self.torch.empty(B, dtype=self.torch.int64, device=self.device)
        self.handle.call("narde_legal_full", _lib.ptr(d), _lib.ptr(out), self._s())
        return out

    def step(self, actions=None, dice=None):
        """NardeEnv.step for all envs.  actions (B,2) codes (rules="full4":
        (B,4,2) int8 (from, die) plays) or None for the in-kernel random
        legal policy; dice (B,2) or None for device dice.  Returns (obs,
        reward, terminated, truncated, info) device tensors; info =
        {'legal': compact list #1, 'actions': codes used} (rules="full4":
        {'legal': first sub-move set + max dice, 'played': sub-moves})."""
        B = self.num_envs
        if self.full:
            a = None if actions is None else self._dev(actions, self.torch.int8, (B, 4, 2))
        else:
            a = None if actions is None else self._dev(actions, self.torch.int16, (B, 2))
        d = None if dice is None else self._dev(dice, self.torch.uint8, (B, 2))
        rc = self._step_fn(self.handle.h, None if a is None else _lib.ptr(a), None if d is None else _lib.ptr(d),
                           *self._step_out, int(self.autoreset), self._s())
        if rc:
            _lib.check(rc, "narde_step_full" if self.full else "narde_step")
        if self.full:
            self._keep = (a, d)
            return (self.obs, self.reward, self.terminated, self.truncated,
                    {"legal": self.legal, "played": self.played})
        return (self.obs, self.reward, self.terminated, self.truncated,
                {"legal": self.legal, "actions": self.actions_used})

    def selfplay(self, plies):
        """plies plies of random-legal self-play in ONE launch (statistics only)."""
        self.handle.call("narde_selfplay_full" if self.full else "narde_selfplay", int(plies),
                         self._s())

    def rollout_buffers(self, plies, obs=True, reward=True, terminated=True, truncated=True,
                        legal=True, actions=True):
        """Allocate [plies][B] rollout buffers for rollout() (rules="full4":
        'actions' holds the played sub-moves, (plies, B) int64)."""
        t, B, dev = self.torch, self.num_envs, self.device
        mk = lambda on, shape, dt: t.empty(shape, dtype=dt, device=dev) if on else None  # noqa: E731
        act = mk(actions, (plies, B), t.int64) if self.full else mk(actions, (plies, B, 2), t.int16)
        return dict(obs=mk(obs, (plies, B, 24), t.int32), reward=mk(reward, (plies, B), t.int32),
                    terminated=mk(terminated, (plies, B), t.uint8),
                    truncated=mk(truncated, (plies, B), t.uint8),
                    legal=mk(legal, (plies, B), t.int64), actions=act)

    def rollout(self, plies, bufs=None):
        """plies plies of random-legal self-play (auto-reset) in ONE launch,
        every ply's outputs streamed into [plies][B] buffers (see
        rollout_buffers); equals `plies` calls of step()."""
        if bufs is None:
            bufs = self.rollout_buffers(plies)
        for v in bufs.values():
            if v is not None and v.shape[0] < plies:
                raise ValueError("rollout buffer shorter than plies")
        self.handle.call("narde_rollout_full" if self.full else "narde_rollout", int(plies),
                         _lib.ptr(bufs["obs"]), _lib.ptr(bufs["reward"]),
                         _lib.ptr(bufs["terminated"]), _lib.ptr(bufs["truncated"]),
                         _lib.ptr(bufs["legal"]), _lib.ptr(bufs["actions"]), self._s())
        return bufs

    def rollout_launcher(self, plies, bufs, events=None, totals=None):
        """rollout(plies, bufs) pre-bound: a zero-argument callable that makes
        exactly one ctypes call (one kernel launch on the stream current
        NOW), for hot loops where the per-call Python of rollout() would
        show (the buffers must stay alive and unmoved while it is used).
        With events, the launch is pre-bound in the library
        (narde_rollout_plan_*: one pointer per call; $NARDE_ROLLOUT_PLAN=0
        takes narde_rollout_timed's per-call arguments instead).
        events = (start, stop) torch.cuda.Event or TimingEvent (either None): recorded on
        that stream right before / after the launch, inside the same call
        (narde_rollout_timed); a torch event must have been recorded once
        already (it creates its HIP event at its first record).
        totals: a (wg_rows(B), 3) int64 device tensor the launch fills with
        the statistics after it summed per 256 envs (.sum(0) = the
        handle's {episodes, white points, black points}) -- no second launch."""
        for v in bufs.values():
            if v is not None and v.shape[0] < plies:
                raise ValueError("rollout buffer shorter than plies")
        if totals is not None:
            t = self.torch
            if (tuple(totals.shape) != (_lib.wg_rows(self.num_envs), 3) or totals.dtype != t.int64
                    or totals.device != self.device or not totals.is_contiguous()):
                raise ValueError(f"totals must be a contiguous ({_lib.wg_rows(self.num_envs)}, 3) int64 "
                                 "tensor on the env's device")
            if plies <= 0:
                raise ValueError("totals need a launch (plies > 0)")
            events = events if events is not None else (None, None)
        bufargs = (_lib.ptr(bufs["obs"]), _lib.ptr(bufs["reward"]), _lib.ptr(bufs["terminated"]),
                   _lib.ptr(bufs["truncated"]), _lib.ptr(bufs["legal"]), _lib.ptr(bufs["actions"]))
        if events is None:
            fn = self.handle.lib.narde_rollout_full if self.full else self.handle.lib.narde_rollout
            name = "narde_rollout_full" if self.full else "narde_rollout"
            args = (self.handle.h, int(plies)) + bufargs + (self._s(),)
        else:
            evs = []
            for ev in events:
                if isinstance(ev, TimingEvent):
                    evs.append(ctypes.c_void_p(ev.handle))
                    continue
                if ev is not None and not ev.cuda_event:
                    raise ValueError("record each event once before binding it (its HIP event is created then)")
                evs.append(ctypes.c_void_p(ev.cuda_event) if ev is not None else None)
            fn, name = self.handle.lib.narde_rollout_timed, "narde_rollout_timed"
            args = (self.handle.h, int(self.full), int(plies)) + bufargs + (evs[0], evs[1], _lib.ptr(totals),
                                                                            self._s())
            if int(plies) > 0 and os.environ.get("NARDE_ROLLOUT_PLAN", "1") == "1":
                # round 6: the same launch pre-bound in the library
                # (narde_rollout_plan_*): the timed call is one pointer
                plan = ctypes.c_void_p()
                _lib.check(self.handle.lib.narde_rollout_plan_create(*args, ctypes.byref(plan)),
                           "narde_rollout_plan_create")
                fn, name, args = self.handle.lib.narde_rollout_plan_launch, "narde_rollout_plan_launch", (plan,)

        def launch():
            rc = fn(*args)
            if rc:
                _lib.check(rc, name)

        if fn is self.handle.lib.narde_rollout_plan_launch:
            weakref.finalize(launch, self.handle.lib.narde_rollout_plan_destroy, args[0])

        launch.bufs = bufs  # keeps the buffers referenced as long as the launcher
        launch.events = events
        launch.totals = totals
        return launch

    def stats(self, out=None):
        """(B,3) int32 {episodes finished, white points, black points} (into
        `out` if given: a preallocated (B,3) int32 device tensor)."""
        if out is None:
            out = self.torch.empty((self.num_envs, 3), dtype=self.torch.int32, device=self.device)
        elif (tuple(out.shape) != (self.num_envs, 3) or out.dtype != self.torch.int32
              or out.device != self.device or not out.is_contiguous()):
            raise ValueError("out must be a contiguous (B,3) int32 tensor on the env's device")
        self.handle.call("narde_get_stats", _lib.ptr(out), self._s())
        return out

    def totals(self, out=None):
        """(64,3) int64 partial sums of stats() over contiguous env ranges
        (narde_get_totals: one launch); .sum(0) gives {episodes, white
        points, black points} of the handle (into `out` if given)."""
        if out is None:
            out = self.torch.empty((_lib.TOTAL_ROWS, 3), dtype=self.torch.int64, device=self.device)
        elif (tuple(out.shape) != (_lib.TOTAL_ROWS, 3) or out.dtype != self.torch.int64
              or out.device != self.device or not out.is_contiguous()):
            raise ValueError("out must be a contiguous (64,3) int64 tensor on the env's device")
        self.handle.call("narde_get_totals", _lib.ptr(out), self._s())
        return out

    def totals_launcher(self, out):
        """totals(out) pre-bound: a zero-argument callable making exactly one
        ctypes call (one launch on the stream current NOW); returns out."""
        t = self.torch
        if (tuple(out.shape) != (_lib.TOTAL_ROWS, 3) or out.dtype != t.int64 or out.device != self.device
                or not out.is_contiguous()):
            raise ValueError("out must be a contiguous (64,3) int64 tensor on the env's device")
        fn, args = self.handle.lib.narde_get_totals, (self.handle.h, _lib.ptr(out), self._s())

        def launch():
            rc = fn(*args)
            if rc:
                _lib.check(rc, "narde_get_totals")
            return out

        launch.out = out
        return launch

    def get_state(self):
        B, t, dev = self.num_envs, self.torch, self.device
        st = dict(board=t.empty((B, 24), dtype=t.int8, device=dev),
                  off=t.empty((B, 2), dtype=t.uint8, device=dev),
                  first_turn=t.empty((B, 2), dtype=t.uint8, device=dev),
                  player=t.empty(B, dtype=t.int8, device=dev),
                  elapsed=t.empty(B, dtype=t.int16, device=dev))
        self.handle.call("narde_get_state", _lib.ptr(st["board"]), _lib.ptr(st["off"]),
                         _lib.ptr(st["first_turn"]), _lib.ptr(st["player"]), _lib.ptr(st["elapsed"]),
                         self._s())
        return st

    def set_state(self, board, off, first_turn, player, elapsed=None):
        B, t = self.num_envs, self.torch
        b = self._dev(board, t.int8, (B, 24))
        o = self._dev(off, t.uint8, (B, 2))
        f = self._dev(first_turn, t.uint8, (B, 2))
        p = self._dev(player, t.int8, (B,))
        e = None if elapsed is None else self._dev(elapsed, t.int16, (B,))
        self.handle.call("narde_set_state", _lib.ptr(b), _lib.ptr(o), _lib.ptr(f), _lib.ptr(p),
                         _lib.ptr(e), self._s())
        self._keep = (b, o, f, p, e)  # keep inputs alive until the kernel has read them

    def apply_moves(self, moves, player=None):
        """execute_rotated_move per env; moves (B,2) int8 (to=24 for off, from<0 skips)."""
        B, t = self.num_envs, self.torch
        m = self._dev(moves, t.int8, (B, 2))
        p = None if player is None else self._dev(player, t.int8, (B,))
        self.handle.call("narde_apply_moves", _lib.ptr(m), _lib.ptr(p), self._s())
        self._keep = (m, p)

    def close(self):
        self.handle.close()


class TimingEvent:
    """A HIP event made by the library (narde_timing_event_create) for
    rollout_launcher(..., events=...).  flags: DISABLE_SYSTEM_FENCE (default)
    makes the record a timing-only marker -- no system-scope cache write-back
    and invalidate when it completes, so the marker after a launch does not
    lengthen the span it measures; 0 = HIP's default event (what a
    torch.cuda.Event is)."""

    DISABLE_SYSTEM_FENCE = 0x20000000

    def __init__(self, device=None, flags=DISABLE_SYSTEM_FENCE):
        import torch

        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.narde_timing_event_create(dev.index or 0, int(flags), ctypes.byref(h)),
                   "narde_timing_event_create")
        self.handle = h.value

    def elapsed_ms(self, stop):
        """Milliseconds from this event to `stop` (both recorded and complete)."""
        ms = ctypes.c_float()
        _lib.check(self._lib.narde_timing_event_elapsed_ms(ctypes.c_void_p(self.handle),
                                                            ctypes.c_void_p(stop.handle), ctypes.byref(ms)),
                   "narde_timing_event_elapsed_ms")
        return float(ms.value)

    def close(self):
        if self.handle:
            self._lib.narde_timing_event_destroy(ctypes.c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
