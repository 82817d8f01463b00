"""FULL4 rules mode (4-move doubles + max dice used) on CPU.

1. The C oracle's composition (oracle/narde_oracle.c or_full4_turn) against
   tests/golden/full4.npz, which tools/capture_full4.py made by composing the
   imported reference's own primitives (Narde.get_valid_moves([die]) and
   execute_rotated_move, narde.py:36-92) -- parity of every sub-move is
   pinned to the reference; the whole-turn rule is the build's (the
   reference env never plays 4 moves: narde_env.py:45-93).
2. The test-only host build of the device engine (tests/hostcheck, the same
   narde_rules.h the HIP kernels compile) against the same fixtures, the
   explicit-play path, and the oracle's FULL4 self-play driver.
"""
import ctypes
import os

import numpy as np
import pytest
from conftest import golden

import oracle as O

# under tools/sanitize.sh (ASan/UBSan build) the big random checks run at a
# tenth of their size: the sanitizers look for memory and UB errors, the
# plain build keeps the coverage
SAN_DIV = 10 if os.environ.get("NARDE_HOSTCHECK_LIB") else 1

P = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731


def compact_c0(d):
    """golden C_0 masks + dice + M -> the device's u64 legal word."""
    hi = np.maximum(d["dice"][:, 0], d["dice"][:, 1]).astype(np.uint64)
    lo = np.minimum(d["dice"][:, 0], d["dice"][:, 1]).astype(np.uint64)
    c = d["cmask"][:, 0, :].astype(np.uint64)
    return (c[:, 0] | (c[:, 1] << np.uint64(24)) | (hi << np.uint64(48)) | (lo << np.uint64(52))
            | (d["max_dice"].astype(np.uint64) << np.uint64(56)))


def played_u64(played):
    """[n,4,2] int8 (from, die) -> u64 (bytes 2k, 2k+1)."""
    b = played.astype(np.uint8).astype(np.uint64)
    v = np.zeros(len(played), np.uint64)
    for k in range(4):
        v |= (b[:, k, 0] | (b[:, k, 1] << np.uint64(8))) << np.uint64(16 * k)
    return v


def test_oracle_full4_golden():
    d = golden("full4.npz")
    r = O.full4_turn(d["board"], d["off"], d["ft"], d["player"], d["dice"], d["words"])
    assert np.array_equal(r["max_dice"], d["max_dice"])
    assert np.array_equal(r["cmask"], d["cmask"])
    assert np.array_equal(r["played"], d["played"])
    assert np.array_equal(r["board"], d["board_after"])
    assert np.array_equal(r["off"], d["off_after"])
    assert np.array_equal(r["first_turn"], d["ft_after"])
    assert np.array_equal(r["reward"], d["reward"])
    assert np.array_equal(r["done"], d["done"])


def test_full4_golden_coverage():
    d = golden("full4.npz")
    M = d["max_dice"]
    dbl = d["dice"][:, 0] == d["dice"][:, 1]
    assert set(np.unique(M).tolist()) == {0, 1, 2, 3, 4}
    assert ((M == 4) & dbl).sum() > 1000 and ((M == 3) & dbl).sum() > 100
    # the higher-die rule (two dice, only one playable, the higher one can)
    one = (M == 1) & ~dbl
    assert one.sum() > 50
    # two head moves on a first-turn 6-6 / 4-4 / 3-3
    heads = (d["played"][:, :, 0] == 23).sum(1)
    assert (heads == 2).any() and heads.max() <= 2
    assert d["done"].sum() > 100


def test_full4_known_answers():
    """Start position turns: hand-checked FULL4 answers."""
    d = golden("full4.npz")
    start = (d["board"][:, 23] == 15) & (d["board"][:, 11] == -15) & (d["ft"] == 1).all(1)
    idx = np.nonzero(start)[0]
    by_roll = {}
    for i in idx:
        by_roll.setdefault((int(d["player"][i]), *map(int, d["dice"][i])), i)
    for pl in (1, -1):
        # 6-6 first turn: two head checkers to 17; 17->11 is blocked by the
        # opponent's head, so only 2 of the 4 dice can be used
        i = by_roll[(pl, 6, 6)]
        assert d["max_dice"][i] == 2
        assert d["played"][i][:2].tolist() == [[23, 6], [23, 6]]
        # 4-4 first turn: 23->19 twice, then 19->15 twice (4 dice)
        i = by_roll[(pl, 4, 4)]
        assert d["max_dice"][i] == 4
        # 5-5: only one head move (5-5 is not a head exception), then that
        # checker moves on: 23->18->13->8 (13 is empty: the opponent is on 11)
        i = by_roll[(pl, 5, 5)]
        assert d["max_dice"][i] == 4 and (d["played"][i][:, 0] == 23).sum() == 1
        # 6-5 from the start: one head move, then the same checker continues
        i = by_roll[(pl, 6, 5)]
        assert d["max_dice"][i] == 2


def test_hostcheck_full4_golden(hostcheck):
    d = golden("full4.npz")
    n = len(d["dice"])
    b, off, ft = d["board"].copy(), d["off"].copy(), d["ft"].copy()
    legal = np.empty(n, np.uint64)
    played = np.empty(n, np.uint64)
    rw = np.empty(n, np.int8)
    dn = np.empty(n, np.uint8)
    hostcheck.hc_full4_batch(ctypes.c_int64(n), P(b), P(off), P(ft), P(d["player"]), P(d["dice"]),
                             P(np.ascontiguousarray(d["words"])), P(legal), P(played), P(rw), P(dn))
    assert np.array_equal(legal, compact_c0(d))
    assert np.array_equal(played, played_u64(d["played"]))
    assert np.array_equal(b, d["board_after"])
    assert np.array_equal(off, d["off_after"])
    assert np.array_equal(ft, d["ft_after"])
    assert np.array_equal(rw, d["reward"]) and np.array_equal(dn, d["done"])


def test_hostcheck_full4_explicit_play(hostcheck):
    """Replaying the golden plays as explicit actions gives the same turn;
    an illegal sub-move ends the turn there (actions are never forced)."""
    d = golden("full4.npz")
    n = len(d["dice"])
    b, off, ft, pl = d["board"].copy(), d["off"].copy(), d["ft"].copy(), d["player"].copy()
    played = np.empty(n, np.uint64)
    play = np.ascontiguousarray(d["played"])
    hostcheck.hc_full4_play_batch(ctypes.c_int64(n), P(b), P(off), P(ft), P(pl), P(d["dice"]),
                                  P(play), P(played))
    assert np.array_equal(played, played_u64(d["played"]))
    assert np.array_equal(off, d["off_after"])
    # truncate every play after its first sub-move with a bogus second one
    bad = play.copy()
    bad[:, 1:, :] = -1
    bad[:, 1, 0] = 30
    b2, off2, ft2, pl2 = d["board"].copy(), d["off"].copy(), d["ft"].copy(), d["player"].copy()
    hostcheck.hc_full4_play_batch(ctypes.c_int64(n), P(b2), P(off2), P(ft2), P(pl2), P(d["dice"]),
                                  P(bad), P(played))
    first = played_u64(d["played"]) & np.uint64(0xFFFF)
    assert np.array_equal(played & np.uint64(0xFFFF), first)
    assert ((played >> np.uint64(16)) == np.uint64(0xFFFFFFFFFFFF)).all()


@pytest.mark.parametrize("dice_mode", [0, 1])
def test_hostcheck_selfplay_full_vs_oracle(hostcheck, dice_mode):
    n, plies, seed, env0 = 384, 300, 0x5EED0F11, 77
    sp = O.SelfPlay(n, seed=seed, env0=env0, dice_mode=dice_mode, max_steps=1000)
    sp.reset(0)
    ro = sp.run_full(plies)
    b = np.zeros((n, 24), np.int8)
    off = np.zeros((n, 2), np.uint8)
    ft = np.zeros((n, 2), np.uint8)
    pl = np.zeros(n, np.int8)
    el = np.zeros(n, np.uint16)
    st = np.zeros((n, 3), np.int32)
    hostcheck.hc_reset_batch(ctypes.c_int64(n), ctypes.c_int64(env0), ctypes.c_uint64(seed),
                             ctypes.c_uint32(0), P(b), P(off), P(ft), P(pl), P(el))
    out = {k: np.empty_like(v) for k, v in ro.items() if k != "dice"}
    hostcheck.hc_selfplay_full(ctypes.c_int64(n), ctypes.c_int64(env0), ctypes.c_uint64(seed),
                               ctypes.c_uint32(0), ctypes.c_int(plies), ctypes.c_int(dice_mode),
                               ctypes.c_int(1000), P(b), P(off), P(ft), P(pl), P(el), P(st),
                               P(out["obs"]), P(out["reward"]), P(out["terminated"]),
                               P(out["truncated"]), P(out["legal"]), P(out["played"]))
    for k in out:
        assert np.array_equal(out[k], ro[k]), k
    assert np.array_equal(st, sp.stats) and np.array_equal(b, sp.board)
    assert sp.stats[:, 0].sum() > 0
    if dice_mode == 0:
        M = (ro["legal"] >> np.uint64(56)).astype(np.int64)
        assert (M == 4).any() and (M == 3).any()


def test_oracle_full4_selfplay_invariants():
    n = 256
    sp = O.SelfPlay(n, seed=3, max_steps=100)
    sp.reset(0)
    r = sp.run_full(400)
    assert r["terminated"].any() and r["truncated"].any()
    w = np.where(sp.board > 0, sp.board, 0).sum(1) + sp.off[:, 0]
    k = np.where(sp.board < 0, -sp.board, 0).sum(1) + sp.off[:, 1]
    assert (w == 15).all() and (k == 15).all()
    # the number of sub-moves played equals max dice used, every ply
    M = (r["legal"] >> np.uint64(56)).astype(np.int64)
    nplayed = sum(((r["played"] >> np.uint64(16 * k)) & np.uint64(0xFF)) != np.uint64(0xFF)
                  for k in range(4))
    assert np.array_equal(nplayed.astype(np.int64), M)
    # FULL4 games are shorter than REF2 ones (doubles move 4 checkers)
    assert sp.stats[:, 0].sum() > 0


def test_hostcheck_pair_bf_matches_per_source(hostcheck):
    """Block-free two-dice turns: the all-sources mask form of the pair check
    (narde_rules.h f4_keep_pair_bf) equals the per-source child check
    (f4_keep_pair) on 300,000 random positions x both dice orders."""
    f = hostcheck.hc_pair_bf_random
    f.restype = ctypes.c_int64
    nt = ctypes.c_int64(0)
    bad = f(ctypes.c_int64(300000 // SAN_DIV), ctypes.c_uint32(7), ctypes.byref(nt))
    assert bad == 0
    assert nt.value > 10000 // SAN_DIV  # the check removes first moves often enough to matter


def test_hostcheck_full4_random_positions(hostcheck):
    """Run-heavy and bear-off positions for both colours, random first-turn
    flags, half doubles: the host engine's turn (block-free shortcuts, mask
    pair checks, exact chain counts, then the search) equals the oracle's
    exhaustive composition on C_0, M, the played sub-moves and the board."""
    from fuzz_positions import random_positions

    n = 6000
    b, off, ft, pl, rng = random_positions(n, 303)
    d0 = rng.integers(1, 7, n)
    d1 = np.where(rng.random(n) < 0.5, d0, rng.integers(1, 7, n))
    dice = np.stack([d0, d1], 1).astype(np.uint8)
    words = rng.integers(0, 2 ** 32, (n, 4), dtype=np.uint64).astype(np.uint32)
    ro = O.full4_turn(b, off, ft, pl, dice, words)
    legal = np.empty(n, np.uint64)
    played = np.empty(n, np.uint64)
    rw = np.empty(n, np.int8)
    dn = np.empty(n, np.uint8)
    b2, off2, ft2 = b.copy(), off.copy(), ft.copy()
    hostcheck.hc_full4_batch(ctypes.c_int64(n), P(b2), P(off2), P(ft2), P(pl), P(dice), P(words),
                             P(legal), P(played), P(rw), P(dn))
    assert np.array_equal(legal, compact_c0({"dice": dice, "cmask": ro["cmask"], "max_dice": ro["max_dice"]}))
    assert np.array_equal(played, played_u64(ro["played"]))
    assert np.array_equal(b2, ro["board"]) and np.array_equal(off2, ro["off"])
    assert all((ro["max_dice"] == m).any() for m in range(5))


def test_hostcheck_open_moves_matches_search(hostcheck):
    """Block-free doubles turns whose bear-off may open mid-turn: the exact
    count (narde_rules.h f4_open_moves, with every C_k = L_k) equals the
    depth-first search's M and first-sub-move set on 100,000 random
    endgames with stragglers outside home."""
    f = hostcheck.hc_open_moves_random
    f.restype = ctypes.c_int64
    up = ctypes.c_int64(0)
    assert f(ctypes.c_int64(100000 // SAN_DIV), ctypes.c_uint32(5), ctypes.byref(up)) == 0
    assert up.value > 3000 // SAN_DIV  # the opening bear-off decides often enough


def test_hostcheck_block_free_is_sound(hostcheck):
    """turn_block_free (narde_rules.h) on 150,000 random block-prone turns:
    a turn it calls block-free never has the block rule remove a candidate
    anywhere in its sub-move tree (exhaustive walk), and its per-window
    test frees many turns the hole count alone calls block-bound.  On the
    doubles among them: dbl_block_free(k) is sound for every k = 1..4 and
    the searches that stop at block-free nodes (f4_depth, f4_reach) equal
    the plain walk; where f4_safe_bound >= 4 (block-bound but settled from
    the never-rejected moves) M = 4 and every first and second sub-move
    keeps the rest playable."""
    f = hostcheck.hc_block_free_random
    f.restype = ctypes.c_int64
    fr, bd, s4 = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
    assert f(ctypes.c_int64(150000 // SAN_DIV), ctypes.c_uint32(11), ctypes.byref(fr), ctypes.byref(bd), ctypes.byref(s4)) == 0
    assert fr.value > 5000 // SAN_DIV and bd.value > 5000 // SAN_DIV and s4.value > 500 // SAN_DIV


def test_hostcheck_sure_pair_is_sound(hostcheck):
    """Block-bound two-dice turns: every first move f4_sure_pair
    (narde_rules.h) marks from the masks keeps a move of the other die
    (the per-source f4_keep_pair) -- 100,000 random block-prone turns."""
    f = hostcheck.hc_sure_pair_random
    f.restype = ctypes.c_int64
    su, tot = ctypes.c_int64(0), ctypes.c_int64(0)
    assert f(ctypes.c_int64(100000 // SAN_DIV), ctypes.c_uint32(3), ctypes.byref(su), ctypes.byref(tot)) == 0
    assert su.value > tot.value // 4  # it settles a real share of the sources


# ---- round 4: the device's straight-line turn (narde_rules.h turn_c0_free,
# turn_c0_pair_bound, turn_moves_sl, turn_block_set_sl, ply_close_sl), host
# mirror hc_full4_batch_sl / hc_selfplay_full_sl (tests/hostcheck)

def test_hostcheck_full4_golden_straight_line(hostcheck):
    d = golden("full4.npz")
    n = len(d["dice"])
    b, off, ft = d["board"].copy(), d["off"].copy(), d["ft"].copy()
    legal = np.empty(n, np.uint64)
    played = np.empty(n, np.uint64)
    rw = np.empty(n, np.int8)
    dn = np.empty(n, np.uint8)
    hostcheck.hc_full4_batch_sl(ctypes.c_int64(n), P(b), P(off), P(ft), P(d["player"]), P(d["dice"]),
                                P(np.ascontiguousarray(d["words"])), P(legal), P(played), P(rw), P(dn))
    assert np.array_equal(legal, compact_c0(d))
    assert np.array_equal(played, played_u64(d["played"]))
    assert np.array_equal(b, d["board_after"])
    assert np.array_equal(off, d["off_after"]) and np.array_equal(ft, d["ft_after"])
    assert np.array_equal(rw, d["reward"]) and np.array_equal(dn, d["done"])


def test_hostcheck_full4_random_positions_straight_line(hostcheck):
    """The straight-line turn on run-heavy / bear-off positions equals the
    oracle's exhaustive composition (block-bound two-dice turns included)."""
    from fuzz_positions import random_positions

    n = 6000
    b, off, ft, pl, rng = random_positions(n, 404)
    d0 = rng.integers(1, 7, n)
    d1 = np.where(rng.random(n) < 0.3, d0, rng.integers(1, 7, n))
    dice = np.stack([d0, d1], 1).astype(np.uint8)
    words = rng.integers(0, 2 ** 32, (n, 4), dtype=np.uint64).astype(np.uint32)
    ro = O.full4_turn(b, off, ft, pl, dice, words)
    legal = np.empty(n, np.uint64)
    played = np.empty(n, np.uint64)
    rw = np.empty(n, np.int8)
    dn = np.empty(n, np.uint8)
    b2, off2, ft2 = b.copy(), off.copy(), ft.copy()
    hostcheck.hc_full4_batch_sl(ctypes.c_int64(n), P(b2), P(off2), P(ft2), P(pl), P(dice), P(words),
                                P(legal), P(played), P(rw), P(dn))
    assert np.array_equal(legal, compact_c0({"dice": dice, "cmask": ro["cmask"], "max_dice": ro["max_dice"]}))
    assert np.array_equal(played, played_u64(ro["played"]))
    assert np.array_equal(b2, ro["board"]) and np.array_equal(off2, ro["off"])


@pytest.mark.parametrize("dice_mode", [0, 1])
def test_hostcheck_selfplay_full_straight_line_vs_oracle(hostcheck, dice_mode):
    n, plies, seed, env0 = 384, 300, 0x5EED0F12, 91
    sp = O.SelfPlay(n, seed=seed, env0=env0, dice_mode=dice_mode, max_steps=100)
    sp.reset(0)
    ro = sp.run_full(plies)
    b = np.zeros((n, 24), np.int8)
    off = np.zeros((n, 2), np.uint8)
    ft = np.zeros((n, 2), np.uint8)
    pl = np.zeros(n, np.int8)
    el = np.zeros(n, np.uint16)
    st = np.zeros((n, 3), np.int32)
    hostcheck.hc_reset_batch(ctypes.c_int64(n), ctypes.c_int64(env0), ctypes.c_uint64(seed),
                             ctypes.c_uint32(0), P(b), P(off), P(ft), P(pl), P(el))
    out = {k: np.empty_like(v) for k, v in ro.items() if k != "dice"}
    hostcheck.hc_selfplay_full_sl(ctypes.c_int64(n), ctypes.c_int64(env0), ctypes.c_uint64(seed),
                                  ctypes.c_uint32(0), ctypes.c_int(plies), ctypes.c_int(dice_mode),
                                  ctypes.c_int(100), P(b), P(off), P(ft), P(pl), P(el), P(st),
                                  P(out["obs"]), P(out["reward"]), P(out["terminated"]),
                                  P(out["truncated"]), P(out["legal"]), P(out["played"]))
    for k in out:
        assert np.array_equal(out[k], ro[k]), k
    assert np.array_equal(st, sp.stats) and np.array_equal(b, sp.board)
    assert ro["truncated"].any() and ro["terminated"].any()


def test_hostcheck_block_set_straight_line(hostcheck):
    f = hostcheck.hc_block_set_sl_random
    f.restype = ctypes.c_int64
    nb = ctypes.c_int64(0)
    assert f(ctypes.c_int64(400000 // SAN_DIV), ctypes.c_uint32(11), ctypes.byref(nb)) == 0
    assert nb.value > 1000 // SAN_DIV


def test_hostcheck_pair_bound_from_failing_windows(hostcheck):
    """Block-bound two-dice turns: C_0 / M from the failing windows
    (turn_c0_pair_bound_w: masks, block_reject_w) equal env_turn_full's bound
    branch (die_filter, f4_keep_pair), and block_reject_w equals die_filter
    at every child of the turn."""
    f = hostcheck.hc_pair_bound_w_random
    f.restype = ctypes.c_int64
    cut = ctypes.c_int64(0)
    assert f(ctypes.c_int64(200000 // SAN_DIV), ctypes.c_uint32(3), ctypes.byref(cut)) == 0
    assert cut.value > 1000 // SAN_DIV


def test_hostcheck_doubles_bound_from_failing_windows(hostcheck):
    """Block-bound doubles turns: block_reject_w (the turn's failing windows)
    equals die_filter at every node to depth 3, and the search over those
    lists (f4_depth_w) equals f4_depth for every first sub-move, and the
    straight-line probe of its first path (f4_probe_w, the device's
    coop_depth_w) is never deeper and equals it whenever it reaches N."""
    f = hostcheck.hc_dbl_bound_w_random
    f.restype = ctypes.c_int64
    cut = ctypes.c_int64(0)
    assert f(ctypes.c_int64(20000 // SAN_DIV), ctypes.c_uint32(9), ctypes.byref(cut)) == 0
    assert cut.value > 1000 // SAN_DIV


def test_hostcheck_windows_few_holes_exhaustive(hostcheck):
    """windows_few_holes (the block test's hole count per 6-window, two
    carry-save adders) equals the plain bit-sliced counter on every one of
    the 2^24 own-point masks, for both hole limits (2: two dice, 4: doubles)."""
    f = hostcheck.hc_windows_few_holes_all
    f.restype = ctypes.c_int64
    assert f() == 0


def test_hostcheck_ply_bound_turn_emulated_wave(hostcheck):
    """ply_bound_turn (full4_wave.h: the rollout's turn for a wave holding a
    block-bound doubles lane, with the f4_safe_bound fast path, the
    cooperative search coop_depth_w and the per-sub-move checks) compiled for
    the CPU with its ballots and readlanes emulated over 64 host threads,
    lane by lane equal to env_turn_full (C_0 | M, played sub-moves, reward,
    done, post-turn state) on waves mixing block-bound doubles, block-bound
    two-dice and free lanes."""
    f = hostcheck.hc_ply_bound_turn_random
    f.restype = ctypes.c_int64
    c = (ctypes.c_int64 * 4)()
    waves = max(4, 160 // SAN_DIV)
    assert f(ctypes.c_int64(waves), ctypes.c_uint32(11), c) == 0
    bd, searched, b2, lanes = list(c)
    assert lanes == 64 * waves
    assert bd > 10 * waves and searched > 5 * waves and b2 > 10 * waves


def test_hostcheck_pair_pass_selfplay_turns(hostcheck):
    """coop_pair_w (full4_wave.h: the block-bound doubles search's root and
    sub-move-1 check in one cooperative pass over source pairs) on the
    searching turns random-legal self-play meets: ply_bound_turn on 64
    emulated lanes == env_turn_full, lane by lane, including the turns whose
    sub-move-1 check differs between one and two more sub-moves (the case
    that tells the pass's two result sets apart; a mutant taking the wrong
    set fails on them); every field of the turn compared (reward, the
    record, the O / P / S1 masks), and both branches of the pass met."""
    f = hostcheck.hc_pair_pass_selfplay
    f.restype = ctypes.c_int64
    c = (ctypes.c_int64 * 5)()
    envs = max(1024, 8192 // SAN_DIV)
    assert f(ctypes.c_int64(envs), ctypes.c_int64(200), c) == 0
    kept, split, waves, fallback, bypass = list(c)
    assert kept > envs // 8 and waves >= kept // 64
    # both branches of the pass ran: sub-move 1 taken from the pairs'
    # checked list, and (rare: 1 of 1,925 kept turns at 8,192 envs) an owner
    # left to coop_depth_w
    assert bypass > kept // 2
    if envs == 8192:
        assert split > 0 and fallback > 0
