"""The batched play set (narde_rules.h play_walk: k_play_set / k_explore_plays'
per-lane body) on the CPU, through the test-only host build of the rules
engine (tests/hostcheck), against the reference's own recordings:

* kind "act" == DQNAgent.act's valid_move_combinations
  (train_deepq_pytorch.py:430-507), list for list -- order and duplicates
  included -- on every step of tests/golden/trainer.npz (the reference
  trainer's loop, recorded on the imported reference: its agent dice, its
  pre-step states, its combination lists);
* play_codes_act(j) (the exploration kernel's index -> codes map) walks the
  same list;
* kind "step": on every golden NardeEnv.step of tests/golden/steps.npz the
  entry of the move 1 the step played holds exactly the reference's list #2
  (sources and die), and the whole set equals a restatement of
  narde_env.py:45-93 over the C oracle's primitives on 4,000 golden states.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
from conftest import golden

P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def _decode(legal, words, kind):
    import sys
    import os

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-narde_amd"))
    from gym_narde.vector import decode_play_set

    return decode_play_set(legal, words, kind)


def _play_set(hc, board, off, ft, player, dice, kind):
    n = board.shape[0]
    legal = np.zeros(n, np.uint64)
    table = np.zeros((n, 48), np.uint32)
    count = np.zeros(n, np.int32)
    c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
    board, off, ft, player, dice = (c(board, np.int8), c(off, np.uint8), c(ft, np.uint8), c(player, np.int8),
                                    c(dice, np.uint8))
    hc.hc_play_set(ctypes.c_int64(n), P(board), P(off), P(ft), P(player), P(dice), ctypes.c_int(kind), P(legal),
                   P(table), P(count))
    return legal, table.view(np.int32).reshape(n, 2, 24), count


def test_act_kind_equals_reference_trainer_combinations(hostcheck):
    t = golden("trainer.npz")
    act = t["nvalid"] > 0  # act() ran (the loop skips it with no legal move)
    starts = np.concatenate([[0], np.cumsum(t["combos_len"])])
    legal, words, count = _play_set(hostcheck, t["pre_board"], t["pre_off"], t["pre_ft"], t["player"], t["dice"], 0)
    assert np.array_equal(count[act], t["combos_len"][act])
    n_checked = 0
    for i in np.nonzero(act)[0]:
        want = [tuple(int(x) for x in r) for r in t["combos"][starts[i]:starts[i + 1]]]
        assert _decode(legal[i], words[i], "act") == want, f"step {i}"
        n_checked += 1
    assert n_checked > 5000


def test_play_codes_act_walks_the_list(hostcheck):
    t = golden("trainer.npz")
    starts = np.concatenate([[0], np.cumsum(t["combos_len"])])
    rows = [i for i in np.nonzero(t["nvalid"] > 0)[0]][:1500]
    codes = np.zeros((64 * 30, 2), np.int16)
    for i in rows:
        b = np.ascontiguousarray(t["pre_board"][i], np.int8)
        o = np.ascontiguousarray(t["pre_off"][i], np.uint8)
        f = np.ascontiguousarray(t["pre_ft"][i], np.uint8)
        d = np.ascontiguousarray(t["dice"][i], np.uint8)
        cnt = hostcheck.hc_play_codes_act(P(b), P(o), P(f), ctypes.c_int8(int(t["player"][i])), P(d), P(codes),
                                          ctypes.c_int(codes.shape[0]))
        assert cnt == t["combos_len"][i]
        assert np.array_equal(codes[:cnt], t["combos"][starts[i]:starts[i + 1]]), f"step {i}"


def _entry_of(list1_row, count1, code1):
    """(from, to) of the move-1 code NardeEnv.step decodes (narde_env.py:47-53)."""
    f, t = divmod(int(code1), 24)
    return (f, 24 if (t == 0 and f <= 5) else t)


def test_step_kind_holds_the_reference_list2(hostcheck):
    s = golden("steps.npz")
    legal, words, count = _play_set(hostcheck, s["board"], s["off"], s["first_turn"], s["player"], s["dice"], 1)
    # list #1 (compact) == the reference's list, every case
    for i in range(0, s["board"].shape[0], 7):
        c = int(legal[i])
        lh, ll, dh, dl = c & 0xFFFFFF, (c >> 24) & 0xFFFFFF, (c >> 48) & 15, (c >> 52) & 15
        got = [(p, 24 if p < d else p - d) for L, d in ((lh, dh), (ll, dl)) for p in range(24) if (L >> p) & 1]
        want = [tuple(int(x) for x in r) for r in s["list1"][i, :s["count1"][i]]]
        assert got == want, f"case {i}"
    played = np.nonzero((s["count2"] >= 0) & (s["count1"] >= 2))[0]
    assert played.size > 10000
    for i in played:
        f, t = _entry_of(s["list1"][i], s["count1"][i], s["action"][i, 0])
        c = int(legal[i])
        dh, dl = (c >> 48) & 15, (c >> 52) & 15
        # the entry the step matched: any list whose die gives this move
        ks = [k for k, d in ((0, dh), (1, dl)) if ((c >> (24 * k)) >> f) & 1
              and ((t == 24 and f < d) or (t != 24 and f - t == d))]
        assert ks, f"case {i}: move 1 not in list #1"
        w = int(words[i, ks[0], f])
        want_src = 0
        for r in s["list2"][i, :s["count2"][i]]:
            want_src |= 1 << int(r[0])
        assert w & 0xFFFFFF == want_src and (w >> 24) & 7 == int(s["roll2"][i]), f"case {i}"


def _step_plays_oracle(board, off, ft, player, dice):
    """narde_env.py:45-93 restated over the C oracle's primitives: the set of
    plays the step carries out (as Narde.get_valid_plays)."""
    roll = np.array([[dice[0], dice[1], 0, 0]], np.uint8)
    mv, cnt = O.legal_moves(board[None], ft[None], np.array([player], np.int8), roll, np.array([2], np.uint8))
    first = []
    for r in mv[0, :cnt[0]]:
        m = (int(r[0]), int(r[1]))
        if m not in first:
            first.append(m)
    if cnt[0] <= 1:
        return {((first[0][0], "off" if first[0][1] == 24 else first[0][1]),)} if cnt[0] else set()
    plays = set()
    for f, t in first:
        b, o, ft2 = O.apply_move(board[None], off[None], ft[None], np.array([player], np.int8),
                                 np.array([[f, t]], np.int8))
        dist = f + 1 if t == 24 else abs(f - t)
        rest = [int(dice[0]), int(dice[1])]
        if dist in rest:
            rest.remove(dist)
        else:
            rest.pop(0)
        mv2, c2 = O.legal_moves(b, ft2, np.array([player], np.int8), np.array([[rest[0], 0, 0, 0]], np.uint8),
                                np.array([1], np.uint8))
        m1 = (f, "off" if t == 24 else t)
        if c2[0] == 0:
            plays.add((m1,))
        for r in mv2[0, :c2[0]]:
            plays.add((m1, (int(r[0]), "off" if int(r[1]) == 24 else int(r[1]))))
    return plays


@pytest.mark.parametrize("kind_seed", [0])
def test_step_kind_equals_oracle_restatement(hostcheck, kind_seed):
    s = golden("steps.npz")
    rng = np.random.default_rng(kind_seed)
    idx = rng.choice(s["board"].shape[0], 4000, replace=False)
    legal, words, count = _play_set(hostcheck, s["board"][idx], s["off"][idx], s["first_turn"][idx],
                                    s["player"][idx], s["dice"][idx], 1)
    for j, i in enumerate(idx):
        want = _step_plays_oracle(s["board"][i], s["off"][i], s["first_turn"][i], int(s["player"][i]), s["dice"][i])
        got = _decode(legal[j], words[j], "step")
        assert got == want, f"case {i}"
        assert count[j] == len(want), f"case {i}"


def test_bad_dice_give_no_play(hostcheck):
    s = golden("steps.npz")
    d = np.array([[0, 3], [7, 1]], np.uint8)
    legal, words, count = _play_set(hostcheck, s["board"][:2], s["off"][:2], s["first_turn"][:2], s["player"][:2], d, 0)
    assert not legal.any() and not words.any() and not count.any()


def test_in_act_plays_helper(hostcheck):
    """conftest.in_act_plays (the GPU tests' vectorised membership check)
    against the reference's recorded combination lists: every recorded
    combination is a member, codes outside the list are not."""
    import torch

    from conftest import in_act_plays

    t = golden("trainer.npz")
    legal, words, count = _play_set(hostcheck, t["pre_board"], t["pre_off"], t["pre_ft"], t["player"], t["dice"], 0)
    starts = np.concatenate([[0], np.cumsum(t["combos_len"])])
    rng = np.random.default_rng(1)
    n = legal.shape[0]
    pick = np.zeros((n, 2), np.int64)
    for i in range(n):
        if count[i]:
            pick[i] = t["combos"][starts[i] + rng.integers(count[i])]
    args = (torch.from_numpy(legal.view(np.int64)), torch.from_numpy(words), torch.from_numpy(count))
    assert bool(in_act_plays(*args, torch.from_numpy(pick)).all())
    # random code pairs: members exactly when the recorded list holds them
    rnd = rng.integers(0, 576, (n, 2))
    got = in_act_plays(*args, torch.from_numpy(rnd)).numpy()
    for i in range(n):
        want = any(tuple(r) == tuple(rnd[i]) for r in t["combos"][starts[i]:starts[i + 1]])
        assert got[i] == want, f"step {i}"
    sel = np.nonzero(count > 0)[0]
    bad = pick.copy()
    bad[sel, 1] = (bad[sel, 1] + 1) % 576  # a neighbouring code is (almost always) not a member
    member = [any(tuple(r) == tuple(bad[i]) for r in t["combos"][starts[i]:starts[i + 1]]) for i in sel]
    assert np.array_equal(in_act_plays(*args, torch.from_numpy(bad)).numpy()[sel], np.array(member))


def _act_masks(hc, t, rows, move1=None):
    n = len(rows)
    c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
    b, o, f, p, d = (c(t["pre_board"][rows], np.int8), c(t["pre_off"][rows], np.uint8),
                     c(t["pre_ft"][rows], np.uint8), c(t["player"][rows], np.int8), c(t["dice"][rows], np.uint8))
    m = np.zeros((n, 9), np.uint64)
    mv = None if move1 is None else c(move1, np.int16)
    hc.hc_act_masks(ctypes.c_int64(n), P(b), P(o), P(f), P(p), P(d), None if mv is None else P(mv), P(m))
    return m


def _expand(m):
    return np.unpackbits(m.view(np.uint8).reshape(m.shape[0], 72), axis=1, bitorder="little")[:, :576].astype(bool)


def test_act_greedy_masks_reproduce_reference_act(hostcheck):
    """narde_rules.h act_masks (k_act_masks' per-lane body): with the Q-values
    the reference's DQNAgent.act was given (tests/golden/act_greedy.npz,
    tools/capture_act_greedy.py), the masked argmax over act_masks' move-1
    codes, then over its move-2 codes for that move 1, picks exactly the
    reference's greedy (move1, move2) -- act()'s candidate sets
    (valid_first_moves' keys; valid_first_moves[move1], pre-move lists)."""
    t = golden("trainer.npz")
    a = golden("act_greedy.npz")
    rows = a["step"]
    tab = np.random.default_rng(int(a["meta"][2])).standard_normal((576, 576)).astype(np.float32)
    q1 = np.stack([np.random.default_rng(int(a["meta"][0]) + int(i)).standard_normal(576).astype(np.float32)
                   for i in rows])
    b2 = np.stack([np.random.default_rng(int(a["meta"][1]) + int(i)).standard_normal(576).astype(np.float32)
                   for i in rows])
    m1 = _expand(_act_masks(hostcheck, t, rows))
    pick1 = np.where(m1, q1, -np.inf).argmax(1)
    assert np.array_equal(pick1, a["action"][:, 0])
    m2 = _expand(_act_masks(hostcheck, t, rows, move1=pick1))
    q2 = b2 + tab[pick1]
    pick2 = np.where(m2, q2, -np.inf).argmax(1)
    assert np.array_equal(pick2, a["action"][:, 1])
    assert m2.any(1).all()  # act() always offers a move 2 (code 0 when none)


def _act_combos_oracle(board, off, ft, player, dice):
    """DQNAgent.act's valid_move_combinations (train_deepq_pytorch.py:430-507)
    restated over the C oracle's get_valid_moves."""
    roll = np.array([[dice[0], dice[1], 0, 0]], np.uint8)
    mv, cnt = O.legal_moves(board[None], ft[None], np.array([player], np.int8), roll, np.array([2], np.uint8))
    combos = []
    for r in mv[0, :cnt[0]]:
        f1, t1 = int(r[0]), int(r[1])
        c1 = f1 * 24 + (0 if t1 == 24 else t1)
        temp = [int(dice[0]), int(dice[1])]
        if t1 == 24:
            match = next((d for d in temp if d >= f1 + 1), None)
            if match is None:
                match = max(temp)
        else:
            match = next((d for d in temp if d == f1 - t1), temp[0])
        temp.remove(match)
        mv2, c2 = O.legal_moves(board[None], ft[None], np.array([player], np.int8),
                                np.array([[temp[0], 0, 0, 0]], np.uint8), np.array([1], np.uint8))
        if c2[0] == 0:
            combos.append((c1, 0))
        for q in mv2[0, :c2[0]]:
            combos.append((c1, int(q[0]) * 24 + (0 if int(q[1]) == 24 else int(q[1]))))
    return combos


def test_play_sets_on_random_positions(hostcheck):
    """Both kinds on 3,000 random run-heavy and bear-off positions (random
    mover, first-turn flags, two-dice rolls including doubles) against
    restatements over the C oracle: act()'s list element for element, the
    step's set as a set."""
    from fuzz_positions import random_positions

    board, off, ft, player, rng = random_positions(3000, 11)
    dice = rng.integers(1, 7, size=(3000, 2)).astype(np.uint8)
    la, wa, ca = _play_set(hostcheck, board, off, ft, player, dice, 0)
    ls, ws, cs = _play_set(hostcheck, board, off, ft, player, dice, 1)
    for i in range(3000):
        want = _act_combos_oracle(board[i], off[i], ft[i], int(player[i]), dice[i])
        assert _decode(la[i], wa[i], "act") == want, f"act {i}"
        assert ca[i] == len(want)
        want_s = _step_plays_oracle(board[i], off[i], ft[i], int(player[i]), dice[i])
        assert _decode(ls[i], ws[i], "step") == want_s, f"step {i}"
        assert cs[i] == len(want_s)
