"""Pin the CPU oracle (and the Python port) to the reference's golden vectors.

The fixtures in tests/golden/ were produced by tools/capture_golden.py, which
imports the reference from /root/reference and drives it with injected dice.
Also diffs the test-only host build of the device rules engine
(tests/hostcheck) against the same fixtures and against the oracle's
self-play -- a CPU pre-check of the bitmask formulation; the GPU parity tests
are in test_gpu_parity.py.
"""
import ctypes
import random

import numpy as np
import pytest
from conftest import golden

import oracle as O
import narde_port as port

P = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None  # noqa: E731


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    assert O.philox((0, 0, 0, 0), (0, 0)) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert O.philox((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2) == (
        0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)
    assert O.philox((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == (
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


def test_oracle_legal_moves_golden():
    d = golden("legal.npz")
    m, c = O.legal_moves(d["board"], d["first_turn"], d["player"], d["roll"], d["nroll"])
    assert np.array_equal(c, d["count"])
    assert np.array_equal(m, d["moves"])


def test_oracle_known_answers_appendix_b():
    d = golden("legal.npz")
    k = int(d["n_kat"])
    lists = [[tuple(x) for x in d["moves"][i][: d["count"][i]].tolist()] for i in range(k)]
    assert lists[0] == [(23, 18)]                       # start, [5,3]
    assert lists[2] == [(23, 17), (23, 17)]             # start, [6,6] first turn: 2 head moves
    assert lists[5] == [(23, 18)]                       # [5,5] is not a head-exception double
    assert lists[7] == [(23, 18)]                       # 4-die roll: never special
    assert lists[11] == [(0, 24), (2, 24), (3, 0), (0, 24), (2, 1), (3, 2)]
    assert lists[13] == [(3, 0), (4, 1), (6, 3), (23, 20), (1, 0), (2, 1), (3, 2), (4, 3)]


def test_oracle_block_rule_golden():
    d = golden("block.npz")
    assert np.array_equal(O.violates_block_rule(d["board"]), d["violates"])
    assert 0.05 < d["violates"].mean() < 0.95  # both outcomes covered


def test_oracle_apply_golden():
    d = golden("apply.npz")
    b, o, f = O.apply_move(d["board"], d["off"], d["first_turn"], d["player"], d["move"])
    assert np.array_equal(b, d["post_board"])
    assert np.array_equal(o, d["post_off"])
    assert np.array_equal(f, d["post_first_turn"])


def test_oracle_step_golden():
    s = golden("steps.npz")
    r = O.step(s["board"], s["off"], s["first_turn"], s["player"], s["dice"], s["action"])
    for mine, ref in [("board", "post_board"), ("off", "post_off"), ("first_turn", "post_first_turn"),
                      ("player", "post_player"), ("obs", "obs"), ("reward", "reward"),
                      ("terminated", "terminated"), ("count1", "count1"), ("list1", "list1"),
                      ("count2", "count2"), ("list2", "list2")]:
        assert np.array_equal(r[mine], s[ref]), mine
    made = s["count2"] >= 0
    assert np.array_equal(r["roll2"][made], s["roll2"][made])
    # coverage of the branches the fixtures must exercise
    assert (s["count1"] == 0).any() and (s["count1"] == 1).any() and (s["count1"] >= 2).any()
    assert (s["terminated"] == 1).sum() > 50 and (s["reward"] == 2).any()
    assert (s["ncalls"] == 2).any()


def test_oracle_compact_legal_is_the_reference_list():
    """The oracle's compact list-#1 word (or_compact2, built from its own list
    and the die loop each entry came from) expands back to the reference's
    list #1 for every golden step, entry by entry: comparing the device's
    compact words with the oracle's is comparing the lists themselves."""
    s = golden("steps.npz")
    r = O.step(s["board"], s["off"], s["first_turn"], s["player"], s["dice"], s["action"])
    moves, count = O.expand_compact(r["legal1"])
    assert np.array_equal(count, s["count1"])
    assert np.array_equal(moves, s["list1"])
    # the self-play driver records the same word
    sp = O.SelfPlay(512, seed=77)
    sp.reset(0)
    rec = sp.run(300)
    m, c = O.expand_compact(rec["legal"])
    assert np.array_equal(c.reshape(300, 512), rec["count1"])
    # doubles lists (duplicate entries, the head filter on the second die) are covered
    dice = rec["dice"]
    assert ((dice[..., 0] == dice[..., 1]) & (rec["count1"] >= 2)).any()


def _port_state(b, off, ft, pl):
    e = port.PortEnv()
    g = e.game
    g.board = b.astype(np.int32).copy()
    g.borne_off_white, g.borne_off_black = int(off[0]), int(off[1])
    g.first_turn_white, g.first_turn_black = bool(ft[0]), bool(ft[1])
    e.current_player = int(pl)
    return e


def test_port_step_golden_sample():
    s = golden("steps.npz")
    idx = np.random.RandomState(0).choice(len(s["dice"]), 3000, replace=False)
    idx = np.concatenate([idx, np.arange(len(s["dice"]) - 4, len(s["dice"]))])  # quirk rows
    for i in idx:
        e = _port_state(s["board"][i], s["off"][i], s["first_turn"][i], s["player"][i])
        obs, rew, done = e.step([int(x) for x in s["dice"][i]], [int(x) for x in s["action"][i]])
        assert np.array_equal(e.game.board, s["post_board"][i].astype(np.int32)), i
        assert (e.game.borne_off_white, e.game.borne_off_black) == tuple(s["post_off"][i]), i
        assert e.current_player == s["post_player"][i], i
        assert np.array_equal(obs, s["obs"][i].astype(np.int32)), i
        assert (rew, done) == (s["reward"][i], bool(s["terminated"][i])), i


def test_port_legal_golden_sample():
    d = golden("legal.npz")
    idx = np.random.RandomState(1).choice(len(d["count"]), 3000, replace=False)
    g = port.PortNarde()
    for i in idx:
        g.board = d["board"][i].astype(np.int32)
        g.first_turn_white, g.first_turn_black = bool(d["first_turn"][i][0]), bool(d["first_turn"][i][1])
        roll = [int(x) for x in d["roll"][i][: d["nroll"][i]]]
        mv = g.get_valid_moves(roll, int(d["player"][i]))
        ref = [(int(f), "off" if t == 24 else int(t)) for f, t in d["moves"][i][: d["count"][i]]]
        assert mv == ref, i


def test_port_selfplay_runs():
    steps, secs, eps = port.selfplay_port(8, plies=300, seed=3)
    assert steps == 2400 and eps > 0


# ---------------------------------------------------------------- hostcheck
def test_hostcheck_legal_golden(hostcheck):
    d = golden("legal.npz")
    n = len(d["count"])
    moves = np.empty((n, 64, 2), np.int8)
    cnt = np.empty(n, np.int16)
    hostcheck.hc_legal_batch(ctypes.c_int64(n), P(d["board"]), P(d["off"]), P(d["first_turn"]),
                             P(d["player"]), P(np.ascontiguousarray(d["roll"])), P(moves), P(cnt))
    assert np.array_equal(cnt, d["count"])
    assert np.array_equal(moves, d["moves"])


def test_hostcheck_step_golden(hostcheck):
    s = golden("steps.npz")
    n = len(s["dice"])
    b, off, ft, pl = (s["board"].copy(), s["off"].copy(), s["first_turn"].copy(), s["player"].copy())
    obs = np.empty((n, 24), np.int8)
    rw = np.empty(n, np.int8)
    tm = np.empty(n, np.uint8)
    l1 = np.empty((n, 64, 2), np.int8)
    c1 = np.empty(n, np.int16)
    l2 = np.empty((n, 64, 2), np.int8)
    c2 = np.empty(n, np.int16)
    hostcheck.hc_step_batch(ctypes.c_int64(n), P(b), P(off), P(ft), P(pl), P(s["dice"]), P(s["action"]),
                            P(obs), P(rw), P(tm), P(l1), P(c1), P(l2), P(c2))
    for a, ref in [(b, "post_board"), (off, "post_off"), (ft, "post_first_turn"), (pl, "post_player"),
                   (obs, "obs"), (rw, "reward"), (tm, "terminated"), (c1, "count1"), (l1, "list1"),
                   (c2, "count2"), (l2, "list2")]:
        assert np.array_equal(a, s[ref]), ref


@pytest.mark.parametrize("fn,max_steps", [("hc_selfplay", 1000), ("hc_selfplay_sl", 1000), ("hc_selfplay_sl", 130)])
@pytest.mark.parametrize("dice_mode", [0, 1])
def test_hostcheck_selfplay_vs_oracle(hostcheck, dice_mode, fn, max_steps):
    """The host build of the device's REF2 ply -- env_ply, and the rollouts'
    straight-line env_ply_policy_sl (round 4) -- equals the oracle's
    self-play on every per-ply output, the compact list-#1 words included."""
    n, plies, seed, env0 = 512, 400, 0xDEADBEEF12345, 1000
    sp = O.SelfPlay(n, seed=seed, env0=env0, dice_mode=dice_mode, max_steps=max_steps)
    sp.reset(0)
    ro = sp.run(plies)
    b = np.zeros((n, 24), np.int8)
    off = np.zeros((n, 2), np.uint8)
    ft = np.zeros((n, 2), np.uint8)
    pl = np.zeros(n, np.int8)
    el = np.zeros(n, np.uint16)
    st = np.zeros((n, 3), np.int32)
    hostcheck.hc_reset_batch(ctypes.c_int64(n), ctypes.c_int64(env0), ctypes.c_uint64(seed),
                             ctypes.c_uint32(0), P(b), P(off), P(ft), P(pl), P(el))
    out = {k: np.empty_like(v) for k, v in ro.items()}
    getattr(hostcheck, fn)(ctypes.c_int64(n), ctypes.c_int64(env0), ctypes.c_uint64(seed),
                          ctypes.c_uint32(0), ctypes.c_int(plies), ctypes.c_int(dice_mode),
                          ctypes.c_int(max_steps), P(b), P(off), P(ft), P(pl), P(el), P(st),
                          P(out["obs"]), P(out["reward"]), P(out["terminated"]), P(out["truncated"]),
                          P(out["dice"]), P(out["action"]), P(out["count1"]), P(out["legal"]))
    for k in ro:
        assert np.array_equal(out[k], ro[k]), k
    assert np.array_equal(st, sp.stats) and np.array_equal(b, sp.board)
    assert sp.stats[:, 0].sum() > 0


def test_oracle_selfplay_invariants():
    n = 256
    sp = O.SelfPlay(n, seed=7, max_steps=130)  # short TimeLimit -> truncations too
    sp.reset(0)
    r = sp.run(300)
    assert r["truncated"].any() and r["terminated"].any()
    # checker conservation: 15 per colour on board + off, no mixed points
    w = np.where(sp.board > 0, sp.board, 0).sum(1) + sp.off[:, 0]
    k = np.where(sp.board < 0, -sp.board, 0).sum(1) + sp.off[:, 1]
    assert (w == 15).all() and (k == 15).all()
    # codes used are legal action codes or 0
    assert ((r["action"] >= 0) & (r["action"] < 576)).all()


def test_oracle_tesauro_bounds():
    d = golden("steps.npz")
    t = O.tesauro198(d["post_board"], d["post_off"], d["post_player"])
    hi = np.ones(198, np.float32)
    hi[[3 + 4 * p for p in range(24)]] = 6.0
    hi[[101 + 4 * p for p in range(24)]] = 6.0
    hi[96] = hi[194] = 7.5
    assert (t >= 0).all() and (t <= hi).all()  # tests/test_observation_space.py:37-234 bounds
    assert np.allclose(t[:, 196] + t[:, 197], 1.0)
    # white block decodes back to the board
    w = t[:, 0:96].reshape(-1, 24, 4)
    cnt = w[..., 0] + w[..., 1] + w[..., 2] + 2 * w[..., 3]
    assert np.array_equal(cnt.astype(np.int64), np.where(d["post_board"] > 0, d["post_board"], 0))
    random.seed(0)



def _prime_boards(n, seed):
    """Random legal positions biased toward 4-5-point own runs with single
    checkers around them: where the block rule's window completion (and its
    single-checker source exception) decides legality.  White moves from
    perspective point 23 down; +counts white, -counts black."""
    rng = np.random.default_rng(seed)
    boards = np.zeros((n, 24), np.int8)
    for i in range(n):
        b = boards[i]
        own = 15
        start = int(rng.integers(0, 20))
        length = int(rng.integers(4, 6))
        for p in range(start, min(24, start + length)):
            c = int(rng.integers(1, 3))
            b[p] = c
            own -= c
        while own > 0:
            p = int(rng.integers(0, 24))
            if b[p] >= 0:
                b[p] += 1
                own -= 1
        opp = 15
        free = np.nonzero(b == 0)[0]
        k = int(rng.integers(1, 5))
        pts = rng.choice(free, size=min(k, len(free)), replace=False)
        for j, p in enumerate(pts):
            c = opp if j == len(pts) - 1 else int(rng.integers(1, opp - (len(pts) - 1 - j) + 1))
            b[p] = -c
            opp -= c
            if opp == 0:
                break
    return boards


def test_hostcheck_legal_random_prime_boards(hostcheck):
    """The bitmask engine's lists (incl. the branch-free block filter) equal
    the oracle's on 20,000 random run-heavy positions and every roll of one
    and two dice."""
    n = 20000
    boards = _prime_boards(n, 7)
    assert (np.where(boards > 0, boards, 0).sum(1) == 15).all()
    assert (np.where(boards < 0, -boards, 0).sum(1) == 15).all()
    rng = np.random.default_rng(8)
    roll4 = np.zeros((n, 4), np.uint8)
    nd = rng.integers(1, 3, n)
    roll4[:, 0] = rng.integers(1, 7, n)
    roll4[:, 1] = np.where(nd == 2, rng.integers(1, 7, n), 0)
    ft = np.zeros((n, 2), np.uint8)
    player = np.ones(n, np.int8)
    off = np.zeros((n, 2), np.uint8)
    ref_moves, ref_cnt = O.legal_moves(boards, ft, player, roll4, nd.astype(np.uint8))
    moves = np.empty((n, 64, 2), np.int8)
    cnt = np.empty(n, np.int16)
    hostcheck.hc_legal_batch(ctypes.c_int64(n), P(boards), P(off), P(ft), P(player), P(roll4), P(moves),
                             P(cnt))
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(moves, ref_moves)
    # the sample reaches the block rule: on one-die rolls, count the
    # positions where a plain candidate (own source, landing not on the
    # opponent, no bear-off) is missing from the list
    one = np.nonzero(nd == 1)[0]
    d = roll4[one, 0].astype(np.int64)
    b = boards[one].astype(np.int64)
    pts = np.arange(24)
    to = pts[None, :] - d[:, None]
    land = np.take_along_axis(b, np.clip(to, 0, 23), 1)
    cand = ((b > 0) & (to >= 0) & (land >= 0)).sum(1)
    normal = ((ref_moves[one, :, 1] != 24) & (np.arange(64)[None, :] < ref_cnt[one, None])).sum(1)
    assert (normal <= cand).all()
    assert int((normal < cand).sum()) > 200


def test_oracle_replays_trainer_fixture_steps():
    """The oracle's NardeEnv.step on every step the reference trainer loop
    took (tests/golden/trainer.npz: pre-step state, the env's own roll, the
    trainer's action): observation, reward and end equal the reference's;
    and where the trainer's own roll had no move, its block-rule probes on
    mutated boards (train_deepq_pytorch.py:1066-1076) equal the oracle's
    _violates_block_rule."""
    d = golden("trainer.npz")
    r = O.step(d["pre_board"], d["pre_off"], d["pre_ft"], d["player"], d["env_dice"], d["action"],
               with_lists=False)
    assert np.array_equal(r["obs"], d["obs"])
    assert np.array_equal(r["reward"].astype(np.int64), d["reward"].astype(np.int64))
    assert np.array_equal(r["terminated"], d["done"] & ~d["truncated"].astype(bool))
    # shaping as the reference computes it, from the oracle's post-step state
    # (float64, train_deepq_pytorch.py:892-912)
    assert (d["shaped"] >= d["reward"]).all()
    assert len(d["blocks"]) == int(d["blocks_len"].sum()) > 0


def test_hostcheck_step_policy_straight_line_random(hostcheck):
    """env_step_policy_sl (the rollouts' straight-line REF2 step) equals
    env_step with the random-legal policy on random run-heavy, head-heavy
    and bear-off positions: state, both lists, codes, reward, end."""
    f = hostcheck.hc_step_sl_random
    f.restype = ctypes.c_int64
    nb = ctypes.c_int64(0)
    assert f(ctypes.c_int64(300000), ctypes.c_uint32(5), ctypes.byref(nb)) == 0
    assert nb.value > 1000  # the block rule cuts list #1 often enough to matter
