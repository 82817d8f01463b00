"""GPU parity of the FULL4 rules mode (whole turns: 4-move doubles, max dice
used) through libnarde.so's C ABI.

Against tests/golden/full4.npz (turns composed of the reference's own
single-die primitives by tools/capture_full4.py) and against the C oracle's
FULL4 self-play driver.  Bit-exact (integer work).  Whole-turn semantics have
no reference arithmetic (the reference env stops after two checker moves,
narde_env.py:45-93): parity of each sub-move is pinned, the composition rule
is the build's.
"""
import numpy as np
import pytest
from conftest import golden

import oracle as O
import replay as R
from bench import available_cores

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

THREADS = available_cores()[0]  # the oracle replay's thread pool (oracle/replay.py)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def vec(n, **kw):
    from gym_narde.vector import VecNardeEnv

    return VecNardeEnv(n, device="cuda:0", rules="full4", **kw)


def np_(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def golden_legal_word(d):
    hi = np.maximum(d["dice"][:, 0], d["dice"][:, 1]).astype(np.uint64)
    lo = np.minimum(d["dice"][:, 0], d["dice"][:, 1]).astype(np.uint64)
    c = d["cmask"][:, 0, :].astype(np.uint64)
    return (c[:, 0] | (c[:, 1] << np.uint64(24)) | (hi << np.uint64(48)) | (lo << np.uint64(52))
            | (d["max_dice"].astype(np.uint64) << np.uint64(56)))


def played_word(played):
    b = played.astype(np.uint8).astype(np.uint64)
    v = np.zeros(len(played), np.uint64)
    for k in range(4):
        v |= (b[:, k, 0] | (b[:, k, 1] << np.uint64(8))) << np.uint64(16 * k)
    return v


def set_golden(env, d):
    env.set_state(torch.from_numpy(d["board"]), torch.from_numpy(d["off"]),
                  torch.from_numpy(d["ft"]), torch.from_numpy(d["player"]))


def test_full4_legal_first_golden():
    d = golden("full4.npz")
    env = vec(len(d["dice"]))
    set_golden(env, d)
    w = env.legal_full(torch.from_numpy(d["dice"]))
    assert np.array_equal(np_(w).view(np.uint64), golden_legal_word(d))
    # the query applies nothing
    assert np.array_equal(np_(env.get_state()["board"]), d["board"])


def test_full4_step_replays_golden_plays():
    """Explicit plays = the golden sub-moves: same post-turn state."""
    d = golden("full4.npz")
    n = len(d["dice"])
    env = vec(n, max_episode_steps=0, autoreset=False)
    set_golden(env, d)
    obs, rew, term, trunc, info = env.step(torch.from_numpy(d["played"]),
                                           torch.from_numpy(d["dice"]))
    assert np.array_equal(np_(info["legal"]).view(np.uint64), golden_legal_word(d))
    assert np.array_equal(np_(info["played"]).view(np.uint64), played_word(d["played"]))
    assert np.array_equal(np_(rew), d["reward"].astype(np.int32))
    assert np.array_equal(np_(term), d["done"])
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), d["board_after"])
    assert np.array_equal(np_(st["off"]), d["off_after"])
    assert np.array_equal(np_(st["first_turn"]), d["ft_after"])
    # the mover flips unless the game ended (narde_env.py:96-100)
    exp_player = np.where(d["done"] == 1, d["player"], -d["player"]).astype(np.int8)
    assert np.array_equal(np_(st["player"]), exp_player)


def test_full4_illegal_play_is_ignored():
    d = golden("full4.npz")
    n = len(d["dice"])
    env = vec(n, max_episode_steps=0, autoreset=False)
    set_golden(env, d)
    bad = np.full((n, 4, 2), -1, np.int8)
    bad[:, 0, 0] = 30  # not a point: the turn ends before any sub-move
    _, _, term, _, info = env.step(torch.from_numpy(bad), torch.from_numpy(d["dice"]))
    assert (np_(info["played"]).view(np.uint64) == np.uint64(0xFFFFFFFFFFFFFFFF)).all()
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), d["board"])
    assert not np_(term).any()


@pytest.mark.parametrize("dice_mode,max_steps", [("all36", 1000), ("nodoubles", 1000), ("all36", 80)])
def test_full4_selfplay_trajectory_vs_oracle(dice_mode, max_steps):
    n, plies, seed, env0 = 4096, 200, 0xF4F4F4, 999
    dm = 0 if dice_mode == "all36" else 1
    env = vec(n, seed=seed, env_id_offset=env0, dice_mode=dice_mode, max_episode_steps=max_steps)
    ref = O.SelfPlay(n, seed=seed, env0=env0, dice_mode=dm, max_steps=max_steps)
    ref.reset(0)
    rec = ref.run_full(plies)
    for p in range(plies):
        assert np.array_equal(np_(env.dice()), rec["dice"][p]), p
        obs, rew, term, trunc, info = env.step()
        assert np.array_equal(np_(obs), rec["obs"][p].astype(np.int32)), p
        assert np.array_equal(np_(rew), rec["reward"][p].astype(np.int32)), p
        assert np.array_equal(np_(term), rec["terminated"][p]), p
        assert np.array_equal(np_(trunc), rec["truncated"][p]), p
        assert np.array_equal(np_(info["legal"]).view(np.uint64), rec["legal"][p]), p
        assert np.array_equal(np_(info["played"]).view(np.uint64), rec["played"][p]), p
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), ref.board)
    assert np.array_equal(np_(env.stats()), ref.stats)


@pytest.mark.parametrize("max_steps", [1000, 30])
def test_full4_rollout_equals_steps(max_steps):
    """narde_rollout_full over launch boundaries == per-ply k_step<full>:
    launches of 1, 29, 70 and 100 plies (k_rollout_pp_full), ragged odd n (the
    last workgroup partly empty, odd plies' rows not 64-B aligned); with
    TimeLimit 30 every env truncates several times inside the launches."""
    n, seed = 2048 + 77, 31337
    a = vec(n, seed=seed, max_episode_steps=max_steps)
    b = vec(n, seed=seed, max_episode_steps=max_steps)
    bufs = a.rollout_buffers(100)
    got = {k: [] for k in bufs}
    for plies in (1, 29, 70, 100):
        a.rollout(plies, bufs)
        for k, v in bufs.items():
            got[k].append(np_(v[:plies]).copy())
    got = {k: np.concatenate(v) for k, v in got.items()}
    for p in range(200):
        obs, rew, term, trunc, info = b.step()
        assert np.array_equal(got["obs"][p], np_(obs)), p
        assert np.array_equal(got["reward"][p], np_(rew)), p
        assert np.array_equal(got["terminated"][p], np_(term)), p
        assert np.array_equal(got["truncated"][p], np_(trunc)), p
        assert np.array_equal(got["legal"][p], np_(info["legal"])), p
        assert np.array_equal(got["actions"][p], np_(info["played"])), p
    assert np.array_equal(np_(a.stats()), np_(b.stats()))
    if max_steps == 30:
        assert got["truncated"].sum() > n  # truncations inside the rollout launches


def test_full4_rollout_ring_boundaries():
    """k_rollout_pp_full launches at the edges of its hand-over: lengths
    around the LDS ring depth (kPpR = 8 plies: 7, 8, 9, 16, 17; the consumer
    draws min(8, plies) ahead) and on both sides of the store-policy switch
    (32 plies non-temporal, 33 plain), n = 300 (a full workgroup and a
    partial one) == per-ply k_step<full>, entry by entry."""
    n, seed = 300, 4242
    lens = (7, 8, 9, 16, 17, 32, 33)
    a = vec(n, seed=seed)
    b = vec(n, seed=seed)
    bufs = a.rollout_buffers(max(lens))
    got = {k: [] for k in bufs}
    for plies in lens:
        a.rollout(plies, bufs)
        for k, v in bufs.items():
            got[k].append(np_(v[:plies]).copy())
    got = {k: np.concatenate(v) for k, v in got.items()}
    for p in range(sum(lens)):
        obs, rew, term, trunc, info = b.step()
        assert np.array_equal(got["obs"][p], np_(obs)), p
        assert np.array_equal(got["reward"][p], np_(rew)), p
        assert np.array_equal(got["terminated"][p], np_(term)), p
        assert np.array_equal(got["truncated"][p], np_(trunc)), p
        assert np.array_equal(got["legal"][p], np_(info["legal"])), p
        assert np.array_equal(got["actions"][p], np_(info["played"])), p
    assert np.array_equal(np_(a.stats()), np_(b.stats()))


@pytest.mark.parametrize("plies,seed", [(120, 7), (20, 0)])
def test_full4_full_batch_vs_oracle_and_invariants(plies, seed):
    """B = 65,536 (the bench shape; 120-ply launches, and the driver's 20-ply
    launch at the bench's seed 0 and env ids 0..65,535; k_rollout_pp_full):
    EVERY env's every output and final state equal the C oracle replaying
    the launch (oracle/replay.py, the bench's parity_check leg); checker
    conservation and played == max dice everywhere."""
    n = 65536
    env = vec(n, seed=seed)
    bufs = env.rollout_buffers(plies)
    before = R.snapshot(env)
    env.rollout(plies, bufs)
    after = R.snapshot(env)
    res = R.check(before, {k: np_(v) for k, v in bufs.items()}, after, plies, seed, full=True,
                  threads=THREADS)
    assert res["mismatches"] == 0 and res["envs"] == n, res
    b = after["board"].astype(np.int64)
    off = after["off"].astype(np.int64)
    assert ((np.where(b > 0, b, 0).sum(1) + off[:, 0]) == 15).all()
    assert ((np.where(b < 0, -b, 0).sum(1) + off[:, 1]) == 15).all()
    legal = np_(bufs["legal"]).view(np.uint64)
    played = np_(bufs["actions"]).view(np.uint64)
    M = (legal >> np.uint64(56)).astype(np.int64)
    nplayed = sum((((played >> np.uint64(16 * k)) & np.uint64(0xFF)) != np.uint64(0xFF)).astype(np.int64)
                  for k in range(4))
    assert np.array_equal(nplayed, M)
    assert (M == 4).mean() > 0.08


def test_full4_steady_state_full_batch_after_selfplay():
    """The driver's 20-ply launch at B = 65,536 in the steady state (300
    plies of stats-only self-play first: the envs spread over every game
    phase, so block-bound two-dice and doubles turns, the failing-window
    loops per kind and the doubles search all occur in every launch,
    tools/diag/wave_kinds.cpp): every env's outputs and final state equal
    the oracle replaying the launch from the state before it."""
    n, seed, pre, plies = 65536, 11, 300, 20
    env = vec(n, seed=seed)
    env.selfplay(pre)
    bufs = env.rollout_buffers(plies)
    before = R.snapshot(env)
    env.rollout(plies, bufs)
    res = R.check(before, {k: np_(v) for k, v in bufs.items()}, R.snapshot(env), plies, seed, full=True,
                  threads=THREADS)
    assert res["mismatches"] == 0 and res["envs"] == n, res


@pytest.mark.parametrize("n", [1, 63, 65])
def test_tiny_batches_both_rules_both_kernels(n):
    """One env, one wave less one lane, one wave plus one lane: REF2 rollouts
    of 20 plies (k_rollout_pc<true>: 2-ply barrier blocks) and 60 plies
    (4-ply blocks), FULL4 rollouts of 20 and 60 plies (k_rollout_pp_full)
    equal the oracle ply for ply."""
    from gym_narde.vector import VecNardeEnv

    seed, env0 = 4242, 3
    for rules in ("ref2", "full4"):
        env = VecNardeEnv(n, device="cuda:0", seed=seed, env_id_offset=env0, rules=rules)
        ref = O.SelfPlay(n, seed=seed, env0=env0)
        ref.reset(0)
        for plies in (20, 60):
            bufs = env.rollout(plies)
            rec = ref.run_full(plies) if rules == "full4" else ref.run(plies)
            assert np.array_equal(np_(bufs["obs"]), rec["obs"].astype(np.int32)), (rules, plies)
            assert np.array_equal(np_(bufs["reward"]), rec["reward"].astype(np.int32)), (rules, plies)
            assert np.array_equal(np_(bufs["terminated"]), rec["terminated"]), (rules, plies)
            if rules == "full4":
                assert np.array_equal(np_(bufs["actions"]).view(np.uint64), rec["played"]), plies
            else:
                assert np.array_equal(np_(bufs["actions"]), rec["action"]), plies
        st = env.get_state()
        assert np.array_equal(np_(st["board"]), ref.board), rules
        assert np.array_equal(np_(env.stats()), ref.stats), rules
