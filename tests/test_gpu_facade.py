"""GPU: the scalar drop-in facade (gym_narde.envs) reproduces the reference.

Episodes in episodes.npz were recorded from the reference NardeEnv with
reset(seed=s) and a seeded random legal policy; the facade draws its dice
from numpy's global legacy RNG exactly like the reference, so replaying the
recorded actions after reset(seed=s) must reproduce every observation,
reward, termination and mover."""
import numpy as np
import pytest
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _moves(row, count):
    return [(int(f), "off" if t == 24 else int(t)) for f, t in row[:count]]


def test_episodes_replay_bit_exact():
    from gym_narde.envs import NardeEnv

    d = golden("episodes.npz")
    pos = 0
    for e, (seed, length) in enumerate(zip(d["seed"], d["length"])):
        env = NardeEnv()
        obs, info = env.reset(seed=int(seed))
        assert np.array_equal(obs, d["reset_obs"][e].astype(np.int32))
        assert env.current_player == d["reset_player"][e]
        for k in range(int(length)):
            st = np.random.get_state()
            dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
            np.random.set_state(st)
            assert dice == d["dice"][pos].tolist(), (e, k)
            obs, r, term, trunc, _ = env.step(tuple(int(x) for x in d["action"][pos]))
            assert np.array_equal(obs, d["obs"][pos].astype(np.int32)), (e, k)
            assert (r, term, trunc) == (int(d["reward"][pos]), bool(d["terminated"][pos]), False)
            assert env.current_player == d["player"][pos], (e, k)
            pos += 1
        assert term or length == 1000
    assert pos == len(d["action"])


def test_reset_draw_pattern():
    from gym_narde.envs import NardeEnv

    d = golden("resets.npz")
    env = NardeEnv()
    for s, pl, nxt in zip(d["seed"], d["player"], d["next_draw"]):
        env.reset(seed=int(s))
        assert env.current_player == pl
        assert np.random.randint(0, 2 ** 31 - 1) == nxt  # same number of RNG draws


def test_get_valid_moves_sample_incl_3_and_4_dice():
    from gym_narde.envs.narde import Narde

    d = golden("legal.npz")
    g = Narde()
    idx = list(range(int(d["n_kat"])))
    idx += list(np.random.RandomState(2).choice(len(d["count"]), 1500, replace=False))
    idx += list(np.nonzero(d["nroll"] >= 3)[0][:300])
    for i in idx:
        g.board = d["board"][i].astype(np.int32)
        g.borne_off_white, g.borne_off_black = int(d["off"][i][0]), int(d["off"][i][1])
        g.first_turn_white, g.first_turn_black = bool(d["first_turn"][i][0]), bool(d["first_turn"][i][1])
        roll = [int(x) for x in d["roll"][i][: d["nroll"][i]]]
        assert g.get_valid_moves(roll, int(d["player"][i])) == _moves(d["moves"][i], d["count"][i]), i


def test_reference_unit_tests_equivalent():
    """tests/test_move_validation.py:13-29 of the reference."""
    from gym_narde.envs.narde import Narde

    g = Narde()
    valid = g.get_valid_moves([3, 5], current_player=1)
    assert len(valid) > 0
    assert g.validate_move(valid[0], [3, 5], current_player=1)
    assert not g.validate_move((23, 20), [3, 5], current_player=1)  # smaller die's head move


def test_execute_rotated_move_and_block_rule():
    from gym_narde.envs.narde import Narde

    d = golden("apply.npz")
    g = Narde()
    for i in range(0, len(d["player"]), 37):
        g.board = d["board"][i].astype(np.int32)
        g.borne_off_white, g.borne_off_black = int(d["off"][i][0]), int(d["off"][i][1])
        g.first_turn_white, g.first_turn_black = bool(d["first_turn"][i][0]), bool(d["first_turn"][i][1])
        f, t = int(d["move"][i][0]), int(d["move"][i][1])
        g.execute_rotated_move((f, "off" if t == 24 else t), int(d["player"][i]))
        assert np.array_equal(g.board, d["post_board"][i].astype(np.int32)), i
        assert (g.borne_off_white, g.borne_off_black) == tuple(d["post_off"][i])
        assert (g.first_turn_white, g.first_turn_black) == tuple(bool(x) for x in d["post_first_turn"][i])
    b = golden("block.npz")
    for i in range(0, len(b["violates"]), 53):
        assert g._violates_block_rule(b["board"][i].astype(np.int32)) == bool(b["violates"][i])


def test_make_timelimit_truncates_at_1000():
    import gym_narde

    env = gym_narde.make("gym_narde:narde-v0")
    env.reset(seed=0)
    trunc = False
    for k in range(1000):
        _, _, term, trunc, _ = env.step((0, 0))  # (0,'off') is never legal early: no move
        if term:
            break
    assert trunc and k == 999


def test_observe_host_pinned():
    """f-4: observations land in pinned host memory, equal to the device ones."""
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(4096, device="cuda:0", seed=8)
    env.selfplay(17)
    host, ev = env.observe_host("int24")
    ev.synchronize()
    assert host.is_pinned() and torch.equal(host, env.observe().cpu())
    h2, ev2 = env.observe_host("tesauro198")
    ev2.synchronize()
    assert h2.is_pinned() and torch.equal(h2, env.tesauro198().cpu())
    h3, ev3 = env.observe_host("int24", out=host)  # reuse the pinned buffer
    ev3.synchronize()
    assert h3.data_ptr() == host.data_ptr()


def test_example_play_random_agent_runs():
    """configs[0] plumbing: the examples/play_random_agent.py counterpart
    plays whole games through gym_narde.make (both agent modes)."""
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(__file__), "..", "examples", "play_random_agent.py")
    spec = importlib.util.spec_from_file_location("play_random_agent", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    wins, lengths = mod.make_plays(games=3, seed=0, legal=True)
    assert len(lengths) == 3 and sum(wins.values()) + sum(1 for x in lengths if x >= 1000) >= 3
    wins, lengths = mod.make_plays(games=1, seed=1, legal=False)
    assert len(lengths) == 1


@pytest.mark.parametrize("rules", ["ref2", "full4"])
def test_timed_rollout_launcher(rules):
    """VecNardeEnv.rollout_launcher(events=...) -> narde_rollout_timed (the
    bench's timed launch): the same outputs and state as plain launches, the
    events bracket the launch on its stream; an event never recorded is
    refused."""
    from gym_narde.vector import VecNardeEnv

    n, plies = 4096, 24
    a = VecNardeEnv(n, device="cuda:0", seed=5, rules=rules)
    b = VecNardeEnv(n, device="cuda:0", seed=5, rules=rules)
    ba, bb = a.rollout_buffers(plies), b.rollout_buffers(plies)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with pytest.raises(ValueError):
        a.rollout_launcher(plies, ba, events=(e0, e1))
    e0.record()
    e1.record()
    timed = a.rollout_launcher(plies, ba, events=(e0, e1))
    plain = b.rollout_launcher(plies, bb)
    for _ in range(2):
        timed()
        plain()
    torch.cuda.synchronize()
    assert e0.elapsed_time(e1) > 0.0
    for k in ba:
        assert torch.equal(ba[k], bb[k]), k
    assert torch.equal(a.stats(), b.stats())
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    # the bench's timing-only events (narde_timing_event_*): the same launch
    from gym_narde.vector import TimingEvent

    t0, t1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    timed2 = a.rollout_launcher(plies, ba, events=(t0, t1))
    timed2()
    plain()
    torch.cuda.synchronize()
    assert t0.elapsed_ms(t1) > 0.0
    for k in ba:
        assert torch.equal(ba[k], bb[k]), k
    t0.close()
    t1.close()


def test_get_valid_plays_vs_reference_lists():
    """Narde.get_valid_plays / NardeEnv.get_valid_actions (the README's
    get_valid_actions) on 600 golden reference steps: the first moves are
    exactly the reference's list #1; for the move 1 the reference step played,
    the second moves are exactly the reference's list #2 after it (captured
    inside the reference step); a one-move list gives that move alone, an
    empty list no play."""
    from gym_narde.envs import NardeEnv
    from gym_narde.envs.narde import Narde

    d = golden("steps.npz")
    dec = lambda m: (int(m[0]), "off" if int(m[1]) == 24 else int(m[1]))  # noqa: E731
    rng = np.random.default_rng(5)
    seen = {0: 0, 1: 0, 2: 0}
    for i in rng.choice(len(d["board"]), 600, replace=False):
        g = Narde()
        g.board[:] = d["board"][i].astype(np.int32)
        g.borne_off_white, g.borne_off_black = (int(x) for x in d["off"][i])
        g.first_turn_white, g.first_turn_black = (bool(x) for x in d["first_turn"][i])
        player, dice = int(d["player"][i]), [int(x) for x in d["dice"][i]]
        plays = g.get_valid_plays(dice, player)
        list1 = [dec(m) for m in d["list1"][i][:d["count1"][i]]]
        seen[min(len(list1), 2)] += 1
        if not list1:
            assert plays == set()
            continue
        if len(list1) == 1:
            assert plays == {(list1[0],)}
            continue
        assert {p[0] for p in plays} == set(list1)
        if d["ncalls"][i] == 2:  # the recorded move 1 was legal: its list #2
            c1 = int(d["action"][i][0])
            m1 = (c1 // 24, "off" if (c1 % 24 == 0 and c1 // 24 <= 5) else c1 % 24)
            list2 = {dec(m) for m in d["list2"][i][:d["count2"][i]]}
            got = {p[1] for p in plays if p[0] == m1 and len(p) == 2}
            assert got == list2
            assert ((m1,) in plays) == (not list2)
    assert seen[2] > 300
    # the env method: the same set for the env's own position and player
    env = NardeEnv()
    env.reset(seed=3)
    assert env.get_valid_actions([6, 1]) == env.game.get_valid_plays([6, 1], env.current_player)
    # the start: one checker may leave the head, the higher die first
    # (narde.py:94-137), so list #1 holds one move and the step plays it alone
    assert env.get_valid_actions([6, 1]) == {((23, 17),)}


@pytest.mark.parametrize("n", [1, 37, 64, 65, 4099])
def test_totals_rows_equal_stats(n):
    """VecNardeEnv.totals() (narde_get_totals: 64 partial rows over
    contiguous env ranges) sums to stats(), for batches smaller than, equal
    to and just above the row count (rows past the last env are zero)."""
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(n, device="cuda:0", seed=n)
    env.selfplay(300)
    rows = env.totals()
    st = env.stats().to(torch.int64)
    assert rows.shape == (64, 3) and rows.dtype == torch.int64
    assert torch.equal(rows.sum(0), st.sum(0))
    per = -(-n // 64)
    for b in range(64):
        assert torch.equal(rows[b], st[b * per:min(n, (b + 1) * per)].sum(0)), b
    env.close()
