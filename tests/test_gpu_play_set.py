"""The batched play set on the GPU (VecNardeEnv.play_set / explore_plays ->
k_play_set / k_explore_plays), through the C ABI (VERDICT r02 missing #2):

* kind "act" == DQNAgent.act's valid_move_combinations
  (train_deepq_pytorch.py:430-507) on every step of the reference trainer's
  recording (tests/golden/trainer.npz: its pre-step states, agent dice and
  combination lists), list for list;
* kind "step": list #1 == the reference's list #1 and the played move 1's
  entry == the reference's list #2 (sources and die) on every golden
  NardeEnv.step (tests/golden/steps.npz); the decoded set ==
  Narde.get_valid_plays (the scalar facade) on 300 self-play positions;
* device dice (dice=None) == the same call with env.dice();
* the driver's exploration: each exploring row's (move1, move2) is play
  mulhi(r1, count) of act()'s list for Philox4x32-10({tag, row, 0, 5}, seed)
  -- exact, so the law is uniform over combinations by construction.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _env_at(board, off, ft, player, seed=3):
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(board.shape[0], device="cuda:0", seed=seed)
    env.set_state(board, off, ft, player)
    return env


def test_act_kind_equals_reference_trainer_combinations():
    from gym_narde.vector import decode_play_set

    t = golden("trainer.npz")
    env = _env_at(t["pre_board"], t["pre_off"], t["pre_ft"], t["player"])
    legal, words, count = env.play_set(dice=t["dice"], kind="act")
    legal, words, count = legal.cpu().numpy(), words.cpu().numpy(), count.cpu().numpy()
    act = t["nvalid"] > 0
    assert np.array_equal(count[act], t["combos_len"][act])
    starts = np.concatenate([[0], np.cumsum(t["combos_len"])])
    for i in np.nonzero(act)[0]:
        want = [tuple(int(x) for x in r) for r in t["combos"][starts[i]:starts[i + 1]]]
        assert decode_play_set(legal[i], words[i], "act") == want, f"step {i}"
    env.close()


def test_step_kind_holds_the_reference_lists():
    s = golden("steps.npz")
    env = _env_at(s["board"], s["off"], s["first_turn"], s["player"])
    legal, words, count = (x.cpu().numpy() for x in env.play_set(dice=s["dice"], kind="step"))
    for i in range(s["board"].shape[0]):
        c = int(np.uint64(np.int64(legal[i])))
        dh, dl = (c >> 48) & 15, (c >> 52) & 15
        got = [(p, 24 if p < d else p - d) for L, d in ((c & 0xFFFFFF, dh), ((c >> 24) & 0xFFFFFF, dl))
               for p in range(24) if (L >> p) & 1]
        want = [tuple(int(x) for x in r) for r in s["list1"][i, :s["count1"][i]]]
        assert got == want, f"case {i}"
        if s["count2"][i] < 0 or s["count1"][i] < 2:
            continue
        f, t = divmod(int(s["action"][i, 0]), 24)
        if t == 0 and f <= 5:
            t = 24
        ks = [k for k, d in ((0, dh), (1, dl)) if ((c >> (24 * k)) >> f) & 1
              and ((t == 24 and f < d) or (t != 24 and f - t == d))]
        w = int(words[i, ks[0], f])
        src = 0
        for r in s["list2"][i, :s["count2"][i]]:
            src |= 1 << int(r[0])
        assert w & 0xFFFFFF == src and (w >> 24) & 7 == int(s["roll2"][i]), f"case {i}"
    env.close()


def test_step_kind_equals_facade_get_valid_plays():
    from gym_narde.envs.narde import Narde
    from gym_narde.vector import VecNardeEnv, decode_play_set

    n = 300
    env = VecNardeEnv(n, device="cuda:0", seed=41)
    env.selfplay(57)
    dice = env.dice().cpu().numpy()
    st = {k: v.cpu().numpy() for k, v in env.get_state().items()}
    legal, words, count = (x.cpu().numpy() for x in env.play_set(kind="step"))  # device dice
    g = Narde()
    for i in range(n):
        g.board[:] = st["board"][i]
        g.borne_off_white, g.borne_off_black = int(st["off"][i, 0]), int(st["off"][i, 1])
        g.first_turn_white, g.first_turn_black = bool(st["first_turn"][i, 0]), bool(st["first_turn"][i, 1])
        want = g.get_valid_plays([int(dice[i, 0]), int(dice[i, 1])], int(st["player"][i]))
        assert decode_play_set(legal[i], words[i], "step") == want, f"env {i}"
        assert count[i] == len(want)
    env.close()


def test_device_dice_equal_given_dice():
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(8192, device="cuda:0", seed=5)
    env.selfplay(33)
    d = env.dice()
    for kind in ("act", "step"):
        a = env.play_set(kind=kind)
        b = env.play_set(dice=d, kind=kind)
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    # a die outside 1..6: no play
    bad = d.clone()
    bad[::2, 0] = 7
    legal, words, count = env.play_set(dice=bad)
    assert int(count[::2].abs().sum()) == 0 and int(legal[::2].abs().sum()) == 0
    env.close()


@pytest.mark.parametrize("eps", [1.0, 0.4])
def test_explore_plays_draws_act_combinations(eps):
    import oracle as O

    from gym_narde.vector import VecNardeEnv, decode_play_set

    n, seed, tag = 4096, 0x1234_5678_9ABC, 17
    env = VecNardeEnv(n, device="cuda:0", seed=9)
    env.selfplay(21)
    legal, words, count = (x.cpu().numpy() for x in env.play_set(kind="act"))
    acts = torch.full((n, 2), -7, dtype=torch.int64, device="cuda:0")
    e = torch.tensor(eps, dtype=torch.float32, device="cuda:0")
    tg = torch.tensor(tag, dtype=torch.int64, device="cuda:0")
    env.explore_plays(acts, e, seed, tg)
    got = acts.cpu().numpy()
    thr = int(min(1.0, eps) * 2 ** 32)
    explored = 0
    for i in range(n):
        r = O.philox((tag, i, 0, 5), (seed & 0xFFFFFFFF, seed >> 32))
        if not (r[0] < thr) or count[i] == 0:
            assert tuple(got[i]) == (-7, -7), f"env {i} untouched"
            continue
        combos = decode_play_set(legal[i], words[i], "act")
        j = (r[1] * int(count[i])) >> 32
        assert tuple(got[i]) == combos[j], f"env {i}"
        explored += 1
    assert explored > (0.9 if eps == 1.0 else 0.3) * n
    env.close()


def test_driver_explores_over_act_combinations():
    """BatchedDQNDriver(explore="plays") at epsilon 1: every row's action is
    one of act()'s combinations for the step's own dice, and its move 1 is
    a code the step accepts unless it is act()'s (f, 0)/(f, 'off') code
    collision."""
    from gym_narde.dqn import BatchedDQNDriver, expand_mask
    from gym_narde.vector import VecNardeEnv, decode_play_set

    env = VecNardeEnv(2048, device="cuda:0", seed=19)
    drv = BatchedDQNDriver(env, capacity=1 << 14, train_batch=256)
    env.selfplay(31)
    drv.resync()
    legal, words, count = (x.cpu().numpy() for x in env.play_set(kind="act"))
    acc1 = expand_mask(env.legal_mask())
    a = drv.act(drv.state)
    got = a.cpu().numpy()
    for i in range(env.num_envs):
        if count[i] == 0:
            assert tuple(got[i]) == (0, 0)
            continue
        assert tuple(got[i]) in set(decode_play_set(legal[i], words[i], "act")), f"env {i}"
    rows = torch.arange(env.num_envs, device="cuda:0")
    ok = acc1[rows, a[:, 0]] | ~acc1.any(1)
    # the only move-1 codes of act()'s list the step does not accept: a
    # normal move (f, 0), f <= 5, whose code f * 24 the step decodes as
    # (f, 'off') (narde_env.py:50-53) -- the reference's own collision
    quirk = (a[:, 0] % 24 == 0) & (a[:, 0] // 24 <= 5)
    assert bool((ok | quirk).all())
    assert float(ok.float().mean()) > 0.8
    env.close()


def test_act_masks_reproduce_reference_greedy_act():
    """k_act_masks (VecNardeEnv.act_masks) + the policy kernel on the
    Q-values the reference's DQNAgent.act was given
    (tests/golden/act_greedy.npz, tools/capture_act_greedy.py): the same
    greedy (move1, move2) as the reference on 2,500 trainer steps."""
    from gym_narde.dqn import policy_576

    t = golden("trainer.npz")
    a = golden("act_greedy.npz")
    rows = a["step"]
    env = _env_at(t["pre_board"][rows], t["pre_off"][rows], t["pre_ft"][rows], t["player"][rows])
    tab = np.random.default_rng(int(a["meta"][2])).standard_normal((576, 576)).astype(np.float32)
    q1 = np.stack([np.random.default_rng(int(a["meta"][0]) + int(i)).standard_normal(576).astype(np.float32)
                   for i in rows])
    b2 = np.stack([np.random.default_rng(int(a["meta"][1]) + int(i)).standard_normal(576).astype(np.float32)
                   for i in rows])
    dice = torch.as_tensor(t["dice"][rows], device="cuda:0")
    m1 = env.act_masks(dice=dice)
    a1 = policy_576(torch.as_tensor(q1, device="cuda:0"), m1, 0.0, seed=0, tag=0, head=0)
    assert np.array_equal(a1.cpu().numpy(), a["action"][:, 0])
    m2 = env.act_masks(move1=a1, dice=dice)
    q2 = torch.as_tensor(b2 + tab[a1.cpu().numpy()], device="cuda:0")
    a2 = policy_576(q2, m2, 0.0, seed=0, tag=0, head=1)
    assert np.array_equal(a2.cpu().numpy(), a["action"][:, 1])
    env.close()


def test_driver_reference_greedy_uses_act_sets():
    """BatchedDQNDriver(greedy="reference") at epsilon 0: move 1 is the
    fused heads' argmax over act()'s move-1 codes, move 2 over act()'s
    move-2 codes for it (pre-move lists)."""
    from gym_narde.dqn import BatchedDQNDriver, expand_mask
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(4096, device="cuda:0", seed=27)
    drv = BatchedDQNDriver(env, capacity=1 << 14, train_batch=256, epsilon=0.0, greedy="reference")
    env.selfplay(45)
    drv.resync()
    a = drv.act(drv.state)
    m1 = expand_mask(env.act_masks())
    rows = torch.arange(env.num_envs, device="cuda:0")
    has1 = m1.any(1)
    assert bool(m1[rows, a[:, 0]][has1].all()) and bool((a[:, 0][~has1] == 0).all())
    m2 = expand_mask(env.act_masks(move1=a[:, 0].contiguous()))
    assert bool(m2[rows, a[:, 1]][has1].all())
    with torch.no_grad():
        q1 = drv.model(drv.state)
    best = q1.masked_fill(~m1, -np.inf).max(1).values
    got = q1.gather(1, a[:, :1]).squeeze(1)
    assert bool((got >= best - 1e-5 * (1 + best.abs()))[has1].all())
    env.close()
