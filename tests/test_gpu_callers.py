"""f-3: the reference's caller loops, run through the
drop-in facade, replay what the same loops did on the imported reference
(tests/golden/{callers,trainer}.npz from tools/capture_callers.py), step for
step:

  evaluate_model.py   the trained checkpoint's decisions (recorded: the
                      checkpoint never travels) against the random agent
  play_against_ai.py  the AI against a scripted keyboard, every printed
                      line and env.render() grid included
  train_deepq_pytorch.py:855-1081
                      the trainer's env-facing calls: get_valid_moves on its
                      own dice and on act()'s remaining dice, the step, the
                      borne-off reward shaping, first_turn_* reads and
                      _violates_block_rule on mutated board copies

The trainer fixture also pins the batched DQN driver's fused shaping
(narde_dqn_transition) against the reference trainer's shaped rewards."""
import ctypes

import numpy as np
import pytest
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_evaluate_loop_replays_reference_games():
    import callers
    from gym_narde import make

    d = golden("callers.npz")
    games, np_seed, py_seed = (int(x) for x in d["meta"])
    ai = callers.ReplayAI(d, "ai")
    rec = callers.play(lambda: make("gym_narde:narde-v0"), ai, games, np_seed, py_seed)
    assert ai.k == len(d["ai_action"])  # every decision of the trained policy replayed
    assert len(rec["action"]) == len(d["action"])
    for k in ("game", "ai_color", "dice", "action", "obs", "reward", "done", "player"):
        assert np.array_equal(rec[k], d[k]), k
    assert d["done"].sum() == games


def test_play_against_ai_loop_replays_reference_game():
    import callers
    from gym_narde import make

    d = golden("callers.npz")
    np_seed, key_seed = (int(x) for x in d["human_meta"])
    ai = callers.ReplayAI(d, "human_ai")
    rec = callers.play_human(lambda **k: make("gym_narde:narde-v0", **k), ai, np_seed, key_seed)
    assert ai.k == len(d["human_ai_action"])
    for k in ("dice", "action", "obs", "reward", "done", "player", "human_color"):
        assert np.array_equal(rec[k], d[f"human_{k}"]), k
    # every line the game printed: the prompts, the move lists and the
    # rendered 4 x 6 grids (narde_env.py:122-129)
    assert bytes(rec["text"]) == bytes(d["human_text"])


def test_trainer_loop_replays_reference_calls():
    import callers
    from gym_narde import make

    d = golden("trainer.npz")
    episodes, np_seed, py_seed = (int(x) for x in d["meta"])
    rec = callers.train_loop(lambda: make("gym_narde:narde-v0"), episodes, np_seed, py_seed)
    assert len(rec["action"]) == len(d["action"])
    for k in ("episode", "dice", "env_dice", "player", "nvalid", "action", "obs", "reward", "done",
              "truncated", "seen_w", "seen_b", "pre_board", "pre_off", "pre_ft", "ft_read", "combos",
              "combos_len", "blocks", "blocks_len"):
        assert np.array_equal(rec[k], d[k]), k
    assert np.array_equal(rec["shaped"], d["shaped"])  # float64, the same Python arithmetic
    assert (d["nvalid"] == 0).any() and len(d["blocks"]) > 0


def test_fused_shaping_matches_reference_trainer():
    """Every recorded trainer step as one env of a batch: set the pre-step
    state, step with the env's own dice and the trainer's action (auto-reset
    on), then k_dqn_transition with the trainer's trackers and its own
    roll's list #1 (the reference shapes only when that list is non-empty):
    the shaped reward equals the reference trainer's to fp32 rounding (the
    reference adds in float64), including the terminal steps whose record
    has already been reset, and the trackers carry over exactly."""
    from gym_narde import _lib
    from gym_narde.vector import VecNardeEnv

    d = golden("trainer.npz")
    n = len(d["action"])
    dev = "cuda:0"
    env = VecNardeEnv(n, device=dev, seed=1, max_episode_steps=1000)
    # the step's index within its episode -> the TimeLimit count before it
    ep = d["episode"].astype(np.int64)
    first = np.r_[0, np.nonzero(np.diff(ep))[0] + 1]
    elapsed = (np.arange(n) - np.repeat(first, np.diff(np.r_[first, n]))).astype(np.int16)
    env.set_state(torch.from_numpy(d["pre_board"]), torch.from_numpy(d["pre_off"]),
                  torch.from_numpy(d["pre_ft"]), torch.from_numpy(d["player"]), torch.from_numpy(elapsed))
    # list #1 of the TRAINER's roll (train_deepq_pytorch.py:866-873 shapes only if non-empty)
    _, _, legal_trainer = env.legal_moves(dice=torch.from_numpy(d["dice"]), expanded=False)
    legal_trainer = legal_trainer.clone()
    pre = torch.from_numpy(d["pre_off"].astype(np.int32))
    misc = (pre[:, 0] | (pre[:, 1] << 4) | ((torch.from_numpy(d["player"]) == -1).to(torch.int32) << 10)).to(dev)
    # trackers before each step: the previous step's (0 at an episode start)
    seen = np.stack([d["seen_w"], d["seen_b"]], 1).astype(np.float32)
    before = np.zeros_like(seen)
    before[1:] = seen[:-1]
    before[first] = 0.0
    off_seen = torch.from_numpy(before).to(dev)
    obs, reward, term, trunc, _ = env.step(torch.from_numpy(d["action"]), torch.from_numpy(d["env_dice"]))
    assert np.array_equal(reward.cpu().numpy(), d["reward"].astype(np.int32))
    assert np.array_equal(term.cpu().numpy() | trunc.cpu().numpy(), d["done"])
    cap = 2 * n
    z = dict(device=dev)
    state = torch.empty((n, 198), dtype=torch.float32, **z)
    acts = torch.from_numpy(d["action"].astype(np.int64)).to(dev)
    r_obs = torch.zeros((cap, 198), dtype=torch.float32, **z)
    r_act = torch.zeros((cap, 2), dtype=torch.int64, **z)
    r_rew, r_done, r_prio = (torch.zeros(cap, dtype=torch.float32, **z) for _ in range(3))
    max_prio = torch.ones((), dtype=torch.float32, **z)
    pos = torch.zeros((), dtype=torch.int64, **z)
    env.handle.call("narde_dqn_transition", _lib.ptr(state), _lib.ptr(acts), _lib.ptr(reward), _lib.ptr(term),
                    _lib.ptr(trunc), _lib.ptr(legal_trainer), _lib.ptr(misc), _lib.ptr(off_seen), 1,
                    _lib.ptr(r_obs), _lib.ptr(r_act), _lib.ptr(r_rew), _lib.ptr(r_done), _lib.ptr(r_prio),
                    _lib.ptr(max_prio), _lib.ptr(pos), cap, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    got = r_rew[:n].cpu().numpy().astype(np.float64)
    assert np.allclose(got, d["shaped"], rtol=0, atol=2e-6)  # fp32 vs the reference's float64
    assert (d["done"] == 1).sum() == d["meta"][0]
    done = d["done"].astype(bool)
    shaped_end = done & (d["nvalid"] > 0)
    assert got[shaped_end].min() >= 1 + 1.5  # the winner: reward + 15 * 0.1 (+ its last checkers)
    # trackers after the step: the reference's (zeroed where an episode ended)
    want = seen.copy()
    want[done] = 0.0
    assert np.array_equal(off_seen.cpu().numpy(), want)
