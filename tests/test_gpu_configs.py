"""GPU: BASELINE.json's configs at their full sizes, the device reset with the
reference's own opening draws, the ABI's edge cases (dice outside 1..6,
moves the record cannot hold) and the RCCL code path.  Bit-exact against the
oracle / the reference's fixtures wherever the reference defines the answer.

  configs[4]  batch 524,288 = 8 x 65,536, one shard of global env ids per GPU
              (narde_env.py:27-103 per env)
  configs[3]  batch 65,536 DQN driver (train_deepq_pytorch.py:855-935 batched)
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from conftest import ROOT, golden

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def vec(n, **kw):
    from gym_narde.vector import VecNardeEnv

    return VecNardeEnv(n, device="cuda:0", **kw)


def np_(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


# ------------------------------------------------------------- configs[4]
def test_config4_eight_shards_of_65536():
    """configs[4] on the one GPU we have: 8 handles of 65,536 envs with
    env_id_offset = r * 65,536 (the shards the 8 ranks own) run self-play and
    then a rollout with every output.  Each shard's 2,048-env window equals
    the oracle on those global ids, and the 8 shards together equal ONE
    524,288-env handle output for output (the sharded run IS the big run)."""
    S, W, seed, p1, p2, m = 65536, 8, 4242, 300, 40, 2048
    shards = [vec(S, seed=seed, env_id_offset=r * S) for r in range(W)]
    whole = vec(S * W, seed=seed)
    for e in shards + [whole]:
        e.selfplay(p1)
    wb = whole.rollout(p2)
    for r, e in enumerate(shards):
        b = e.rollout(p2)
        cols = slice(r * S, (r + 1) * S)
        for k in ("obs", "reward", "terminated", "truncated", "legal", "actions"):
            assert torch.equal(b[k], wb[k][:, cols]), (r, k)
        lo = 1000 + 7919 * r
        ref = O.SelfPlay(m, seed=seed, env0=r * S + lo)
        ref.reset(0)
        ref.run(p1, record=False)
        rec = ref.run(p2)
        sl = slice(lo, lo + m)
        assert np.array_equal(np_(b["obs"][:, sl]), rec["obs"].astype(np.int32)), r
        assert np.array_equal(np_(b["reward"][:, sl]), rec["reward"].astype(np.int32)), r
        assert np.array_equal(np_(b["terminated"][:, sl]), rec["terminated"]), r
        assert np.array_equal(np_(b["actions"][:, sl]), rec["action"]), r
        assert np.array_equal(np_(e.get_state()["board"])[sl], ref.board), r
        assert np.array_equal(np_(e.stats())[sl], ref.stats), r
        del b
    from gym_narde import distributed as D

    st = torch.cat([D.gather_stats(e.stats()) for e in shards])
    assert torch.equal(st, whole.stats())
    # the per-rank totals the bench gathers (one kernel per shard) add up to
    # the whole batch's, and each shard's rows to its own statistics
    rows = torch.cat([D.gather_total_rows(e.totals()) for e in shards])
    assert rows.shape == (W, 64, 3)
    for r, e in enumerate(shards):
        assert torch.equal(rows[r].sum(0), e.stats().to(torch.int64).sum(0)), r
    assert torch.equal(rows.sum((0, 1)), whole.totals().sum(0))
    s = D.summarize(st)
    assert s["episodes"] > S * W // 4  # ~340 plies: several hundred thousand games ended
    for e in shards + [whole]:
        e.close()


# ------------------------------------------------------------- configs[3]
def test_config3_dqn_driver_at_65536():
    """configs[3] at its stated batch: every move-1 / move-2 code the driver
    sends is one the env accepts (the env's exact masks), and on a 2,048-env
    window the env's step equals the oracle's NardeEnv.step on the same
    (state, dice, actions) -- post-board for the games that go on, reward and
    termination for all; learning runs (finite loss, epsilon decays)."""
    from conftest import in_act_plays
    from gym_narde.dqn import BatchedDQNDriver, expand_mask

    B, lo, m = 65536, 30000, 2048
    env = vec(B, seed=77)
    drv = BatchedDQNDriver(env, capacity=1 << 20, train_batch=4096)
    rows = torch.arange(B, device="cuda:0")
    sl = slice(lo, lo + m)
    for step in range(8):
        x = drv.state
        m1 = expand_mask(env.legal_mask())
        a = drv.act(x)
        m2 = expand_mask(env.legal_mask_move2(a[:, 0].to(torch.int16)))
        has1, has2 = m1.any(1), m2.any(1)
        greedy_ok = torch.where(has1, m1[rows, a[:, 0]], a[:, 0] == 0) & (~has2 | m2[rows, a[:, 1]])
        # exploring rows: one of act()'s (move1, move2) combinations
        assert bool((greedy_ok | in_act_plays(*env.play_set(kind="act"), a)).all()), step
        st = {k: np_(v)[sl] for k, v in env.get_state().items()}
        dice = np_(env.dice())[sl]
        ref = O.step(st["board"], st["off"], st["first_turn"], st["player"], dice,
                     np_(a)[sl].astype(np.int16), with_lists=False)
        pos = drv.replay.pos
        drv.step()  # the same actions: act() is a function of (state, epsilon, tag)
        assert torch.equal(drv.replay.action[pos:pos + B], a), step
        post = {k: np_(v)[sl] for k, v in env.get_state().items()}
        done = ref["terminated"].astype(bool)
        assert np.array_equal(post["board"][~done], ref["board"][~done]), step
        assert np.array_equal(post["player"][~done], ref["player"][~done]), step
        assert np.array_equal(np_(env.reward)[sl], ref["reward"].astype(np.int32)), step
        assert np.array_equal(np_(env.terminated)[sl], ref["terminated"]), step
    torch.cuda.synchronize()
    assert drv.train_steps >= 1 and torch.isfinite(drv.last_loss)
    assert drv.epsilon < 1.0
    env.close()


# ------------------------------------------------ reset with injected draws
def _reference_opening_draws(seed):
    """The draws NardeEnv.reset(seed) consumes (narde_env.py:107-115): the
    global legacy MT19937 reseeded, pairs until unequal.  Pinned to the
    reference by resets.npz (first player + the next draw)."""
    np.random.seed(seed)
    pairs = []
    while True:
        w, b = np.random.randint(1, 7), np.random.randint(1, 7)
        pairs.append((w, b))
        if w != b:
            return pairs


def _opening_rows(seeds):
    draws = [_reference_opening_draws(int(s)) for s in seeds]
    rows = np.zeros((len(seeds), max(len(d) for d in draws), 2), np.uint8)  # 0 = padding
    for i, d in enumerate(draws):
        rows[i, :len(d)] = d
    return rows, draws


def test_device_reset_replays_reference_opening_draws():
    """narde_reset with injected opening draws: the first player of every
    resets.npz seed (and the reset observation of every episodes.npz seed)
    comes out of the DEVICE reset, not only the host facade."""
    d = golden("resets.npz")
    rows, draws = _opening_rows(d["seed"])
    for s, nxt, dr in zip(d["seed"], d["next_draw"], draws):
        np.random.seed(int(s))
        for _ in range(2 * len(dr)):
            np.random.randint(1, 7)
        assert np.random.randint(0, 2 ** 31 - 1) == nxt  # the restated draw count is the reference's
    assert max(len(x) for x in draws) >= 2  # some seed needed a redraw
    n = len(d["seed"])
    env = vec(n, seed=3)
    env.selfplay(77)  # mid-game states, so the reset really rewrites them
    obs = np_(env.reset(opening=torch.from_numpy(rows)))
    st = env.get_state()
    assert np.array_equal(np_(st["player"]), d["player"])
    start = np.zeros(24, np.int8)
    start[23], start[11] = 15, -15
    assert (np_(st["board"]) == start).all()
    assert (np_(st["first_turn"]) == 1).all() and (np_(st["off"]) == 0).all()
    assert (np_(st["elapsed"]) == 0).all() and (np_(env.stats()) == 0).all()
    assert (obs == start.astype(np.int32)).all()  # both perspectives of the start look alike

    e = golden("episodes.npz")
    rows, _ = _opening_rows(e["seed"])
    env2 = vec(len(e["seed"]), seed=9)
    obs2 = np_(env2.reset(opening=rows))
    assert np.array_equal(np_(env2.get_state()["player"]), e["reset_player"])
    assert np.array_equal(obs2, e["reset_obs"].astype(np.int32))
    # masked reset with draws: only the masked envs change; a row without a
    # deciding pair falls back to the device draw (same as opening=None)
    env3, env4 = vec(n, seed=3), vec(n, seed=3)
    for x in (env3, env4):
        x.selfplay(50)
    mask = torch.zeros(n, dtype=torch.uint8)
    mask[::3] = 1
    before = np_(env3.get_state()["board"])
    undecided = np.full((n, 2, 2), 4, np.uint8)
    env3.reset(mask=mask, opening=undecided)
    env4.reset(mask=mask)
    after = np_(env3.get_state()["board"])
    keep = np_(mask) == 0
    assert np.array_equal(after[keep], before[keep])
    assert np.array_equal(np_(env3.get_state()["player"]), np_(env4.get_state()["player"]))


# ----------------------------------------------------------- ABI edge cases
def test_dice_outside_1_to_6_make_a_no_move_ply():
    """narde_step / narde_step_full / narde_legal_full / move-2 mask with a
    given die outside 1..6: no checker moves, the player changes, t and the
    TimeLimit count advance; other envs of the launch are unaffected."""
    n = 4096
    src = vec(n, seed=12)
    src.selfplay(60)
    st = {k: v.clone() for k, v in src.get_state().items()}
    dice = np.random.RandomState(1).randint(1, 7, size=(n, 2)).astype(np.uint8)
    bad = np.zeros(n, bool)
    bad[::5] = True
    dice_bad = dice.copy()
    ib = np.nonzero(bad)[0]
    dice_bad[ib, 0] = np.where(np.arange(len(ib)) % 2, 0, 7)
    dice_bad[ib[::3], 0] = dice[ib[::3], 0]  # some envs: only the second die is bad
    dice_bad[ib[::3], 1] = 200
    acts = np.zeros((n, 2), np.int16)
    for rules in ("ref2", "full4"):
        e, ref_env = vec(n, seed=12, rules=rules), vec(n, seed=12, rules=rules)
        for x in (e, ref_env):
            x.set_state(st["board"], st["off"], st["first_turn"], st["player"], st["elapsed"])
        if rules == "ref2":
            obs, rew, term, trunc, info = e.step(torch.from_numpy(acts), torch.from_numpy(dice_bad))
            ref_env.step(torch.from_numpy(acts), torch.from_numpy(dice))
            lg = np_(info["legal"]).view(np.uint64)
            assert ((lg[bad] & np.uint64(0xFFFFFFFFFFFF)) == 0).all()
        else:
            play = torch.full((n, 4, 2), -1, dtype=torch.int8)
            obs, rew, term, trunc, info = e.step(play, torch.from_numpy(dice_bad))
            ref_env.step(play, torch.from_numpy(dice))
            assert (np_(info["legal"])[bad] == 0).all()
            assert (np_(info["played"])[bad] == -1).all()
        a, b = e.get_state(), ref_env.get_state()
        assert np.array_equal(np_(a["board"])[bad], np_(st["board"])[bad])
        assert np.array_equal(np_(a["player"])[bad], -np_(st["player"])[bad])
        assert np.array_equal(np_(a["elapsed"])[bad], np_(st["elapsed"])[bad] + 1)
        assert not np_(rew)[bad].any() and not np_(term)[bad].any()
        for k in ("board", "off", "first_turn", "player"):  # the other envs: as with their real dice
            assert np.array_equal(np_(a[k])[~bad], np_(b[k])[~bad]), (rules, k)
    f = vec(n, rules="full4")
    f.set_state(st["board"], st["off"], st["first_turn"], st["player"])
    lw = np_(f.legal_full(torch.from_numpy(dice_bad)))
    lw_ok = np_(f.legal_full(torch.from_numpy(dice)))
    assert (lw[bad] == 0).all() and np.array_equal(lw[~bad], lw_ok[~bad])
    r = vec(n)
    r.set_state(st["board"], st["off"], st["first_turn"], st["player"])
    m1 = np_(r.legal_mask()).view(np.uint64)
    mv1 = np.array([next((c for c in range(576) if (int(m1[i][c >> 6]) >> (c & 63)) & 1), 0)
                    for i in range(n)], np.int16)
    m2 = np_(r.legal_mask_move2(torch.from_numpy(mv1), dice=torch.from_numpy(dice_bad)))
    assert (m2[bad] == 0).all()


def test_unexecutable_moves_leave_state_unchanged():
    """narde_apply_moves / execute_rotated_move with a move the record cannot
    hold (empty source, opponent target): the device leaves that env
    unchanged, the host facade raises ValueError and keeps the game as it
    was; executable moves in the same launch apply (reference:
    narde.py:36-56,108-125 would conjure / cancel checkers instead)."""
    from gym_narde.envs.narde import Narde

    g = Narde()
    with pytest.raises(ValueError):
        g.execute_rotated_move((5, 2), 1)  # no white checker on 5
    with pytest.raises(ValueError):
        g.execute_rotated_move((23, 11), 1)  # black's 15 on 11
    assert g.board[23] == 15 and g.board[11] == -15 and g.first_turn_white
    g.execute_rotated_move((23, 18), 1)
    assert g.board[23] == 14 and g.board[18] == 1 and not g.first_turn_white

    n = 1024
    e = vec(n, seed=4)
    before = np_(e.get_state()["board"]).copy()
    player = np_(e.get_state()["player"])
    moves = np.zeros((n, 2), np.int8)
    moves[0::3] = (23, 18)   # from the head: executable for either mover
    moves[1::3] = (5, 2)     # empty source
    moves[2::3] = (23, 11)   # the opponent's head, from the mover's view
    e.apply_moves(torch.from_numpy(moves))
    after = np_(e.get_state()["board"])
    assert np.array_equal(after[1::3], before[1::3]) and np.array_equal(after[2::3], before[2::3])
    ok = after[0::3].astype(int)
    mover_abs = lambda p, pl: p if pl == 1 else (p + 12) % 24  # noqa: E731
    for j, i in enumerate(range(0, n, 3)):
        pl = int(player[i])
        assert ok[j][mover_abs(23, pl)] == 14 * pl and ok[j][mover_abs(18, pl)] == pl


# ------------------------------------------------------------------- RCCL
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_NCCL_CHILD = r"""
import os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "gym-narde_amd")]
import torch
import torch.distributed as dist
from gym_narde import distributed as D
from gym_narde.vector import VecNardeEnv
r, w, local = D.init_from_env(backend="nccl", force=True)
assert (r, w) == (0, 1) and dist.get_backend() == "nccl"
env = VecNardeEnv(8192, device="cuda:0", seed=5)
env.selfplay(300)
st = env.stats()
g = D.gather_stats(st)  # all_gather_into_tensor over RCCL on device tensors
torch.cuda.synchronize()
assert g.is_cuda and g.shape == st.shape and torch.equal(g, st)
tot = D.gather_totals(st)  # per-rank totals
torch.cuda.synchronize()
assert tot.is_cuda and tot.shape == (1, 3) and torch.equal(tot[0], st.to(torch.int64).sum(0))
rows = D.gather_total_rows(env.totals())  # the bench's timed-region gather: one kernel + one all-gather
torch.cuda.synchronize()
assert rows.is_cuda and rows.shape == (1, 64, 3) and torch.equal(rows.sum(1), tot)
# the bench's timed-region gather at N > 1: the last launch's per-256-env
# totals rows through RCCL's own ncclAllGather (D.RcclGather)
from gym_narde import _lib
wrows = torch.empty((_lib.wg_rows(8192), 3), dtype=torch.int64, device="cuda:0")
L = env.rollout_launcher(20, env.rollout_buffers(20), totals=wrows)
L()
G = D.RcclGather(wrows)
out = G()
torch.cuda.synchronize()
assert out.shape == (1,) + tuple(wrows.shape) and torch.equal(out[0], wrows)
L()
out = G()  # the rows of the next launch, same buffers
torch.cuda.synchronize()
assert torch.equal(out[0], wrows) and torch.equal(wrows.sum(0), env.stats().long().sum(0))
G.close()
t = torch.tensor([1.5, 2.5], dtype=torch.float64, device="cuda:0")
dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks timing
dist.barrier()
dist.destroy_process_group()
env.close()
print("RCCL_OK", int(st[:, 0].sum()))
"""


def test_rccl_world1_process_group_gathers_device_stats():
    """The nccl (= RCCL) branch of init_from_env (device_id bound) and the
    all-gather of device statistics, as the N-GPU bench runs them, in a
    world of one process (RCCL cannot put two ranks on one GPU)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _NCCL_CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


_NCCL_RANK = r"""
import os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "gym-narde_amd")]
import torch
import torch.distributed as dist
from gym_narde import distributed as D, _lib
from gym_narde.vector import VecNardeEnv
r, w, local = D.init_from_env(backend="nccl", force=True)
assert w == 2 and dist.get_backend() == "nccl"
n = 4096
env = VecNardeEnv(n, device=f"cuda:{local}", seed=3, env_id_offset=r * n)
rows = torch.empty((_lib.wg_rows(n), 3), dtype=torch.int64, device=env.device)
L = env.rollout_launcher(20, env.rollout_buffers(20), totals=rows)
L()
G = D.RcclGather(rows)
out = G()
torch.cuda.synchronize()
mine = env.totals().sum(0)
allt = [torch.empty_like(mine) for _ in range(w)]
dist.all_gather(allt, mine)  # every rank's env.totals(), by the torch collective
assert out.shape == (w,) + tuple(rows.shape)
for k in range(w):
    assert torch.equal(out[k].sum(0), allt[k]), (k, out[k].sum(0), allt[k])
G.close()
dist.barrier()
dist.destroy_process_group()
env.close()
print("RCCL2_OK", r)
"""


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="two ranks over RCCL need two GPUs")
def test_rccl_two_ranks_gather_equals_every_rank_totals():
    """the N > 1 timed-region gather (D.RcclGather, RCCL's
    ncclAllGather through its C API) at world size 2 on two GPUs: the
    gathered per-256-env rows of rank k sum to rank k's env.totals(), and
    both ranks exit cleanly."""
    port = str(_free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2")
        procs.append(subprocess.Popen([sys.executable, "-c", _NCCL_RANK, ROOT], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"RCCL2_OK {r}" in o, o[-2000:] + e[-4000:]


@pytest.mark.parametrize("rules,plies,n", [("ref2", 20, 65536), ("ref2", 1000, 1000), ("full4", 20, 4099),
                                           ("full4", 60, 65536), ("ref2", 7, 300)])
def test_rollout_launch_totals_rows(rules, plies, n):
    """narde_rollout_timed(totals=...): the launch writes its envs'
    statistics after it, summed per 256 envs -- equal to stats() of the same
    handle grouped the same way (and .sum(0) to totals()), for every rollout
    kernel (REF2 producer/consumer at both store policies, FULL4
    k_rollout_pp_full) and ragged env counts."""
    from gym_narde import _lib

    env = vec(n, seed=13, rules=rules)
    bufs = env.rollout_buffers(plies)
    rows = torch.full((_lib.wg_rows(n), 3), -1, dtype=torch.int64, device="cuda:0")
    env.rollout(150, env.rollout_buffers(150))  # some episodes finished already
    L = env.rollout_launcher(plies, bufs, totals=rows)
    for _ in range(2):
        L()
    st = env.stats().long()
    pad = torch.zeros((rows.shape[0] * 256, 3), dtype=torch.int64, device="cuda:0")
    pad[:n] = st
    assert torch.equal(rows, pad.view(-1, 256, 3).sum(1))
    assert torch.equal(rows.sum(0), env.totals().sum(0))
    assert int(rows[:, 0].sum()) > 0
    env.close()
