"""GPU parity: the HIP kernels (through libnarde.so's C ABI) vs the reference's
golden vectors and vs the CPU oracle.  Bit-exact everywhere (integer work)."""
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

    return VecNardeEnv(n, device="cuda:0", **kw)


def np_(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def set_from(env, d, board="board", off="off", ft="first_turn", player="player"):
    env.set_state(torch.from_numpy(d[board]), torch.from_numpy(d[off]), torch.from_numpy(d[ft]),
                  torch.from_numpy(d[player]))


# ------------------------------------------------------------------ goldens
def test_legal_moves_golden():
    d = golden("legal.npz")
    n = len(d["count"])
    env = vec(n)
    set_from(env, d)
    count, moves, compact = env.legal_moves(dice=torch.from_numpy(d["roll"]))
    assert np.array_equal(np_(count), d["count"])
    assert np.array_equal(np_(moves), d["moves"])
    # compact form encodes the same ordered list for <= 2 dice
    from gym_narde.vector import decode_compact

    c = np_(compact).view(np.uint64)
    two = np.nonzero(d["nroll"] == 2)[0]
    m2, c2 = O.expand_compact(c[two])  # every two-dice case, entry by entry
    assert np.array_equal(c2, d["count"][two]) and np.array_equal(m2, d["moves"][two])
    for i in two[:200]:  # the product's own decoder agrees
        ref = [(int(f), "off" if t == 24 else int(t)) for f, t in d["moves"][i][: d["count"][i]]]
        assert decode_compact(c[i]) == ref, i


def test_step_golden():
    s = golden("steps.npz")
    n = len(s["dice"])
    env = vec(n, max_episode_steps=0, autoreset=False)
    set_from(env, s)
    obs, rew, term, trunc, info = env.step(torch.from_numpy(s["action"]), torch.from_numpy(s["dice"]))
    assert np.array_equal(np_(obs), s["obs"].astype(np.int32))
    assert np.array_equal(np_(rew), s["reward"].astype(np.int32))
    assert np.array_equal(np_(term), s["terminated"])
    assert not np_(trunc).any()
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), s["post_board"])
    assert np.array_equal(np_(st["off"]), s["post_off"])
    assert np.array_equal(np_(st["first_turn"]), s["post_first_turn"])
    assert np.array_equal(np_(st["player"]), s["post_player"])
    # list #1 of all 44,004 golden steps, entry by entry (vectorised expansion
    # of the compact words), and the words equal the oracle's own (or_compact2)
    c = np_(info["legal"]).view(np.uint64)
    moves, count = O.expand_compact(c)
    assert np.array_equal(count, s["count1"])
    assert np.array_equal(moves, s["list1"])
    ref = O.step(s["board"], s["off"], s["first_turn"], s["player"], s["dice"], s["action"], with_lists=False)
    assert np.array_equal(c, ref["legal1"])


def test_apply_golden():
    d = golden("apply.npz")
    n = len(d["player"])
    env = vec(n)
    set_from(env, d)
    env.apply_moves(torch.from_numpy(d["move"]), torch.from_numpy(d["player"]))
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), d["post_board"])
    assert np.array_equal(np_(st["off"]), d["post_off"])
    assert np.array_equal(np_(st["first_turn"]), d["post_first_turn"])


def test_block_rule_golden():
    import ctypes

    from gym_narde import _lib

    d = golden("block.npz")
    b = torch.from_numpy(d["board"]).cuda()
    out = torch.empty(len(b), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().narde_violates_block_rule(0, _lib.ptr(b), len(b), _lib.ptr(out),
                                                      ctypes.c_void_p(0)), "block")
    assert np.array_equal(np_(out), d["violates"])


# -------------------------------------------------------- oracle self-play
@pytest.mark.parametrize("dice_mode,max_steps", [("all36", 1000), ("nodoubles", 1000), ("all36", 90)])
def test_selfplay_trajectory_vs_oracle(dice_mode, max_steps):
    n, plies, seed, env0 = 4096, 260, 0x5EED0001, 12345
    dm = 0 if dice_mode == "all36" else 1
    env = vec(n, seed=seed, env_id_offset=env0, dice_mode=dice_mode, max_episode_steps=max_steps)
    ref = O.SelfPlay(n, seed=seed, env0=env0, dice_mode=dm, max_steps=max_steps)
    ref.reset(0)
    rec = ref.run(plies)
    for p in range(plies):
        dice = np_(env.dice())
        obs, rew, term, trunc, info = env.step()
        assert np.array_equal(dice, rec["dice"][p]), p
        assert np.array_equal(np_(obs), rec["obs"][p].astype(np.int32)), p
        assert np.array_equal(np_(rew), rec["reward"][p].astype(np.int32)), p
        assert np.array_equal(np_(term), rec["terminated"][p]), p
        assert np.array_equal(np_(trunc), rec["truncated"][p]), p
        assert np.array_equal(np_(info["actions"]), rec["action"][p]), p
        assert np.array_equal(np_(info["legal"]).view(np.uint64), rec["legal"][p]), p
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), ref.board)
    assert np.array_equal(np_(st["elapsed"]).view(np.uint16), ref.elapsed)
    assert np.array_equal(np_(env.stats()), ref.stats)
    if max_steps < 200:
        assert rec["truncated"].any()


@pytest.mark.parametrize("n", [8192, 1337])
def test_fused_selfplay_vs_oracle(n):
    seed = 99
    env = vec(n, seed=seed)
    ref = O.SelfPlay(n, seed=seed)
    ref.reset(0)
    for k in (1, 7, 150, 342):  # continuity across launches of different length
        env.selfplay(k)
        ref.run(k, record=False)
    st = env.get_state()
    assert np.array_equal(np_(st["board"]), ref.board)
    assert np.array_equal(np_(st["off"]), ref.off)
    assert np.array_equal(np_(st["first_turn"]), ref.ft)
    assert np.array_equal(np_(st["player"]), ref.player)
    assert np.array_equal(np_(env.stats()), ref.stats)
    assert env.ply == 500
    # the per-ply kernel and the fused kernel are the same function of (state, t)
    env2 = vec(n, seed=seed)
    for _ in range(500):
        env2.step()
    assert np.array_equal(np_(env2.get_state()["board"]), ref.board)


@pytest.mark.parametrize("n", [4096, 1000, 37])
def test_rollout_vs_oracle_and_step(n):
    """k_rollout (P plies per launch, outputs streamed) == the oracle per ply,
    across launch boundaries of different lengths, also for env counts that
    leave partial workgroups and waves (ragged tails)."""
    seed, env0 = 0xABCDEF, 777
    env = vec(n, seed=seed, env_id_offset=env0, max_episode_steps=150)
    stepper = vec(n, seed=seed, env_id_offset=env0, max_episode_steps=150)
    ref = O.SelfPlay(n, seed=seed, env0=env0, max_steps=150)
    ref.reset(0)
    for plies in (1, 20, 64, 235):  # <= 32 plies: 2-ply barrier blocks, else 4
        rec = ref.run(plies)
        bufs = env.rollout(plies)
        # the compact legal sets and codes, bit for bit, against the per-ply
        # API kernel (k_step), whose outputs are per env (no packed rows)
        for p in range(plies):
            _, _, _, _, info = stepper.step()
            assert np.array_equal(np_(bufs["legal"][p]), np_(info["legal"])), p
            assert np.array_equal(np_(bufs["actions"][p]), np_(info["actions"])), p
        assert np.array_equal(np_(bufs["obs"]), rec["obs"].astype(np.int32))
        assert np.array_equal(np_(bufs["reward"]), rec["reward"].astype(np.int32))
        assert np.array_equal(np_(bufs["terminated"]), rec["terminated"])
        assert np.array_equal(np_(bufs["truncated"]), rec["truncated"])
        assert np.array_equal(np_(bufs["actions"]), rec["action"])
        # list #1 of every ply against the oracle's own list, word for word
        assert np.array_equal(np_(bufs["legal"]).view(np.uint64), rec["legal"])
    assert np.array_equal(np_(env.stats()), ref.stats)
    assert env.ply == 320


def test_rollout_block_boundaries_vs_oracle():
    """k_rollout_pc launches at the edges of its barrier blocks (blocks of 1,
    2, then 4 plies: launches of 2, 3, 4, 5 and 7 plies end in each kind of
    block) and on both sides of the store-policy switch (32 plies
    non-temporal, 33 plain), n = 300 (a full workgroup and a partial one):
    every output and list #1 of every ply == the oracle's."""
    n, seed, env0 = 300, 0x5EED, 91
    env = vec(n, seed=seed, env_id_offset=env0)
    ref = O.SelfPlay(n, seed=seed, env0=env0)
    ref.reset(0)
    for plies in (2, 3, 4, 5, 7, 32, 33):
        rec = ref.run(plies)
        bufs = env.rollout(plies)
        assert np.array_equal(np_(bufs["obs"]), rec["obs"].astype(np.int32)), plies
        assert np.array_equal(np_(bufs["reward"]), rec["reward"].astype(np.int32)), plies
        assert np.array_equal(np_(bufs["terminated"]), rec["terminated"]), plies
        assert np.array_equal(np_(bufs["truncated"]), rec["truncated"]), plies
        assert np.array_equal(np_(bufs["actions"]), rec["action"]), plies
        assert np.array_equal(np_(bufs["legal"]).view(np.uint64), rec["legal"]), plies
    assert np.array_equal(np_(env.stats()), ref.stats)


@pytest.mark.parametrize("rules", ["ref2", "full4"])
@pytest.mark.parametrize("n", [37, 130, 4097])
def test_rollout_writes_only_its_buffers(rules, n):
    """Every output of a rollout launch lands inside its [plies][n] buffer and
    nowhere else, for batches that end inside a wave and inside a workgroup,
    at both REF2 block schedules (<= 32 plies: 2-ply barrier blocks; longer:
    4-ply) of the raw buffer stores, whose extents drop the rows past n, and
    the FULL4 kernel: each buffer is a view into a larger sentinel-filled
    tensor, with guard regions before and after it, and the guards must come
    back untouched while the buffer itself matches a plain rollout."""
    G = 4096  # guard elements on each side
    fills = {torch.uint8: 0x5A, torch.int16: -0x2B2B, torch.int32: -0x2B2B2B2B, torch.int64: -0x2B2B2B2B2B}
    for plies in (20, 33):
        ref = vec(n, seed=5, rules=rules, max_episode_steps=60)
        env = vec(n, seed=5, rules=rules, max_episode_steps=60)
        want = ref.rollout(plies)
        bufs, bigs = {}, {}
        for k, v in env.rollout_buffers(plies).items():
            if v is None:
                bufs[k] = None
                continue
            flat = v.numel()
            big = torch.full((flat + 2 * G,), fills[v.dtype], dtype=v.dtype, device=v.device)
            bigs[k] = big
            bufs[k] = big[G:G + flat].view(v.shape)
        env.rollout(plies, bufs)
        for k, big in bigs.items():
            b = np_(big)
            assert (b[:G] == fills[big.dtype]).all() and (b[-G:] == fills[big.dtype]).all(), (k, plies)
            assert np.array_equal(np_(bufs[k]), np_(want[k])), (k, plies)
        env.close()
        ref.close()


def test_step_graph_replay_vs_oracle():
    """k_step captured in a hipGraph and replayed advances each env's own RNG
    counter, so replays reproduce consecutive plies exactly."""
    n, seed, G, R = 4096, 4242, 20, 5
    env = vec(n, seed=seed)
    ref = O.SelfPlay(n, seed=seed)
    ref.reset(0)
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        with torch.cuda.graph(graph, stream=cap):
            for _ in range(G):
                env.step()
    torch.cuda.current_stream().wait_stream(cap)
    torch.cuda.synchronize()
    # capture does not execute: state untouched
    assert np.array_equal(np_(env.get_state()["board"]), ref.board)
    for _ in range(R):
        graph.replay()
    torch.cuda.synchronize()
    ref.run(G * R, record=False)
    assert np.array_equal(np_(env.get_state()["board"]), ref.board)
    assert np.array_equal(np_(env.stats()), ref.stats)
    rec = ref.run(1)
    obs, *_ = env.step()
    assert np.array_equal(np_(obs), rec["obs"][0].astype(np.int32))


def test_full_batch_selfplay_vs_oracle():
    """B = 65536 (BASELINE configs[2]): 400 plies of stats-only self-play
    (k_selfplay) leave every env's state and statistics equal to the
    oracle's, whole batch, and the whole batch conserves checkers."""
    B, plies, seed = 65536, 400, 2024
    env = vec(B, seed=seed)
    before = R.snapshot(env)
    env.selfplay(plies)
    after = R.snapshot(env)
    board = after["board"].astype(np.int64)
    off = after["off"].astype(np.int64)
    w = np.where(board > 0, board, 0).sum(1) + off[:, 0]
    k = np.where(board < 0, -board, 0).sum(1) + off[:, 1]
    assert (w == 15).all() and (k == 15).all()
    state, _ = R.replay(before, plies, 0, seed, threads=THREADS)
    for key in ("board", "off", "first_turn", "player", "stats"):
        assert np.array_equal(after[key], state[key]), key
    assert np.array_equal(after["elapsed"].astype(np.int64), state["elapsed"].astype(np.int64))
    assert after["stats"][:, 0].sum() > B  # several episodes per env on average


def test_bench_launches_full_batch_vs_oracle():
    """The launches bench.py times (k_rollout_pc<true>: B = 65,536, 1,000
    plies, every output), then a 100-ply one and the driver's 20-ply one
    (non-temporal stores), at the bench's own seed 0 and env ids 0..65,535:
    EVERY env's every output -- the legal sets included, the metric's
    "legal-move bit-exact vs CPU" -- and final state equal the C oracle
    replaying the launch from the state before it (oracle/replay.py, the
    bench's parity_check leg); the outputs obey the rules' invariants (at
    most 15 checkers a side, reward only on a finished game (1 or 2),
    truncation only of an unfinished game)."""
    B, seed = 65536, 0
    env = vec(B, seed=seed)
    for P in (1000, 100, 20):
        bufs = env.rollout_buffers(P)
        before = R.snapshot(env)
        env.rollout(P, bufs)
        host = {k: np_(v) for k, v in bufs.items()}
        res = R.check(before, host, R.snapshot(env), P, seed, threads=THREADS)
        assert res["mismatches"] == 0 and res["envs"] == B, res
        obs = bufs["obs"]
        assert int(obs.abs().max()) <= 15
        assert bool((obs.clamp(min=0).sum(-1) <= 15).all()) and bool(((-obs).clamp(min=0).sum(-1) <= 15).all())
        rew, term, trunc = bufs["reward"], bufs["terminated"].bool(), bufs["truncated"].bool()
        # narde_env.py:134-141: 1 for a win, 2 for a mars (loser bore off nothing)
        assert bool(((rew == 0) | (((rew == 1) | (rew == 2)) & term)).all())
        assert bool((rew[term] > 0).all())
        # TimeLimit 1000: a truncation ends an unfinished game (rare: at seed
        # 0 a few games of the 65,536 reach 1,000 plies in the 1,000-ply launch)
        assert not bool((trunc & term).any()) and float(trunc.float().mean()) < 1e-3
        del bufs, obs, rew, term, trunc, host
    assert env.ply == 1120


def test_bench_timed_launch_totals_rows_vs_oracle():
    """The bench's timed launch shape with its totals rows
    (narde_rollout_timed: the launch writes its envs' statistics summed per
    256 envs): rows and every output against the oracle, whole batch."""
    from gym_narde.vector import TimingEvent

    B, seed, P = 65536, 0, 20
    env = vec(B, seed=seed)
    env.selfplay(137)  # mid-game, odd ply: the Philox block of a ply pair re-derived
    bufs = env.rollout_buffers(P)
    rows = torch.empty(((B + 255) // 256, 3), dtype=torch.int64, device="cuda:0")
    ev0, ev1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    launch = env.rollout_launcher(P, bufs, events=(ev0, ev1), totals=rows)
    before = R.snapshot(env)
    launch()
    host = {k: np_(v) for k, v in bufs.items()}
    res = R.check(before, host, R.snapshot(env), P, seed, threads=THREADS, totals_rows=np_(rows))
    assert res["mismatches"] == 0 and res["by_field"]["totals_rows"] == 0, res
    assert ev0.elapsed_ms(ev1) > 0


def test_sharded_handles_equal_single():
    B, seed, plies = 8192, 31337, 200
    full = vec(B, seed=seed)
    a = vec(B // 2, seed=seed, env_id_offset=0)
    b = vec(B // 2, seed=seed, env_id_offset=B // 2)
    for e in (full, a, b):
        e.selfplay(plies)
    fb = np_(full.get_state()["board"])
    ab = np.concatenate([np_(a.get_state()["board"]), np_(b.get_state()["board"])])
    assert np.array_equal(fb, ab)
    assert np.array_equal(np_(full.stats()), np.concatenate([np_(a.stats()), np_(b.stats())]))


def test_mask576_matches_reference_acceptance():
    n, seed = 4096, 5
    env = vec(n, seed=seed)
    env.selfplay(37)
    mask = np_(env.legal_mask()).view(np.uint64)
    count, moves, _ = env.legal_moves()
    moves, count = np_(moves), np_(count)
    for i in range(0, n, 7):
        lst = {(int(f), int(t)) for f, t in moves[i][: count[i]]}
        for c in range(576):
            f, t = c // 24, c % 24
            if t == 0 and f <= 5:
                t = 24
            accepted = (f, t) in lst
            bit = (int(mask[i][c >> 6]) >> (c & 63)) & 1
            assert bit == accepted, (i, c)


@pytest.mark.parametrize("n", [4096, 4099, 17, 65536])
def test_tesauro198_vs_oracle(n):
    """k_tesauro198_rows (16 envs a wave, rows staged in LDS): every row of a
    ragged batch (a partial last wave, an odd row count ending inside a 16-B
    piece) equals the oracle's; the int32[24] observation (k_observe, whole
    waves through LDS) equals the perspective board."""
    env = vec(n, seed=3)
    env.selfplay(120)
    st = env.get_state()
    t = np_(env.tesauro198())
    ref = O.tesauro198(np_(st["board"]), np_(st["off"]), np_(st["player"]))
    assert np.array_equal(t, ref)  # exact: every value is k/2 or k/15 computed once in f32
    # a fresh buffer full of NaN: nothing past the last row is written, nothing is left unwritten
    out = torch.full((n + 3, 198), float("nan"), device="cuda")
    env.tesauro198(out=out[:n])
    assert np.array_equal(np_(out[:n]), ref) and torch.isnan(out[n:]).all()
    obs = np_(env.observe()).astype(np.int64)
    board = np_(st["board"]).astype(np.int64)
    persp = np.where((np_(st["player"]) == 1)[:, None], board, -np.roll(board, 12, axis=1))
    assert np.array_equal(obs, persp)


def test_reset_mask_and_opening_law():
    n = 65536
    env = vec(n, seed=11)
    env.selfplay(50)
    before = np_(env.get_state()["board"])
    mask = torch.zeros(n, dtype=torch.uint8)
    mask[::2] = 1
    env.reset(mask)
    st = env.get_state()
    after = np_(st["board"])
    start = np.zeros(24, np.int8)
    start[23], start[11] = 15, -15
    assert (after[::2] == start).all()
    assert np.array_equal(after[1::2], before[1::2])
    pl = np_(st["player"])[::2]
    assert abs((pl == 1).mean() - 0.5) < 0.02
    assert (np_(st["first_turn"])[::2] == 1).all()


def _codes_of(moves, count):
    """the reference's requestable codes of a list: encode(f, t), except a
    normal (f, 0) with f <= 5, which decodes to (f, 'off')"""
    out = set()
    for f, t in moves[:count]:
        f, t = int(f), int(t)
        if t == 0 and f <= 5:
            continue
        out.add(f * 24 + (0 if t == 24 else t))
    return out


def _bits(row):
    return {c for c in range(576) if (int(row[c >> 6]) >> (c & 63)) & 1}


def test_mask576_move2_golden():
    """move-2 mask for the recorded (state, dice, move1) of every golden step
    == the requestable codes of the reference's list #2 (empty when the
    reference made no second list)."""
    s = golden("steps.npz")
    n = len(s["dice"])
    env = vec(n)
    set_from(env, s)
    m2 = np_(env.legal_mask_move2(torch.from_numpy(s["action"][:, 0].copy()),
                                  dice=torch.from_numpy(s["dice"]))).view(np.uint64)
    for i in range(n):
        exp = _codes_of(s["list2"][i], s["count2"][i]) if s["count2"][i] >= 0 else set()
        assert _bits(m2[i]) == exp, i


def test_mask576_move2_device_dice_vs_oracle():
    n, seed = 4096, 21
    env = vec(n, seed=seed)
    env.selfplay(53)
    m1 = np_(env.legal_mask()).view(np.uint64)
    rng = np.random.RandomState(0)
    move1 = np.zeros(n, np.int16)
    for i in range(n):
        legal = sorted(_bits(m1[i]))
        move1[i] = legal[rng.randint(len(legal))] if legal and rng.rand() < 0.9 else rng.randint(576)
    m2 = np_(env.legal_mask_move2(torch.from_numpy(move1))).view(np.uint64)
    st = {k: np_(v) for k, v in env.get_state().items()}
    dice = np_(env.dice())
    ref = O.step(st["board"], st["off"], st["first_turn"], st["player"], dice,
                 np.stack([move1, np.zeros(n, np.int16)], 1))
    for i in range(n):
        exp = _codes_of(ref["list2"][i], ref["count2"][i]) if ref["count2"][i] >= 0 else set()
        assert _bits(m2[i]) == exp, i


@pytest.mark.parametrize("rules,plies", [("ref2", 20), ("ref2", 40), ("full4", 20)])
def test_rollout_plan_equals_timed_call(rules, plies, monkeypatch):
    """narde_rollout_plan_launch (the pre-bound timed launch, round 6) ==
    narde_rollout_timed's per-call form: the same outputs, totals rows and
    final state from the same start, ragged n, both rules, both store
    policies."""
    from gym_narde.vector import TimingEvent

    n, seed = 3000 + 17, 77
    got = []
    for plan in ("1", "0"):
        monkeypatch.setenv("NARDE_ROLLOUT_PLAN", plan)
        env = vec(n, seed=seed, rules=rules)
        env.selfplay(33)
        bufs = env.rollout_buffers(plies)
        rows = torch.empty(((n + 255) // 256, 3), dtype=torch.int64, device="cuda:0")
        ev0, ev1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
        launch = env.rollout_launcher(plies, bufs, events=(ev0, ev1), totals=rows)
        launch()
        launch()
        got.append(({k: np_(v) for k, v in bufs.items()}, np_(rows), np_(env.get_state()["board"]), env.ply))
        assert ev0.elapsed_ms(ev1) > 0
        env.close()
    (a, ra, ba, pa), (b, rb, bb, pb) = got
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(ra, rb) and np.array_equal(ba, bb) and pa == pb == 33 + 2 * plies
