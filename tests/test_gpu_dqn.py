"""The batched DQN driver (gym_narde/dqn.py, config 4) on the GPU: every
chosen action is legal per the env's own masks, greedy actions are the masked
argmax of the network, and learning updates run (finite loss, replay grows,
target sync, epsilon decay)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def make(n=4096, **kw):
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(n, device="cuda:0", seed=17)
    return env, BatchedDQNDriver(env, capacity=1 << 16, train_batch=1024, **kw)


@pytest.mark.parametrize("obs", ["tesauro198", "int24"])
def test_driver_actions_are_legal_and_learning_runs(obs):
    from gym_narde.dqn import expand_mask

    env, drv = make(obs=obs)
    n = env.num_envs
    for step in range(12):
        x = drv.state
        m1 = expand_mask(env.legal_mask())
        a = drv.act(x)
        m2 = expand_mask(env.legal_mask_move2(a[:, 0].to(torch.int16)))
        rows = torch.arange(n, device=a.device)
        has1 = m1.any(1)
        assert bool(m1[rows, a[:, 0]][has1].all())
        assert bool((a[:, 0][~has1] == 0).all())
        has2 = m2.any(1)
        assert bool(m2[rows, a[:, 1]][has2].all())
        drv.step()  # (draws its own actions; the env advances)
    torch.cuda.synchronize()
    assert drv.replay.size == 12 * n
    assert drv.train_steps >= 10
    assert torch.isfinite(drv.last_loss)
    assert drv.epsilon < 1.0
    assert drv.state.shape == (n, drv.state_size)


def test_greedy_is_masked_argmax():
    from gym_narde.dqn import expand_mask

    env, drv = make(epsilon=0.0)
    x = drv.state
    m1 = expand_mask(env.legal_mask())
    q1 = drv.model(x)
    a = drv.act(x)
    q1m = q1.masked_fill(~m1, -np.inf)
    has1 = m1.any(1)
    assert torch.equal(a[:, 0][has1], q1m.argmax(1)[has1])
    m2 = expand_mask(env.legal_mask_move2(a[:, 0].to(torch.int16)))
    q2 = drv.model(x, a[:, 0]).masked_fill(~m2, -np.inf)
    has2 = m2.any(1)
    assert torch.equal(a[:, 1][has2], q2.argmax(1)[has2])


def test_reference_step_accepts_driver_actions():
    """Played through the oracle's NardeEnv.step with the same dice, the
    driver's greedy/explore codes are never ignored: move1 is played whenever
    list #1 has >= 2 entries of which one can be requested by a code."""
    import oracle as O

    from gym_narde.dqn import expand_mask

    env, drv = make(n=2048)
    env.selfplay(40)
    drv.state = drv._observe()
    has1 = expand_mask(env.legal_mask()).any(1).cpu().numpy()
    a = drv.act(drv.state).cpu().numpy().astype(np.int16)
    st = {k: v.cpu().numpy() for k, v in env.get_state().items()}
    dice = env.dice().cpu().numpy()
    ref = O.step(st["board"], st["off"], st["first_turn"], st["player"], dice, a)
    played1 = ref["count2"] >= 0
    # list #1 may hold only moves no action code can request ((f, 0) with
    # f <= 5): then the mask is empty and the driver sends the no-move code
    assert (played1 | (ref["count1"] < 2) | ~has1).all()


def test_policy_kernel_matches_torch_and_explores_legally():
    from gym_narde.dqn import expand_mask, masked_argmax, policy_576
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(8192, device="cuda:0", seed=3)
    env.selfplay(29)
    words = env.legal_mask()
    m = expand_mask(words)
    q = torch.randn((8192, 576), device="cuda:0")
    q[:, 100] = q[:, 7]  # ties: the lowest legal code wins, as torch.argmax
    greedy = policy_576(q, words, 0.0, seed=1, tag=0, head=0)
    assert torch.equal(greedy, masked_argmax(q, m))
    ex = policy_576(q, words, 1.0, seed=1, tag=5, head=0)
    rows = torch.arange(8192, device="cuda:0")
    has = m.any(1)
    assert bool(m[rows, ex][has].all()) and bool((ex[~has] == 0).all())
    # uniform over the legal codes: per-row counts of the picked rank
    ranks = (m.long().cumsum(1)[rows, ex] - 1)[has].float()
    cnt = m.sum(1)[has].float()
    u = (ranks + 0.5) / cnt
    assert abs(float(u.mean()) - 0.5) < 0.02
    # one shared explore decision per (seed, tag, row) for both heads
    e1 = policy_576(q, words, 0.5, seed=9, tag=11, head=0) != greedy
    e2 = policy_576(q, words, 0.5, seed=9, tag=11, head=1) != greedy
    both = has & (m.sum(1) > 3)
    agree = (e1 == e2)[both].float().mean()
    assert float(agree) > 0.6


def test_graph_replay_matches_driver_semantics():
    """capture_graph(): every replay reads the CURRENT params, observation,
    epsilon and tag (greedy move 1 == masked argmax of the live network), the
    host mirrors and device scalars advance one step per replay, and the
    target sync keeps running between replays."""
    from gym_narde.dqn import expand_mask, masked_argmax

    n = 4096
    env, drv = make(n=n)
    drv.capture_graph(warmup=2)
    cap = drv.replay.capacity
    assert drv.replay.size == cap
    steps0, train0 = drv.steps, drv.train_steps
    drv.eps_t.fill_(0.0)
    for k in range(12):
        with torch.no_grad():
            m1 = expand_mask(env.legal_mask())
            want = masked_argmax(drv.model(drv.state), m1)
        pos = drv.replay.pos
        tag = int(drv.tag_t)
        loss = drv.step()
        assert int(drv.tag_t) == tag + 1
        assert drv.replay.pos == (pos + n) % cap == int(drv.replay.pos_t)
        got = drv.replay.action[pos:pos + n, 0]
        has = m1.any(1)
        assert torch.equal(got[has], want[has])
        assert bool((got[~has] == 0).all())
        assert torch.isfinite(loss)
    assert drv.steps == steps0 + 12 and drv.train_steps == train0 + 12
    drv.eps_t.fill_(0.5)
    drv.step()
    assert drv.epsilon == pytest.approx(0.5 * 0.995, rel=1e-6)
    # the target net was synced at a multiple of 10 updates inside the replays
    drv.step()
    while drv.train_steps % drv.target_update:
        drv.step()
    torch.cuda.synchronize()
    for p, q in zip(drv.model.parameters(), drv.target.parameters()):
        assert torch.equal(p, q)


def test_policy_kernel_device_scalars_and_fused_addend():
    """The _dev entry point: epsilon / tag from device memory give the same
    codes as the scalar entry point, and the fused addend row equals the
    argmax of q + table[rows] (the move-2 head's one-hot column)."""
    from gym_narde.dqn import expand_mask, masked_argmax, policy_576
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(4096, device="cuda:0", seed=5)
    env.selfplay(13)
    words = env.legal_mask()
    m = expand_mask(words)
    q = torch.randn((4096, 576), device="cuda:0")
    for eps in (0.0, 0.3, 1.0):
        want = policy_576(q, words, eps, seed=7, tag=21, head=1)
        got = policy_576(q, words, torch.tensor(eps, device="cuda:0"), seed=7,
                         tag=torch.tensor(21, device="cuda:0"), head=1)
        assert torch.equal(got, want)
    tab = torch.randn((576, 576), device="cuda:0")
    rows = torch.randint(0, 576, (4096,), device="cuda:0")
    got = policy_576(q, words, 0.0, seed=7, tag=0, head=1, add=(tab, rows))
    assert torch.equal(got, masked_argmax(q + tab[rows], m))


@pytest.mark.parametrize("shaping", [True, False])
def test_fused_transition_matches_torch_restatement(shaping):
    """k_dqn_transition (observation + reward shaping + replay write + s <- s')
    is bit-exact against the driver's torch restatement on the same step,
    including a replay-ring wrap and games that end in the step."""
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    n = 4096
    env = VecNardeEnv(n, device="cuda:0", seed=23)
    env.selfplay(260)
    drv = BatchedDQNDriver(env, capacity=3 * n, train_batch=1024, shaping=shaping)
    drv.state = drv._observe()
    g = torch.Generator(device="cuda:0").manual_seed(4)
    off0 = torch.randint(0, 16, (n, 2), device="cuda:0", generator=g).float()
    state0 = drv.state.clone()
    rp = drv.replay
    rp.pos_t.fill_(3 * n - 100)
    rp.max_prio.fill_(2.5)
    a = drv.act(drv.state)
    _, reward, term, trunc, _ = env.step(a.to(torch.int16))
    reward, term, trunc = reward.clone(), term.clone(), trunc.clone()
    assert int((term | trunc).sum()) > 0

    def run(fn):
        drv.state.copy_(state0)
        drv.off_seen.copy_(off0)
        for t in (rp.obs, rp.next_obs, rp.action, rp.reward, rp.done, rp.prio):
            t.zero_()
        rp.pos_t.fill_(3 * n - 100)
        fn()
        return [t.clone() for t in (drv.state, drv.off_seen, rp.obs, rp.next_obs, rp.action, rp.reward,
                                    rp.done, rp.prio, rp.pos_t)]

    fused = run(lambda: drv._transition_fused(a, reward, term, trunc))
    ref = run(lambda: drv._transition_torch(drv.state, a, reward, term, trunc))
    names = ["state", "off_seen", "obs", "next_obs", "action", "reward", "done", "prio", "pos"]
    for nm, x, y in zip(names, fused, ref):
        assert torch.equal(x, y), nm
    # the wrap really happened: rows at both ends of the ring were written
    assert float(ref[7][0]) == 2.5 and float(ref[7][3 * n - 1]) == 2.5
