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


def greedy_ok(got, q, m, rel=1e-5):
    """got (B,) int64 picks: legal under m (B,576) bool wherever m has a legal
    code (0 elsewhere), and within fp32 rounding of the masked maximum of q
    (the fused heads sum in another order than the dense GEMM: a pick may
    differ from q's argmax only between near-equal codes).  Returns the
    share of exact argmax matches."""
    has = m.any(1)
    assert bool((got[~has] == 0).all())
    qm = q.masked_fill(~m, -np.inf)
    best, arg = qm.max(1)
    g = got.view(-1, 1)
    assert bool(m.gather(1, g).squeeze(1)[has].all())
    val = q.gather(1, g).squeeze(1)
    assert bool((val >= best - rel * (1.0 + best.abs()))[has].all())
    return float((got == arg)[has].double().mean())


def make(n=4096, **kw):
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(n, device="cuda:0", seed=17)
    return env, BatchedDQNDriver(env, capacity=1 << 16, train_batch=1024, **kw)


@pytest.mark.parametrize("obs,explore", [("tesauro198", "plays"), ("int24", "plays"), ("tesauro198", "codes")])
def test_driver_actions_are_legal_and_learning_runs(obs, explore):
    """Every action is legal: greedy and explore="codes" rows per the env's
    acceptance masks; explore="plays" rows one of act()'s combinations."""
    from conftest import in_act_plays
    from gym_narde.dqn import expand_mask

    env, drv = make(obs=obs, explore=explore)
    n = env.num_envs
    for step in range(12):
        x = drv.state
        m1 = expand_mask(env.legal_mask())
        a = drv.act(x)
        m2 = expand_mask(env.legal_mask_move2(a[:, 0].to(torch.int16)))
        rows = torch.arange(n, device=a.device)
        has1, has2 = m1.any(1), m2.any(1)
        ok1 = torch.where(has1, m1[rows, a[:, 0]], a[:, 0] == 0)
        ok2 = ~has2 | m2[rows, a[:, 1]]
        if explore == "codes":
            assert bool(ok1.all()) and bool(ok2.all())
        else:
            assert bool((in_act_plays(*env.play_set(kind="act"), a) | (ok1 & ok2)).all())
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
    assert greedy_ok(a[:, 0], q1, m1) > 0.99
    m2 = expand_mask(env.legal_mask_move2(a[:, 0].to(torch.int16)))
    assert greedy_ok(a[:, 1], drv.model(x, a[:, 0]), m2) > 0.99
    # the dense heads (policy_576 over hipBLASLt's Q): torch's argmax exactly
    env, drv = make(epsilon=0.0, fused_heads=False)
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

    env, drv = make(n=2048, explore="codes")
    env.selfplay(40)
    drv.resync()
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
    assert drv.replay.rows == cap and drv.replay.size == cap - n
    steps0, train0 = drv.steps, drv.train_steps
    drv.eps_t.fill_(0.0)
    for k in range(12):
        with torch.no_grad():
            m1 = expand_mask(env.legal_mask())
            q1 = drv.model(drv.state)
        pos = drv.replay.pos
        tag = int(drv.tag_t)
        loss = drv.step()
        assert int(drv.tag_t) == tag + 1
        assert drv.replay.pos == (pos + n) % cap == int(drv.replay.pos_t)
        got = drv.replay.action[pos:pos + n, 0]
        assert greedy_ok(got, q1, m1) > 0.99  # the live network, fused heads
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


@pytest.mark.parametrize("shaping,pos", [(True, "wrap"), (False, "wrap"), (True, "aligned"), (True, "wrap_next")])
def test_fused_transition_matches_torch_restatement(shaping, pos):
    """k_dqn_transition (observation + reward shaping + replay write + s <- s')
    is bit-exact against the driver's torch restatement on the same step,
    including a replay-ring wrap, games that end in the step (terminated and
    truncated: the shaping reads the pre-step record there), and envs with
    no legal move (no shaping)."""
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    n = 4096
    # the step after 119 plies: random games end after 104-131 plies, so
    # some end in this step and the TimeLimit (120) cuts others
    env = VecNardeEnv(n, device="cuda:0", seed=23, max_episode_steps=120)
    env.selfplay(119)
    drv = BatchedDQNDriver(env, capacity=3 * n, train_batch=1024, shaping=shaping)
    drv.resync()
    g = torch.Generator(device="cuda:0").manual_seed(4)
    off0 = torch.randint(0, 16, (n, 2), device="cuda:0", generator=g).float()
    state0, misc0 = drv.state.clone(), drv.misc.clone()
    rp = drv.replay
    # ring wrap of this step's rows / of its s' rows (inside a 16-row group
    # of the staged store: row by row) / contiguous rows
    p0 = {"wrap": 3 * n - 100, "wrap_next": 2 * n - 99, "aligned": n}[pos]
    rp.max_prio.fill_(2.5)
    a = drv.act(drv.state)
    _, reward, term, trunc, info = env.step(a.to(torch.int16))
    reward, term, trunc, legal = reward.clone(), term.clone(), trunc.clone(), info["legal"].clone()
    assert int(term.sum()) > 0 and int(trunc.sum()) > 0
    assert int(((legal & 0xFFFFFFFFFFFF) == 0).sum()) > 0

    def run(fn):
        drv.state.copy_(state0)
        drv.off_seen.copy_(off0)
        drv.misc.copy_(misc0)
        for t in (rp.obs, rp.action, rp.reward, rp.done, rp.prio):
            t.zero_()
        rp.pos_t.fill_(p0)
        fn()
        return [t.clone() for t in (drv.state, drv.off_seen, drv.misc, rp.obs, rp.action, rp.reward,
                                    rp.done, rp.prio, rp.pos_t)]

    fused = run(lambda: drv._transition_fused(a, reward, term, trunc, legal))
    ref = run(lambda: drv._transition_torch(a, reward, term, trunc, legal))
    names = ["state", "off_seen", "misc", "obs", "action", "reward", "done", "prio", "pos"]
    for nm, x, y in zip(names, fused, ref):
        assert torch.equal(x, y), nm
    prio, obs = ref[7], ref[3]
    rows = (torch.arange(n, device="cuda:0") + p0) % (3 * n)
    nrows = (rows + n) % (3 * n)
    assert bool((prio[rows] == 2.5).all()) and bool((prio[nrows] == 0).all())
    assert torch.equal(obs[nrows], ref[0])  # s' stored once, in the next step's rows
    if shaping:  # the winner of a terminal step is credited its 15 checkers off
        r = ref[5][rows]
        t = term.bool()
        assert bool((r[t] >= reward[t].float() + 1.5).all())


# ------------------------------------------------ fused learner kernels
def test_per_sample_kernel_vs_torch():
    """k_per_sample: for its own uniforms u, idx == torch.searchsorted(cdf,
    u * total, right=True) clamped (up to the rounding of the prefix sums),
    weights == (N p[idx] / total)^-beta / max
    (fp32, 1 ulp of powf), beta annealed and the counter advanced."""
    from gym_narde.dqn import DeviceReplay

    n, B = 300000, 4096
    rp = DeviceReplay(n, 4, "cuda:0", stride=1)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    rp.prio.copy_(torch.rand(n, device="cuda:0", generator=g) * 3 + 0.01)
    rp.prio[:1000] = 50.0  # a heavy head
    rp.size = n
    u = torch.empty(B, device="cuda:0")
    beta0 = float(rp.beta_t)
    idx, w = rp.sample_fused(B, seed=11, u_out=u)
    p = rp.prio ** rp.alpha
    cdf = torch.cumsum(p, 0)
    total = cdf[-1]
    v = u * total
    want = torch.searchsorted(cdf, v, right=True).clamp_(max=n - 1)
    # the sampler's prefix sums (narde_per_prefix, chunked) and torch's
    # cumsum (a rocPRIM look-back scan) sum in other associations, so they
    # differ by rounding -- over 300,000 rows by more than the spacing of a
    # few rows' sums here and there: a pick may differ only where v lies
    # within rounding of a prefix sum
    off = idx != want
    assert float(off.double().mean()) < 0.05
    lo = torch.minimum(idx, want)[off]
    assert bool(((cdf[lo] - v[off]).abs() <= 1e-4 * total).all())
    x = (n * (p[idx] / total)) ** (-beta0)
    assert torch.allclose(w, x / x.max(), rtol=2e-6, atol=0)
    assert float(rp.beta_t) == pytest.approx(beta0 + rp.beta_increment)
    assert int(rp.sample_ctr) == 1
    idx2, _ = rp.sample_fused(B, seed=11)
    assert not torch.equal(idx, idx2)  # a new counter, new draws
    # proportional to priority^alpha over many draws
    counts = torch.zeros(n, device="cuda:0")
    for _ in range(20):
        i, _ = rp.sample_fused(B, seed=11)
        counts += torch.bincount(i, minlength=n).float()
    head = float(counts[:1000].sum() / counts.sum())
    assert head == pytest.approx(float(p[:1000].sum() / total), rel=0.05)


@pytest.mark.parametrize("n", [1, 3, 4, 17, 1023, 1024, 1025, 4097, 300001])
def test_per_prefix_vs_torch_pow_cumsum(n):
    """narde_per_prefix (round 6): p == prio ** alpha to powf's rounding,
    cdf == the fp64 prefix sum of p to fp32 rounding, for ragged sizes and
    zero-priority runs; deterministic (a second call equal bit for bit)."""
    from gym_narde.dqn import DeviceReplay

    rp = DeviceReplay(max(n, 2), 4, "cuda:0", stride=1)
    g = torch.Generator(device="cuda:0").manual_seed(n)
    rp.prio.copy_(torch.rand(rp.capacity, device="cuda:0", generator=g) * 3 + 0.01)
    if n > 8:
        rp.prio[torch.rand(rp.capacity, device="cuda:0", generator=g) < 0.2] = 0.0
        rp.prio[n // 3:n // 3 + n // 5] = 0.0
    p, cdf = rp.prefix(n)
    torch.cuda.synchronize()
    want_p = rp.prio[:n] ** rp.alpha
    assert torch.allclose(p, want_p, rtol=3e-7, atol=0)
    assert bool((p[rp.prio[:n] == 0] == 0).all())
    ref = torch.cumsum(p.double(), 0)
    assert torch.allclose(cdf.double(), ref, rtol=2e-6, atol=1e-6)
    p2, cdf2 = rp.prefix(n)
    assert torch.equal(p2, p) and torch.equal(cdf2, cdf)


def test_gather_batch_and_rowmax_addend_exact():
    from gym_narde.dqn import DeviceReplay, rowmax_addend

    rp = DeviceReplay(5000, 198, "cuda:0", stride=1234)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    for t in (rp.obs, rp.reward, rp.done):
        t.copy_(torch.rand(t.shape, device="cuda:0", generator=g))
    rp.action.copy_(torch.randint(0, 576, rp.action.shape, device="cuda:0", generator=g))
    idx = torch.randint(0, 5000, (4096,), device="cuda:0", generator=g)
    s, ns, a, r, d = rp.gather(idx)
    nxt = (idx + 1234) % 5000
    for got, src in ((s, rp.obs[idx]), (ns, rp.obs[nxt]), (a, rp.action[idx]), (r, rp.reward[idx]),
                     (d, rp.done[idx])):
        assert torch.equal(got, src)
    base = torch.randn((4096, 576), device="cuda:0", generator=g)
    tab = torch.randn((576, 576), device="cuda:0", generator=g)
    rows = torch.randint(0, 576, (4096,), device="cuda:0", generator=g)
    assert torch.equal(rowmax_addend(base, tab, rows), (base + tab[rows]).max(1).values)


def test_dqn_loss_kernel_vs_torch_autograd():
    """k_dqn_loss: TD errors and dloss/dq bit-exact against torch's autograd
    of the reference loss (batch a power of two), the loss to fp32 summation
    order."""
    from gym_narde.dqn import DQNLoss

    B, gamma = 4096, 0.99
    g = torch.Generator(device="cuda:0").manual_seed(9)
    rnd = lambda: torch.randn(B, device="cuda:0", generator=g)  # noqa: E731
    q1, q2, m1, m2 = rnd(), rnd(), rnd(), rnd()
    r = (torch.rand(B, device="cuda:0", generator=g) < 0.1).float() * 2
    d = (torch.rand(B, device="cuda:0", generator=g) < 0.2).float()
    w = torch.rand(B, device="cuda:0", generator=g)
    q1r, q2r = q1.clone().requires_grad_(), q2.clone().requires_grad_()
    t1 = r + (1 - d) * gamma * m1
    t2 = r + (1 - d) * gamma * m2
    td_ref = torch.clamp((t1 - q1r).abs() + (t2 - q2r).abs(), 0.0, 100.0).detach()
    loss_ref = (w * (q1r - t1) ** 2).mean() + (w * (q2r - t2) ** 2).mean()
    loss_ref.backward()
    q1f, q2f = q1.clone().requires_grad_(), q2.clone().requires_grad_()
    td = torch.empty(B, device="cuda:0")
    copy = torch.zeros((), device="cuda:0")
    loss = DQNLoss.apply(q1f, q2f, m1, m2, r, d, w, gamma, td, copy)
    loss.backward()
    assert torch.equal(td, td_ref)
    assert torch.equal(q1f.grad, q1r.grad) and torch.equal(q2f.grad, q2r.grad)
    assert float(loss.detach()) == pytest.approx(float(loss_ref.detach()), rel=1e-6)
    assert float(copy) == float(loss.detach())


def test_prio_update_kernel_exact():
    from gym_narde.dqn import DeviceReplay

    rp = DeviceReplay(10000, 4, "cuda:0", stride=1)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    idx = torch.randperm(10000, device="cuda:0", generator=g)[:4096]
    td = torch.rand(4096, device="cuda:0", generator=g) * 7
    eps = torch.full((), 0.5, device="cuda:0")
    rp.update_fused(idx, td, eps, 0.01, 0.995)
    pr = td + rp.epsilon
    assert torch.equal(rp.prio[idx], pr)
    assert float(rp.max_prio) == float(torch.maximum(torch.ones((), device="cuda:0"), pr.max()))
    want = torch.where(torch.full((), 0.5, device="cuda:0") > 0.01,
                       torch.full((), 0.5, device="cuda:0") * 0.995, torch.full((), 0.5, device="cuda:0"))
    assert float(eps) == float(want)


def test_fused_and_torch_learners_agree_on_one_update():
    """One update from the same state: the fused learner (its own sampler)
    and the torch restatement given the fused learner's minibatch produce
    the same loss and parameters to fp32 rounding."""
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(4096, device="cuda:0", seed=41)
    drv = BatchedDQNDriver(env, capacity=1 << 14, train_batch=1024, seed=3)
    for _ in range(5):
        drv.step()
    torch.cuda.synchronize()
    rp = drv.replay
    state = {k: v.clone() for k, v in drv.model.state_dict().items()}
    sample_state = (rp.sample_ctr.clone(), rp.beta_t.clone(), rp.prio.clone())
    loss_f = drv._update_fused().clone()
    after_f = {k: v.clone() for k, v in drv.model.state_dict().items()}
    assert torch.isfinite(loss_f)
    assert any(not torch.equal(state[k], after_f[k]) for k in state)
    # the fused minibatch, replayed through torch ops on a copy of the model
    rp.sample_ctr.copy_(sample_state[0]); rp.beta_t.copy_(sample_state[1]); rp.prio.copy_(sample_state[2])
    idx, w = rp.sample_fused(drv.train_batch, drv.seed)
    s, ns, a, r, d = (rp.obs[idx], rp.obs[rp.next_index(idx)], rp.action[idx], rp.reward[idx], rp.done[idx])
    import copy as _copy
    model = _copy.deepcopy(drv.model)
    model.load_state_dict(state)
    f = model.features(s)
    q1 = model.move1_head(f).gather(1, a[:, :1]).squeeze(1)
    q2 = model.move2_from_features(f, a[:, 0]).gather(1, a[:, 1:]).squeeze(1)
    with torch.no_grad():
        tf = drv.target.features(ns)
        nq1 = drv.target.move1_head(tf)
        t1 = r + (1 - d) * drv.gamma * nq1.max(1)[0]
        t2 = r + (1 - d) * drv.gamma * drv.target.move2_from_features(tf, nq1.argmax(1)).max(1)[0]
    loss_t = (w * (q1 - t1) ** 2).mean() + (w * (q2 - t2) ** 2).mean()
    assert float(loss_f) == pytest.approx(float(loss_t.detach()), rel=1e-5)


@pytest.mark.parametrize("scale", [1e-3, 50.0])  # clip inactive / active
def test_fused_adam_clip_matches_torch(scale):
    """narde_adam_clip == clip_grad_norm_(10) + torch.optim.Adam over three
    steps, to fp32 rounding (operation order differs)."""
    import copy

    from gym_narde.dqn import DecomposedDQN, FusedAdamClip

    torch.manual_seed(0)
    a = DecomposedDQN(198).cuda()
    b = copy.deepcopy(a)
    ref = torch.optim.Adam(a.parameters(), lr=1e-3)
    fus = FusedAdamClip(b.parameters(), lr=1e-3, max_norm=10.0)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    for _ in range(3):
        grads = [torch.randn(p.shape, device="cuda:0", generator=g) * scale for p in a.parameters()]
        for p, q, gr in zip(a.parameters(), b.parameters(), grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(a.parameters(), max_norm=10.0)
        ref.step()
        fus.step()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6)
    assert int(fus.step_t) == 3


def test_head_policy_kernel_vs_fp64_heads():
    """k_head_policy576 (the fused heads): greedy picks are legal and within
    fp32 rounding of the fp64 masked maximum of f @ W^T + b (+ the one-hot
    column for head 2), nearly always the exact argmax; exploration is
    policy_576's, draw for draw; device-scalar epsilon / tag."""
    from gym_narde.dqn import expand_mask, head_policy_576, policy_576
    from gym_narde.vector import VecNardeEnv

    n = 8192
    env = VecNardeEnv(n, device="cuda:0", seed=23)
    env.selfplay(37)
    words = env.legal_mask()
    m = expand_mask(words)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    f = torch.relu(torch.randn((n, 256), device="cuda:0", generator=g))
    w1 = torch.randn((576, 256), device="cuda:0", generator=g) * 0.06
    w2 = torch.randn((576, 256 + 576), device="cuda:0", generator=g) * 0.06
    b1 = torch.randn(576, device="cuda:0", generator=g) * 0.1
    b2 = torch.randn(576, device="cuda:0", generator=g) * 0.1
    zero = torch.zeros((), device="cuda:0")
    tag = torch.tensor(4, dtype=torch.int64, device="cuda:0")
    a1 = head_policy_576(f, w1, b1, words, zero, 11, tag, 0)
    q1 = (f.double() @ w1.double().t() + b1.double())
    assert greedy_ok(a1, q1, m) > 0.995
    # head 2: the one-hot column of move 1 (move-2 masks from the env)
    words2 = env.legal_mask_move2(a1.to(torch.int16))
    m2 = expand_mask(words2)
    a2 = head_policy_576(f, w2, b2, words2, zero, 11, tag, 1, move1=a1)
    q2 = f.double() @ w2[:, :256].double().t() + b2.double() + w2[:, 256:].double().t()[a1]
    assert greedy_ok(a2, q2, m2) > 0.995
    # exploration: policy_576's draws exactly (epsilon 1 and 0.5, both heads)
    for eps in (1.0, 0.5):
        e = torch.tensor(eps, device="cuda:0")
        for head in (0, 1):
            got = head_policy_576(f, w1, b1, words, e, 11, tag, head)
            q = (f @ w1.t() + b1).contiguous()
            want = policy_576(q, words, e, 11, tag, head)
            explored = got != head_policy_576(f, w1, b1, words, zero, 11, tag, head)
            assert torch.equal(got[explored], want[explored])
            assert bool(m.gather(1, got.view(-1, 1)).squeeze(1)[m.any(1)].all())


@pytest.mark.parametrize("n", [4096, 5000, 37])
def test_gathered_heads_vs_dense_autograd(n):
    """GatheredHeads (narde_dqn_heads_forward / _backward) == the dense heads
    + gather of _update_torch under torch autograd: q1, q2 and every gradient
    (features, both heads' weights and biases) to fp32 rounding; codes
    skewed so some hold hundreds of rows and most of the 576 hold none; a
    row count past one LDS tile (4,096) and a ragged one; deterministic
    from call to call."""
    import copy

    from gym_narde.dqn import DecomposedDQN, gathered_heads

    torch.manual_seed(5)
    model = DecomposedDQN(198).cuda()
    ref = copy.deepcopy(model)
    g = torch.Generator(device="cuda:0").manual_seed(9)
    f0 = torch.relu(torch.randn((n, 256), device="cuda:0", generator=g))
    skew = torch.randint(0, 40, (n, 2), device="cuda:0", generator=g)
    wide = torch.randint(0, 576, (n, 2), device="cuda:0", generator=g)
    a = torch.where(torch.rand((n, 2), device="cuda:0", generator=g) < 0.7, skew, wide).to(torch.int64)
    a[: n // 10, 0] = 0  # the no-move code, common in the ring
    up1 = torch.randn(n, device="cuda:0", generator=g)
    up2 = torch.randn(n, device="cuda:0", generator=g)

    def run(m, gathered):
        f = f0.clone().requires_grad_(True)
        if gathered:
            q1, q2 = gathered_heads(m, f, a)
        else:
            q1 = m.move1_head(f).gather(1, a[:, :1]).squeeze(1)
            q2 = m.move2_from_features(f, a[:, 0]).gather(1, a[:, 1:]).squeeze(1)
        for p in m.parameters():
            p.grad = None
        ((q1 * up1).sum() + (q2 * up2).sum()).backward()
        heads = [m.move1_head.weight.grad, m.move1_head.bias.grad, m.move2_head.weight.grad,
                 m.move2_head.bias.grad]
        return q1.detach(), q2.detach(), f.grad, [h.clone() for h in heads]

    q1, q2, gf, gh = run(model, True)
    r1, r2, rf, rh = run(ref, False)
    assert torch.allclose(q1, r1, rtol=1e-5, atol=1e-5)
    assert torch.allclose(q2, r2, rtol=1e-5, atol=1e-5)
    assert torch.allclose(gf, rf, rtol=1e-5, atol=1e-6)
    for x, y in zip(gh, rh):
        assert x.shape == y.shape
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-4), float((x - y).abs().max())
    # rows no code holds: exactly zero, as the dense path's
    used1 = torch.zeros(576, dtype=torch.bool, device="cuda:0")
    used1[a[:, 0]] = True
    assert bool((gh[0][~used1] == 0).all()) and bool((gh[1][~used1] == 0).all())
    # deterministic: a second call gives the same bits
    s1, s2, sf, sh = run(model, True)
    assert torch.equal(s1, q1) and torch.equal(s2, q2) and torch.equal(sf, gf)
    assert all(torch.equal(x, y) for x, y in zip(sh, gh))


@pytest.mark.parametrize("n", [4096, 1000, 37])
def test_fused_feature_layers_vs_module_autograd(n):
    """features_fused (LinearReLU: narde_relu_bias_grad for the ReLU mask and
    the bias gradient) == model.features under torch autograd: forward
    values, the weight / bias / input gradients of both layers to fp32
    rounding (the weight GEMMs are the same hipBLASLt calls); ragged row
    counts (partial 64-row slices); repeated calls give the same bits."""
    import copy

    from gym_narde.dqn import DecomposedDQN, features_fused, relu_bias_grad_scratch

    torch.manual_seed(7)
    model = DecomposedDQN(198).cuda()
    ref = copy.deepcopy(model)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    x0 = torch.randn((n, 198), device="cuda:0", generator=g)
    up = torch.randn((n, 256), device="cuda:0", generator=g)
    scratch = relu_bias_grad_scratch(n, 256, "cuda:0")

    def run(m, fused):
        x = x0.clone().requires_grad_(True)
        f = features_fused(m, x, scratch) if fused else m.features(x)
        for p in m.parameters():
            p.grad = None
        (f * up).sum().backward()
        grads = [m.feature_network[i].weight.grad.clone() for i in (0, 2)]
        grads += [m.feature_network[i].bias.grad.clone() for i in (0, 2)]
        return f.detach(), x.grad, grads

    f, gx, gr = run(model, True)
    rf, rgx, rgr = run(ref, False)
    assert torch.allclose(f, rf, rtol=1e-5, atol=1e-5)
    assert torch.allclose(gx, rgx, rtol=1e-4, atol=1e-5)
    for a, b in zip(gr, rgr):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4), float((a - b).abs().max())
    f2, gx2, gr2 = run(model, True)
    assert torch.equal(f2, f) and torch.equal(gx2, gx)
    assert all(torch.equal(a, b) for a, b in zip(gr2, gr))


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 4097, 300000])
def test_per_sample_search_exact_on_given_cdf(n):
    """narde_per_sample's 64-ary search (one wave per sample) on a GIVEN
    prefix sum: idx == torch.searchsorted(cdf, u * cdf[-1], right=True)
    clamped to n - 1, exactly, with runs of zero-priority rows (flat
    stretches of the cdf, the ring's pending rows) and ragged sizes; the
    weights normalised by their max; the scratch word left zero."""
    import ctypes

    from gym_narde import _lib

    g = torch.Generator(device="cuda:0").manual_seed(n)
    p = torch.rand(n, device="cuda:0", generator=g) + 0.05
    if n > 4:
        p[torch.rand(n, device="cuda:0", generator=g) < 0.3] = 0.0  # pending rows
        p[0] = 0.0
        p[n // 2:n // 2 + min(100, n // 4)] = 0.0
    p[-1] = 0.5  # (u * total may round to total: the clamp then picks the last row)
    cdf = torch.cumsum(p, 0)
    B = 4096
    idx = torch.empty(B, dtype=torch.int64, device="cuda:0")
    w = torch.empty(B, device="cuda:0")
    u = torch.empty(B, device="cuda:0")
    ctr = torch.zeros((), dtype=torch.int64, device="cuda:0")
    beta = torch.full((), 0.4, dtype=torch.float64, device="cuda:0")
    scratch = torch.zeros(2, dtype=torch.int32, device="cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = _lib.ptr
    _lib.check(_lib.load().narde_per_sample(0, P(p), P(cdf), n, B, 77, P(ctr), P(beta), 0.001, P(idx), P(w), P(u),
                                            P(scratch), st), "narde_per_sample")
    torch.cuda.synchronize()
    want = torch.searchsorted(cdf, u * cdf[-1], right=True).clamp_(max=n - 1)
    assert torch.equal(idx, want)
    x = (n * (p[idx] / cdf[-1])) ** (-0.4)
    assert torch.allclose(w, x / x.max(), rtol=2e-6, atol=0)
    assert int(scratch.abs().sum()) == 0 and int(ctr) == 1
    assert float(beta) == pytest.approx(0.401)


def test_head_policy_strided_outputs_equal_contiguous():
    """k_head_policy576 writing straight into the columns of (B, 2) action
    rows (int64, stride 2), move 1 also as int16, and reading move 1 from
    such a column: the same codes as the contiguous calls."""
    from gym_narde.dqn import head_policy_576
    from gym_narde.vector import VecNardeEnv

    n = 4099
    env = VecNardeEnv(n, device="cuda:0", seed=29)
    env.selfplay(23)
    g = torch.Generator(device="cuda:0").manual_seed(8)
    f = torch.relu(torch.randn((n, 256), device="cuda:0", generator=g))
    w1 = torch.randn((576, 256), device="cuda:0", generator=g) * 0.06
    w2 = torch.randn((576, 256 + 576), device="cuda:0", generator=g) * 0.06
    b1 = torch.randn(576, device="cuda:0", generator=g) * 0.1
    b2 = torch.randn(576, device="cuda:0", generator=g) * 0.1
    eps = torch.tensor(0.3, device="cuda:0")
    tag = torch.tensor(9, dtype=torch.int64, device="cuda:0")
    words = env.legal_mask()
    a1 = head_policy_576(f, w1, b1, words, eps, 5, tag, 0)
    m2 = env.legal_mask_move2(a1.to(torch.int16))
    a2 = head_policy_576(f, w2, b2, m2, eps, 5, tag, 1, move1=a1)
    acts = torch.full((n, 2), -7, dtype=torch.int64, device="cuda:0")
    m1 = torch.empty(n, dtype=torch.int16, device="cuda:0")
    head_policy_576(f, w1, b1, words, eps, 5, tag, 0, out=acts[:, 0], out16=m1)
    head_policy_576(f, w2, b2, env.legal_mask_move2(m1), eps, 5, tag, 1, out=acts[:, 1], move1=acts[:, 0])
    assert torch.equal(acts[:, 0], a1) and torch.equal(acts[:, 1], a2)
    assert torch.equal(m1.to(torch.int64), a1)


def test_target_onehot_rows_cache_follows_target_syncs():
    """The learner's cached (576, 576) one-hot rows of the target move-2 head
    equal the target's weights after every sync, eagerly and across graph
    replays (refreshed in place outside the graph)."""
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    env = VecNardeEnv(2048, device="cuda:0", seed=17)
    drv = BatchedDQNDriver(env, capacity=1 << 13, train_batch=512, seed=4, target_update=2)

    def fresh():
        return drv.target.move2_head.weight[:, 256:].t()

    for _ in range(8):
        drv.step()
    torch.cuda.synchronize()
    assert drv._wm_rows is not None and torch.equal(drv._target_onehot_rows(), fresh())
    drv.capture_graph(warmup=2)
    syncs = 0
    for _ in range(6):
        before = drv.train_steps
        drv.step()
        syncs += (drv.train_steps // 2) - (before // 2)
    torch.cuda.synchronize()
    assert syncs >= 2
    assert torch.equal(drv._wm_rows, fresh())


def test_policies_nan_rows_follow_torch_argmax():
    """A diverging learner's NaN Q-values: both policy
    kernels return a legal code per torch.argmax's rule over the legal codes
    -- the first NaN if any, else the first maximum -- never a sentinel; a
    move-1 code outside 0..575 as the one-hot column index is clamped (no
    out-of-bounds read)."""
    from gym_narde.dqn import expand_mask, head_policy_576, masked_argmax, policy_576
    from gym_narde.vector import VecNardeEnv

    n = 4096
    env = VecNardeEnv(n, device="cuda:0", seed=29)
    env.selfplay(41)
    words = env.legal_mask()
    m = expand_mask(words)
    has = m.any(1)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    f = torch.relu(torch.randn((n, 256), device="cuda:0", generator=g))
    f[: n // 4] = float("nan")  # every code's Q is NaN
    w1 = torch.randn((576, 256), device="cuda:0", generator=g) * 0.06
    w1[300] = float("nan")  # one NaN code in every row (first NaN wins where legal)
    b1 = torch.randn(576, device="cuda:0", generator=g) * 0.1
    zero = torch.zeros((), device="cuda:0")
    tag = torch.zeros((), dtype=torch.int64, device="cuda:0")
    q = (f @ w1.t() + b1).contiguous()
    want = masked_argmax(q, m)
    # the dense policy kernel equals torch.argmax over the masked row exactly
    got = policy_576(q, words, 0.0, seed=1, tag=0, head=0)
    assert torch.equal(got, want)
    # the fused heads: same rule (NaN rows are exact; finite rows within rounding)
    a1 = head_policy_576(f, w1, b1, words, zero, 1, tag, 0)
    nanrow = torch.isnan(q).logical_and(m).any(1)
    assert torch.equal(a1[nanrow], want[nanrow])
    rows = torch.arange(n, device="cuda:0")
    assert bool(m[rows, a1][has].all()) and bool((a1[~has] == 0).all())
    assert int(a1.min()) >= 0 and int(a1.max()) < 576
    # move 2 with out-of-range move-1 codes (as a NaN-era sentinel would be)
    w2 = torch.randn((576, 256 + 576), device="cuda:0", generator=g) * 0.06
    b2 = torch.randn(576, device="cuda:0", generator=g) * 0.1
    bogus = torch.full((n,), 2 ** 31 - 1, dtype=torch.int64, device="cuda:0")
    bogus[::3] = -5
    a2 = head_policy_576(f, w2, b2, words, zero, 1, tag, 1, move1=bogus)
    assert bool(m[rows, a2][has].all())
    tab = torch.randn((576, 576), device="cuda:0", generator=g)
    a2d = policy_576(q, words, 0.0, seed=1, tag=0, head=1, add=(tab, bogus))
    assert torch.equal(a2d, masked_argmax(q + tab[bogus.clamp(0, 575)], m))


@pytest.mark.parametrize("fused", [True, False])
def test_sampler_never_returns_zero_priority_rows(fused):
    """a prefix sum whose flat run (pending rows, p = 0)
    steps up -- a scan's association differs across tiles -- or u * total
    rounded up to total must not pick a zero-priority row, whose weight would
    be inf and turn the batch's weights NaN.  A deliberately stepped cdf puts
    a third of the mass on pending rows: every pick has p > 0, the weights
    are finite, and the kernel's picks equal the torch rule
    (nearest_positive) on the same uniforms."""
    from gym_narde import _lib
    from gym_narde.dqn import DeviceReplay, nearest_positive

    n, B = 6000, 4096
    p = torch.rand(n, device="cuda:0") + 0.05
    p[2000:3000] = 0.0  # a pending run in the middle (a wrapped ring)
    p[n - 500:] = 0.0  # ... and at the end (the fill phase)
    p[:10] = 0.0  # ... and at the start
    cdf = torch.cumsum(p, 0)
    step = float(cdf[-1]) * 0.25
    cdf[2500:3000] += step  # a flat run that steps up (mass on pending rows)
    cdf[3000:] += step
    cdf[n - 200:] += step  # ... and the tail past the last positive row
    if fused:
        import ctypes

        idx = torch.empty(B, dtype=torch.int64, device="cuda:0")
        w = torch.empty(B, device="cuda:0")
        u = torch.empty(B, device="cuda:0")
        ctr = torch.zeros((), dtype=torch.int64, device="cuda:0")
        beta = torch.full((), 0.4, dtype=torch.float64, device="cuda:0")
        scratch = torch.zeros(2, dtype=torch.int32, device="cuda:0")
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        P = _lib.ptr
        _lib.check(_lib.load().narde_per_sample(0, P(p), P(cdf), n, B, 3, P(ctr), P(beta), 0.001, P(idx), P(w),
                                                P(u), P(scratch), st), "narde_per_sample")
        torch.cuda.synchronize()
        raw = torch.searchsorted(cdf, u * cdf[-1], right=True).clamp_(max=n - 1)
        assert bool((p[raw] == 0).float().mean() > 0.2)  # the stepped runs were hit
        assert torch.equal(idx, nearest_positive(p, raw))
    else:
        rp = DeviceReplay(n, 4, "cuda:0", stride=1)
        rp.prio.copy_(p ** (1 / rp.alpha))
        rp.size = n - 1  # rows = size + stride = n
        idx, w = rp.sample(B)
    assert bool((p[idx] > 0).all())
    assert bool(torch.isfinite(w).all()) and float(w.max()) == pytest.approx(1.0)
    # the rule itself: the last positive row before, else the first after
    k = torch.tensor([2500, 5999, 0, 5, 10, 1999], device="cuda:0")
    assert nearest_positive(p, k).tolist() == [1999, 5499, 10, 10, 10, 1999]


# ------------------------------------- round 6: the one-launch learner chains
def _filled_replay(n=5000, ss=198, stride=1234, seed=5):
    from gym_narde.dqn import DeviceReplay

    rp = DeviceReplay(n, ss, "cuda:0", stride=stride)
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    for t in (rp.obs, rp.reward, rp.done):
        t.copy_(torch.rand(t.shape, device="cuda:0", generator=g))
    rp.action.copy_(torch.randint(0, 576, rp.action.shape, device="cuda:0", generator=g))
    rp.prio.copy_(torch.rand(n, device="cuda:0", generator=g) * 3 + 0.01)
    rp.prio[n - stride:] = 0.0  # pending rows: never sampled
    rp.size = n - stride
    return rp


def test_per_sample_gather_equals_sample_then_gather():
    """k_per_sample_gather == k_per_sample + k_per_finish + k_gather_batch:
    the same rows and minibatch, its raw weights normalised by their max are
    the sampler's weights bit for bit; beta and the counter left untouched
    (the loss block steps them)."""
    rp = _filled_replay()
    ctr, beta = rp.sample_ctr.clone(), rp.beta_t.clone()
    idx, w = rp.sample_fused(4096, seed=21)
    want = rp.gather(idx)
    rp.sample_ctr.copy_(ctr)
    rp.beta_t.copy_(beta)
    idx2, w_raw, *got = rp.sample_gather_fused(4096, seed=21)
    assert torch.equal(idx2, idx)
    for x, y in zip(got, want):
        assert torch.equal(x, y)
    assert torch.equal(w_raw / w_raw.max(), w)
    assert int(rp.sample_ctr) == int(ctr) and float(rp.beta_t) == float(beta)
    assert bool((rp.prio[idx2] > 0).all())


def test_target_max2_vs_torch_max_and_rowmax():
    """k_target_max2: (values, indices) of torch.max(dim=1) -- exact ties go to
    the lowest code, a NaN row's first NaN wins -- and the move-2 maximum of
    k_rowmax_addend at that argmax, bit for bit."""
    from gym_narde.dqn import rowmax_addend, target_max2

    g = torch.Generator(device="cuda:0").manual_seed(8)
    n = 4099
    nq1 = torch.randn((n, 576), device="cuda:0", generator=g)
    nq1[::7] = torch.round(nq1[::7])          # many exact ties
    nq1[5, 300] = float("nan")
    nq1[6, 17] = float("nan")
    nq1[6, 400] = float("nan")
    base = torch.randn((n, 576), device="cuda:0", generator=g)
    tab = torch.randn((576, 576), device="cuda:0", generator=g)
    m1, am1, m2 = target_max2(nq1, base, tab)
    v, i = nq1.max(1)
    assert torch.equal(am1, i)
    assert torch.equal(m1[~v.isnan()], v[~v.isnan()]) and bool(m1[v.isnan()].isnan().all())
    assert int(am1[5]) == 300 and int(am1[6]) == 17
    assert torch.equal(m2, rowmax_addend(base, tab, am1))
    # ties: the lowest code holding the row maximum
    rows = torch.arange(0, n, 7, device="cuda:0")
    first = (nq1[rows] == v[rows, None]).int().argmax(1)
    assert torch.equal(am1[rows], first)


def test_loss_prio_block_equals_the_three_kernels():
    """k_dqn_loss_prio == the weight normalisation, k_dqn_loss and
    k_prio_update (+ beta / counter steps): td, dloss/dq, the loss, the
    priorities, max priority, epsilon, cursor and tag, bit for bit."""
    from gym_narde.dqn import DQNLoss

    B, gamma = 4096, 0.99
    rp = _filled_replay(n=20000, stride=64)
    g = torch.Generator(device="cuda:0").manual_seed(12)
    rnd = lambda: torch.randn(B, device="cuda:0", generator=g)  # noqa: E731
    q1, q2, m1, m2 = rnd(), rnd(), rnd(), rnd()
    r = (torch.rand(B, device="cuda:0", generator=g) < 0.1).float() * 2
    d = (torch.rand(B, device="cuda:0", generator=g) < 0.2).float()
    w_raw = torch.rand(B, device="cuda:0", generator=g) * 5 + 0.1
    idx = torch.randperm(20000 - 64, device="cuda:0", generator=g)[:B]
    # the unfused sequence on copies
    prio0, maxp0, ctr0, beta0 = rp.prio.clone(), rp.max_prio.clone(), rp.sample_ctr.clone(), rp.beta_t.clone()
    pos0 = rp.pos_t.clone()
    eps_a = torch.full((), 0.5, device="cuda:0")
    tag_a = torch.zeros((), dtype=torch.int64, device="cuda:0")
    w_n = w_raw / w_raw.max()
    td_a = torch.empty(B, device="cuda:0")
    loss_a, g1a, g2a = DQNLoss.compute(q1, q2, m1, m2, r, d, w_n, gamma, td_a, None)
    rp.update_fused(idx, td_a, eps_a, 0.01, 0.995, cursor_add=64, tag=tag_a)
    prio_a, maxp_a, pos_a = rp.prio.clone(), rp.max_prio.clone(), rp.pos_t.clone()
    # the fused block from the same state
    rp.prio.copy_(prio0); rp.max_prio.copy_(maxp0); rp.pos_t.copy_(pos0)
    eps_b = torch.full((), 0.5, device="cuda:0")
    tag_b = torch.zeros((), dtype=torch.int64, device="cuda:0")
    td_b = torch.empty(B, device="cuda:0")
    loss_b = torch.empty((), device="cuda:0")
    w_b = w_raw.clone()
    g1b, g2b = rp.loss_prio_fused(q1, q2, m1, m2, r, d, w_b, gamma, td_b, loss_b, idx, eps_b, 0.01, 0.995,
                                  cursor_add=64, tag=tag_b)
    assert torch.equal(w_b, w_n)
    assert torch.equal(td_b, td_a) and torch.equal(g1b, g1a) and torch.equal(g2b, g2a)
    assert float(loss_b) == float(loss_a)
    assert torch.equal(rp.prio, prio_a) and float(rp.max_prio) == float(maxp_a) and int(rp.pos_t) == int(pos_a)
    assert float(eps_b) == float(eps_a) and int(tag_b) == int(tag_a) == 1
    assert int(rp.sample_ctr) == int(ctr0) + 1
    assert float(rp.beta_t) == min(1.0, float(beta0) + rp.beta_increment)


def test_adam_float4_vs_scalar_kernels():
    """narde_adam_clip's float4 passes (round 6) against round 5's scalar
    ones: the same clipped Adam steps to fp32 rounding, both deterministic."""
    import copy

    from gym_narde.dqn import DecomposedDQN, FusedAdamClip, learner_variant

    torch.manual_seed(4)
    a = DecomposedDQN(198).cuda()
    b = copy.deepcopy(a)
    fa = FusedAdamClip(a.parameters(), lr=1e-3, max_norm=10.0)
    fb = FusedAdamClip(b.parameters(), lr=1e-3, max_norm=10.0)
    g = torch.Generator(device="cuda:0").manual_seed(6)
    prev = learner_variant(2)
    try:
        for _ in range(3):
            grads = [torch.randn(p.shape, device="cuda:0", generator=g) * 5 for p in a.parameters()]
            for p, q, gr in zip(a.parameters(), b.parameters(), grads):
                p.grad = gr.clone()
                q.grad = gr.clone()
            learner_variant(2)
            fa.step()
            learner_variant(0)
            fb.step()
    finally:
        learner_variant(prev)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6)
    assert int(fa.step_t) == int(fb.step_t) == 3


def test_one_launch_learner_equals_round5_learner():
    """Two drivers from the same seed, one with round 6's one-launch chains
    and one with round 5's: the same losses, priorities and parameters over
    three updates (the fused chains compute the same fp32 values; only the
    clip's norm sums in another order)."""
    from gym_narde.dqn import BatchedDQNDriver
    from gym_narde.vector import VecNardeEnv

    drv = []
    for one in (True, False):
        env = VecNardeEnv(4096, device="cuda:0", seed=41)
        drv.append(BatchedDQNDriver(env, capacity=1 << 14, train_batch=1024, seed=3, one_launch_chains=one))
    losses = [[], []]
    for _ in range(6):
        for k, d in enumerate(drv):
            l = d.step()
            if l is not None:
                losses[k].append(float(l))
    torch.cuda.synchronize()
    assert len(losses[0]) >= 2 and len(losses[0]) == len(losses[1])
    for x, y in zip(*losses):
        assert x == pytest.approx(y, rel=1e-4, abs=1e-6)
    for (k, p), (_, q) in zip(drv[0].model.state_dict().items(), drv[1].model.state_dict().items()):
        assert torch.allclose(p, q, rtol=1e-4, atol=1e-5), k
    assert int(drv[0].replay.sample_ctr) == int(drv[1].replay.sample_ctr)
    assert float(drv[0].replay.beta_t) == float(drv[1].replay.beta_t)
    assert float(drv[0].eps_t) == float(drv[1].eps_t) and int(drv[0].tag_t) == int(drv[1].tag_t)
