"""Host-side logic of the batched DQN driver (gym_narde/dqn.py) on CPU tensors:
the network is the reference's (train_deepq_pytorch.py:184-222), the move-2
column-gather equals the reference's one-hot concat, the mask helpers, and the
prioritized replay rules (:279-342).  The env-facing parts run on the GPU
(tests/test_gpu_dqn.py)."""
import os

import numpy as np
import pytest
import torch

from gym_narde.dqn import DecomposedDQN, DeviceReplay, expand_mask, masked_argmax


def reference_move2(model, x, m1):
    """train_deepq_pytorch.py:219-231: cat(features, onehot(move1)) @ move2_head."""
    f = model.feature_network(x)
    onehot = torch.zeros(x.shape[0], 576)
    onehot.scatter_(1, m1.unsqueeze(1), 1)
    return model.move2_head(torch.cat((f, onehot), 1))


def test_move2_column_gather_equals_onehot_concat():
    torch.manual_seed(0)
    m = DecomposedDQN(198)
    x = torch.rand(257, 198)
    a1 = torch.randint(0, 576, (257,))
    got = m(x, a1)
    ref = reference_move2(m, x, a1)
    # same math, different fp32 summation order: tolerance 1e-5 absolute on
    # O(0.1) values (the one-hot columns add exact zeros in the reference)
    assert torch.allclose(got, ref, rtol=0, atol=1e-5)
    assert torch.equal(m(x), m.move1_head(m.feature_network(x)))


def test_parameter_names_match_reference():
    m = DecomposedDQN(24)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert shapes == {
        "feature_network.0.weight": (256, 24), "feature_network.0.bias": (256,),
        "feature_network.2.weight": (256, 256), "feature_network.2.bias": (256,),
        "move1_head.weight": (576, 256), "move1_head.bias": (576,),
        "move2_head.weight": (576, 832), "move2_head.bias": (576,)}


@pytest.mark.skipif(not os.path.exists("/root/reference/saved_models/narde_model_final.pt"),
                    reason="reference checkpoint not present (it never travels to the GPU box)")
def test_reference_checkpoint_loads():
    sd = torch.load("/root/reference/saved_models/narde_model_final.pt", weights_only=True,
                    map_location="cpu")
    m = DecomposedDQN(24)
    m.load_state_dict(sd, strict=True)


def test_expand_mask_and_masked_argmax():
    rng = np.random.RandomState(1)
    bits = rng.rand(50, 576) < 0.02
    bits[7] = False  # an env with no legal code
    words = np.zeros((50, 9), np.uint64)
    for c in range(576):
        words[:, c >> 6] |= bits[:, c].astype(np.uint64) << np.uint64(c & 63)
    m = expand_mask(torch.from_numpy(words.view(np.int64)))
    assert torch.equal(m, torch.from_numpy(bits))
    q = torch.randn(50, 576)
    a = masked_argmax(q, m)
    for i in range(50):
        if bits[i].any():
            legal = np.nonzero(bits[i])[0]
            assert int(a[i]) == legal[np.argmax(q[i].numpy()[legal])]
        else:
            assert int(a[i]) == 0


def test_replay_priority_rules():
    """DeviceReplay's ring (each observation once, s' = row + stride) and the
    reference's PER rules (train_deepq_pytorch.py:279-342)."""
    r = DeviceReplay(10, 4, "cpu", stride=3)
    obs = [torch.full((3, 4), float(k)) for k in range(6)]
    r.seed(obs[0])
    act = lambda k: torch.full((3, 2), k, dtype=torch.int64)  # noqa: E731
    r.add(act(0), torch.ones(3), obs[1], torch.zeros(3))
    assert r.size == 3 and r.pos == 3 and r.rows == 6
    assert torch.equal(r.obs[0:3], obs[0]) and torch.equal(r.obs[3:6], obs[1])
    assert r.prio[0:3].tolist() == [1.0] * 3 and r.prio[3:6].tolist() == [0.0] * 3  # s' rows pending
    for k in range(1, 4):
        r.add(act(k), torch.ones(3), obs[k + 1], torch.zeros(3))
    # 12 rows written into 10: the ring wrapped; the live transitions are the
    # 7 = capacity - stride rows that are not pending
    assert r.pos == 2 and r.size == 7 and r.rows == 10
    pend = r.next_index(torch.arange(9, 12) % 10)  # the last step's s' rows: 2, 3, 4
    assert sorted(pend.tolist()) == [2, 3, 4] and float(r.prio[pend].sum()) == 0.0
    for j in range(10):  # every live row's next observation is its env's next s
        if float(r.prio[j]) > 0:
            k = int(r.action[j, 0])
            assert torch.equal(r.obs[j], obs[k][0]) and torch.equal(r.obs[(j + 3) % 10], obs[k + 1][0])
    r.update(torch.tensor([6]), torch.tensor([5.0]))
    assert float(r.prio[6]) == pytest.approx(5.01) and float(r.max_prio) == pytest.approx(5.01)
    g = torch.Generator().manual_seed(0)
    idx, w = r.sample(20000, generator=g)
    p = r.prio ** r.alpha
    p = p / p.sum()
    freq = torch.bincount(idx, minlength=10).float() / 20000
    assert torch.allclose(freq, p, atol=0.02)
    assert float(freq[pend].sum()) == 0.0  # pending rows are never sampled
    # importance weights: (N p)^-beta normalised by the max
    beta = r.beta - r.beta_increment
    exp = (10 * p[idx]) ** (-beta)
    assert torch.allclose(w, exp / exp.max())
    # new transitions get the running max priority
    r.add(act(9), torch.ones(3), obs[0], torch.zeros(3))
    assert float(r.prio[2]) == pytest.approx(5.01) and float(r.prio[5]) == 0.0
    with pytest.raises(ValueError):
        DeviceReplay(5, 4, "cpu", stride=3)  # capacity below twice the stride


def test_features_nograd_matches_module():
    from gym_narde.dqn import DecomposedDQN

    torch.manual_seed(0)
    m = DecomposedDQN(198)
    x = torch.randn(64, 198)
    with torch.no_grad():
        assert torch.allclose(m.features_nograd(x), m.features(x), rtol=1e-6, atol=1e-6)
