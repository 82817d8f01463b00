"""GPU differential fuzzing ("CPU-twin vs HIP differential
fuzzing on the GPU box"): random positions far from self-play -- run-heavy
boards where the block rule decides (narde.py:139-184) and bear-off
endgames (narde.py:73-77) -- for both colours, with random first-turn
flags and rolls of 1-4 dice, through libnarde.so's C ABI against the CPU
oracle (oracle/narde_oracle.c, pinned to the reference's golden vectors).
Bit-exact (integer work)."""
import numpy as np
import pytest
from fuzz_positions import random_positions

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


def test_legal_moves_random_positions_vs_oracle():
    n = 65536
    board, off, ft, player, rng = random_positions(n, 101)
    nd = rng.integers(1, 5, n).astype(np.uint8)
    roll = np.zeros((n, 4), np.uint8)
    d0 = rng.integers(1, 7, n)
    roll[:, 0] = d0
    roll[:, 1] = np.where(nd >= 2, np.where(rng.random(n) < 0.3, d0, rng.integers(1, 7, n)), 0)
    roll[:, 2] = np.where(nd >= 3, d0, 0)  # 3- and 4-die rolls: doubles as the web manager rolls them
    roll[:, 3] = np.where(nd >= 4, d0, 0)
    ref_moves, ref_cnt = O.legal_moves(board, ft, player, roll, nd)
    env = vec(n)
    env.set_state(torch.from_numpy(board), torch.from_numpy(off), torch.from_numpy(ft),
                  torch.from_numpy(player))
    count, moves, _ = env.legal_moves(dice=torch.from_numpy(roll))
    assert np.array_equal(np_(count), ref_cnt)
    assert np.array_equal(np_(moves), ref_moves)
    # the sample reaches the rules that decide on these positions
    assert (ref_cnt == 0).any() and (ref_moves[..., 1] == 24).any()


def test_full4_random_positions_vs_oracle():
    """FULL4 turns on the same kind of positions, half
    of them doubles: the first-sub-move set and max dice of the device turn
    (block-free shortcuts, mask pair checks, chain counts, cooperative
    searches) against the oracle's exhaustive composition; the oracle's own
    sub-moves replayed as explicit plays reach the same board."""
    n = 32768
    board, off, ft, player, rng = random_positions(n, 202)
    d0 = rng.integers(1, 7, n)
    d1 = np.where(rng.random(n) < 0.5, d0, rng.integers(1, 7, n))
    dice = np.stack([d0, d1], 1).astype(np.uint8)
    words = rng.integers(0, 2 ** 32, (n, 4), dtype=np.uint64).astype(np.uint32)
    ro = O.full4_turn(board, off, ft, player, dice, words)
    hi = np.maximum(d0, d1).astype(np.uint64)
    lo = np.minimum(d0, d1).astype(np.uint64)
    c = ro["cmask"][:, 0, :].astype(np.uint64)
    want = (c[:, 0] | (c[:, 1] << np.uint64(24)) | (hi << np.uint64(48)) | (lo << np.uint64(52))
            | (ro["max_dice"].astype(np.uint64) << np.uint64(56)))
    env = vec(n, rules="full4", max_episode_steps=0, autoreset=False)
    env.set_state(torch.from_numpy(board), torch.from_numpy(off), torch.from_numpy(ft),
                  torch.from_numpy(player))
    w = env.legal_full(torch.from_numpy(dice))
    assert np.array_equal(np_(w).view(np.uint64), want)
    env.step(torch.from_numpy(np.ascontiguousarray(ro["played"])), torch.from_numpy(dice))
    s = env.get_state()
    assert np.array_equal(np_(s["board"]), ro["board"])
    assert np.array_equal(np_(s["off"]), ro["off"])
    M = ro["max_dice"]
    assert all((M == m).any() for m in range(5))
