import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "gym-narde_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden(name):
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


@pytest.fixture(scope="session")
def hostcheck():
    """Test-only host build of the device rules engine (tests/hostcheck)."""
    import ctypes

    path = os.environ.get("NARDE_HOSTCHECK_LIB",  # tools/sanitize.sh: an ASan/UBSan build
                          os.path.join(ROOT, "tests", "hostcheck", "build", "libhostcheck.so"))
    if not os.path.exists(path):
        import __graft_entry__ as g

        g.build()
    return ctypes.CDLL(path)


def in_act_plays(legal, words, count, acts):
    """Per row: (move1, move2) codes `acts` (B,2) int64 are one of
    DQNAgent.act's combinations (train_deepq_pytorch.py:430-507) encoded by
    VecNardeEnv.play_set(kind="act") -> (legal, words, count); (0, 0) for a
    row with no play.  Vectorised (torch, on the device)."""
    import torch

    legal, words, acts = legal.long(), words.long(), acts.long()
    c1, c2 = acts[:, 0], acts[:, 1]
    p, t = (c1 // 24)[:, None], (c1 % 24)[:, None]
    L = torch.stack([legal & 0xFFFFFF, (legal >> 24) & 0xFFFFFF], 1)
    D = torch.stack([(legal >> 48) & 15, (legal >> 52) & 15], 1)
    first = ((L >> p) & 1).bool() & (((t == p - D) & (p >= D)) | ((t == 0) & (p < D)))
    w = words.gather(2, p.clamp(0, 23)[:, :, None].expand(-1, 2, 1)).squeeze(2)
    m2, rem = w & 0xFFFFFF, (w >> 24) & 7
    q, u = (c2 // 24)[:, None], (c2 % 24)[:, None]
    second = torch.where(m2 == 0, (c2 == 0)[:, None],
                         ((m2 >> q.clamp(0, 23)) & 1).bool() & (((u == q - rem) & (q >= rem)) | ((u == 0) & (q < rem))))
    none = (count == 0) & (c1 == 0) & (c2 == 0)
    return (first & second).any(1) | none
