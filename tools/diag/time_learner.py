"""DIAGNOSTIC: time the DQN learner kernels in isolation (torch events)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.dqn import DeviceReplay  # noqa: E402


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for n in (1 << 14, 1 << 17, 1 << 20):
    rp = DeviceReplay(n, 4, "cuda:0")
    rp.prio.copy_(torch.rand(n, device="cuda:0") + 0.01)
    rp.size = n
    p = rp.prio ** rp.alpha
    cdf = torch.cumsum(p, 0)
    for B in (1024, 4096):
        u = torch.rand(B, device="cuda:0")
        t_f = timed(lambda: rp.sample_fused(B, 1))
        t_pc = timed(lambda: (rp.prio ** rp.alpha).cumsum(0))
        t_ss = timed(lambda: torch.searchsorted(cdf, u * cdf[-1], right=True))
        print(f"n={n} B={B}: sample_fused {t_f:.1f} us (pow+cumsum alone {t_pc:.1f}); torch searchsorted {t_ss:.1f} us")
