#!/usr/bin/env python3
"""DIAGNOSTIC: k_heads_grad_w (+ k_heads_grad_f) time per call at the
config-4 learner shape (4,096 rows) for code distributions of different
skew, and the code histogram of a real DQN replay ring (config 4 after a
short run).  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.dqn import BatchedDQNDriver, DecomposedDQN  # noqa: E402
from gym_narde.vector import VecNardeEnv  # noqa: E402


def time_backward(model, f, a, reps=200):
    """back-to-back narde_dqn_heads_backward calls (k_heads_grad_f +
    k_heads_grad_w), microseconds per call"""
    from gym_narde import _lib

    n = f.shape[0]
    g1 = torch.randn(n, device="cuda:0")
    g2 = torch.randn(n, device="cuda:0")
    w1, w2 = model.move1_head.weight, model.move2_head.weight
    gf = torch.empty((n, 256), device="cuda:0")
    gw1, gw2 = torch.empty_like(w1), torch.empty_like(w2)
    gb1 = torch.empty(576, device="cuda:0")
    gb2 = torch.empty(576, device="cuda:0")
    a = a.contiguous()
    lib = _lib.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = _lib.ptr
    args = (0, P(g1), P(g2), P(f), f.stride(0), P(w1), w1.stride(0), P(w2), w2.stride(0), P(a), n, P(gf), P(gw1),
            P(gb1), P(gw2), P(gb2), st)

    for _ in range(5):
        _lib.check(lib.narde_dqn_heads_backward(*args), "bwd")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        lib.narde_dqn_heads_backward(*args)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 2)


def main():
    out = {}
    n = 4096
    model = DecomposedDQN(198).cuda()
    g = torch.Generator(device="cuda:0").manual_seed(1)
    f = torch.relu(torch.randn((n, 256), device="cuda:0", generator=g))
    uni = torch.randint(0, 576, (n, 2), device="cuda:0", generator=g)
    out["bwd_us_uniform"] = time_backward(model, f, uni)
    for frac in (0.05, 0.25, 0.5):
        a = uni.clone()
        a[torch.rand(n, device="cuda:0", generator=g) < frac, 1] = 0
        out[f"bwd_us_code0_{frac}"] = time_backward(model, f, a)
    env = VecNardeEnv(65536, device="cuda:0", seed=1)
    drv = BatchedDQNDriver(env, train_batch=4096, capacity=1 << 20)
    for _ in range(25):
        drv.step()
    torch.cuda.synchronize()
    rows = drv.replay.rows
    act = drv.replay.action[:rows]
    for h in (0, 1):
        cnt = torch.bincount(act[:, h], minlength=576).float() / rows
        top = torch.topk(cnt, 5)
        out[f"ring_head{h}_top5"] = [(int(i), round(float(v), 4)) for v, i in zip(top.values, top.indices)]
        out[f"ring_head{h}_codes_used"] = int((cnt > 0).sum())
    idx, _ = drv.replay.sample_fused(4096, drv.seed)
    a = drv.replay.action[idx].contiguous()
    out["bwd_us_ring_sample"] = time_backward(model, f, a)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
