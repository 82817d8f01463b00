#!/usr/bin/env python3
"""DIAGNOSTIC: the config-4 act path's first feature layer (65,536 x K ->
256, fp32, bias + ReLU epilogue) for K = 198 as stored, 198 over rows
padded to 200 floats (lda = 200), and zero-padded K = 200 / 208 / 256;
microseconds per GEMM, back to back.  $NARDE_TUNED_GEMMS=1 loads the
TunableOp results file first (as bench.py does)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 2)


def main():
    if os.environ.get("NARDE_TUNED_GEMMS") == "1":
        from gym_narde.dqn import use_tuned_gemms

        use_tuned_gemms()
    B, N = 65536, 256
    g = torch.Generator(device="cuda:0").manual_seed(0)
    bias = torch.randn(N, device="cuda:0", generator=g)
    out = {"tuned": os.environ.get("NARDE_TUNED_GEMMS") == "1"}
    w198 = torch.randn((N, 198), device="cuda:0", generator=g)
    x198 = torch.randn((B, 198), device="cuda:0", generator=g)
    out["k198"] = timeit(lambda: torch._addmm_activation(bias, x198, w198.t()))
    xp = torch.zeros((B, 200), device="cuda:0")
    xp[:, :198] = x198
    out["k198_lda200"] = timeit(lambda: torch._addmm_activation(bias, xp[:, :198], w198.t()))
    for K in (200, 208, 256):
        x = torch.zeros((B, K), device="cuda:0")
        x[:, :198] = x198
        w = torch.zeros((N, K), device="cuda:0")
        w[:, :198] = w198
        out[f"k{K}_padded"] = timeit(lambda: torch._addmm_activation(bias, x, w.t()))
        ref = torch._addmm_activation(bias, x198, w198.t())
        got = torch._addmm_activation(bias, x, w.t())
        out[f"k{K}_maxdiff"] = float((ref - got).abs().max())
    w256 = torch.randn((N, 256), device="cuda:0", generator=g)
    x256 = torch.randn((B, 256), device="cuda:0", generator=g)
    out["layer2_k256"] = timeit(lambda: torch._addmm_activation(bias, x256, w256.t()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
