#!/usr/bin/env python3
"""The per-call API kernels warm, at B = 65,536:
k_step<false> (REF2 VecNardeEnv.step), k_step<true> (FULL4 step),
k_observe's 198-float Tesauro observation and its int32[24] one.  Each runs
`--warm` untimed then `--reps` timed calls back to back; HIP events around
each run give microseconds per eager call (`us`: the host's call rate when
the kernel is shorter than the call, as k_observe's is), and the same calls
replayed from a CUDA graph give the device time per call (`graph_us`: the
kernel plus the gap between dispatches).  The same command under
`rocprofv3 --kernel-trace --stats` gives the per-dispatch durations
(tools/gpu_round.sh commits that summary).  Prints one JSON line.

`floor_*`: torch's zero_ / fill_ / copy_ kernels at the same byte counts
(what a traced dispatch of that size costs).

Algorithmic bytes per env: k_step 64 (record r+w) +
114 (REF2 outputs) / 118 (FULL4) B; the observations 32 (record read) +
792 / 96 B."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))

import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402

HBM_PEAK = 8.0e12


def timed(fn, warm, reps):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def graphed(fn, reps, per_graph=50):
    """Device time per call: `per_graph` calls captured in one CUDA graph,
    replayed until `reps` calls ran, HIP events around the replays -- no
    host launch cost between kernels (an eager call of a ~4-us kernel is
    bound by the host's ~6-us call, so HIP events around eager calls measure
    the host, not the kernel)."""
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for _ in range(per_graph):
                fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    R = max(1, reps // per_graph)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(R):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (R * per_graph)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    n = a.envs
    out = {"envs": n, "reps": a.reps}
    for rules, per_env in (("ref2", 64 + 114), ("full4", 64 + 118)):
        env = VecNardeEnv(n, device="cuda:0", seed=0, rules=rules)
        us = timed(env.step, a.warm, a.reps)
        gus = graphed(env.step, a.reps)
        out[f"k_step_{rules}"] = {"us": round(us, 2), "graph_us": round(gus, 2), "bytes": n * per_env,
                                  "frac": round(n * per_env / (us * 1e-6) / HBM_PEAK, 4),
                                  "graph_frac": round(n * per_env / (gus * 1e-6) / HBM_PEAK, 4)}
        env.close()
    env = VecNardeEnv(n, device="cuda:0", seed=0)
    env.selfplay(100)
    obs198 = torch.empty((n, 198), dtype=torch.float32, device="cuda:0")
    for kind, per_env, fn in (("tesauro198", 32 + 792, lambda: env.tesauro198(out=obs198)),
                              ("observe_int24", 32 + 96, env.observe)):
        us = timed(fn, a.warm, a.reps)
        gus = graphed(fn, a.reps)
        out[kind] = {"us": round(us, 2), "graph_us": round(gus, 2), "bytes": n * per_env,
                     "frac": round(n * per_env / (us * 1e-6) / HBM_PEAK, 4),
                     "graph_frac": round(n * per_env / (gus * 1e-6) / HBM_PEAK, 4)}
    env.close()
    # floors (round 6): torch's own kernels writing the same
    # bytes, so the trace shows what a dispatch of this size costs there --
    # a 4-byte zero_ (the launch alone), fill_ of k_observe's 6.3 MB and of
    # k_step's 7.5 MB of outputs, a copy_ of k_observe's 8.4 MB
    floors = {"zero_4B": torch.empty(1, dtype=torch.int32, device="cuda:0"),
              "fill_obs24": torch.empty((n, 24), dtype=torch.int32, device="cuda:0"),
              "fill_step_outputs": torch.empty(n * 114 // 4, dtype=torch.int32, device="cuda:0")}
    src = torch.zeros(n * 64 // 4, dtype=torch.int32, device="cuda:0")  # 4.2 MB read + 4.2 written
    dst = torch.empty_like(src)
    for kind, fn in (("zero_4B", floors["zero_4B"].zero_), ("fill_obs24", lambda: floors["fill_obs24"].fill_(7)),
                     ("fill_step_outputs", lambda: floors["fill_step_outputs"].fill_(7)),
                     ("copy_observe_bytes", lambda: dst.copy_(src))):
        us = timed(fn, a.warm, a.reps)
        gus = graphed(fn, a.reps)
        out["floor_" + kind] = {"us": round(us, 2), "graph_us": round(gus, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
