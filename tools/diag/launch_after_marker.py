#!/usr/bin/env python3
"""DIAGNOSTIC: how long the HOST call of a launch takes when it follows the
driver-shape rollout launch (20 plies, with / without its two timing
markers).  bench.py's timed region at round 3 showed ~110-130 us inside the
totals call (tools/diag/gpu_benchcmp2.sh).  For each case: the host time of
the second call (first occurrence after a fresh handle, then the median of
20 repeats), and the whole region (launch + second call + synchronize).
Second calls: the totals kernel (pre-bound), a torch op on the same stream,
an RCCL all-gather on a world-1 process group (ProcessGroupNCCL, and
RCCL's own ncclAllGather through gym_narde.distributed.RcclGather).  argv: plies (20)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gym_narde.vector import TimingEvent, VecNardeEnv  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    b = env.rollout_buffers(P)
    e0, e1 = TimingEvent("cuda:0"), TimingEvent("cuda:0")
    launches = {"marked": env.rollout_launcher(P, b, events=(e0, e1)), "bare": env.rollout_launcher(P, b)}
    rows = torch.empty((64, 3), dtype=torch.int64, device="cuda:0")
    gat = torch.empty((1, 64, 3), dtype=torch.int64, device="cuda:0")
    x = torch.zeros(16, device="cuda:0")
    from gym_narde.distributed import RcclGather

    G = RcclGather(rows)
    seconds = {"totals": env.totals_launcher(rows), "torch_add": lambda: x.add_(1.0),
               "allgather": lambda: dist.all_gather_into_tensor(gat, rows.unsqueeze(0)),
               "rccl_direct": G}
    for f in seconds.values():  # every path once
        f()
    torch.cuda.synchronize()
    out = {"plies": P}
    for lname, L in launches.items():
        for sname, S in seconds.items():
            call, region = [], []
            for _ in range(21):
                for _ in range(3):
                    ramp()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                L()
                t1 = time.perf_counter()
                S()
                t2 = time.perf_counter()
                torch.cuda.synchronize()
                t3 = time.perf_counter()
                call.append((t2 - t1) * 1e6)
                region.append((t3 - t0) * 1e6)
            first = call[0]
            call, region = sorted(call[1:]), sorted(region[1:])
            out[f"{lname}+{sname}"] = {"call_first_us": round(first, 1), "call_med_us": round(call[10], 1),
                                       "region_med_us": round(region[10], 1)}
    # the launch alone
    for lname, L in launches.items():
        region = []
        for _ in range(21):
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L()
            torch.cuda.synchronize()
            region.append((time.perf_counter() - t0) * 1e6)
        out[f"{lname} alone"] = {"region_med_us": round(sorted(region)[10], 1)}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
