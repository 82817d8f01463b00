#!/usr/bin/env python3
"""DIAGNOSTIC: which host calls block right after the driver-shape rollout
launch (20 plies, ctypes, on torch's current stream).  For each probe: the
host time of the probe call just after the launch (median of 15, first),
and whether torch's current stream is the null stream.  Probes: ctypes
hipGetDevice, torch.cuda.current_stream(), a view (unsqueeze), is_initialized,
a torch kernel (add_), hipStreamQuery on the launch stream.  Then the same
launch made on a torch-created stream (torch.cuda.Stream) instead."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")
    torch.cuda.set_device(0)
    env = VecNardeEnv(65536, device="cuda:0", seed=0)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    b = env.rollout_buffers(20)
    rows = torch.zeros((256, 3), dtype=torch.int64, device="cuda:0")
    x = torch.zeros(16, device="cuda:0")
    dev = ctypes.c_int()
    out = {"current_stream_handle": int(torch.cuda.current_stream().cuda_stream)}

    def probes(stream_handle):
        return {
            "nothing": lambda: None,
            "hipGetDevice": lambda: hip.hipGetDevice(ctypes.byref(dev)),
            "current_stream": lambda: torch.cuda.current_stream(),
            "unsqueeze": lambda: rows.unsqueeze(0),
            "dist_is_initialized": lambda: dist.is_initialized(),
            "torch_add": lambda: x.add_(1.0),
            "hipStreamQuery": lambda: hip.hipStreamQuery(ctypes.c_void_p(stream_handle)),
        }

    for where in ("current", "side"):
        s = torch.cuda.Stream() if where == "side" else torch.cuda.current_stream()
        with torch.cuda.stream(s):
            L = env.rollout_launcher(20, b)
            L()
            torch.cuda.synchronize()
            for name, P in probes(s.cuda_stream).items():
                times = []
                for _ in range(16):
                    for _ in range(3):
                        ramp()
                    torch.cuda.synchronize()
                    L()
                    t1 = time.perf_counter()
                    P()
                    times.append((time.perf_counter() - t1) * 1e6)
                    torch.cuda.synchronize()
                first, rest = times[0], sorted(times[1:])
                out[f"{where}:{name}"] = [round(first, 1), round(rest[7], 1)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
