#!/usr/bin/env python3
"""DIAGNOSTIC: the anatomy of ONE rollout launch at the driver's bench shape
(bench.py --steps P --warmup 5: device ramped, GPU idle, one launch timed).
For P in argv (default 1 2 5 10 20 40) prints the median over 30 trials of
the host round trip (launch + torch.cuda.synchronize) and of the kernel's
own span (hipExtLaunchKernel events), plus the back-to-back time per launch.
$NARDE_LIB selects the library; argv[1] may be 'full4'; $NARDE_TOTALS=1
gives the timed launch the totals rows, as bench.py's timed launch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.vector import VecNardeEnv  # noqa: E402


def main():
    args = sys.argv[1:]
    rules = "ref2"
    if args and args[0] in ("ref2", "full4"):
        rules, args = args[0], args[1:]
    plies = [int(a) for a in args] or [1, 2, 5, 10, 20, 40]
    env = VecNardeEnv(65536, device="cuda:0", seed=0, rules=rules)
    big = env.rollout_buffers(1000)
    ramp = env.rollout_launcher(1000, big)
    for _ in range(120):
        ramp()
    torch.cuda.synchronize()
    out = {"lib": os.path.basename(os.environ.get("NARDE_LIB", "libnarde.so")), "rules": rules}
    # $NARDE_EVENTS: torch (torch.cuda.Event) | nofence | default | todevice
    # (library TimingEvents with hipEventDisableSystemFence / 0 / ReleaseToDevice)
    kind = os.environ.get("NARDE_EVENTS", "torch")
    out["events"] = kind
    if kind == "torch":
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e1.record()
        span_of = lambda: e0.elapsed_time(e1)  # noqa: E731
    else:
        from gym_narde.vector import TimingEvent

        fl = {"nofence": TimingEvent.DISABLE_SYSTEM_FENCE, "default": 0, "todevice": 0x40000000}[kind]
        e0, e1 = TimingEvent("cuda:0", fl), TimingEvent("cuda:0", fl)
        span_of = lambda: e0.elapsed_ms(e1)  # noqa: E731
    for P in plies:
        b = env.rollout_buffers(P)
        tot = None
        if os.environ.get("NARDE_TOTALS") == "1":
            from gym_narde import _lib

            tot = torch.zeros((_lib.wg_rows(env.num_envs), 3), dtype=torch.int64, device="cuda:0")
        L = env.rollout_launcher(P, b, events=(e0, e1), totals=tot)
        Lb = env.rollout_launcher(P, b)
        trip, span, bare = [], [], []
        for _ in range(30):
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            Lb()
            torch.cuda.synchronize()
            bare.append((time.perf_counter() - t0) * 1e6)
            for _ in range(3):
                ramp()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L()
            torch.cuda.synchronize()
            trip.append((time.perf_counter() - t0) * 1e6)
            span.append(span_of() * 1e3)
        trip.sort()
        span.sort()
        bare.sort()
        for _ in range(3):
            ramp()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(30):
            Lb()
        s1.record()
        torch.cuda.synchronize()
        out[P] = {"trip_us": round(trip[15], 2), "trip_bare_us": round(bare[15], 2), "span_us": round(span[15], 2),
                  "span_min_us": round(span[0], 2), "b2b_us": round(s0.elapsed_time(s1) * 1e3 / 30, 2)}
        del L, Lb, b
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
