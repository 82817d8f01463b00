#!/usr/bin/env python3
"""DIAGNOSTIC: the write rate a plain streaming fill reaches on this device
(torch fill_ of a 7.5 GB int32 tensor: 16-B vector stores, no reads), after
~0.5 s of warm-up -- the practical roof for a write-only kernel."""
import json
import time

import torch


def main():
    n = 7475298304 // 4
    x = torch.empty(n, dtype=torch.int32, device="cuda:0")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        x.fill_(1)
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 40
    s.record()
    for i in range(reps):
        x.fill_(i)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(json.dumps({"fill_bytes": n * 4, "ms": round(ms, 4), "TBps": round(n * 4 / (ms * 1e-3) / 1e12, 3)}))


if __name__ == "__main__":
    main()
