#!/usr/bin/env python3
"""Per-step breakdown of the configs[3] DQN driver from a kernel trace.

  rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o dqn \
      -- python3 tools/dqn_target.py 65536 20
  python3 tools/dqn_breakdown.py OUT [--out profiles/.../dqn_breakdown.json]

Splits every graph-replayed step of the trace (BatchedDQNDriver._step_body,
gym_narde/dqn.py) at its env step: `act` = the kernels from the previous
step's last learner kernel (k_prio_update, or round 6's k_adam4) up to k_step (the 65,536-row
feature GEMMs, the two head-policy kernels, the masks, the exploration
draw), `env` = k_step + k_dqn_transition, `update` = the rest (the 4,096-row
learner: sampling, gathers, GEMMs, loss, gradients, clip + Adam, priority
update).  The act GEMMs are the feature layers (DecomposedDQN,
train_deepq_pytorch.py:184-231: 198 -> 256 -> 256 on B = 65,536 rows; both
256 -> 576 heads are evaluated inside k_head_policy576 for the legal codes
only, no dense head GEMM): 2 x B x (198*256 + 256*256) = 15.2 GFLOP per
step, priced against the fp32 MFMA dense peak (MI355X_MICROARCH.md:
157.3 TFLOP/s).  Measurement tool, never shipped.
"""
import argparse
import csv
import glob
import json
import os

FP32_MFMA_PEAK = 157.3e12
ACT_DIMS = 198 * 256 + 256 * 256  # the feature layers (the heads run in k_head_policy576)


def is_gemm(name):
    return name.startswith("Cijk_") or "gemm" in name.lower() or "Gemm" in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--out")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    step_ix = [j for j, k in enumerate(ks) if "k_step<false>" in k[0]]
    # a learner ends at k_prio_update (round 5) or at its clip + Adam
    # (round 6: the priorities ride in k_dqn_loss_prio, before the backward)
    prio_ix = [j for j, k in enumerate(ks) if "k_prio_update" in k[0] or "k_adam" in k[0]]
    steps = []
    for s0, s1 in zip(step_ix, step_ix[1:]):
        before = [p for p in prio_ix if p < s0]
        if not before:
            continue
        a0 = before[-1] + 1
        end = max(p for p in prio_ix if p < s1)  # this step's learner ends at its last marker
        act = ks[a0:s0]
        env = [k for k in ks[s0:end + 1] if "k_step<false>" in k[0] or "k_dqn_transition" in k[0]]
        upd = [k for k in ks[s0:end + 1] if k not in env]
        dur = lambda ls: sum(e - b for _, b, e in ls) / 1e3  # noqa: E731  (us, kernel time)
        steps.append({
            "act_us": dur(act), "act_gemm_us": dur([k for k in act if is_gemm(k[0])]),
            "env_us": dur(env), "update_us": dur(upd),
            "update_gemm_us": dur([k for k in upd if is_gemm(k[0])]),
            "kernels": len(act) + len(env) + len(upd),
            "wall_us": (ks[end][2] - ks[a0][1]) / 1e3,
        })
    steps = steps[-10:]  # the steady replays
    mean = {k: round(sum(s[k] for s in steps) / len(steps), 2) for k in steps[0]}
    act_flops = 2.0 * a.envs * ACT_DIMS
    mean["act_gemm_gflop"] = round(act_flops / 1e9, 2)
    g = mean["act_gemm_us"] * 1e-6
    mean["act_gemm_tflops"] = round(act_flops / g / 1e12, 1) if g > 0 else None
    mean["act_gemm_frac_of_fp32_mfma_peak"] = round(act_flops / g / FP32_MFMA_PEAK, 3) if g > 0 else None
    mean["steps_averaged"] = len(steps)
    mean["source"] = os.path.relpath(path)
    text = json.dumps(mean, indent=1)
    if a.out:
        open(a.out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
