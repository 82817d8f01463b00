#!/usr/bin/env python3
"""Benchmark: env steps/s of batched random-policy Narde self-play.

Workload (BASELINE.json metric, configs[2] at N=1): 65,536 envs per GPU in
lockstep; one bench step = one ply of NardeEnv.step over every env (device
dice uniform over the 36 ordered pairs, list #1, in-kernel random legal
policy, the reference's action decode and die bookkeeping, list #2, end
check, flip, TimeLimit 1000, auto-reset) writing every per-env output
(int32[24] obs, reward, terminated, truncated, compact legal set, actions) --
one k_step launch per step.  N GPUs = N processes (torchrun), each owning a
contiguous shard of global env ids (weak scaling); the timed region ends with
the RCCL all-gather of per-env episode statistics.

Prints ONE JSON line on rank 0 (see README/DESIGN.md for the fields).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "env steps/sec at batch=65536, 1 MI355X (+ legal-move bit-exact vs CPU)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes per env-step of k_step:
# record read 32 + write 32, obs 96, reward 4, terminated 1, truncated 1,
# compact legal set 8, actions 4
BYTES_PER_STEP = 178
BYTES_PER_STEP_FUSED_STATE = 64  # per env per fused launch (record r+w), amortised over plies


def _port_worker(args):
    seed, seconds = args
    import narde_port

    steps, wall, eps = narde_port.selfplay_port(64, seconds=seconds, seed=seed)
    return steps, wall


def cpu_baseline(seconds, cores):
    """Python restatement of the reference env (same per-env loop structure),
    one process per core, plus the C oracle on one core.  Runs BEFORE any GPU
    initialisation (fork is safe then)."""
    import multiprocessing as mp

    import oracle as O

    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(_port_worker, [(s, seconds) for s in range(cores)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    sp = O.SelfPlay(4096, seed=1)
    sp.reset(0)
    t0 = time.perf_counter()
    plies = 0
    while time.perf_counter() - t0 < min(2.0, seconds):
        sp.run(25, record=False)
        plies += 25
    c_rate = 4096 * plies / (time.perf_counter() - t0)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(steps / wall, 1),
        "unit": "env steps/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle/narde_port.py (Python restatement of NardeEnv.step, reference loop "
                   f"structure) random-legal self-play, 64 envs x {seconds:.1f}s per process, "
                   f"{cores} processes, {steps} env steps; CPU: {cpu_model}"),
        "c_oracle_1core": round(c_rate, 1),
    }


def load_traffic(path, envs):
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if d.get("envs") != envs:
        return None
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--fused-plies", type=int, default=100)
    ap.add_argument("--fused-launches", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--cpu-cores", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_k_step.json"))
    args = ap.parse_args()

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank_env = int(os.environ.get("RANK", "0"))
    cpu = None
    if world_env == 1 and rank_env == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_cores)

    import torch
    import torch.distributed as dist

    from gym_narde import distributed as D
    from gym_narde.vector import VecNardeEnv

    rank, world, local = D.init_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    first, per = D.env_shard(world * args.envs, rank, world)
    env = VecNardeEnv(per, device=dev, seed=args.seed, env_id_offset=first, max_episode_steps=1000)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        env.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()

    K = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record()
        env.step()
        ev[i][1].record()
    stats = D.gather_stats(env.stats())
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(s.elapsed_time(e) for s, e in ev) / K

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    total_steps = world * per * K
    value = total_steps / elapsed
    summary = D.summarize(stats)

    # secondary: fused self-play (K plies per launch, state in VGPRs, no per-ply outputs)
    P, L = args.fused_plies, args.fused_launches
    env.selfplay(P)
    torch.cuda.synchronize()
    barrier()
    fe = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(L)]
    f0 = time.perf_counter()
    for i in range(L):
        fe[i][0].record()
        env.selfplay(P)
        fe[i][1].record()
    torch.cuda.synchronize()
    barrier()
    f_elapsed = time.perf_counter() - f0
    f_kern_ms = sum(s.elapsed_time(e) for s, e in fe) / L
    ft = torch.tensor([f_elapsed, f_kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ft, op=dist.ReduceOp.MAX)
    f_elapsed, f_kern_ms = float(ft[0]), float(ft[1])

    if rank == 0:
        achieved = BYTES_PER_STEP * per / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(args.traffic_json, per)
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Philox dice, random legal policy, start position + auto-reset)",
            "config": {
                "workload": ("configs[2]: batch=65536 random-policy self-play per GPU; rules = "
                             "reference NardeEnv.step (REF2: <=2 checker moves per step, also on "
                             "doubles); dice uniform over 36 ordered pairs; TimeLimit 1000; one "
                             "k_step launch per ply writing obs/reward/terminated/truncated/"
                             "legal set/actions for every env"),
                "envs_per_gpu": per,
                "global_envs": world * per,
                "parallelism": f"dp{world} (env-id shards, 1 RCCL all-gather of stats)",
                "episodes_finished": summary["episodes"],
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_step",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "bytes_per_env_step": BYTES_PER_STEP,
                "kernel_ms": round(kern_ms, 5),
            },
            "cpu_baseline": cpu,
            "fused_selfplay": {
                "value": round(world * per * P * L / f_elapsed, 1),
                "unit": "env steps/s",
                "plies_per_launch": P,
                "kernel": "k_selfplay",
                "kernel_ms": round(f_kern_ms, 5),
                "outputs": "per-env statistics only",
            },
        }
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
