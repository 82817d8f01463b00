#!/usr/bin/env python3
"""Benchmark: env steps/s of batched random-policy Narde self-play.

Workload (BASELINE.json metric, configs[2] at N=1): 65,536 envs per GPU in
lockstep.  One bench step = one ply of NardeEnv.step over every env: device
dice uniform over the 36 ordered pairs, list #1, in-kernel random legal
policy, the reference's action decode and die bookkeeping, list #2, end
check, flip, TimeLimit 1000, auto-reset -- and every per-env output of the
ply written to HBM (int32[24] obs, reward, terminated, truncated, compact
legal set, actions).  The timed path is k_rollout: P plies per launch with
the env record in VGPRs, each ply's outputs streamed to [P][B] rollout
buffers (K steps = ceil(K/P) launches).  The per-ply API kernel k_step is
measured beside it (eager and hipGraph-replayed).  N GPUs = N processes,
each owning a contiguous shard of global env ids (weak scaling): under
torchrun (WORLD_SIZE set) the bench is one rank and checks that the world
size equals --gpus; run plainly with --gpus N > 1 it starts the N ranks
itself (torch.distributed.run, 127.0.0.1) before touching the GPU.  The
timed region ends with every rank's episode totals (one kernel) and, at
N > 1, the RCCL all-gather of them.

Prints ONE JSON line on rank 0 (fields: DESIGN.md section 6).
"""
import argparse
import gc
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-narde_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "env steps/sec at batch=65536, 1 MI355X (+ legal-move bit-exact vs CPU)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes: per env and ply the outputs
# obs 96 + reward 4 + terminated 1 + truncated 1 + compact legal set 8 +
# actions 4 = 114 B; per env and launch the 32-B record read + written = 64 B
OUT_BYTES_PER_STEP = 114
RECORD_BYTES = 64
# FULL4: the same per-ply outputs with the 8-B played
# sub-moves instead of the 4-B action codes = 118 B
OUT_BYTES_PER_STEP_FULL = 118
# speed of oracle/narde_port.py over the imported reference, same core
# (tools/calibrate_port.py)
PORT_OVER_REFERENCE = 1.015
# plies per launch of the untimed device ramp
RAMP_PLIES = 1000


def launch_bytes(envs, plies, full=False):
    return envs * ((OUT_BYTES_PER_STEP_FULL if full else OUT_BYTES_PER_STEP) * plies + RECORD_BYTES)


def _port_worker(args):
    seed, seconds = args
    import narde_port

    steps, wall, eps = narde_port.selfplay_port(64, seconds=seconds, seed=seed)
    return steps, wall


def available_cores():
    """(cores, how): the CPUs this process may run on -- its affinity set,
    capped by a cgroup CPU quota if one is set (on the GPU pool the affinity
    set is the whole machine, the quota the box's share)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:  # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is None:
        return aff, f"{aff} CPUs in the affinity set, no cgroup CPU quota"
    n = max(1, min(aff, int(quota)))
    return n, f"{aff} CPUs in the affinity set, cgroup CPU quota {quota:g} CPUs"


def cpu_baseline(seconds, cores, how):
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
                   f"{cores} processes (one per available core: {how}), {steps} env steps; "
                   f"CPU: {cpu_model}"),
        "cpu_model": cpu_model,
        # tools/calibrate_port.py in the build container: the port runs
        # 12,293 steps/s/core against the imported reference's 12,116
        "port_over_reference": PORT_OVER_REFERENCE,
        "c_oracle_1core": round(c_rate, 1),
    }


# the parity_check leg's cost model: the C oracle's self-play rate per host
# core (env steps/s; conservative -- measured 0.6-1.7e6 REF2 and 0.04-0.11e6
# FULL4 on the build container and the GPU box's EPYC 9575F)
ORACLE_RATE = {"ref2": 1.0e6, "full4": 8.0e4}
PARITY_MIN_ENVS = 16384


def parity_envs(per, plies, rules, core_s):
    """Envs the checker replays for `plies` plies within `core_s` core-seconds
    of oracle work: the whole shard when it fits, else a prefix of at least
    PARITY_MIN_ENVS envs (a multiple of 256, one workgroup's envs)."""
    fit = int(core_s * ORACLE_RATE[rules] / max(1, plies))
    if fit >= per:
        return per
    return min(per, max(PARITY_MIN_ENVS, fit // 256 * 256))


def host_bufs(bufs, plies, envs):
    """Host copies of the first `plies` rows and `envs` envs of rollout
    buffers (the checker's input; untimed)."""
    return {k: (v[:plies, :envs].cpu().numpy() if v is not None else None) for k, v in bufs.items()}


def run_parity(item, threads):
    """The checker leg (oracle/replay.py): the oracle replays what the device
    played from the snapshot taken before it and compares every output.
    Same standing as cpu_baseline: test infrastructure, run after the GPU
    work it checks, never inside a timed region."""
    import replay as R

    res = R.check(item["before"], item["bufs"], item["after"], item["plies"], item["seed"],
                  env0=item["env0"], full=item["rules"] == "full4", envs=item["envs"], threads=threads,
                  totals_rows=item.get("totals_rows"))
    res["scope"] = item["scope"]
    res["env_ids"] = f"{item['env0']}..{item['env0'] + item['envs'] - 1}"
    return res


def kernel_name(full4, plies):
    """The kernel narde_rollout[_full] launches with outputs (narde.hip):
    REF2 is the producer/consumer workgroup k_rollout_pc, FULL4 the pairwise
    producer/consumer k_rollout_pp_full; one store form at every launch
    length since round 6 (round 5's had a second one past 32 plies)."""
    return "k_rollout_pp_full<true>" if full4 else "k_rollout_pc<true>"


def load_traffic(path, envs, plies, kernel):
    """HBM bytes per k_rollout launch from the committed rocprofv3 PMC
    summary (tools/pmc_summary.py), if it was measured at this shape on this
    kernel (its `kernel` filter is a prefix of the launched kernel's name)."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    k = d.get("kernel")
    if d.get("envs") != envs or d.get("plies") != plies or not k or k not in kernel:
        return None
    return d.get("hbm_bytes_per_launch")


# SURVEY.md 8(d)'s secondary figure: VALU wave-instructions per launch (a
# committed SQ-counter summary at the launch shape, tools/sq_summary.py)
# against the chip's integer VALU issue peak -- one VALU wave-instruction per
# 4 cycles per SIMD: what one wave issues of any kind, and two waves of the
# slow kinds; two waves issue the fast kinds every 2 cycles
# (profiles/r05/issue_probe/summary.json, tools/sq_summary.py's docstring)
ISSUE_PEAK = 1024 * 2.4e9 / 4
ISSUE_BASIS = ("1,024 SIMDs x 2.4 GHz / 4 cycles per VALU wave-instruction: one wave's rate (any kind) "
               "and two waves' rate on the slow kinds, measured in profiles/r05/issue_probe/summary.json")


def load_issue(full4, envs, plies, kernel_ms):
    """The issue roofline of a launch of this shape: profiles/sq_k_rollout
    [_full]_p<plies>.json's VALU wave-instructions per launch over the
    launch's live duration (kernel_ms), or None if no summary was measured
    at this shape."""
    path = os.path.join(ROOT, "profiles", f"sq_k_rollout{'_full' if full4 else ''}_p{plies}.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if d.get("envs") != envs or d.get("plies") != plies or not d.get("valu_per_launch") or not kernel_ms:
        return None
    k = d.get("kernel")
    if not k or k not in kernel_name(full4, plies):  # no kernel named, or another kernel's summary
        return None
    achieved = d["valu_per_launch"] / (kernel_ms * 1e-3)
    return {
        "bound": "valu-issue",
        "valu_per_launch": d["valu_per_launch"],
        "salu_per_launch": d.get("salu_per_launch"),
        "valu_per_wave_ply": d.get("valu_per_env_ply"),
        "achieved": round(achieved / 1e9, 2),
        "peak": round(ISSUE_PEAK / 1e9, 2),
        "unit": "G VALU wave-instructions/s",
        "frac": round(achieved / ISSUE_PEAK, 4),
        "basis": ISSUE_BASIS,
        "frac_of_two_wave_fast_peak": round(achieved / (2 * ISSUE_PEAK), 4),
        "valu_busy_of_wave_cycles": d.get("valu_busy_of_wave_cycles"),
        "source": os.path.relpath(path, ROOT),
    }


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# the launching process's CPU baseline, handed to rank 0 (spawn_ranks)
CPU_BASELINE_ENV = "NARDE_BENCH_CPU_BASELINE"


def spawn_ranks(n, argv, cpu=None):
    """Start the N-rank bench as the driver would (torch.distributed.run,
    one process per GPU, rendezvous on 127.0.0.1) and return its exit code.
    Called before this process touches the GPU; the ranks are children (no
    exec), and rank 0's JSON line reaches our stdout.  `cpu`: the CPU
    baseline this process measured before starting them (rank 0 reports it
    instead of measuring it again)."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.pop(CPU_BASELINE_ENV, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL on this host driver)
    if cpu is not None:
        # marked for this launch only: rank 0 accepts it when the marker's
        # port is its MASTER_PORT and the marker's pid one of its ancestors
        env[CPU_BASELINE_ENV] = json.dumps({"launcher_pid": os.getpid(), "master_port": port, "cpu": cpu})
    return subprocess.call(cmd, env=env)


def _ancestors(depth=64):
    """pids of this process's parent, grandparent, ... up to pid 1 (Linux
    /proc; any number of wrapper processes between the launcher and the
    rank)."""
    out, pid = [], os.getpid()
    while pid > 1 and len(out) < depth:
        try:
            with open(f"/proc/{pid}/stat") as f:
                pid = int(f.read().rsplit(")", 1)[1].split()[1])
        except (OSError, ValueError, IndexError):
            break
        out.append(pid)
    return out


def handed_cpu_baseline():
    """The CPU baseline spawn_ranks measured for THIS launch, or None: a
    value inherited from an outer shell or another launch is ignored (and
    then rank 0 measures its own)."""
    raw = os.environ.get(CPU_BASELINE_ENV)
    if not raw:
        return None
    try:
        d = json.loads(raw)
        ok = (str(d["master_port"]) == os.environ.get("MASTER_PORT")
              and int(d["launcher_pid"]) in _ancestors())
    except (ValueError, KeyError, TypeError):
        ok = False
    if not ok:
        print(f"bench.py: {CPU_BASELINE_ENV} is set but is not this launch's; measuring the CPU "
              "baseline here", file=sys.stderr)
        return None
    return d["cpu"]


def measure_cpu_baseline(args):
    """The CPU baseline leg (before any GPU call: the pool forks)."""
    cores, how = available_cores()
    if args.cpu_cores > 0:
        cores, how = args.cpu_cores, f"--cpu-cores {args.cpu_cores}"
    return cpu_baseline(args.cpu_seconds, cores, how)


class GpuEngine:
    """The product: VecNardeEnv (libnarde.so) on this rank's GPU."""

    name = None

    def __init__(self, local_rank):
        import torch

        torch.cuda.set_device(local_rank)
        self.torch = torch
        self.device = torch.device("cuda", local_rank)

    def make_env(self, per, first, seed, rules):
        from gym_narde.vector import VecNardeEnv

        return VecNardeEnv(per, device=self.device, seed=seed, env_id_offset=first, max_episode_steps=1000,
                           rules=rules)

    def timing_event(self):
        from gym_narde.vector import TimingEvent

        return TimingEvent(self.device)

    def sync(self):
        self.torch.cuda.synchronize()


def load_engine(local_rank):
    """GpuEngine, or the test-only host engine NARDE_BENCH_TEST_ENGINE names
    (tests/bench_host_engine.py: the N-rank plumbing on a CPU-only machine;
    never a measurement)."""
    path = os.environ.get("NARDE_BENCH_TEST_ENGINE")
    if not path:
        return GpuEngine(local_rank)
    spec = importlib.util.spec_from_file_location("narde_bench_test_engine", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Engine(local_rank)


def single_node(world):
    """Every rank on this node (torchrun's LOCAL_WORLD_SIZE == WORLD_SIZE)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world


def aligned_start(world, dev):
    """After the barrier + synchronize: every rank starts its clock at the
    same instant of the node's monotonic clock (CLOCK_MONOTONIC is one clock
    for every process of a node) -- a little after the slowest rank has left
    the barrier (one MAX all-reduce of each rank's exit time).  Ranks leave
    a barrier at different times (host wake-up jitter), and with the max
    over ranks of per-rank spans that jitter would be timed as work.
    Returns this rank's barrier-exit lag behind the slowest rank (us), or
    None where the clocks are not one clock (ranks on several nodes: the
    plain barrier stands)."""
    if world == 1:
        return 0.0
    if not single_node(world):
        return None
    import torch
    import torch.distributed as dist

    mine = time.monotonic()
    t = torch.tensor([mine], dtype=torch.float64)
    if dist.get_backend() != "gloo":
        t = t.to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    latest = float(t.cpu()[0])
    go = latest + 0.002  # after the all-reduce has returned on every rank
    while time.monotonic() < go:
        pass
    return round((latest - mine) * 1e6, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); under torchrun it must equal WORLD_SIZE, otherwise "
                         "N > 1 starts the N ranks itself (default: WORLD_SIZE, or 1)")
    # 200 launches of 1,000 plies timed, after 100 untimed: the device needs
    # ~100 back-to-back 0.14-ms launches to reach its sustained rate
    # (tools/diag/ramp_rollout.py)
    ap.add_argument("--steps", type=int, default=200000)
    ap.add_argument("--warmup", type=int, default=100000)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--plies-per-launch", type=int, default=1000)
    ap.add_argument("--ramp-launches", type=int, default=100,
                    help="untimed 1,000-ply launches before --warmup (device clock ramp; 0 = none)")
    ap.add_argument("--ramp-ms", type=float, default=150.0,
                    help="... and at least this long")
    ap.add_argument("--api-steps", type=int, default=200)
    ap.add_argument("--fused-plies", type=int, default=1000)
    ap.add_argument("--fused-launches", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="processes of the CPU baseline (0 = every available core: the CPU "
                         "affinity set, capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rules", choices=("ref2", "full4"), default="ref2",
                    help="rules of the timed path (value); the other mode is reported beside it")
    ap.add_argument("--dqn-steps", type=int, default=30,
                    help="timed steps of the config-4 DQN driver leg (0 = skip)")
    ap.add_argument("--dqn-train-batch", type=int, default=4096)
    ap.add_argument("--other-launches", type=int, default=20,
                    help="k_rollout launches of the other rules mode, timed beside the headline")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (tools/pmc_summary.py); default profiles/pmc_k_rollout[_full].json")
    ap.add_argument("--no-parity-check", action="store_true",
                    help="skip the checker leg (the C oracle replaying the timed launches)")
    ap.add_argument("--parity-core-s", type=float, default=160.0,
                    help="oracle work the checker may spend per leg (host core-seconds): the whole "
                         "shard when it fits, else a prefix of >= 16,384 envs")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus is not None and args.gpus > 1:
            # the N ranks, started here before any GPU call (no exec); the CPU
            # baseline first, on this launching process, so the N-GPU line
            # carries it too
            cpu = None if args.no_cpu_baseline else measure_cpu_baseline(args)
            return spawn_ranks(args.gpus, sys.argv[1:], cpu)
        world_env = "1"
    world_env = int(world_env)
    if args.gpus is None:
        args.gpus = world_env
    if args.gpus != world_env:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env} ranks were started")
    rank_env = int(os.environ.get("RANK", "0"))
    if rank_env != 0:
        # ONE JSON line on stdout, from rank 0: the other ranks' stdout (RCCL /
        # gloo print banners there at init) goes to /dev/null, fd level
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        os.close(devnull)
    # the CPU baseline on rank 0 at every world size, before any GPU call:
    # the launching process's (spawn_ranks), else measured here (under an
    # outside launcher the other ranks wait in the rendezvous meanwhile)
    cpu = None
    if rank_env == 0 and not args.no_cpu_baseline:
        cpu = handed_cpu_baseline()
        if cpu is None:
            cpu = measure_cpu_baseline(args)

    import torch
    import torch.distributed as dist

    from gym_narde import distributed as D

    rank, world, local = D.init_from_env()
    if world > 1:
        assert dist.get_world_size() == args.gpus == world, (dist.get_world_size(), args.gpus, world)
    eng = load_engine(local)
    dev = eng.device
    first, per = D.env_shard(world * args.envs, rank, world)
    is_full4 = args.rules == "full4"
    env = eng.make_env(per, first, args.seed, args.rules)
    if eng.name is not None:  # the test-only host engine: the plumbing, no secondary legs
        args.ramp_launches = 0
        args.ramp_ms = 0.0
        args.api_steps = args.fused_launches = args.other_launches = args.dqn_steps = 0

    def barrier():
        if world > 1:
            dist.barrier()

    P = max(1, min(args.plies_per_launch, args.steps))
    bufs = env.rollout_buffers(P)
    full_launch = env.rollout_launcher(P, bufs)

    def run_plies(k):
        launches = []
        done = 0
        while done < k:
            p = min(P, k - done)
            if p == P:
                full_launch()  # pre-bound: one ctypes call per launch
            else:
                env.rollout(p, bufs)
            launches.append(p)
            done += p
        return launches

    # untimed device ramp, whatever --warmup is: a cold MI355X runs its first
    # ~100 back-to-back launches of this kernel at DVFS-reduced clocks
    # (DESIGN.md section 6), so the ramp plays RAMP_PLIES-ply launches of the
    # same kernel for at least --ramp-ms and --ramp-launches
    ramp_n, ramp_t0 = 0, time.perf_counter()
    if args.ramp_launches > 0:
        rbufs = bufs if P == RAMP_PLIES else env.rollout_buffers(RAMP_PLIES)
        ramp = env.rollout_launcher(RAMP_PLIES, rbufs)
        while ramp_n < args.ramp_launches or (time.perf_counter() - ramp_t0) * 1e3 < args.ramp_ms:
            for _ in range(10):
                ramp()
            ramp_n += 10
            eng.sync()
        del ramp, rbufs
    ramp_ms = (time.perf_counter() - ramp_t0) * 1e3

    # the timed region's launches, pre-bound: K plies as launches of P (the
    # last one shorter if P does not divide K), the two timing events recorded
    # inside the first and the last launch's own call (narde_rollout_timed:
    # no separate event-record calls on the host path; hipExtLaunchKernel's
    # packet events cost ~12 us more per round trip than these markers).
    # The events are timing-only markers (TimingEvent: HIP events with
    # hipEventDisableSystemFence -- a default event's record writes back and
    # invalidates the caches, which lengthens the span it measures by ~1 us
    # at the driver's shape).  The launch path is warmed up untimed.
    K = args.steps
    ev0, ev1 = eng.timing_event(), eng.timing_event()
    sizes = [P] * (K // P) + ([K % P] if K % P else [])
    # the episode totals land here at every world size: the LAST launch of
    # the region writes its envs' statistics summed per 256 envs
    # (narde_rollout_timed's totals rows -- no second launch); at N > 1 the
    # region ends with the one RCCL all-gather of every rank's rows
    # (wg_rows(B) x 24 B per rank), summed afterwards
    rows_buf = torch.empty((-(-per // 256), 3), dtype=torch.int64, device=dev)
    calls = []
    for j, p in enumerate(sizes):
        last = j == len(sizes) - 1
        evs = (ev0 if j == 0 else None, ev1 if last else None)
        calls.append(full_launch if evs == (None, None) else
                     env.rollout_launcher(p, bufs, events=evs, totals=rows_buf if last else None))
    for _ in range(3):
        calls[0]()
        if len(calls) > 1:
            calls[-1]()
    eng.sync()
    ramp_n += 3 if len(calls) == 1 else 6

    run_plies(args.warmup)
    # the checker leg (rank 0's shard, after the GPU work it checks): when
    # the oracle can replay the whole timed region within --parity-core-s,
    # the state before it is snapshotted here (untimed, before the barrier)
    # and every timed ply is replayed; otherwise one launch of the timed
    # kernel at the timed shape right after the region is checked instead
    check_parity = rank == 0 and eng.name is None and not args.no_parity_check
    parity_items, snap0 = [], None
    if check_parity:
        import replay as R

        cores_p, _ = available_cores()
        if parity_envs(per, K, args.rules, args.parity_core_s) == per:
            # two small stream-ordered kernels into device tensors, no
            # synchronize: the device goes from the warm-up into the region
            # as without the checker (a host copy here left the GPU idle for
            # ~ms before the region and the timed 20-ply launch ran 46 us
            # instead of 37, profiles/r06/parity/)
            snap0 = R.snapshot_async(env)
    # the rows' all-gather at N > 1: RCCL's own ncclAllGather on the
    # launching stream (D.RcclGather, one library call) -- ProcessGroupNCCL's
    # all_gather_into_tensor costs ~80 us of host time after a marked launch
    # (tools/diag/launch_after_marker.py); the process group's collective if
    # RCCL's C API cannot be set up
    rows_view = D.gather_total_rows(rows_buf)  # one rank: the (1, R, 3) view, no collective
    gather, gather_impl = (lambda: rows_view), "none (one rank)"
    rccl = None
    if world > 1:
        gather = lambda: D.gather_total_rows(rows_buf)  # noqa: E731
        gather_impl = "ProcessGroup all_gather_into_tensor"
        if dist.get_backend() == "nccl":
            # RcclGather agrees across ranks at every stage: when every rank's
            # RCCL calls return, it either builds on every rank or raises on
            # every rank, so the fallback is common (an init that never
            # returns on some rank ends with the launcher's timeout)
            try:
                rccl = D.RcclGather(rows_buf)
                gather, gather_impl = rccl, "ncclAllGather (RCCL C API, launching stream)"
            except RuntimeError as exc:
                gather_impl += f" (RCCL C API unavailable: {exc})"
    # every call of the timed region once, untimed: a first call pays one-off
    # host costs (the first unsqueeze of this process took ~150 us,
    # tools/diag/after_launch_calls.py; an RCCL collective sets itself up)
    gather()
    eng.sync()
    barrier()
    eng.sync()
    start_skew_us = aligned_start(world, dev)
    if start_skew_us is None:  # several nodes: no shared clock, the barrier stands
        start_skew_us = "n/a (ranks on several nodes: plain barrier)"

    # HIP events on the launching stream around the launches of the timed
    # region (no per-launch event between them): kernel time per launch =
    # that span / launches, i.e. the launches' durations plus the gaps
    # between them (an upper bound on the dispatch duration rocprof shows)
    gc.disable()  # no collector pass inside a region this short
    t0 = time.perf_counter()
    for call in calls:
        call()
    launches = sizes
    t_sub = time.perf_counter()
    gathered = gather()
    t_tot = time.perf_counter()
    eng.sync()
    # the region ends when this rank's stream has run its launches and the
    # all-gather -- which completes only once EVERY rank's rows are in, so
    # no rank stops its clock before the slowest rank's last launch is done;
    # the closing barrier follows, and the max over ranks is taken
    elapsed = time.perf_counter() - t0
    barrier()
    if world > 1:  # (one process: no barrier, and the device is idle already)
        eng.sync()
    t_close = time.perf_counter() - t0
    gc.enable()
    host_us = {"start_skew_removed": start_skew_us,
               "submit": round((t_sub - t0) * 1e6, 1), "gather_call": round((t_tot - t_sub) * 1e6, 1),
               "wait": round((elapsed - (t_tot - t0)) * 1e6, 1),
               "closing_barrier_untimed": round((t_close - elapsed) * 1e6, 1)}
    span_ms = ev0.elapsed_ms(ev1)
    rank_totals = gathered.sum(1).cpu()  # (world, 3): each rank's {episodes, white pts, black pts}
    totals = rank_totals
    # algorithmic bytes of every launch in the span (a last partial launch
    # included), and the mean duration of a full-length launch
    span_bytes = sum(launch_bytes(per, p, is_full4) for p in launches)
    kern_ms = span_ms * launch_bytes(per, P, is_full4) / span_bytes

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        if dist.get_backend() == "gloo":  # D.rehearsal(): host tensors
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    total_steps = world * per * K
    value = total_steps / elapsed
    summary = D.summarize(totals)

    if check_parity:
        # the checker's inputs, copied to the host before any other leg runs
        # on this env (untimed)
        last_p = sizes[-1]
        if snap0 is not None:
            parity_items.append(dict(
                rules=args.rules, before=R.to_host(snap0), bufs=host_bufs(bufs, last_p, per), after=R.snapshot(env),
                plies=K, envs=per, seed=args.seed, env0=first, totals_rows=rows_buf.cpu().numpy(),
                scope=(f"the timed region itself: all {K} timed plies replayed from the state snapshotted "
                       f"before it; the last launch's {last_p} plies of per-ply outputs, the final state "
                       f"and its per-256-env totals rows compared")))
        else:
            n_chk = parity_envs(per, P, args.rules, args.parity_core_s)
            before = R.snapshot(env)
            full_launch()
            eng.sync()
            parity_items.append(dict(
                rules=args.rules, before=before, bufs=host_bufs(bufs, P, n_chk), after=R.snapshot(env),
                plies=P, envs=n_chk, seed=args.seed, env0=first,
                scope=(f"the {K} timed plies are more than --parity-core-s lets the oracle replay: one "
                       f"untimed launch of the timed kernel at the timed shape ({P} plies) right after "
                       f"the region, its per-ply outputs and final state compared")))

    # secondary 1: per-ply API kernel k_step (eager, then hipGraph replay)
    api = None
    S = args.api_steps
    if S > 0:
        for _ in range(10):
            env.step()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(S)]
        for i in range(S):  # per-launch kernel time (events cost host time: not in the rate below)
            ev[i][0].record()
            env.step()
            ev[i][1].record()
        torch.cuda.synchronize()
        step_ms = sum(x.elapsed_time(y) for x, y in ev) / S
        a0 = time.perf_counter()
        for i in range(S):
            env.step()
        torch.cuda.synchronize()
        api_eager = per * S / (time.perf_counter() - a0)
        G = 50
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            env.step()  # warm the capture stream
            torch.cuda.synchronize()
            with torch.cuda.graph(graph, stream=cap):
                for _ in range(G):
                    env.step()
        torch.cuda.current_stream().wait_stream(cap)
        graph.replay()
        torch.cuda.synchronize()
        reps = max(1, S // G)
        g0 = time.perf_counter()
        for _ in range(reps):
            graph.replay()
        torch.cuda.synchronize()
        api_graph = per * G * reps / (time.perf_counter() - g0)
        api = {
            "kernel": "k_step (one ply per launch, same outputs)",
            "eager": round(api_eager, 1),
            "hipgraph": round(api_graph, 1),
            "unit": "env steps/s",
            "kernel_ms": round(step_ms, 5),
            "achieved_GBps": round(((OUT_BYTES_PER_STEP_FULL if is_full4 else OUT_BYTES_PER_STEP) + RECORD_BYTES)
                                   * per / (step_ms * 1e-3) / 1e9, 2),
        }

    # secondary 2: fused self-play with no per-ply outputs (statistics only)
    fused = None
    F = args.fused_plies
    if args.fused_launches > 0:
        env.selfplay(F)
        torch.cuda.synchronize()
        f0 = time.perf_counter()
        for _ in range(args.fused_launches):
            env.selfplay(F)
        torch.cuda.synchronize()
        fused = {
            "kernel": f"k_rollout without per-ply outputs, {F} plies per launch",
            "value": round(per * F * args.fused_launches / (time.perf_counter() - f0), 1),
            "unit": "env steps/s",
        }

    # secondary 3: the other rules mode through the same rollout kernel shape
    other_rules = "ref2" if is_full4 else "full4"
    other = None
    if args.other_launches > 0:
        env_o = eng.make_env(per, first, args.seed, other_rules)
        bufs_o = env_o.rollout_buffers(P)
        env_o.rollout(P, bufs_o)
        env_o.rollout(P, bufs_o)
        torch.cuda.synchronize()
        ev_o = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.other_launches)]
        n_o = parity_envs(per, P, other_rules, args.parity_core_s) if check_parity else 0
        snap_o = None
        o0 = time.perf_counter()
        for j, (s_, e_) in enumerate(ev_o):
            if n_o and j == len(ev_o) - 1:
                # the checker's snapshot of the state before the last timed
                # launch: two small stream-ordered kernels into device
                # tensors and the host ply counter, outside the launch's
                # events (in the wall rate: ~0.2 % of 20 launches)
                snap_o = R.snapshot_async(env_o)
            s_.record()
            env_o.rollout(P, bufs_o)
            e_.record()
        torch.cuda.synchronize()
        if snap_o is not None:
            parity_items.append(dict(
                rules=other_rules, before=R.to_host(snap_o), bufs=host_bufs(bufs_o, P, n_o), after=R.snapshot(env_o),
                plies=P, envs=n_o, seed=args.seed, env0=first, leg="other_rules",
                scope=f"the last of the {len(ev_o)} timed launches of this leg ({P} plies): its per-ply "
                      f"outputs and final state compared"))
        other_rate = per * P * args.other_launches / (time.perf_counter() - o0)
        other_ms = sum(s_.elapsed_time(e_) for s_, e_ in ev_o) / len(ev_o)
        other_M = None
        if other_rules == "full4":
            M = ((bufs_o["legal"] >> 56) & 7).flatten()
            other_M = [round(float(x), 4) for x in (torch.bincount(M, minlength=5).double() / M.numel()).tolist()]
        env_o.close()
        obytes = launch_bytes(per, P, not is_full4)
        other = {
            "rules": other_rules,
            "kernel": f"{kernel_name(other_rules == 'full4', P)} ({other_rules.upper()}), {P} plies per launch, all outputs",
            "value": round(other_rate, 1),
            "unit": "env steps/s",
            "kernel_ms": round(other_ms, 5),
            "bytes_per_launch": obytes,
            "achieved_GBps": round(obytes / (other_ms * 1e-3) / 1e9, 2),
            "frac": round(obytes / (other_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "issue": load_issue(other_rules == "full4", per, P, other_ms),
            "max_dice_hist": other_M,
        }

    # secondary 4: configs[3] -- the batched DQN driver (198-d obs + legal
    # masks -> DecomposedDQN -> env step -> device replay -> one PER update)
    dqn = None
    if args.dqn_steps > 0 and not is_full4:
        from gym_narde.dqn import BatchedDQNDriver, use_tuned_gemms

        tuned = use_tuned_gemms()  # TunableOp GEMM choices measured on MI355X

        env_q = eng.make_env(per, first, args.seed + 1, "ref2")
        drv = BatchedDQNDriver(env_q, obs="tesauro198", train_batch=args.dqn_train_batch,
                               capacity=max(1 << 20, 4 * per))
        for _ in range(5):
            drv.step()
        torch.cuda.synchronize()
        q0 = time.perf_counter()
        for _ in range(args.dqn_steps):
            drv.step()
        torch.cuda.synchronize()
        q_el = time.perf_counter() - q0
        # split: action selection + env step vs the learner update
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        x = drv.state
        a = drv.act(x)
        env_q.step(a.to(torch.int16))
        ev[1].record()
        drv.update()
        ev[2].record()
        torch.cuda.synchronize()
        # the same step captured once as a CUDA graph and replayed
        drv.capture_graph(warmup=2)
        for _ in range(3):
            drv.step()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(args.dqn_steps):
            drv.step()
        torch.cuda.synchronize()
        g_el = time.perf_counter() - g0
        dqn = {
            "config": "configs[3]: batch=65536, legal-action masks + 198-d obs -> DecomposedDQN "
                      "(train_deepq_pytorch.py:184-277) on PyTorch-ROCm, fp32",
            "value": round(world * per * args.dqn_steps / g_el, 1),
            "unit": "env steps/s",
            "ms_per_step": round(g_el / args.dqn_steps * 1e3, 4),
            "mode": "hipGraph replay of the whole step (BatchedDQNDriver.capture_graph)",
            "eager_value": round(world * per * args.dqn_steps / q_el, 1),
            "eager_ms_per_step": round(q_el / args.dqn_steps * 1e3, 4),
            "act_plus_env_ms": round(ev[0].elapsed_time(ev[1]), 4),
            "update_ms": round(ev[1].elapsed_time(ev[2]), 4),
            "train_batch": args.dqn_train_batch,
            "updates_per_step": 1,
            "dtype": "f32",
            "gemms": "TunableOp results (gym_narde/tunableop_gfx950.csv)" if tuned else "torch heuristics",
            "final_loss": float(drv.last_loss) if drv.last_loss is not None else None,
        }
        env_q.close()

    # the checker leg, after every GPU leg (rank 0's shard)
    parity = {}
    for item in parity_items:
        parity[item.get("leg", "headline")] = run_parity(item, cores_p)
    del parity_items

    if rank == 0:
        nbytes = launch_bytes(per, P, is_full4)
        achieved = nbytes / (kern_ms * 1e-3) / 1e9  # = span bytes / span time (max over ranks)
        # the PMC summary measured at this launch shape (plies per launch):
        # profiles/pmc_k_rollout[_full]_p<P>.json, else the 1,000-ply one
        base = os.path.join(ROOT, "profiles", "pmc_k_rollout_full" if is_full4 else "pmc_k_rollout")
        traffic = None
        for tj in ([args.traffic_json] if args.traffic_json else [f"{base}_p{P}.json", f"{base}.json"]):
            traffic = load_traffic(tj, per, P, kernel_name(is_full4, P))
            if traffic is not None:
                break
        # what each rules mode is, and which BASELINE.json config it times
        rules_txt = {
            "ref2": ("REF2 = the reference's NardeEnv.step (narde_env.py:27-103: <=2 checker moves "
                     "per step, also on doubles); legal sets bit-exact vs the reference"),
            "full4": ("FULL4 whole turns (4-move doubles, max dice used, higher-die rule; DESIGN.md "
                      "section 10); every sub-move is the reference's single-die primitive, the "
                      "whole-turn composition is the build's (parity unpinned: the reference never "
                      "plays a whole turn)"),
        }
        config_txt = {
            "ref2": ("configs[2]'s batch and dice (65536 envs/GPU, all 36 ordered pairs) under REF2, "
                     "the rules the metric's 'legal-move bit-exact vs CPU' is defined on; "
                     "configs[2] as written ('full rules incl. 4-move doubles') is the FULL4 leg, "
                     "other_rules"),
            "full4": ("configs[2] as written: 65536 envs/GPU, full rules incl. 4-move doubles "
                      "(FULL4); the REF2 leg is other_rules"),
        }
        if world > 1:
            # configs[4]: 524,288 envs sharded over 8 GPUs (its N = 2 / 4
            # points: the same 65,536-env shards on fewer GPUs)
            c4 = ("configs[4]: batch=524288 sharded 8 x MI355X (8 x 65536 contiguous global env ids), "
                  "one RCCL all-gather of the episode totals" if world * per == 524288 else
                  f"configs[4]'s layout at {world} GPUs: {world} x {per} = {world * per} envs, contiguous "
                  f"global env-id shards, one RCCL all-gather of the episode totals")
            config_txt = {k: f"{c4}; per GPU {v}" for k, v in config_txt.items()}
        parity_txt = {
            "ref2": ("bit-exact vs the reference's golden vectors and the CPU oracle; unpinned: "
                     "TimeLimit truncation (gymnasium semantics, gymnasium absent) and the device "
                     "RNG (the build's own synthetic workload)"),
            "full4": ("sub-moves pinned to the reference (tests/golden/full4.npz); whole-turn "
                      "composition unpinned (the build's rule, held to the build's oracle)"),
        }
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 6),
            "device_ramp_launches": ramp_n,
            "device_ramp_ms": round(ramp_ms, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Philox dice, random legal policy, start position + auto-reset)",
            "config": {
                "workload": (f"{config_txt[args.rules]}: random-policy self-play; rules = "
                             f"{rules_txt[args.rules]}; TimeLimit 1000; every ply writes obs/"
                             f"reward/terminated/truncated/legal set/actions for every env"),
                "rules": args.rules,
                "parity": parity_txt[args.rules],
                "kernel": f"{kernel_name(is_full4, P)} ({'FULL4' if is_full4 else 'REF2'}), {P} plies per launch",
                "envs_per_gpu": per,
                "global_envs": world * per,
                "parallelism": f"dp{world} (env-id shards, 1 RCCL all-gather of episode totals)",
                "episodes_finished": summary["episodes"],
                # every rank's {episodes, white points, black points}, as gathered in the timed region
                "rank_totals": rank_totals.tolist(),
                "collective": {"backend": dist.get_backend() if dist.is_initialized() else None,
                               "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                               "timed": (f"the last launch writes its {rows_buf.shape[0]} per-256-env totals "
                                         f"rows; one all-gather of them ({rows_buf.shape[0] * 24} B per rank)"
                                         if world > 1 else f"the last launch writes its {rows_buf.shape[0]} "
                                         "per-256-env totals rows (no process group at N=1)"),
                               "impl": gather_impl,
                               "region_end": "this rank's synchronize after the all-gather (complete only once "
                                             "every rank's rows are in); the closing barrier is untimed; max over "
                                             "ranks"},
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel_name(is_full4, P),
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "bytes_per_launch": nbytes,
                "kernel_ms": round(kern_ms, 5),
                # the same launch against the integer VALU issue peak
                "issue": load_issue(is_full4, per, P, kern_ms),
            },
            # rank 0's wall split of the timed region: launches submitted,
            # waiting for them (and the gather), the closing barrier + sync
            "timed_region_host_us": host_us,
            "cpu_baseline": cpu,
            # the metric's "legal-move bit-exact vs CPU", checked on this
            # run's own launches: the C oracle (oracle/replay.py) replays
            # them from the snapshotted state; mismatches counts (ply, env)
            # entries of every output plus envs whose final state differs
            "parity_check": parity.get("headline"),
            "api_step": api,
            "other_rules": other,
            "config4_dqn": dqn,
            "selfplay_stats_only": fused,
        }
        if other is not None:
            other["workload"] = f"{config_txt[other_rules]}; rules = {rules_txt[other_rules]}"
            other["parity"] = parity_txt[other_rules]
            other["parity_check"] = parity.get("other_rules")
        if eng.name is not None:
            line["engine"] = eng.name
        # (a fresh line: a library banner on stdout may lack its newline)
        sys.stdout.write("\n" + json.dumps(line) + "\n")
        sys.stdout.flush()
    env.close()
    if rccl is not None:  # its communicator before the process group's
        eng.sync()
        rccl.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
