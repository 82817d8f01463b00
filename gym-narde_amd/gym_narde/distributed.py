"""Multi-GPU: one process per GPU, env-id sharding, one RCCL all-gather.

Envs never interact, so the batch shards with no data-path collective
(SURVEY.md 8e): rank r of W owns global env ids [r*B/W, (r+1)*B/W).  The
device RNG is keyed by the global env id, so any W reproduces the W=1 run
bit for bit.  The only collective is one all_gather_into_tensor of the
per-env statistics {episodes, white points, black points} at the end of a
run (backend "nccl" = RCCL over xGMI on ROCm; "gloo" on CPU for tests).
"""
import ctypes
import os

import torch
import torch.distributed as dist


def env_shard(global_envs, rank, world):
    """(first global env id, count) owned by `rank`."""
    if global_envs % world:
        raise ValueError(f"{global_envs} envs do not split evenly over {world} ranks")
    per = global_envs // world
    return rank * per, per


def rehearsal():
    """NARDE_REHEARSAL=1: run every rank on GPU 0 over gloo, so the N-rank
    bench path can be exercised on a one-GPU box (tools/diag/gpu_rehearse.sh).
    Never set for measurements."""
    return os.environ.get("NARDE_REHEARSAL", "0") == "1"


def init_from_env(backend=None, force=False):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/
    LOCAL_RANK/MASTER_*).  Returns (rank, world, local_rank); local_rank is the
    GPU index to use (0 for every rank under rehearsal()).  A world of one
    process gets no process group unless `force` (then gather_stats runs the
    real collective, e.g. to exercise the RCCL path on a one-GPU box)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = 0 if rehearsal() else int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "gloo" if rehearsal() or not torch.cuda.is_available() else "nccl"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def gather_stats(local_stats):
    """All-gather (B_local, 3) int32 statistics -> (B_global, 3) on every rank,
    ordered by global env id (the local tensor itself when no process group
    is initialised)."""
    if not dist.is_initialized():
        return local_stats
    world = dist.get_world_size()
    src = local_stats.contiguous()
    if dist.get_backend() == "gloo" and src.is_cuda:  # gloo gathers host tensors
        src = src.cpu()
    out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src)
    return out.to(local_stats.device)


def gather_totals(local_stats):
    """Per-rank totals {episodes, white points, black points} of (B_local, 3)
    statistics, all-gathered: (world, 3) int64 on every rank, rank order (the
    local totals as (1, 3) when no process group is initialised).  One 24-B
    RCCL all-gather per rank -- what the self-play driver reports per run --
    instead of gather_stats' 12 B per env."""
    tot = local_stats.to(torch.int64).sum(0, keepdim=True)
    if not dist.is_initialized():
        return tot
    if dist.get_backend() == "gloo" and tot.is_cuda:  # gloo gathers host tensors
        tot = tot.cpu()
    out = torch.empty((dist.get_world_size(), 3), dtype=torch.int64, device=tot.device)
    dist.all_gather_into_tensor(out, tot)
    return out


def gather_total_rows(rows):
    """All-gather of a rank's VecNardeEnv.totals() partial rows ((R, 3)
    int64, one kernel on the device): (world, R, 3) on every rank, rank
    order ((1, R, 3) without a process group).  1.5 KB per rank in one RCCL
    call; .sum(1) gives gather_totals' (world, 3) -- done by the reader,
    after the timed region."""
    rows = rows.unsqueeze(0)
    if not dist.is_initialized():
        return rows
    if dist.get_backend() == "gloo" and rows.is_cuda:  # gloo gathers host tensors
        rows = rows.cpu()
    out = torch.empty((dist.get_world_size(),) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(out, rows)
    return out


def summarize(stats):
    """{episodes, white_points, black_points} of a (B, 3) statistics tensor."""
    s = stats.to(torch.int64).sum(0).tolist()
    return {"episodes": int(s[0]), "white_points": int(s[1]), "black_points": int(s[2])}


# ---------------------------------------------------------------- RCCL, direct
_NCCL_INT64 = 4  # ncclDataType_t ncclInt64 (rccl.h)


class _NcclUniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES


def _rccl():
    """The RCCL library torch's ProcessGroupNCCL already uses (torch/lib)."""
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    lib = ctypes.CDLL(path if os.path.exists(path) else "librccl.so.1")
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_NcclUniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _NcclUniqueId, ctypes.c_int]
    lib.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    lib.ncclGetErrorString.argtypes = [ctypes.c_int]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    return lib


def agree(ok, device=None):
    """True on every rank iff `ok` is true on every rank: one MIN all-reduce
    (a device tensor on the nccl backend, a host one on gloo).  Without a
    process group: `ok` itself."""
    if not dist.is_initialized():
        return bool(ok)
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.cpu()[0]))


class RcclGather:
    """gather_total_rows through RCCL's own C API: one ncclAllGather on the
    caller's stream (ring / direct xGMI transfers of every rank's rows into
    every rank's (world, R, 3) buffer) -- one library call in the timed
    region, where ProcessGroupNCCL's all_gather_into_tensor adds its stream
    and event bookkeeping on the host (~20 us after a bare launch, ~80 us
    after a launch bracketed by timing markers: tools/diag/launch_after_marker.py).
    Built collectively from an initialised process group (the unique id is
    broadcast through it); the same bytes as gather_total_rows.

    Every stage ends with the ranks agreeing (`agree`, or rank 0's status
    byte riding with the unique id), so when every rank's calls RETURN,
    either every rank gets a communicator or every rank raises RuntimeError
    -- a caller that falls back to the process group's collective on that
    error falls back on every rank alike (a rank deciding alone
    would leave the others in a broadcast, or in a different collective,
    forever).  ncclCommInitRank itself is collective and blocking: a rank
    whose init never returns (a peer that died inside its own init) leaves
    the others inside theirs, and no agreement can follow; that case ends
    with the launcher's timeout, not with the fallback.  (The non-blocking
    init, ncclCommInitRankConfig with blocking = 0, would make every later
    call on the communicator -- the timed ncclAllGather included -- liable
    to return ncclInProgress and need polling, so it is not used.)"""

    def __init__(self, rows):
        self.comm = ctypes.c_void_p()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        dev = rows.device
        err = None
        try:
            self.lib = _rccl()
        except (OSError, AttributeError) as exc:
            self.lib, err = None, f"librccl: {exc}"
        if not agree(err is None, dev):
            raise RuntimeError(err or "RCCL C API unavailable on another rank")
        # rank 0's unique id, with its status in byte 128 (one broadcast)
        uid = _NcclUniqueId()
        ok0 = 1
        if self.rank == 0:
            rc = self.lib.ncclGetUniqueId(ctypes.byref(uid))
            if rc != 0:
                ok0, err = 0, self._msg(rc, "ncclGetUniqueId")
        idb = ctypes.string_at(ctypes.addressof(uid), 128) + bytes([ok0])  # (c_char arrays stop at a NUL)
        raw = torch.tensor(list(idb), dtype=torch.uint8, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.broadcast(raw, 0)
        host = raw.cpu().tolist()
        if host[128] != 1:
            raise RuntimeError(err or "ncclGetUniqueId failed on rank 0")
        uid = _NcclUniqueId()
        ctypes.memmove(ctypes.addressof(uid), bytes(host[:128]), 128)
        rc = self.lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank)
        if rc != 0:
            self.comm, err = ctypes.c_void_p(), self._msg(rc, "ncclCommInitRank")
        if not agree(rc == 0, dev):
            self.close()
            raise RuntimeError(err or "ncclCommInitRank failed on another rank")
        self.src = rows
        self.out = torch.empty((self.world,) + tuple(rows.shape), dtype=rows.dtype, device=dev)
        self.count = rows.numel()

    def _msg(self, rc, what):
        return f"{what} failed ({rc}): {self.lib.ncclGetErrorString(rc).decode()}"

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(self._msg(rc, what))

    def __call__(self, stream=None):
        """All-gather the rows tensor given at construction (its current
        contents) on `stream` (default: torch's current stream of its
        device); returns the (world, R, 3) output."""
        st = stream if stream is not None else torch.cuda.current_stream(self.src.device).cuda_stream
        self._check(self.lib.ncclAllGather(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.out.data_ptr()),
                                           self.count, _NCCL_INT64, self.comm, ctypes.c_void_p(st)),
                    "ncclAllGather")
        return self.out

    def close(self):
        if self.comm and self.lib is not None:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
