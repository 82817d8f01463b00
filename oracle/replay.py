"""Whole-batch oracle replay of a device launch -- the checker of bench.py's
parity_check leg and of the full-batch GPU parity tests.

TEST INFRASTRUCTURE ONLY -- imported by tests/ and bench.py's checker leg
(after the timed region, never inside it), never by the product package.

A device handle's state at ply t (VecNardeEnv.get_state() + stats(), and
the handle's ply counter) is all the self-play drivers depend on: the dice
and picks of ply t for global env e are Philox({t >> 1, e, 0, 0}, seed)
(oracle/narde_oracle.c or_ply_draw), so the C oracle, loaded with the same
state, replays the same plies (or_selfplay restates narde_env.py:27-103,
or_selfplay_full DESIGN.md section 10's whole turns).  The batch is cut into
contiguous env chunks run on a thread pool: the ctypes calls release the
GIL, so the replay scales with the host cores.
"""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle as O

# fields compared, device rollout buffer key -> oracle record key
FIELDS_REF2 = (("obs", "obs"), ("reward", "reward"), ("terminated", "terminated"),
               ("truncated", "truncated"), ("actions", "action"), ("legal", "legal"))
FIELDS_FULL4 = (("obs", "obs"), ("reward", "reward"), ("terminated", "terminated"),
                ("truncated", "truncated"), ("actions", "played"), ("legal", "legal"))


def _host(x):
    """numpy view of a device tensor / numpy array (synchronising copy)."""
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def snapshot_async(env):
    """A VecNardeEnv's replay state as device tensors: two stream-ordered
    kernels (narde_get_state, narde_get_stats) and the host ply counter, no
    synchronize -- to_host() copies it later."""
    return env.get_state(), env.stats(), int(env.ply)


def to_host(snap):
    """snapshot_async's tensors -> the host dict replay() / check() take."""
    st, stats, t = snap
    out = {k: _host(v).copy() for k, v in st.items()}
    out["stats"] = _host(stats).copy()
    out["t"] = int(t)
    return out


def snapshot(env):
    """The host copy of a VecNardeEnv's replay state: board, off,
    first_turn, player, elapsed, stats and the ply counter (synchronises
    the env's stream)."""
    return to_host(snapshot_async(env))


def _run_chunk(snap, lo, hi, seed, env0, full, skip, record, dice_mode, max_steps):
    sp = O.SelfPlay(hi - lo, seed=seed, env0=env0 + lo, dice_mode=dice_mode, max_steps=max_steps)
    sp.load(snap["board"][lo:hi], snap["off"][lo:hi], snap["first_turn"][lo:hi], snap["player"][lo:hi],
            snap["elapsed"][lo:hi], snap["stats"][lo:hi], snap["t"])
    run = sp.run_full if full else sp.run
    if skip:
        run(skip, record=False)
    rec = run(record) if record else None
    return lo, hi, sp, rec


def replay(snap, plies, record, seed, env0=0, full=False, envs=None, threads=8, dice_mode=0,
           max_steps=1000, chunk=4096):
    """Replay `plies` plies from `snap` for envs [0, envs) on `threads`
    threads; the last `record` of them are recorded.  Returns (final state
    dict, records dict with [record][envs] arrays or None)."""
    n = len(snap["player"]) if envs is None else int(envs)
    skip = plies - record
    assert 0 <= record <= plies
    bounds = [(lo, min(n, lo + chunk)) for lo in range(0, n, chunk)]
    with ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
        parts = list(pool.map(lambda b: _run_chunk(snap, b[0], b[1], seed, env0, full, skip, record,
                                                   dice_mode, max_steps), bounds))
    parts.sort(key=lambda p: p[0])
    state = {k: np.concatenate([getattr(p[2], a) for p in parts])
             for k, a in (("board", "board"), ("off", "off"), ("first_turn", "ft"), ("player", "player"),
                          ("elapsed", "elapsed"), ("stats", "stats"))}
    recs = None
    if record:
        recs = {k: np.concatenate([p[3][k] for p in parts], axis=1) for k in parts[0][3]}
    return state, recs


def _as_oracle(key, dev):
    """A device buffer in the oracle record's dtype/view (the device widens
    obs/reward to int32 and keeps the 64-bit words signed)."""
    if key in ("legal", "played"):
        return dev.view(np.uint64)
    return dev


def check(snap, bufs, after, plies, seed, env0=0, full=False, envs=None, threads=8, dice_mode=0,
          max_steps=1000, totals_rows=None):
    """Compare a device run with the oracle: `snap` the state before it,
    `bufs` (host numpy, [P][B] rollout buffers) the outputs of its last P
    plies, `after` the snapshot after it.  Returns the parity_check dict:
    mismatching (ply, env) entries per output field, mismatching envs of
    the final state, the envs / plies compared and the oracle's wall time.
    totals_rows: the launch's per-256-env statistics rows (narde_rollout_timed),
    compared with the oracle's final statistics summed per 256 envs."""
    t0 = time.perf_counter()
    P = next(v.shape[0] for v in bufs.values() if v is not None)
    n = len(snap["player"]) if envs is None else int(envs)
    state, rec = replay(snap, plies, P, seed, env0, full, n, threads, dice_mode, max_steps)
    oracle_s = time.perf_counter() - t0
    fields = FIELDS_FULL4 if full else FIELDS_REF2
    mism = {}
    for dk, ok in fields:
        d = bufs.get(dk)
        if d is None:
            continue
        d = _as_oracle(ok, d[:P, :n])
        r = rec[ok]
        if dk in ("obs", "reward"):
            r = r.astype(np.int32)
        neq = d != r
        if neq.ndim == 3:
            neq = neq.any(-1)
        mism[dk] = int(neq.sum())
    st_bad = np.zeros(n, bool)
    for k in ("board", "off", "first_turn"):
        st_bad |= (after[k][:n].reshape(n, -1) != state[k].reshape(n, -1)).any(1)
    for k in ("player", "elapsed"):
        st_bad |= after[k][:n].astype(np.int64) != state[k].astype(np.int64)
    st_bad |= (after["stats"][:n] != state["stats"]).any(1)
    mism["final_state_envs"] = int(st_bad.sum())
    if totals_rows is not None:
        rows = np.asarray(totals_rows, dtype=np.int64)
        pad = np.zeros((rows.shape[0] * 256, 3), np.int64)
        pad[:n] = state["stats"]
        mism["totals_rows"] = int((pad.reshape(-1, 256, 3).sum(1) != rows).any(1).sum())
    return {
        "rules": "full4" if full else "ref2",
        "envs": n,
        "plies": plies,
        "plies_compared_per_output": P,
        "mismatches": int(sum(mism.values())),
        "by_field": mism,
        "oracle_s": round(oracle_s, 3),
        "threads": threads,
    }
