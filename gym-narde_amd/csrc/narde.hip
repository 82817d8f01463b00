// narde.hip -- HIP kernels (gfx950) + the C ABI of libnarde (include/narde.h).
//
// One lane = one env.  Each env is a 32-byte record split into two planar
// 16-byte planes (narde_rules.h), so every wave-wide load/store of state is
// a single contiguous 1 KiB transaction.  The rules engine (narde_rules.h) is
// branch-light bitmask arithmetic on 24-bit point masks held in VGPRs.
//
// One translation unit; the device code is split by role into headers
// included below, in order:
//   device_common.h     build knobs, env planes, the device RNG draws
//   kernels_state.h     reset, set/get state, peek dice, get_valid_moves
//                       (k_legal), apply, statistics, block rule
//   kernels_full4.h     k_legal_full, with full4_wave.h: the
//                       wave-cooperative FULL4 turn
//   kernels_rollout.h   the timed path: per-ply outputs, k_step (API step),
//                       the producer/consumer rollouts k_rollout_pc (REF2)
//                       and k_rollout_pp_full (FULL4)
//   kernels_agent.h     observations, move masks, the policy kernel, the DQN
//                       transition
// This file keeps the handle, the host-side checks and every C entry point.
// The DQN learner kernels are a second translation unit (dqn_learner.hip).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <type_traits>

#include "../../include/narde.h"
#include "narde_rules.h"

using namespace narde;

namespace {

constexpr int64_t kHostCap = 4096;

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(NARDE_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

}  // namespace

#include "device_common.h"
#include "kernels_state.h"
#include "kernels_full4.h"
#include "kernels_rollout.h"
#include "kernels_agent.h"

namespace {

inline int grid(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }

}  // namespace

// ---------------------------------------------------------------- handle
struct narde_env {
  int device;
  int64_t n;
  int64_t env0;
  uint64_t seed;
  int dice_mode;
  int max_steps;
  uint32_t epoch;
  Planes pl;
  // host-call staging (scalar facade)
  Planes hpl;
  uint8_t* h_in;   // pinned
  uint8_t* h_out;  // pinned
  uint8_t* d_in;
  uint8_t* d_out;
  hipStream_t hstream;
  size_t stage_bytes;
};

namespace {

Rng rng_of(const narde_env* e) {
  Rng g;
  g.env0 = (uint32_t)e->env0;
  g.k0 = (uint32_t)e->seed;
  g.k1 = (uint32_t)(e->seed >> 32);
  g.dice_mode = e->dice_mode;
  return g;
}

// the handle's device for the call; the caller's restored after it (no
// runtime call on the way out when they are the same -- the usual case, and
// the timed launch's host path)
struct DeviceGuard {
  int prev = -1;
  bool switched = false;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) switched = hipSetDevice(d) == hipSuccess;
  }
  ~DeviceGuard() {
    if (switched && prev >= 0) (void)hipSetDevice(prev);
  }
};

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(NARDE_EHIP, "%s launch: %s", what, hipGetErrorString(e));
  return NARDE_OK;
}

bool valid_position(const int8_t* board, const uint8_t* off, const uint8_t* ft, const int8_t* player,
                    int64_t i) {
  int w = 0, b = 0;
  for (int p = 0; p < 24; ++p) {
    const int v = board[i * 24 + p];
    if (v > 15 || v < -15) return false;
    if (v > 0) w += v; else b -= v;
  }
  if (off[2 * i] > 15 || off[2 * i + 1] > 15) return false;
  if (w + off[2 * i] > 15 || b + off[2 * i + 1] > 15) return false;
  if (player && player[i] != 1 && player[i] != -1) return false;
  (void)ft;
  return true;
}

}  // namespace

namespace narde_abi {
// the other translation units' (dqn_learner.hip) way into narde_last_error()
int set_error(int code, const char* what) { return fail(code, "%s", what); }
}  // namespace narde_abi

extern "C" {

int narde_version(void) { return 2; }
const char* narde_last_error(void) { return g_err; }

int narde_create(int device, int64_t num_envs, int64_t env_id_offset, uint64_t seed, int dice_mode,
                 int max_episode_steps, narde_env** out) {
  if (!out) return fail(NARDE_EINVAL, "out is NULL");
  *out = nullptr;
  if (num_envs <= 0 || num_envs > (int64_t(1) << 31) - kBlock)
    return fail(NARDE_EINVAL, "num_envs %lld out of range", (long long)num_envs);
  if (env_id_offset < 0 || env_id_offset + num_envs > (int64_t(1) << 32))
    return fail(NARDE_EINVAL, "global env ids must fit in 32 bits");
  if (dice_mode != NARDE_DICE_ALL36 && dice_mode != NARDE_DICE_NODOUBLES)
    return fail(NARDE_EINVAL, "bad dice_mode %d", dice_mode);
  if (max_episode_steps < 0 || max_episode_steps > 65535)
    return fail(NARDE_EINVAL, "max_episode_steps must be in [0, 65535]");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(NARDE_EINVAL, "device %d of %d", device, ndev);
  DeviceGuard dg(device);
  narde_env* e = new (std::nothrow) narde_env();
  if (!e) return fail(NARDE_ENOMEM, "host alloc");
  e->device = device;
  e->n = num_envs;
  e->env0 = env_id_offset;
  e->seed = seed;
  e->dice_mode = dice_mode;
  e->max_steps = max_episode_steps;
  e->stage_bytes = (size_t)kHostCap * 512;
  hipError_t err = hipSuccess;
  err = hipMalloc(&e->pl.p0, num_envs * sizeof(uint4));
  if (err == hipSuccess) err = hipMalloc(&e->pl.p1, num_envs * sizeof(uint4));
  if (err == hipSuccess) err = hipMalloc(&e->pl.stats, num_envs * sizeof(int4));
  if (err == hipSuccess) err = hipMalloc(&e->hpl.p0, kHostCap * sizeof(uint4));
  if (err == hipSuccess) err = hipMalloc(&e->hpl.p1, kHostCap * sizeof(uint4));
  if (err == hipSuccess) err = hipMalloc(&e->hpl.stats, kHostCap * sizeof(int4));
  if (err == hipSuccess) err = hipMalloc(&e->d_in, e->stage_bytes);
  if (err == hipSuccess) err = hipMalloc(&e->d_out, e->stage_bytes);
  if (err == hipSuccess) err = hipHostMalloc(&e->h_in, e->stage_bytes, hipHostMallocDefault);
  if (err == hipSuccess) err = hipHostMalloc(&e->h_out, e->stage_bytes, hipHostMallocDefault);
  if (err == hipSuccess) err = hipStreamCreateWithFlags(&e->hstream, hipStreamNonBlocking);
  if (err != hipSuccess) {
    narde_destroy(e);
    return fail(NARDE_ENOMEM, "device alloc for %lld envs: %s", (long long)num_envs,
                hipGetErrorString(err));
  }
  k_reset<<<grid(num_envs), kBlock, 0, e->hstream>>>(e->pl, (int)num_envs, rng_of(e), 0u, nullptr,
                                                     (int64_t)0, nullptr, 0);
  int rc = check_launch("k_reset");
  if (rc == NARDE_OK) {
    err = hipStreamSynchronize(e->hstream);
    if (err != hipSuccess) rc = fail(NARDE_EHIP, "reset sync: %s", hipGetErrorString(err));
  }
  if (rc != NARDE_OK) {
    narde_destroy(e);
    return rc;
  }
  e->epoch = 1;
  *out = e;
  return NARDE_OK;
}

int narde_destroy(narde_env* e) {
  if (!e) return NARDE_OK;
  DeviceGuard dg(e->device);
  if (e->hstream) (void)hipStreamSynchronize(e->hstream);
  (void)hipFree(e->pl.p0); (void)hipFree(e->pl.p1); (void)hipFree(e->pl.stats);
  (void)hipFree(e->hpl.p0); (void)hipFree(e->hpl.p1); (void)hipFree(e->hpl.stats);
  (void)hipFree(e->d_in); (void)hipFree(e->d_out);
  if (e->h_in) (void)hipHostFree(e->h_in);
  if (e->h_out) (void)hipHostFree(e->h_out);
  if (e->hstream) (void)hipStreamDestroy(e->hstream);
  delete e;
  return NARDE_OK;
}

int64_t narde_num_envs(const narde_env* e) { return e ? e->n : -1; }

int narde_get_ply(const narde_env* e, uint32_t* t) {
  if (!e || !t) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(t, reinterpret_cast<const char*>(e->pl.p1) + 12, sizeof(uint32_t),
                    hipMemcpyDeviceToHost));
  return NARDE_OK;
}

int narde_set_ply(narde_env* e, uint32_t t) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  DeviceGuard dg(e->device);
  // every step / rollout still queued on any stream of the device first (they
  // advance t): the private stream alone is not ordered with the caller's
  HIP_TRY(hipDeviceSynchronize());
  k_set_ply<<<grid(e->n), kBlock, 0, e->hstream>>>(e->pl, (int)e->n, t);
  int rc = check_launch("k_set_ply");
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->hstream));
  return NARDE_OK;
}

int narde_reset(narde_env* e, const uint8_t* mask, const uint8_t* opening, int pairs, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  if (opening && pairs <= 0) return fail(NARDE_EINVAL, "opening draws need pairs >= 1");
  DeviceGuard dg(e->device);
  k_reset<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), e->epoch, mask,
                                                           (int64_t)-1, opening, opening ? pairs : 0);
  e->epoch += 1;
  return check_launch("k_reset");
}

int narde_set_state(narde_env* e, const int8_t* board, const uint8_t* off, const uint8_t* ft,
                    const int8_t* player, const uint16_t* elapsed, void* stream) {
  if (!e || !board || !off || !ft || !player) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_set_state<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, board, off, ft, player,
                                                              elapsed, 1);
  return check_launch("k_set_state");
}

int narde_get_state(narde_env* e, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                    uint16_t* elapsed, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  DeviceGuard dg(e->device);
  k_get_state<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, board, off, ft, player,
                                                              elapsed);
  return check_launch("k_get_state");
}

int narde_peek_dice(narde_env* e, uint8_t* dice, void* stream) {
  if (!e || !dice) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_peek_dice<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), dice);
  return check_launch("k_peek_dice");
}

int narde_legal_moves(narde_env* e, const uint8_t* dice, int16_t* out_count, int8_t* out_moves,
                      uint64_t* out_compact, void* stream) {
  if (!e || !out_count) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_legal<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), dice,
                                                          out_count, out_moves, out_compact);
  return check_launch("k_legal");
}

int narde_step(narde_env* e, const int16_t* actions, const uint8_t* dice, int32_t* obs,
               int32_t* reward, uint8_t* terminated, uint8_t* truncated, uint64_t* legal_compact,
               int16_t* actions_out, int autoreset, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  DeviceGuard dg(e->device);
  StepArgs a;
  a.pl = e->pl;
  a.n = (int)e->n;
  a.g = rng_of(e);
  a.max_steps = e->max_steps;
  a.autoreset = autoreset;
  a.actions = actions;
  a.dice = dice;
  a.play = nullptr;
  a.out = Outs{obs, reward, terminated, truncated, legal_compact, actions_out, nullptr};
  k_step<false><<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(a);
  return check_launch("k_step");
}

int narde_step_full(narde_env* e, const int8_t* play, const uint8_t* dice, int32_t* obs, int32_t* reward,
                    uint8_t* terminated, uint8_t* truncated, uint64_t* legal_first, uint64_t* played,
                    int autoreset, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  DeviceGuard dg(e->device);
  StepArgs a;
  a.pl = e->pl;
  a.n = (int)e->n;
  a.g = rng_of(e);
  a.max_steps = e->max_steps;
  a.autoreset = autoreset;
  a.actions = nullptr;
  a.play = play;
  a.dice = dice;
  a.out = Outs{obs, reward, terminated, truncated, legal_first, nullptr, played};
  k_step<true><<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(a);
  return check_launch("k_step<full>");
}

// The rollout launches.  narde_rollout_timed brackets them with two
// hipEventRecord markers: hipExtLaunchKernel's packet-level start / stop
// events were measured too and cost ~12 us more per host round trip of one
// launch than the markers' ~4 us (tools/diag/single_launch.py, one box).
namespace {

int launch_rollout_ref2(narde_env* e, int plies, const Outs& out, bool any, hipStream_t stream) {
  const dim3 g((unsigned)((e->n + kPcEnvs - 1) / kPcEnvs)), b(kPcThreads);
  if (any)
    k_rollout_pc<true><<<g, b, 0, stream>>>(e->pl, (int)e->n, rng_of(e), plies, e->max_steps, out);
  else
    k_rollout_pc<false><<<g, b, 0, stream>>>(e->pl, (int)e->n, rng_of(e), plies, e->max_steps, out);
  return check_launch("k_rollout");
}

int launch_rollout_full(narde_env* e, int plies, const Outs& out, bool any, hipStream_t stream) {
  // producer/consumer pairs (k_rollout_pp_full)
  const dim3 g((unsigned)((e->n + kPcEnvs - 1) / kPcEnvs)), b(kPcThreads);
  if (any)
    k_rollout_pp_full<true><<<g, b, 0, stream>>>(e->pl, (int)e->n, rng_of(e), plies, e->max_steps, out);
  else
    k_rollout_pp_full<false><<<g, b, 0, stream>>>(e->pl, (int)e->n, rng_of(e), plies, e->max_steps, out);
  return check_launch("k_rollout_pp_full");
}

}  // namespace

int narde_rollout(narde_env* e, int plies, int32_t* obs, int32_t* reward, uint8_t* terminated,
                  uint8_t* truncated, uint64_t* legal_compact, int16_t* actions_out, void* stream) {
  if (!e || plies < 0) return fail(NARDE_EINVAL, "bad argument");
  if (plies == 0) return NARDE_OK;
  DeviceGuard dg(e->device);
  const Outs out{obs, reward, terminated, truncated, legal_compact, actions_out, nullptr};
  const bool any = obs || reward || terminated || truncated || legal_compact || actions_out;
  return launch_rollout_ref2(e, plies, out, any, (hipStream_t)stream);
}

int narde_selfplay(narde_env* e, int plies, void* stream) {
  return narde_rollout(e, plies, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int narde_rollout_full(narde_env* e, int plies, int32_t* obs, int32_t* reward, uint8_t* terminated,
                       uint8_t* truncated, uint64_t* legal_first, uint64_t* played, void* stream) {
  if (!e || plies < 0) return fail(NARDE_EINVAL, "bad argument");
  if (plies == 0) return NARDE_OK;
  DeviceGuard dg(e->device);
  const Outs out{obs, reward, terminated, truncated, legal_first, nullptr, played};
  const bool any = obs || reward || terminated || truncated || legal_first || played;
  return launch_rollout_full(e, plies, out, any, (hipStream_t)stream);
}

int narde_selfplay_full(narde_env* e, int plies, void* stream) {
  return narde_rollout_full(e, plies, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int narde_rollout_timed(narde_env* e, int full, int plies, int32_t* obs, int32_t* reward, uint8_t* terminated,
                        uint8_t* truncated, uint64_t* legal, void* last, void* ev_start, void* ev_stop,
                        int64_t* totals, void* stream) {
  if (!e || plies < 0) return fail(NARDE_EINVAL, "bad argument");
  if (totals && plies == 0) return fail(NARDE_EINVAL, "totals rows need a launch (plies > 0)");
  DeviceGuard dg(e->device);
  const bool any = obs || reward || terminated || truncated || legal || last;
  if (ev_start && hipEventRecord((hipEvent_t)ev_start, (hipStream_t)stream) != hipSuccess)
    return fail(NARDE_EHIP, "hipEventRecord(ev_start) failed");
  int rc = NARDE_OK;
  if (plies > 0 && full) {
    const Outs out{obs, reward, terminated, truncated, legal, nullptr, (uint64_t*)last, totals};
    rc = launch_rollout_full(e, plies, out, any, (hipStream_t)stream);
  } else if (plies > 0) {
    const Outs out{obs, reward, terminated, truncated, legal, (int16_t*)last, nullptr, totals};
    rc = launch_rollout_ref2(e, plies, out, any, (hipStream_t)stream);
  }
  if (rc) return rc;
  if (ev_stop && hipEventRecord((hipEvent_t)ev_stop, (hipStream_t)stream) != hipSuccess)
    return fail(NARDE_EHIP, "hipEventRecord(ev_stop) failed");
  return NARDE_OK;
}

// narde_rollout_timed pre-bound (round 6): everything but the launch is done
// once at create -- argument checks, the device check, the kernel chosen,
// its arguments packed -- so the timed call is one ctypes argument and
// three runtime calls (event, hipLaunchKernel, event), no device switch.
struct narde_rollout_plan {
  narde_env* e;
  const void* kernel;
  dim3 grid, block;
  Planes pl;
  int n;
  Rng g;
  int plies;
  int max_steps;
  Outs out;
  void* args[6];
  hipEvent_t ev0, ev1;
  hipStream_t stream;
};

int narde_rollout_plan_create(narde_env* e, int full, int plies, int32_t* obs, int32_t* reward, uint8_t* terminated,
                              uint8_t* truncated, uint64_t* legal, void* last, void* ev_start, void* ev_stop,
                              int64_t* totals, void* stream, void** plan) {
  if (!e || !plan || plies <= 0) return fail(NARDE_EINVAL, "bad argument (a plan needs plies > 0)");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != e->device)
    return fail(NARDE_EINVAL, "the calling thread's current device must be the env's");
  narde_rollout_plan* p = new (std::nothrow) narde_rollout_plan();
  if (!p) return fail(NARDE_ENOMEM, "out of host memory");
  const bool any = obs || reward || terminated || truncated || legal || last;
  if (full) {
    p->out = Outs{obs, reward, terminated, truncated, legal, nullptr, (uint64_t*)last, totals};
    p->kernel = any ? (const void*)k_rollout_pp_full<true> : (const void*)k_rollout_pp_full<false>;
  } else {
    p->out = Outs{obs, reward, terminated, truncated, legal, (int16_t*)last, nullptr, totals};
    p->kernel = any ? (const void*)k_rollout_pc<true> : (const void*)k_rollout_pc<false>;
  }
  p->e = e;
  p->grid = dim3((unsigned)((e->n + kPcEnvs - 1) / kPcEnvs));
  p->block = dim3(kPcThreads);
  p->pl = e->pl;
  p->n = (int)e->n;
  p->g = rng_of(e);  // seed, env ids, dice law (the ply counter is each env's record word)
  p->plies = plies;
  p->max_steps = e->max_steps;
  p->args[0] = &p->pl;
  p->args[1] = &p->n;
  p->args[2] = &p->g;
  p->args[3] = &p->plies;
  p->args[4] = &p->max_steps;
  p->args[5] = &p->out;
  p->ev0 = (hipEvent_t)ev_start;
  p->ev1 = (hipEvent_t)ev_stop;
  p->stream = (hipStream_t)stream;
  *plan = p;
  return NARDE_OK;
}

int narde_rollout_plan_launch(void* plan) {
  narde_rollout_plan* p = (narde_rollout_plan*)plan;
  if (!p) return fail(NARDE_EINVAL, "NULL plan");
  if (p->ev0 && hipEventRecord(p->ev0, p->stream) != hipSuccess) return fail(NARDE_EHIP, "hipEventRecord(ev_start) failed");
  if (hipLaunchKernel(p->kernel, p->grid, p->block, p->args, 0, p->stream) != hipSuccess)
    return fail(NARDE_EHIP, "hipLaunchKernel(k_rollout) failed");
  if (p->ev1 && hipEventRecord(p->ev1, p->stream) != hipSuccess) return fail(NARDE_EHIP, "hipEventRecord(ev_stop) failed");
  return NARDE_OK;
}

int narde_rollout_plan_destroy(void* plan) {
  delete (narde_rollout_plan*)plan;
  return NARDE_OK;
}

int narde_timing_event_create(int device, unsigned flags, void** event) {
  if (!event) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(device);
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, flags) != hipSuccess) return fail(NARDE_EHIP, "hipEventCreateWithFlags failed");
  *event = ev;
  return NARDE_OK;
}

int narde_timing_event_destroy(void* event) {
  if (event && hipEventDestroy((hipEvent_t)event) != hipSuccess) return fail(NARDE_EHIP, "hipEventDestroy failed");
  return NARDE_OK;
}

int narde_timing_event_elapsed_ms(void* start, void* stop, float* ms) {
  if (!start || !stop || !ms) return fail(NARDE_EINVAL, "NULL argument");
  if (hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop) != hipSuccess)
    return fail(NARDE_EHIP, "hipEventElapsedTime failed");
  return NARDE_OK;
}

int narde_legal_full(narde_env* e, const uint8_t* dice, uint64_t* legal_first, void* stream) {
  if (!e || !legal_first) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_legal_full<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), dice,
                                                               legal_first);
  return check_launch("k_legal_full");
}

int narde_get_stats(narde_env* e, int32_t* stats, void* stream) {
  if (!e || !stats) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_get_stats<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, stats);
  return check_launch("k_get_stats");
}

int narde_get_totals(narde_env* e, int64_t* rows, void* stream) {
  if (!e || !rows) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_get_totals<<<kTotalRows, kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rows);
  return check_launch("k_get_totals");
}

int narde_apply_moves(narde_env* e, const int8_t* moves, const int8_t* player, void* stream) {
  if (!e || !moves) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_apply<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, moves, player, nullptr);
  return check_launch("k_apply");
}

int narde_observe(narde_env* e, int32_t* obs, float* tes, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  if (!obs && !tes) return NARDE_OK;
  if (tes && e->n * 198 >= (int64_t(1) << 31)) return fail(NARDE_EINVAL, "too many envs for one observation launch");
  DeviceGuard dg(e->device);
  if (obs) {
    k_observe<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, obs);
    if (const int rc = check_launch("k_observe")) return rc;
  }
  if (tes) {
    // kTesEnvs envs per wave, kBlock / 64 waves per workgroup
    const int64_t per_block = (int64_t)kTesEnvs * (kBlock / 64);
    k_tesauro198_rows<<<(unsigned)((e->n + per_block - 1) / per_block), kBlock, 0, (hipStream_t)stream>>>(
        e->pl, (int)e->n, tes);
    return check_launch("k_tesauro198_rows");
  }
  return NARDE_OK;
}

int narde_dqn_transition(narde_env* e, float* state, const int64_t* actions, const int32_t* reward,
                         const uint8_t* terminated, const uint8_t* truncated, const uint64_t* legal,
                         int32_t* misc, float* off_seen, int shaping, float* r_obs, int64_t* r_action,
                         float* r_reward, float* r_done, float* r_prio, const float* max_prio, const int64_t* pos,
                         int64_t capacity, void* stream) {
  if (!e || !state || !actions || !reward || !terminated || !truncated || !misc || !r_obs || !r_action ||
      !r_reward || !r_done || !r_prio || !max_prio || !pos || (shaping && !off_seen))
    return fail(NARDE_EINVAL, "NULL argument");
  if (capacity < 2 * e->n) return fail(NARDE_EINVAL, "replay capacity below twice the env count");
  if (e->n * 198 >= (int64_t(1) << 31)) return fail(NARDE_EINVAL, "too many envs for one transition launch");
  DeviceGuard dg(e->device);
  TransArgs t{e->pl, (int)e->n, shaping, state, actions, reward, terminated, truncated, legal, misc, off_seen,
              r_obs, r_action, r_reward, r_done, r_prio, max_prio, pos, capacity};
  const int64_t per_block = (int64_t)kTesEnvs * (kBlock / 64);  // s' rows per obs workgroup
  const int obs_blocks = (int)((e->n + per_block - 1) / per_block);
  k_dqn_transition<<<(unsigned)(obs_blocks + grid(e->n)), kBlock, 0, (hipStream_t)stream>>>(t, obs_blocks);
  return check_launch("k_dqn_transition");
}

int narde_legal_mask576(narde_env* e, uint64_t* mask, void* stream) {
  if (!e || !mask) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_mask576<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), mask);
  return check_launch("k_mask576");
}

int narde_legal_mask576_move2(narde_env* e, const int16_t* move1, const uint8_t* dice, uint64_t* mask,
                              void* stream) {
  if (!e || !move1 || !mask) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_mask576_move2<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), move1, dice,
                                                                  mask);
  return check_launch("k_mask576_move2");
}

int narde_play_set(narde_env* e, const uint8_t* dice, int kind, uint64_t* legal, uint32_t* table, int32_t* count,
                   void* stream) {
  if (!e || !table || !count) return fail(NARDE_EINVAL, "NULL argument");
  if (kind != kPlayAct && kind != kPlayStep) return fail(NARDE_EINVAL, "kind must be 0 (act) or 1 (step)");
  DeviceGuard dg(e->device);
  k_play_set<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), dice, kind, legal, table,
                                                             count);
  return check_launch("k_play_set");
}

int narde_act_masks(narde_env* e, const uint8_t* dice, const int64_t* move1, int64_t ld_move1, uint64_t* mask,
                    void* stream) {
  if (!e || !mask) return fail(NARDE_EINVAL, "NULL argument");
  if (move1 && ld_move1 < 1) return fail(NARDE_EINVAL, "bad move1 stride");
  DeviceGuard dg(e->device);
  k_act_masks<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), dice, move1, ld_move1,
                                                              mask);
  return check_launch("k_act_masks");
}

int narde_explore_plays(narde_env* e, const uint8_t* dice, const float* epsilon, uint64_t seed, const int64_t* tag,
                        int64_t* out, int64_t ld_out, void* stream) {
  if (!e || !epsilon || !tag || !out) return fail(NARDE_EINVAL, "NULL argument");
  if (ld_out < 2) return fail(NARDE_EINVAL, "action rows hold two codes (ld_out >= 2)");
  DeviceGuard dg(e->device);
  k_explore_plays<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), dice, epsilon, tag,
                                                                  (uint32_t)seed, (uint32_t)(seed >> 32), out,
                                                                  ld_out);
  return check_launch("k_explore_plays");
}

int narde_policy_masked_argmax576(int device, const float* q, int64_t ldq, const uint64_t* mask, int64_t n,
                                  float epsilon, uint64_t seed, uint32_t tag, int head, int64_t* out,
                                  void* stream) {
  if (!q || !mask || !out || n < 0 || n > (int64_t(1) << 31) - 4 || ldq < 576)
    return fail(NARDE_EINVAL, "bad argument");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_policy576<<<(int)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(q, ldq, mask, (int)n, eps_to_q32(epsilon),
                                                                   (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                                                                   head, out, nullptr, nullptr, nullptr, 0,
                                                                   nullptr);
  return check_launch("k_policy576");
}

int narde_policy_masked_argmax576_dev(int device, const float* q, int64_t ldq, const uint64_t* mask, int64_t n,
                                      const float* epsilon, uint64_t seed, const int64_t* tag, int head,
                                      const float* add_tab, int64_t ld_add, const int64_t* add_row,
                                      int64_t* out, void* stream) {
  if (!q || !mask || !out || !epsilon || !tag || n < 0 || n > (int64_t(1) << 31) - 4 || ldq < 576)
    return fail(NARDE_EINVAL, "bad argument");
  if (add_tab && (!add_row || ld_add < 576)) return fail(NARDE_EINVAL, "bad addend table");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_policy576<<<(int)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(q, ldq, mask, (int)n, 0ull, (uint32_t)seed,
                                                                   (uint32_t)(seed >> 32), 0u, head, out, epsilon,
                                                                   tag, add_tab, ld_add, add_row);
  return check_launch("k_policy576");
}

int narde_head_policy576_dev(int device, const float* f, int64_t ldf, int64_t feat, const float* w, int64_t ldw,
                             const float* bias, const uint64_t* mask, int64_t n, const float* epsilon,
                             uint64_t seed, const int64_t* tag, int head, const float* addcol,
                             const int64_t* add_row, int64_t ld_row, int64_t* out, int64_t ld_out,
                             int16_t* out16, int64_t ld_out16, void* stream) {
  if (!f || !w || !bias || !mask || !out || !epsilon || !tag || n < 0 || n > (int64_t(1) << 31) - 4)
    return fail(NARDE_EINVAL, "bad argument");
  if (ld_out < 1 || (out16 && ld_out16 < 1) || (addcol && ld_row < 1)) return fail(NARDE_EINVAL, "bad strides");
  if (feat != kHeadF || ldf < feat || ldw < feat || (ldf % 4) || (ldw % 4) ||
      (reinterpret_cast<uintptr_t>(f) % 16) || (reinterpret_cast<uintptr_t>(w) % 16))
    return fail(NARDE_EINVAL, "features must be 256 wide, rows 16-B aligned");
  if (addcol && !add_row) return fail(NARDE_EINVAL, "addend column without its rows");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_head_policy576<<<(int)((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(f, ldf, w, ldw, bias, mask, (int)n,
                                                                        (uint32_t)seed, (uint32_t)(seed >> 32),
                                                                        head, out, ld_out, out16, ld_out16,
                                                                        epsilon, tag, addcol, add_row, ld_row);
  return check_launch("k_head_policy576");
}

int narde_violates_block_rule(int device, const int8_t* boards, int64_t n, uint8_t* out, void* stream) {
  if (!boards || !out || n < 0 || n > (int64_t(1) << 31) - kBlock) return fail(NARDE_EINVAL, "bad argument");
  if (n == 0) return NARDE_OK;
  DeviceGuard dg(device);
  k_block<<<grid(n), kBlock, 0, (hipStream_t)stream>>>(boards, (int)n, out);
  return check_launch("k_block");
}

}  // extern "C"

// ------------------------------------------------------- host entry points
namespace {

struct Carve {
  uint8_t* base;
  size_t off = 0;
  template <class T>
  T* take(int64_t count) {
    T* p = reinterpret_cast<T*>(base + off);
    off += ((size_t)count * sizeof(T) + 255) & ~size_t(255);
    return p;
  }
};

int host_check(narde_env* e, int64_t n) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  if (n < 0 || n > kHostCap) return fail(NARDE_EINVAL, "host batch %lld > %lld", (long long)n, (long long)kHostCap);
  return NARDE_OK;
}

int host_validate(int64_t n, const int8_t* board, const uint8_t* off, const uint8_t* ft,
                  const int8_t* player) {
  for (int64_t i = 0; i < n; ++i)
    if (!valid_position(board, off, ft, player, i))
      return fail(NARDE_EINVAL, "invalid position at index %lld", (long long)i);
  return NARDE_OK;
}

int host_sync(narde_env* e) {
  HIP_TRY(hipStreamSynchronize(e->hstream));
  return NARDE_OK;
}

}  // namespace

extern "C" {

int narde_host_legal_moves(narde_env* e, int64_t n, const int8_t* board, const uint8_t* off,
                           const uint8_t* ft, const int8_t* player, const uint8_t* dice4,
                           int16_t* count, int8_t* moves) {
  int rc = host_check(e, n);
  if (rc) return rc;
  if (n == 0) return NARDE_OK;
  if (!board || !off || !ft || !player || !dice4 || !count) return fail(NARDE_EINVAL, "NULL argument");
  if ((rc = host_validate(n, board, off, ft, player))) return rc;
  DeviceGuard dg(e->device);
  Carve hi{e->h_in}, di{e->d_in}, ho{e->h_out}, dq{e->d_out};
  int8_t* hb = hi.take<int8_t>(n * 24); int8_t* db = di.take<int8_t>(n * 24);
  uint8_t* hoff = hi.take<uint8_t>(n * 2); uint8_t* doff = di.take<uint8_t>(n * 2);
  uint8_t* hft = hi.take<uint8_t>(n * 2); uint8_t* dft = di.take<uint8_t>(n * 2);
  int8_t* hp = hi.take<int8_t>(n); int8_t* dp = di.take<int8_t>(n);
  uint8_t* hd = hi.take<uint8_t>(n * 4); uint8_t* dd = di.take<uint8_t>(n * 4);
  memcpy(hb, board, n * 24); memcpy(hoff, off, n * 2); memcpy(hft, ft, n * 2);
  memcpy(hp, player, n); memcpy(hd, dice4, n * 4);
  int16_t* hc = ho.take<int16_t>(n); int16_t* dc = dq.take<int16_t>(n);
  int8_t* hm = ho.take<int8_t>(n * NARDE_MAX_MOVES * 2); int8_t* dm = dq.take<int8_t>(n * NARDE_MAX_MOVES * 2);
  HIP_TRY(hipMemcpyAsync(e->d_in, e->h_in, hi.off, hipMemcpyHostToDevice, e->hstream));
  k_set_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db, doff, dft, dp, nullptr, 0);
  k_legal<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, rng_of(e), dd, dc, moves ? dm : nullptr,
                                              nullptr);
  if ((rc = check_launch("host legal"))) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_out, e->d_out, dq.off, hipMemcpyDeviceToHost, e->hstream));
  if ((rc = host_sync(e))) return rc;
  memcpy(count, hc, n * sizeof(int16_t));
  if (moves) memcpy(moves, hm, n * NARDE_MAX_MOVES * 2);
  return NARDE_OK;
}

int narde_host_step(narde_env* e, int64_t n, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                    const uint8_t* dice2, const int16_t* actions, int32_t* obs, int32_t* reward,
                    uint8_t* terminated) {
  int rc = host_check(e, n);
  if (rc) return rc;
  if (n == 0) return NARDE_OK;
  if (!board || !off || !ft || !player || !dice2 || !actions) return fail(NARDE_EINVAL, "NULL argument");
  if ((rc = host_validate(n, board, off, ft, player))) return rc;
  for (int64_t i = 0; i < 2 * n; ++i)
    if (dice2[i] < 1 || dice2[i] > 6) return fail(NARDE_EINVAL, "die out of range at %lld", (long long)i);
  DeviceGuard dg(e->device);
  Carve hi{e->h_in}, di{e->d_in}, ho{e->h_out}, dq{e->d_out};
  int8_t* hb = hi.take<int8_t>(n * 24); int8_t* db = di.take<int8_t>(n * 24);
  uint8_t* hoff = hi.take<uint8_t>(n * 2); uint8_t* doff = di.take<uint8_t>(n * 2);
  uint8_t* hft = hi.take<uint8_t>(n * 2); uint8_t* dft = di.take<uint8_t>(n * 2);
  int8_t* hp = hi.take<int8_t>(n); int8_t* dp = di.take<int8_t>(n);
  uint8_t* hd = hi.take<uint8_t>(n * 2); uint8_t* dd = di.take<uint8_t>(n * 2);
  int16_t* ha = hi.take<int16_t>(n * 2); int16_t* da = di.take<int16_t>(n * 2);
  memcpy(hb, board, n * 24); memcpy(hoff, off, n * 2); memcpy(hft, ft, n * 2);
  memcpy(hp, player, n); memcpy(hd, dice2, n * 2); memcpy(ha, actions, n * 4);
  int8_t* hb2 = ho.take<int8_t>(n * 24); int8_t* db2 = dq.take<int8_t>(n * 24);
  uint8_t* hoff2 = ho.take<uint8_t>(n * 2); uint8_t* doff2 = dq.take<uint8_t>(n * 2);
  uint8_t* hft2 = ho.take<uint8_t>(n * 2); uint8_t* dft2 = dq.take<uint8_t>(n * 2);
  int8_t* hp2 = ho.take<int8_t>(n); int8_t* dp2 = dq.take<int8_t>(n);
  int32_t* hobs = ho.take<int32_t>(n * 24); int32_t* dobs = dq.take<int32_t>(n * 24);
  int32_t* hr = ho.take<int32_t>(n); int32_t* dr = dq.take<int32_t>(n);
  uint8_t* ht = ho.take<uint8_t>(n); uint8_t* dt = dq.take<uint8_t>(n);
  HIP_TRY(hipMemcpyAsync(e->d_in, e->h_in, hi.off, hipMemcpyHostToDevice, e->hstream));
  k_set_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db, doff, dft, dp, nullptr, 0);
  StepArgs a;
  a.pl = e->hpl;
  a.n = (int)n;
  a.g = rng_of(e);
  a.max_steps = 0;
  a.autoreset = 0;
  a.actions = da;
  a.dice = dd;
  a.play = nullptr;
  a.out = Outs{dobs, dr, dt, nullptr, nullptr, nullptr, nullptr};
  k_step<false><<<grid(n), kBlock, 0, e->hstream>>>(a);
  k_get_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db2, doff2, dft2, dp2, nullptr);
  if ((rc = check_launch("host step"))) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_out, e->d_out, dq.off, hipMemcpyDeviceToHost, e->hstream));
  if ((rc = host_sync(e))) return rc;
  memcpy(board, hb2, n * 24); memcpy(off, hoff2, n * 2); memcpy(ft, hft2, n * 2); memcpy(player, hp2, n);
  if (obs) memcpy(obs, hobs, n * 24 * sizeof(int32_t));
  if (reward) memcpy(reward, hr, n * sizeof(int32_t));
  if (terminated) memcpy(terminated, ht, n);
  return NARDE_OK;
}

int narde_host_apply_moves(narde_env* e, int64_t n, int8_t* board, uint8_t* off, uint8_t* ft,
                           const int8_t* player, const int8_t* moves) {
  int rc = host_check(e, n);
  if (rc) return rc;
  if (n == 0) return NARDE_OK;
  if (!board || !off || !ft || !player || !moves) return fail(NARDE_EINVAL, "NULL argument");
  if ((rc = host_validate(n, board, off, ft, player))) return rc;
  DeviceGuard dg(e->device);
  Carve hi{e->h_in}, di{e->d_in}, ho{e->h_out}, dq{e->d_out};
  int8_t* hb = hi.take<int8_t>(n * 24); int8_t* db = di.take<int8_t>(n * 24);
  uint8_t* hoff = hi.take<uint8_t>(n * 2); uint8_t* doff = di.take<uint8_t>(n * 2);
  uint8_t* hft = hi.take<uint8_t>(n * 2); uint8_t* dft = di.take<uint8_t>(n * 2);
  int8_t* hp = hi.take<int8_t>(n); int8_t* dp = di.take<int8_t>(n);
  int8_t* hm = hi.take<int8_t>(n * 2); int8_t* dm = di.take<int8_t>(n * 2);
  memcpy(hb, board, n * 24); memcpy(hoff, off, n * 2); memcpy(hft, ft, n * 2);
  memcpy(hp, player, n); memcpy(hm, moves, n * 2);
  int8_t* hb2 = ho.take<int8_t>(n * 24); int8_t* db2 = dq.take<int8_t>(n * 24);
  uint8_t* hoff2 = ho.take<uint8_t>(n * 2); uint8_t* doff2 = dq.take<uint8_t>(n * 2);
  uint8_t* hft2 = ho.take<uint8_t>(n * 2); uint8_t* dft2 = dq.take<uint8_t>(n * 2);
  uint8_t* hst = ho.take<uint8_t>(n); uint8_t* dst = dq.take<uint8_t>(n);
  HIP_TRY(hipMemcpyAsync(e->d_in, e->h_in, hi.off, hipMemcpyHostToDevice, e->hstream));
  k_set_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db, doff, dft, dp, nullptr, 0);
  k_apply<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, dm, dp, dst);
  k_get_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db2, doff2, dft2, nullptr, nullptr);
  if ((rc = check_launch("host apply"))) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_out, e->d_out, dq.off, hipMemcpyDeviceToHost, e->hstream));
  if ((rc = host_sync(e))) return rc;
  // a move the record cannot hold (k_apply): nothing is written back
  for (int64_t i = 0; i < n; ++i)
    if (hst[i])
      return fail(NARDE_EINVAL,
                  "move (%d, %d) at index %lld is not executable: the source holds none of the "
                  "mover's checkers or the target holds opponent checkers",
                  (int)moves[2 * i], (int)moves[2 * i + 1], (long long)i);
  memcpy(board, hb2, n * 24); memcpy(off, hoff2, n * 2); memcpy(ft, hft2, n * 2);
  return NARDE_OK;
}

int narde_host_violates_block_rule(narde_env* e, int64_t n, const int8_t* boards, uint8_t* out) {
  int rc = host_check(e, n);
  if (rc) return rc;
  if (n == 0) return NARDE_OK;
  if (!boards || !out) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  Carve hi{e->h_in}, di{e->d_in}, ho{e->h_out}, dq{e->d_out};
  int8_t* hb = hi.take<int8_t>(n * 24); int8_t* db = di.take<int8_t>(n * 24);
  memcpy(hb, boards, n * 24);
  uint8_t* hr = ho.take<uint8_t>(n); uint8_t* dr = dq.take<uint8_t>(n);
  HIP_TRY(hipMemcpyAsync(e->d_in, e->h_in, hi.off, hipMemcpyHostToDevice, e->hstream));
  k_block<<<grid(n), kBlock, 0, e->hstream>>>(db, (int)n, dr);
  if ((rc = check_launch("host block"))) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_out, e->d_out, dq.off, hipMemcpyDeviceToHost, e->hstream));
  if ((rc = host_sync(e))) return rc;
  memcpy(out, hr, n);
  return NARDE_OK;
}

}  // extern "C"
