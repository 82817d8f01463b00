// kernels_rollout.h -- the timed path: per-ply outputs, k_step, k_rollout and the producer/consumer k_rollout_pc
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

namespace {

// per-ply outputs; a rollout writes ply p of env i at [p * n + i]
struct Outs {
  int32_t* __restrict__ obs;      // [.][n][24]
  int32_t* __restrict__ reward;   // [.][n]
  uint8_t* __restrict__ term;     // [.][n]
  uint8_t* __restrict__ trunc;    // [.][n]
  uint64_t* __restrict__ legal;   // [.][n] compact list #1 (FULL4: C_0 | M<<56)
  int16_t* __restrict__ act_out;  // [.][n][2] REF2 codes used
  uint64_t* __restrict__ played;  // [.][n] FULL4 sub-moves (from, die) x 4
};

struct StepArgs {
  Planes pl;
  int n;
  Rng g;
  int max_steps;
  int autoreset;
  const int16_t* __restrict__ actions;  // REF2: i16[n][2] codes
  const int8_t* __restrict__ play;      // FULL4: i8[n][4][2] (from, die)
  const uint8_t* __restrict__ dice;
  Outs out;
};

// (DIAGNOSTIC bit 64: a store guarded by a condition the compiler cannot
// fold but that never holds at run time)
#if NARDE_DIAG_ABLATE & 64
__device__ int g_diag_never;
#define NARDE_DIAG_STORE_GUARD if (g_diag_never != 12345) return;
#else
#define NARDE_DIAG_STORE_GUARD
#endif

template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
  NARDE_DIAG_STORE_GUARD
#if NARDE_OBS_STORE == 2 || NARDE_OBS_STORE == 4
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void st_out(int4* p, int4 v) {
  NARDE_DIAG_STORE_GUARD
#if NARDE_OBS_STORE == 2 || NARDE_OBS_STORE == 3
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<v4i*>(p));
#else
  *p = v;
#endif
}

__device__ __forceinline__ int4 obs_quad(const Side& s, int q) {
  return make_int4(obs_point(s, 4 * q), obs_point(s, 4 * q + 1), obs_point(s, 4 * q + 2),
                   obs_point(s, 4 * q + 3));
}

__device__ __forceinline__ void store_obs(int32_t* __restrict__ obs, size_t ix, const Side& s) {
  int4* o = reinterpret_cast<int4*>(obs + ix * 24);
#pragma unroll
  for (int q = 0; q < 6; ++q) st_out(o + q, obs_quad(s, q));
}

// whole-wave obs store through the wave's 6-KiB LDS slice (all 64 lanes
// active, rows ix - lane .. ix - lane + 63 contiguous)
__device__ __forceinline__ void store_obs_wave(int32_t* __restrict__ obs, size_t ix, const Side& s,
                                               int4* __restrict__ lds) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 6; ++q) lds[lane * 6 + q] = obs_quad(s, q);
  __builtin_amdgcn_wave_barrier();  // LDS ops of one wave retire in issue order
  int4* dst = reinterpret_cast<int4*>(obs + (ix - lane) * 24);
#pragma unroll
  for (int q = 0; q < 6; ++q) st_out(dst + q * 64 + lane, lds[q * 64 + lane]);
  __builtin_amdgcn_wave_barrier();
}

// obs rows through the wave's LDS slice (whole 1-KiB store instructions) or
// straight from each lane (6 x 16 B at a 96-B lane stride).  FULL4 takes
// the direct path: its turn is issue-bound far below the store rate, and the
// LDS round trip costs more than the scattered stores (sustained 1,000-ply
// rollouts, one box: 0.592 vs 0.614 ms per 100 plies); REF2's k_step keeps
// the LDS path (6.1 vs 6.7 us per launch).
#ifndef NARDE_FULL4_OBS_LDS
#define NARDE_FULL4_OBS_LDS 0
#endif
__device__ __forceinline__ void store_common(const Outs& out, size_t ix, const Side& s, int reward,
                                             int term, int trunc, int4* lds, bool via_lds) {
  if (out.obs) {
    if (via_lds) store_obs_wave(out.obs, ix, s, lds);
    else store_obs(out.obs, ix, s);
  }
  if (out.reward) st_out(out.reward + ix, (int32_t)reward);
  if (out.term) st_out(out.term + ix, (uint8_t)term);
  if (out.trunc) st_out(out.trunc + ix, (uint8_t)trunc);
}

__device__ __forceinline__ void store_outs(const Outs& out, size_t ix, const Side& s,
                                           const StepOut& o, int term, int trunc, int4* lds,
                                           bool wave_full) {
  store_common(out, ix, s, o.reward, term, trunc, lds, NARDE_OBS_STORE != 0 && wave_full);
  if (out.legal) st_out(out.legal + ix, (uint64_t)compact_legal(o.l1));
  if (out.act_out)
    st_out(reinterpret_cast<uint32_t*>(out.act_out) + ix,
           ((uint32_t)(uint16_t)o.code1) | ((uint32_t)(uint16_t)o.code2 << 16));
}

__device__ __forceinline__ void store_outs(const Outs& out, size_t ix, const Side& s,
                                           const TurnOut& o, int term, int trunc, int4* lds,
                                           bool wave_full) {
  store_common(out, ix, s, o.reward, term, trunc, lds,
               NARDE_FULL4_OBS_LDS && NARDE_OBS_STORE != 0 && wave_full);
  if (out.legal) st_out(out.legal + ix, o.legal);
  if (out.played) st_out(out.played + ix, o.played);
}

// this wave's slice of the block's obs staging buffer (6 KiB per wave)
#define OBS_LDS_DECL                                   \
  __shared__ int4 obs_lds[kBlock * 6];                 \
  int4* const wave_lds = obs_lds + (threadIdx.x & ~63) * 6;

// the words of ply t with the Philox block kept in R across consecutive
// plies: a new block on the first ply of a launch and on every even t
__device__ __forceinline__ void ply_draw_cached(const Rng& g, uint32_t t, uint32_t i, uint32_t R[4], bool first,
                                                uint32_t r[4]) {
  if (first || (t & 1u) == 0u) ply_block(t, g.env0 + i, g.k0, g.k1, R);
  ply_words_of(R, t, g.dice_mode, r);
}

// one ply for env i: draw with the env's own counter, then the shared
// host/device ply (narde_rules.h)
__device__ __forceinline__ void ply(Side& s, int4& st, const Rng& g, uint32_t i,
                                    const int16_t* actions, const uint8_t* dice, int max_steps,
                                    bool autoreset, StepOut& o, int& term, int& trunc, uint32_t R[4],
                                    bool first) {
  uint32_t r[4];
  ply_draw_cached(g, s.t, i, R, first, r);
  int d0 = 0, d1 = 0, c1 = 0, c2 = 0;
  if (dice) { d0 = dice[2 * i]; d1 = dice[2 * i + 1]; }
  if (actions) { c1 = actions[2 * i]; c2 = actions[2 * i + 1]; }
  env_ply(s, st, r, dice != nullptr, d0, d1, g.dice_mode, actions == nullptr, c1, c2, max_steps,
          autoreset, o, term, trunc);
}

// one FULL4 ply (a whole turn per step), the turn
// played wave-cooperatively: every lane of the wave must call it (lanes past
// the last env pass valid = false and a dummy state)
__device__ __forceinline__ void ply(Side& s, int4& st, const Rng& g, uint32_t i, bool valid,
                                    const int8_t* play, const uint8_t* dice, int max_steps,
                                    bool autoreset, TurnOut& o, int& term, int& trunc, CoopLds& W,
                                    uint32_t R[4], bool first) {
  uint32_t r[4];
  ply_draw_cached(g, s.t, i, R, first, r);
  int d0 = 1, d1 = 2;
  if (dice && valid) { d0 = dice[2 * i]; d1 = dice[2 * i + 1]; }
  // one 8-B load per env: the play's four (from, die) pairs
  const uint64_t pw = (play && valid) ? reinterpret_cast<const uint64_t*>(play)[i] : ~0ull;
  const int lane = (int)(threadIdx.x & 63);
  env_ply_full_with(s, st, r, g.env0 + i, g.k0, g.k1, dice != nullptr, d0, d1, g.dice_mode,
                    play != nullptr, pw, max_steps, autoreset, o, term, trunc,
                    [&](Side& s2, int a, int b, bool pl, uint64_t pw2, const uint32_t* w2, TurnOut& o2) {
                      coop_turn_full(s2, a, b, pl, pw2, w2, o2, W, lane);
                    });
}

__device__ __forceinline__ void add_stats(int4* __restrict__ stats, int i, const int4& st) {
  if (st.x) {
    int4 cur = stats[i];
    cur.x += st.x; cur.y += st.y; cur.z += st.z;
    stats[i] = cur;
  }
}

// NardeEnv.step for every env (API step; one ply of self-play when the
// actions are NULL).  kFull: FULL4 whole turns (TurnOut), else REF2 (StepOut).
template <bool kFull>
__global__ void __launch_bounds__(kBlock) k_step(StepArgs a) {
  OBS_LDS_DECL
  COOP_LDS_DECL
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < a.n;
  if (!kFull && !valid) return;  // FULL4 lanes stay: its turn is wave-cooperative
  Side s = valid ? side_from_record(a.pl.p0[i], a.pl.p1[i]) : side_start(0u);
  int4 st = make_int4(0, 0, 0, 0);
  typename std::conditional<kFull, TurnOut, StepOut>::type o;
  int term, trunc;
  uint32_t R[4];
  if constexpr (kFull)
    ply(s, st, a.g, (uint32_t)i, valid, a.play, a.dice, a.max_steps, a.autoreset != 0, o, term, trunc,
        wave_coop, R, true);
  else
    ply(s, st, a.g, (uint32_t)i, a.actions, a.dice, a.max_steps, a.autoreset != 0, o, term, trunc, R, true);
  if (!valid) return;
  uint4 ra, rb;
  side_to_record(s, ra, rb);
  a.pl.p0[i] = ra;
  a.pl.p1[i] = rb;
  add_stats(a.pl.stats, i, st);
  store_outs(a.out, (size_t)i, s, o, term, trunc, wave_lds, i - (int)(threadIdx.x & 63) + 64 <= a.n);
}

// `plies` plies of random-legal self-play with auto-reset in one launch; the
// record stays in VGPRs, each ply's outputs (if requested) are streamed to
// [ply][n] rollout buffers.  kOut = false: statistics only (a separate
// instantiation, so profiles tell the two apart).
#ifndef NARDE_ROLLOUT_MINW
#define NARDE_ROLLOUT_MINW 1
#endif
template <bool kOut, bool kFull>
__global__ void __launch_bounds__(kBlock, NARDE_ROLLOUT_MINW) k_rollout(Planes pl, int n, Rng g, int plies, int max_steps,
                                                    Outs out) {
  OBS_LDS_DECL
  COOP_LDS_DECL
#ifdef NARDE_DIAG_LDS_PAD
  // DIAGNOSTIC: LDS the kernel never uses, to cap its occupancy
  __shared__ uint32_t diag_pad[NARDE_DIAG_LDS_PAD / 4];
  if (n == -12345) ((volatile uint32_t*)diag_pad)[threadIdx.x] = (uint32_t)plies;
#endif
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < n;
  if (!kFull && !valid) return;  // FULL4 lanes stay: its turn is wave-cooperative
  const bool wave_full = i - (int)(threadIdx.x & 63) + 64 <= n;
  Side s = valid ? side_from_record(pl.p0[i], pl.p1[i]) : side_start(0u);
  int4 st = make_int4(0, 0, 0, 0);
  uint32_t R[4];  // the Philox block of the current ply pair
  for (int p = 0; p < plies; ++p) {
    typename std::conditional<kFull, TurnOut, StepOut>::type o;
    int term, trunc;
    if constexpr (kFull)
      ply(s, st, g, (uint32_t)i, valid, (const int8_t*)nullptr, nullptr, max_steps, true, o, term, trunc,
          wave_coop, R, p == 0);
    else
      ply(s, st, g, (uint32_t)i, (const int16_t*)nullptr, nullptr, max_steps, true, o, term, trunc, R,
          p == 0);
    if (kOut && valid) store_outs(out, (size_t)p * n + i, s, o, term, trunc, wave_lds, wave_full);
  }
  if (!valid) return;
  uint4 ra, rb;
  side_to_record(s, ra, rb);
  pl.p0[i] = ra;
  pl.p1[i] = rb;
  add_stats(pl.stats, i, st);
}

// ---------------------------------------------------------------------------
// k_rollout_pc: the REF2 rollout as a producer/consumer workgroup.
//
// At B = 65,536 one lane per env gives exactly one wave per SIMD, and one wave
// alone issues a VALU instruction only every 4 cycles (MI355X_MICROARCH.md,
// constants table) -- half of what the SIMD can issue.  So each workgroup
// (one per CU) holds 256 envs on 8 waves, two per SIMD:
//   waves 0-3 (producers, the older waves, which win VALU arbitration) run
//     the rules for their env with the record in VGPRs;
//   waves 4-7 (consumers) do the work that does not depend on the state:
//     the Philox draws of the NEXT block of plies (counter-based, so known
//     in advance), and the per-ply outputs of the PREVIOUS block, expanded
//     from the ply results the producers left in LDS and stored so that
//     every wave-wide store is one contiguous 1 KiB.
// Plies go in blocks of kPcR with one workgroup barrier per block; LDS holds
// two slots of each ring (draws and results), 16 + 96 KiB.
// Equivalent, bit for bit, to `plies` narde_step(NULL, NULL, autoreset=1).
#ifndef NARDE_PC_SETS
#define NARDE_PC_SETS 1
#endif
// rule (producer) waves per workgroup, each with its consumer wave(s)
#ifndef NARDE_PC_GROUPS
#define NARDE_PC_GROUPS 4
#endif
constexpr int kPcGroups = NARDE_PC_GROUPS;
constexpr int kPcEnvs = 64 * kPcGroups;        // envs per workgroup
constexpr int kPcSets = NARDE_PC_SETS;        // consumer waves per producer wave
constexpr int kPcThreads = (1 + kPcSets) * kPcEnvs;  // producers + consumers
// plies per barrier block (tuning knob: 3, 4 and 5 time the same)
#ifndef NARDE_PC_R
#define NARDE_PC_R 4
#endif
constexpr int kPcR = NARDE_PC_R;                       // plies per barrier block

// Ring slots and the synchronisation of the two roles:
//   NARDE_PC_FLAGS 0: one workgroup barrier per block, 2 slots;
//   NARDE_PC_FLAGS 1: each rule wave and its consumer wave (they share
//     only their own 64 env columns) hand blocks over through three LDS
//     counters -- drawn, produced, emitted -- with NARDE_PC_SLOTS slots, so
//     neither role waits for the other pairs.  Bit-exact, but slower:
//     sustained 1,000-ply rollouts 0.139 (3 slots) / 0.139-0.143 (2) against
//     0.1315 ms per 100 plies with the barrier on the same box -- the
//     workgroup-wide lockstep keeps the CU's output stream better formed.
//     Kept as an A/B knob (default 0).
#ifndef NARDE_PC_FLAGS
#define NARDE_PC_FLAGS 0
#endif
#ifndef NARDE_PC_SLOTS
#define NARDE_PC_SLOTS (NARDE_PC_FLAGS ? 3 : 2)
#endif
constexpr int kPcSlots = NARDE_PC_SLOTS;
static_assert(!NARDE_PC_FLAGS || kPcSets == 1, "flag hand-over needs one consumer wave per rule wave");
static_assert(NARDE_PC_FLAGS || kPcSlots == 2, "barrier hand-over uses two slots");

struct PcLds {
  uint2 draw[kPcSlots][kPcR][kPcEnvs];        // the ply's (wa, wb) per env and ply
  // ply results (kOut only), structure-of-arrays (a wave's reads of one
  // field are contiguous; 1 % faster than three uint4 per env, and 8 KiB
  // less LDS):
  uint4 nib0[kPcSlots][kPcR][kPcEnvs];               // {own w0, own w1, own w2, opp w0}
  uint2 nib1[kPcSlots][kPcR][kPcEnvs];               // {opp w1, opp w2}  (next mover's view)
  uint2 legal[kPcSlots][kPcR][kPcEnvs];              // compact legal set (lo, hi)
  uint2 cf[kPcSlots][kPcR][kPcEnvs];                 // {code1 | code2 << 16, reward | term << 8 | trunc << 16}
};

__device__ __forceinline__ void pc_put(PcLds& L, int slot, int k, int le, const Side& s,
                                       const StepOut& o, int term, int trunc) {
  const uint64_t lg = compact_legal(o.l1);
  L.nib0[slot][k][le] = make_uint4(s.own.w[0], s.own.w[1], s.own.w[2], s.opp.w[0]);
  L.nib1[slot][k][le] = make_uint2(s.opp.w[1], s.opp.w[2]);
  L.legal[slot][k][le] = make_uint2((uint32_t)lg, (uint32_t)(lg >> 32));
  L.cf[slot][k][le] = make_uint2(((uint32_t)(uint16_t)o.code1) | ((uint32_t)(uint16_t)o.code2 << 16),
                                 (uint32_t)o.reward | ((uint32_t)term << 8) | ((uint32_t)trunc << 16));
}

// consumer: outputs of plies p0 .. p0+np-1 for the 64 envs of consumer wave cw
__device__ __forceinline__ void pc_emit(const PcLds& L, int slot, int np, int p0, int n, int wg_env0,
                                        int cw, int lane, const Outs& out, int k0, int kstep) {
  const int e0 = cw * 64;          // first env of this wave, workgroup-local
  const int g0 = wg_env0 + e0;     // ... global (handle) index
  const bool mine = g0 + lane < n;
  for (int k = k0; k < np; k += kstep) {
    const size_t row0 = (size_t)(p0 + k) * n + g0;
    if (out.obs) {
      // the wave's 64 obs rows are 384 contiguous int4 quads: lane takes
      // quads lane + 64 q, so every store instruction covers 1 KiB
      int4* dst = reinterpret_cast<int4*>(out.obs + row0 * 24);
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const int j = lane + 64 * q;
        const int el = j / 6, qq = j - 6 * el;
        if (g0 + el >= n) continue;
        const int wi = qq >> 1, sh = (qq & 1) * 16;
        // read only the two words this quad needs: own word wi is dword wi
        // of nib0, opponent word wi is dword 3 of nib0 or wi - 1 of nib1
        const uint32_t* n0w = reinterpret_cast<const uint32_t*>(&L.nib0[slot][k][e0 + el]);
        const uint32_t* n1w = reinterpret_cast<const uint32_t*>(&L.nib1[slot][k][e0 + el]);
        const uint32_t own = n0w[wi];
        const uint32_t opp = wi == 0 ? n0w[3] : n1w[wi - 1];
        int4 v;
#if NARDE_DIAG_ABLATE & 8
        st_out(dst + j, make_int4(own, opp, 0, 0)); continue;
#endif
        v.x = (int)((own >> sh) & 15u) - (int)((opp >> sh) & 15u);
        v.y = (int)((own >> (sh + 4)) & 15u) - (int)((opp >> (sh + 4)) & 15u);
        v.z = (int)((own >> (sh + 8)) & 15u) - (int)((opp >> (sh + 8)) & 15u);
        v.w = (int)((own >> (sh + 12)) & 15u) - (int)((opp >> (sh + 12)) & 15u);
        st_out(dst + j, v);
      }
    }
#if NARDE_DIAG_ABLATE & 512
    if (false) {  // DIAGNOSTIC timing only: obs rows only
#else
    if (mine) {
#endif
      const uint2 lg = L.legal[slot][k][e0 + lane];
      const uint2 c = L.cf[slot][k][e0 + lane];
      const size_t ix = row0 + lane;
      if (out.reward) st_out(out.reward + ix, (int32_t)(c.y & 0xFFu));
      if (out.term) st_out(out.term + ix, (uint8_t)((c.y >> 8) & 1u));
      if (out.trunc) st_out(out.trunc + ix, (uint8_t)((c.y >> 16) & 1u));
      if (out.legal) st_out(out.legal + ix, (uint64_t)lg.x | ((uint64_t)lg.y << 32));
      if (out.act_out) st_out(reinterpret_cast<uint32_t*>(out.act_out) + ix, c.x);
    }
  }
}

// DIAGNOSTIC (-DNARDE_DIAG_CLOCK=1 builds only): per workgroup, wave 0's
// (s_memtime, s_memrealtime) at entry and exit of the last k_rollout_pc
// launch, for the in-kernel clock (MI355X_MICROARCH.md, DVFS give-back
// item 6).  Read by narde_diag_clock; no output depends on it.
#if NARDE_DIAG_CLOCK
__device__ unsigned long long g_diag_clock[4096][4];
#endif

// flag hand-over (NARDE_PC_FLAGS): wait until *f >= target (wave-uniform
// spin with s_sleep; bounded, so a logic error can never hang the device --
// it would show as wrong results in the parity tests instead)
__device__ __forceinline__ void pc_wait(volatile uint32_t* f, int target) {
  if (target <= 0) return;
  for (int guard = 0; guard < (1 << 21); ++guard) {
    if (__builtin_amdgcn_readfirstlane((int)*f) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no LDS access hoisted above the wait
}
// publish *f = v once this wave's LDS reads and writes have retired
__device__ __forceinline__ void pc_signal(volatile uint32_t* f, int v) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: stores to HBM stay in flight
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  *f = (uint32_t)v;
}

template <bool kOut>
__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(Planes pl, int n, Rng g, int plies,
                                                           int max_steps, Outs out) {
  __shared__ PcLds L;
#if NARDE_DIAG_CLOCK
  const unsigned long long clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool producer = wave < kPcGroups;
#if NARDE_PC_PRIO == 1
  if (!producer) __builtin_amdgcn_s_setprio(1);
#elif NARDE_PC_PRIO == 2
  if (producer) __builtin_amdgcn_s_setprio(1);
#endif
  const int le = (wave % kPcGroups) * 64 + lane;    // workgroup-local env
  // consumer set: with kPcSets > 1 the consumer waves of one env group split
  // the plies of each block (set c takes plies k = c, c + kPcSets, ...)
  const int cset = producer ? 0 : (wave - kPcGroups) / kPcGroups;
  const int wg_env0 = blockIdx.x * kPcEnvs;
  const int i = wg_env0 + le;
  const bool valid = i < n;
  const int nb = (plies + kPcR - 1) / kPcR;

  Side s;
  int4 st = make_int4(0, 0, 0, 0);
  uint32_t t0 = 0;
  if (producer) {
    if (valid) s = side_from_record(pl.p0[i], pl.p1[i]);
  } else if (valid) {
    t0 = pl.p1[i].w;
  }
  // consumer: draws of block b into slot b & 1: one Philox block (ctr
  // {t >> 1, env, 0, 0}) per ply pair, its halves to plies 2j and 2j + 1
  // (narde_rules.h ply_words)
  auto draw_block = [&](int b) {
    const int p0 = b * kPcR;
    const int np = min(kPcR, plies - p0);
    uint32_t R[4];
    for (int k = cset; k < np; k += kPcSets) {
      const uint32_t t = t0 + (uint32_t)(p0 + k);
#if NARDE_DIAG_ABLATE & 16
      R[0] = t * 0x9E3779B9u ^ (uint32_t)i; R[1] = R[0] * 0x85EBCA6Bu; R[2] = R[1] ^ 0xC2B2AE35u; R[3] = R[0] + 7u;
#else
      if (k == cset || (t & 1u) == 0u || kPcSets > 1) ply_block(t, g.env0 + (uint32_t)i, g.k0, g.k1, R);
#endif
      const bool odd = (t & 1u) != 0u;
      L.draw[b % kPcSlots][k][le] = odd ? make_uint2(R[2], R[3]) : make_uint2(R[0], R[1]);
    }
  };
  // one ply of the rule wave: block b's draw k, results into b's slot
  auto one_ply = [&](int b, int k) {
    const uint2 rv = L.draw[b % kPcSlots][k][le];
    uint32_t r[4];
    ply_words(rv.x, rv.y, g.dice_mode, r);
    StepOut o;
    int term, trunc;
#if NARDE_DIAG_ABLATE & 32
    o.l1.L[0] = r[1] & MASK24; o.l1.L[1] = r[2] & MASK24; o.l1.d[0] = 6; o.l1.d[1] = 1; o.l1.n = 2;
    o.code1 = (int)(r[1] >> 23); o.code2 = (int)(r[2] >> 23); o.reward = 0; o.term = 0;
    term = 0; trunc = 0;
    s.own.w[0] ^= r[1]; s.opp.w[1] ^= r[2]; s.t += 1u;
#else
    env_ply(s, st, r, false, 0, 0, g.dice_mode, true, 0, 0, max_steps, true, o, term, trunc);
#endif
    if (kOut) pc_put(L, b % kPcSlots, k, le, s, o, term, trunc);
  };
#if NARDE_PC_FLAGS
  __shared__ uint32_t flag_drawn[kPcGroups], flag_prod[kPcGroups], flag_emit[kPcGroups];
  const int pr = wave % kPcGroups;  // this wave's pair
  if (producer) flag_prod[pr] = 0u;
  else { flag_drawn[pr] = 0u; flag_emit[pr] = 0u; }
  __syncthreads();  // the one workgroup barrier: counters initialised
  if (producer) {
    for (int b = 0; b < nb; ++b) {
      const int np = min(kPcR, plies - b * kPcR);
      pc_wait(&flag_drawn[pr], b + 1);                     // block b's draws written
      if (kOut) pc_wait(&flag_emit[pr], b + 1 - kPcSlots);  // the slot's last results read
      if (valid)
        for (int k = 0; k < np; ++k) one_ply(b, k);
      pc_signal(&flag_prod[pr], b + 1);
    }
  } else {
    for (int j = 0; j <= nb; ++j) {
      if (j < nb) {
        pc_wait(&flag_prod[pr], j + 1 - kPcSlots);  // the slot's last draws read
        draw_block(j);
        pc_signal(&flag_drawn[pr], j + 1);
      }
      if (kOut && j >= 1) {
        const int p0 = (j - 1) * kPcR;
        pc_wait(&flag_prod[pr], j);  // block j - 1's results written
        pc_emit(L, (j - 1) % kPcSlots, min(kPcR, plies - p0), p0, n, wg_env0, pr, lane, out, 0, 1);
        pc_signal(&flag_emit[pr], j);
      }
    }
  }
#else
  if (!producer) draw_block(0);
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    const int p0 = b * kPcR;
    const int np = min(kPcR, plies - p0);
    if (producer) {
      if (valid) {
#if NARDE_PC_UNROLL
        if (np == kPcR) {
#pragma unroll
          for (int k = 0; k < kPcR; ++k) one_ply(b, k);
        } else {
          for (int k = 0; k < np; ++k) one_ply(b, k);
        }
#else
        for (int k = 0; k < np; ++k) one_ply(b, k);
#endif
      }
    } else {
      if (b + 1 < nb) draw_block(b + 1);
      if (kOut && b > 0)
        pc_emit(L, (b - 1) & 1, kPcR, p0 - kPcR, n, wg_env0, wave % kPcGroups, lane, out, cset, kPcSets);
    }
    __syncthreads();
  }
  if (kOut && !producer && nb > 0) {
    const int p0 = (nb - 1) * kPcR;
    pc_emit(L, (nb - 1) & 1, plies - p0, p0, n, wg_env0, wave % kPcGroups, lane, out, cset, kPcSets);
  }
#endif
  if (producer && valid) {
    uint4 ra, rb;
    side_to_record(s, ra, rb);
    pl.p0[i] = ra;
    pl.p1[i] = rb;
    add_stats(pl.stats, i, st);
  }
#if NARDE_DIAG_CLOCK
  if (threadIdx.x == 0 && blockIdx.x < 4096) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    g_diag_clock[blockIdx.x][0] = clk0; g_diag_clock[blockIdx.x][1] = clk1;
    g_diag_clock[blockIdx.x][2] = rt0; g_diag_clock[blockIdx.x][3] = rt1;
  }
#endif
}

}  // namespace
