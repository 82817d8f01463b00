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

// Every per-ply output is a plain store.  Measured against non-temporal
// stores on sustained 1,000-ply REF2 rollouts (one box): plain 0.1265 ms
// per 100 plies, non-temporal obs rows 0.135 (the narrow outputs' policy
// did not matter).
template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
  *p = v;
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
  store_common(out, ix, s, o.reward, term, trunc, lds, wave_full);
  if (out.legal) st_out(out.legal + ix, (uint64_t)compact_legal(o.l1));
  if (out.act_out)
    st_out(reinterpret_cast<uint32_t*>(out.act_out) + ix,
           ((uint32_t)(uint16_t)o.code1) | ((uint32_t)(uint16_t)o.code2 << 16));
}

__device__ __forceinline__ void store_outs(const Outs& out, size_t ix, const Side& s,
                                           const TurnOut& o, int term, int trunc, int4* lds,
                                           bool wave_full) {
  (void)wave_full;
  store_common(out, ix, s, o.reward, term, trunc, lds, false);
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
template <bool kOut, bool kFull>
__global__ void __launch_bounds__(kBlock, 1) k_rollout(Planes pl, int n, Rng g, int plies, int max_steps,
                                                       Outs out) {
  OBS_LDS_DECL
  COOP_LDS_DECL
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
// Plies go in barrier blocks (pc_block) with one workgroup barrier per
// block; LDS holds two slots of each ring (draws and results), 16 + 96 KiB.
// Equivalent, bit for bit, to `plies` narde_step(NULL, NULL, autoreset=1).
//
// Shape measured on sustained 1,000-ply rollouts:
// one consumer wave per rule wave (two or three timed the same), four rule
// waves per workgroup (two or one: 0.173 / 0.179 against 0.132 ms per 100
// plies -- the dispatcher then no longer pairs a rule wave with a consumer
// wave on every SIMD), 4-ply blocks (3 / 5 / 6: 2-8 % slower), one
// workgroup barrier per block (a pairwise hand-over through LDS counters
// was bit-exact but 6 % slower), no wave priorities, no unrolled plies.
constexpr int kPcGroups = 4;                    // rule (producer) waves per workgroup
constexpr int kPcEnvs = 64 * kPcGroups;         // envs per workgroup
constexpr int kPcThreads = 2 * kPcEnvs;         // producers + one consumer wave each
constexpr int kPcR = 4;                         // plies per full barrier block
constexpr int kPcSlots = 2;                     // ring slots (block b uses slot b & 1)

// Barrier blocks of 1, 2, then kPcR plies: the output stream (the
// consumers' stores of block b - 1 while the rule waves play block b) only
// starts after the first block, and the kernel is store-bound, so a short
// first block shortens the stretch with no stores -- worth ~3 us of a 20-ply
// launch (~35 us), nothing at 1,000 plies.
__device__ __forceinline__ int pc_nblocks(int plies) {
  return plies <= 1 ? 1 : (plies <= 3 ? 2 : 2 + (plies - 3 + kPcR - 1) / kPcR);
}
__device__ __forceinline__ void pc_block(int b, int plies, int& p0, int& np) {
  p0 = b == 0 ? 0 : (b == 1 ? 1 : 3 + (b - 2) * kPcR);
  const int sz = b == 0 ? 1 : (b == 1 ? 2 : kPcR);
  np = max(0, min(sz, plies - p0));
}

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
                                        int cw, int lane, const Outs& out) {
  const int e0 = cw * 64;          // first env of this wave, workgroup-local
  const int g0 = wg_env0 + e0;     // ... global (handle) index
  const bool mine = g0 + lane < n;
  for (int k = 0; k < np; ++k) {
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
        v.x = (int)((own >> sh) & 15u) - (int)((opp >> sh) & 15u);
        v.y = (int)((own >> (sh + 4)) & 15u) - (int)((opp >> (sh + 4)) & 15u);
        v.z = (int)((own >> (sh + 8)) & 15u) - (int)((opp >> (sh + 8)) & 15u);
        v.w = (int)((own >> (sh + 12)) & 15u) - (int)((opp >> (sh + 12)) & 15u);
        st_out(dst + j, v);
      }
    }
    if (mine) {
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

template <bool kOut>
__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(Planes pl, int n, Rng g, int plies,
                                                           int max_steps, Outs out) {
  __shared__ PcLds L;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool producer = wave < kPcGroups;
  const int cw = wave % kPcGroups;                  // the env group of this wave
  const int le = cw * 64 + lane;                    // workgroup-local env
  const int wg_env0 = blockIdx.x * kPcEnvs;
  const int i = wg_env0 + le;
  const bool valid = i < n;
  const int nb = pc_nblocks(plies);

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
    int p0, np;
    pc_block(b, plies, p0, np);
    uint32_t R[4];
    for (int k = 0; k < np; ++k) {
      const uint32_t t = t0 + (uint32_t)(p0 + k);
      if (k == 0 || (t & 1u) == 0u) ply_block(t, g.env0 + (uint32_t)i, g.k0, g.k1, R);
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
    env_ply(s, st, r, false, 0, 0, g.dice_mode, true, 0, 0, max_steps, true, o, term, trunc);
    if (kOut) pc_put(L, b % kPcSlots, k, le, s, o, term, trunc);
  };
  if (!producer) draw_block(0);
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    int p0, np;
    pc_block(b, plies, p0, np);
    if (producer) {
      if (valid)
        for (int k = 0; k < np; ++k) one_ply(b, k);
    } else {
      if (b + 1 < nb) draw_block(b + 1);
      if (kOut && b > 0) {
        int q0, nq;
        pc_block(b - 1, plies, q0, nq);
        pc_emit(L, (b - 1) % kPcSlots, nq, q0, n, wg_env0, cw, lane, out);
      }
    }
    __syncthreads();
  }
  if (kOut && !producer && nb > 0) {
    int p0, np;
    pc_block(nb - 1, plies, p0, np);
    pc_emit(L, (nb - 1) % kPcSlots, np, p0, n, wg_env0, cw, lane, out);
  }
  if (producer && valid) {
    uint4 ra, rb;
    side_to_record(s, ra, rb);
    pl.p0[i] = ra;
    pl.p1[i] = rb;
    add_stats(pl.stats, i, st);
  }
}

}  // namespace
