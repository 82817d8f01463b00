// kernels_rollout.h -- the timed path: per-ply outputs, k_step, the producer/consumer rollouts k_rollout_pc (REF2) and k_rollout_pp_full (FULL4) (DESIGN.md sections 5, 10)
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
  int64_t* __restrict__ totals;   // [workgroup][3] statistics after the launch (wg_totals), or null
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

// The per-call API kernels (k_step, k_observe) store non-temporally: a
// launch's outputs are all it writes, and their L2 write-back is otherwise
// on the call's critical path (with the straight-line REF2 ply below,
// k_step<false> 5.25 -> 5.09-5.12 us and k_observe 2.88 -> 2.71 us per
// graph-replayed call; profiles/r05/ab/api_kstep_variants.log).  The
// rollouts store through raw buffer stores (pc_st* below).
template <class T>
__device__ __forceinline__ void st_nt(T* p, T v) {
  if constexpr (sizeof(T) == 16) {
    typedef int v4nt __attribute__((ext_vector_type(4)));
    v4nt x;
    __builtin_memcpy(&x, &v, 16);
    __builtin_nontemporal_store(x, reinterpret_cast<v4nt*>(p));
  } else {
    __builtin_nontemporal_store(v, p);
  }
}

// the nibble of x at bit `off` (a multiple of 4, below 32) as one v_bfe_u32:
// with a per-lane offset the compiler emits a shift and a mask (two VALU)
__device__ __forceinline__ int nib_at(uint32_t x, int off) {
  return (int)__builtin_amdgcn_ubfe(x, (uint32_t)off, 4u);
}

// a - b of byte B of each operand as one VALU (v_sub_u32 with SDWA byte
// selects; written out because the compiler folds the byte masks below back
// into per-nibble extracts)
template <int B>
__device__ __forceinline__ int sub_byte(uint32_t a, uint32_t b) {
  int r;
  if constexpr (B == 0)
    asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0"
        : "=v"(r) : "v"(a), "v"(b));
  else if constexpr (B == 1)
    asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1"
        : "=v"(r) : "v"(a), "v"(b));
  else if constexpr (B == 2)
    asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2"
        : "=v"(r) : "v"(a), "v"(b));
  else
    asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3"
        : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// obs points 4q .. 4q + 3 (obs_point: own - opponent count; the two never
// share a point) from nibble words `own` / `opp` holding them (q odd: the
// word's upper half): the even and odd nibbles spread to bytes, then one
// byte-select subtraction per point -- 1.75 VALU a point instead of 3
template <int Q>
__device__ __forceinline__ int4 obs_quad_w(uint32_t own, uint32_t opp) {
  const uint32_t ol = own & 0x0F0F0F0Fu, oh = (own >> 4) & 0x0F0F0F0Fu;
  const uint32_t pl = opp & 0x0F0F0F0Fu, ph = (opp >> 4) & 0x0F0F0F0Fu;
  if constexpr ((Q & 1) == 0)
    return make_int4(sub_byte<0>(ol, pl), sub_byte<0>(oh, ph), sub_byte<1>(ol, pl), sub_byte<1>(oh, ph));
  else
    return make_int4(sub_byte<2>(ol, pl), sub_byte<2>(oh, ph), sub_byte<3>(ol, pl), sub_byte<3>(oh, ph));
}

template <int Q>
__device__ __forceinline__ int4 obs_quad(const Side& s) {
  return obs_quad_w<Q>(s.own.w[Q >> 1], s.opp.w[Q >> 1]);
}

__device__ __forceinline__ void store_obs(int32_t* __restrict__ obs, size_t ix, const Side& s) {
  int4* o = reinterpret_cast<int4*>(obs + ix * 24);
  st_nt(o + 0, obs_quad<0>(s));
  st_nt(o + 1, obs_quad<1>(s));
  st_nt(o + 2, obs_quad<2>(s));
  st_nt(o + 3, obs_quad<3>(s));
  st_nt(o + 4, obs_quad<4>(s));
  st_nt(o + 5, obs_quad<5>(s));
}

// whole-wave obs store through the wave's 6-KiB LDS slice (all 64 lanes
// active, rows ix - lane .. ix - lane + 63 contiguous)
__device__ __forceinline__ void store_obs_wave(int32_t* __restrict__ obs, size_t ix, const Side& s,
                                               int4* __restrict__ lds) {
  const int lane = threadIdx.x & 63;
  lds[lane * 6 + 0] = obs_quad<0>(s);
  lds[lane * 6 + 1] = obs_quad<1>(s);
  lds[lane * 6 + 2] = obs_quad<2>(s);
  lds[lane * 6 + 3] = obs_quad<3>(s);
  lds[lane * 6 + 4] = obs_quad<4>(s);
  lds[lane * 6 + 5] = obs_quad<5>(s);
  wave_lds_handoff();
  int4* dst = reinterpret_cast<int4*>(obs + (ix - lane) * 24);
#pragma unroll
  for (int q = 0; q < 6; ++q) st_nt(dst + q * 64 + lane, lds[q * 64 + lane]);
  wave_lds_handoff();  // the slice's next writes stay behind these reads
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
  if (out.reward) st_nt(out.reward + ix, (int32_t)reward);
  if (out.term) st_nt(out.term + ix, (uint8_t)term);
  if (out.trunc) st_nt(out.trunc + ix, (uint8_t)trunc);
}

__device__ __forceinline__ void store_outs(const Outs& out, size_t ix, const Side& s,
                                           const StepOut& o, int term, int trunc, int4* lds,
                                           bool wave_full) {
  store_common(out, ix, s, o.reward, term, trunc, lds, wave_full);
  if (out.legal) st_nt(out.legal + ix, (uint64_t)compact_legal(o.l1));
  if (out.act_out)
    st_nt(reinterpret_cast<uint32_t*>(out.act_out) + ix,
           ((uint32_t)(uint16_t)o.code1) | ((uint32_t)(uint16_t)o.code2 << 16));
}

__device__ __forceinline__ void store_outs(const Outs& out, size_t ix, const Side& s,
                                           const TurnOut& o, int term, int trunc, int4* lds,
                                           bool wave_full) {
  (void)wave_full;
  store_common(out, ix, s, o.reward, term, trunc, lds, false);
  if (out.legal) st_nt(out.legal + ix, o.legal);
  if (out.played) st_nt(out.played + ix, o.played);
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
  // self-play with auto-reset (every argument a kernel argument: a
  // wave-uniform branch): the rollouts' straight-line ply
  if (!dice && !actions && autoreset) env_ply_policy_sl(s, st, r, g.dice_mode, max_steps, o, term, trunc);
  else env_ply(s, st, r, dice != nullptr, d0, d1, g.dice_mode, actions == nullptr, c1, c2, max_steps,
               autoreset, o, term, trunc);
}

// the words of ply p of a launch (env counter t): the Philox block on the
// launch's first ply and on every even t.  par >= 0: every lane's counter
// had parity par at ply 0 (every env's t advances by one per ply), so the
// test is a scalar branch; par < 0: per lane
__device__ __forceinline__ void ply_draw_wave(const Rng& g, uint32_t t, uint32_t i, uint32_t R[4], int p, int par,
                                              uint32_t r[4]) {
  if (par >= 0) {
    if (p == 0 || ((par + p) & 1) == 0) ply_block(t, g.env0 + i, g.k0, g.k1, R);
  } else if (p == 0 || (t & 1u) == 0u) {
    ply_block(t, g.env0 + i, g.k0, g.k1, R);
  }
  ply_words_of(R, t, g.dice_mode, r);
}

// the wave's counter parity for ply_draw_wave (0 / 1, or -1 if mixed)
__device__ __forceinline__ int wave_parity(bool valid, uint32_t t) {
  const uint64_t odd = __ballot(valid && (t & 1u)), vm = __ballot(valid);
  return odd == 0ull ? 0 : (odd == vm ? 1 : -1);
}

// one FULL4 ply of the random-legal policy with device dice (ply p of the
// launch): the draw, the block test (turn_block_set_sl: the failing
// windows), the turn of every lane (ply_free_turn, or kernels_full4.h
// ply_bound_turn in a wave with a block-bound doubles lane), the end of the
// ply.  Every lane of the wave must call it.  (Round 3 -- turn_free /
// turn_free<true> / coop_turn_full by kind of wave, per-lane branches: 0.460
// ms per 100 plies of 20-ply k_rollout_wave launches)
// a wave with no block-bound doubles lane: every lane's C_0 / M from the
// masks (turn_c0_free), the block-bound two-dice lanes' (kFilt: the wave has
// one) from the failing windows (turn_c0_pair_bound_w), the sub-moves
// straight-line (turn_moves_sl)
template <bool kFilt>
__device__ __forceinline__ void ply_free_turn(Side& s, int dh, int dl, uint32_t bs, uint32_t fw, const uint32_t w[4],
                                              bool flip_always, TurnOut& o, const TurnC0& c) {
  uint32_t Lh = c.Lh, Ll = c.Ll, Ch = c.Ch, Cl = c.Cl;
  int M = c.M;
  const bool b2 = kFilt && bs != 0u;
  if (kFilt && b2) turn_c0_pair_bound_w(s, dh, dl, bs, fw, Lh, Ll, Ch, Cl, M);
  turn_moves_sl(s, dh, dl, Ch, Cl, M, c.hl0, w, b2, fw, flip_always, o);
}

// the turn and the end of the ply once the block test (bs, fw) and
// turn_c0_free's results (c) are known; w = turn_words of the ply's words r,
// rb = reset_black(r[3]) (auto-reset only); every lane of the wave must call
// it
__device__ __forceinline__ void ply_full_turn(Side& s, int4& st, int dh, int dl, uint32_t bs, uint32_t fw,
                                              const TurnC0& c, const uint32_t w[4], uint32_t rb, int max_steps,
                                              bool autoreset, TurnOut& o, int& term, int& trunc) {
  const uint32_t mover_black = s.black;
  // three kinds of wave (one instruction stream each): no block-bound
  // lane, block-bound two-dice lanes only, a block-bound doubles lane
  // (one copy of the turn for all three: 0.448 against 0.437 ms per 100
  // plies of 20-ply launches, tools/diag/gpu_ab_f4.sh)
  if (__ballot(bs != 0u && dh == dl) == 0ull) {
    if (__ballot(bs != 0u) == 0ull) ply_free_turn<false>(s, dh, dl, bs, fw, w, autoreset, o, c);
    else ply_free_turn<true>(s, dh, dl, bs, fw, w, autoreset, o, c);
  } else {
    ply_bound_turn_c0(s, dh, dl, bs, fw, w, autoreset, o, (int)(threadIdx.x & 63), c);
  }
  if (autoreset) ply_close_sl_b(s, st, o.term, o.reward, mover_black, rb, max_steps, term, trunc);
  else ply_close(s, st, o.term, o.reward, mover_black, 0u, max_steps, false, term, trunc);
}

// the ply from what its words give (dice dh >= dl, the pick words w, the
// auto-reset side rb); every lane of the wave must call it
__device__ __forceinline__ void ply_full_dice(Side& s, int4& st, int dh, int dl, const uint32_t w[4], uint32_t rb,
                                              int max_steps, bool autoreset, TurnOut& o, int& term, int& trunc) {
  const uint32_t low = block_lowmask(s.P);
  uint32_t fw;
  const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, low, dh, dl, fw);
  TurnC0 c;
  turn_c0_free(s, dh, dl, c.Lh, c.Ll, c.Ch, c.Cl, c.M, c.hl0);
  ply_full_turn(s, st, dh, dl, bs, fw, c, w, rb, max_steps, autoreset, o, term, trunc);
}

// what a ply's words r give ply_full_dice, packed: dh | dl << 4 | rb << 8
// (and the pick words w) -- computed by the rollout's consumer wave, off the
// turn's stream
__device__ __forceinline__ uint32_t ply_dice_word(const uint32_t r[4], int dice_mode, uint32_t w[4]) {
  int d0, d1;
  dice_from(r[0], dice_mode, d0, d1);
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  turn_words(r, w);
  return (uint32_t)dh | ((uint32_t)dl << 4) | (reset_black(r[3]) << 8);
}

// the ply with its words r already drawn (ply_words); every lane of the wave
// must call it
__device__ __forceinline__ void ply_full_words(Side& s, int4& st, const uint32_t r[4], int dice_mode,
                                               int max_steps, bool autoreset, TurnOut& o, int& term,
                                               int& trunc) {
  uint32_t w[4];
  const uint32_t dw = ply_dice_word(r, dice_mode, w);
  ply_full_dice(s, st, (int)(dw & 15u), (int)((dw >> 4) & 15u), w, autoreset ? dw >> 8 : 0u, max_steps, autoreset,
                o, term, trunc);
}

__device__ __forceinline__ void ply_policy_full(Side& s, int4& st, const Rng& g, uint32_t i, int max_steps,
                                                bool autoreset, TurnOut& o, int& term, int& trunc,
                                                uint32_t R[4], int p, int par) {
  uint32_t r[4];
  ply_draw_wave(g, s.t, i, R, p, par, r);
  ply_full_words(s, st, r, g.dice_mode, max_steps, autoreset, o, term, trunc);
}

// one FULL4 ply (a whole turn per step), the turn
// played wave-cooperatively: every lane of the wave must call it (lanes past
// the last env pass valid = false and a dummy state)
__device__ __forceinline__ void ply(Side& s, int4& st, const Rng& g, uint32_t i, bool valid,
                                    const int8_t* play, const uint8_t* dice, int max_steps,
                                    bool autoreset, TurnOut& o, int& term, int& trunc, uint32_t R[4],
                                    bool first) {
  if (!play && !dice) {  // kernel arguments: a wave-uniform branch
    ply_policy_full(s, st, g, i, max_steps, autoreset, o, term, trunc, R, 0, 0);
    return;
  }
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
                      coop_turn_full(s2, a, b, pl, pw2, w2, o2, lane);
                    });
}

__device__ __forceinline__ void add_stats(int4* __restrict__ stats, int i, const int4& st) {
  if (st.x) {
    int4 cur = stats[i];
    cur.x += st.x; cur.y += st.y; cur.z += st.z;
    stats[i] = cur;
  }
}

// add_stats, returning env i's statistics after it when `want` (read even
// if this launch finished no episode of the env); zeros otherwise
__device__ __forceinline__ int4 stats_after(int4* __restrict__ stats, int i, const int4& st, bool want) {
  int4 cur = make_int4(0, 0, 0, 0);
  if (st.x || want) {
    cur = stats[i];
    cur.x += st.x; cur.y += st.y; cur.z += st.z;
    if (st.x) stats[i] = cur;
  }
  return cur;
}

// k_rollout_pp_full's form of stats_after: env i's statistics read at the
// start of the launch (pre) -- there the load at the end, after the
// workgroup's closing barrier, sat on a short launch's critical path (one
// 20-ply FULL4 launch at the driver's shape: medians of 8, 74.4 -> 73.6 us;
// k_rollout_pc's producers finish while their consumers still store the
// last block, and it gained nothing there) -- and stored back only when the
// launch finished an episode of the env
__device__ __forceinline__ int4 stats_read(const int4* __restrict__ stats, int i, bool valid) {
  return valid ? stats[i] : make_int4(0, 0, 0, 0);
}
__device__ __forceinline__ int4 stats_after_pre(int4* __restrict__ stats, int i, int4 pre, const int4& st) {
  pre.x += st.x;
  pre.y += st.y;
  pre.z += st.z;
  if (st.x) stats[i] = pre;
  return pre;
}

// The rollout's episode totals without a second launch: every thread of
// the workgroup passes its env's statistics after the launch (zeros for
// threads with no env), and the workgroup writes their sum
// {episodes, white points, black points} to rows[blockIdx.x] -- one row per
// 256 envs (every rollout kernel holds 256 envs per workgroup).  A
// workgroup barrier: every thread must call it.  (narde_get_totals after
// the launch costs a second dispatch; right behind a launch bracketed by
// timing markers its host call also blocked for ~110 us,
// tools/diag/gpu_benchcmp2.sh.)
__device__ __forceinline__ void wg_totals(const int4& cum, int64_t* __restrict__ rows) {
  __shared__ long long red[16][3];
  long long e = cum.x, w = cum.y, k = cum.z;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    e += __shfl_xor(e, o, 64);
    w += __shfl_xor(w, o, 64);
    k += __shfl_xor(k, o, 64);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[wave][0] = e; red[wave][1] = w; red[wave][2] = k; }
  __syncthreads();
  if (threadIdx.x < 3) {
    long long t = 0;
    const int nw = (int)(blockDim.x >> 6);
    for (int q = 0; q < nw; ++q) t += red[q][threadIdx.x];
    rows[3 * blockIdx.x + threadIdx.x] = (int64_t)t;
  }
}

// NardeEnv.step for every env (API step; one ply of self-play when the
// actions are NULL).  kFull: FULL4 whole turns (TurnOut), else REF2 (StepOut).
template <bool kFull>
__global__ void __launch_bounds__(kBlock) k_step(StepArgs a) {
  OBS_LDS_DECL
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < a.n;
  if (!kFull && !valid) return;  // FULL4 lanes stay: its turn is wave-cooperative
  Side s = valid ? side_from_record(a.pl.p0[i], a.pl.p1[i]) : side_start(0u);
  int4 st = make_int4(0, 0, 0, 0);
  typename std::conditional<kFull, TurnOut, StepOut>::type o;
  int term, trunc;
  uint32_t R[4];
  if constexpr (kFull)
    ply(s, st, a.g, (uint32_t)i, valid, a.play, a.dice, a.max_steps, a.autoreset != 0, o, term, trunc, R,
        true);
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

// ---------------------------------------------------------------------------
// k_rollout_pc: the REF2 rollout as a producer/consumer workgroup.
//
// At B = 65,536 one lane per env gives exactly one wave per SIMD, and one wave
// alone issues a VALU instruction only every 4 cycles, whatever the kind;
// a second wave on the SIMD adds issue slots for the "fast" kinds (add/sub,
// and/or/xor, bitop3, shift right: every 2 cycles across two waves) and
// hides the first one's waits (profiles/r05/issue_probe/summary.json,
// tools/issue_probe.hip).  So each workgroup
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

// Barrier blocks of 1, then R plies: the output stream (the consumers'
// stores of block b - 1 while the rule waves play block b) only starts
// after the first block, and the kernel is store-bound, so a short first
// block shortens the stretch with no stores -- worth ~3 us of a 20-ply
// launch (~35 us), nothing at 1,000 plies.  (Round 5's 1, 2, then R: one
// 20-ply launch 32.0 -> 31.2-31.7 us, sustained 0.1518 -> 0.1498 ms per 100
// plies at 20 plies, 1,000 plies unchanged; 1, 1, then R lost at 1,000
// plies, 0.1288; profiles/r06/blocks/)
// R: the full blocks' plies (<= kPcR, the rings' depth) -- kPcRShort in
// launches of at most kPcShortPlies plies, where the more frequent barriers
// cost less than the stretch with no stores at the end (one launch's last
// block is stored after every rule wave is done): 20 plies 33.5 -> 33.0 us
// event span with 2-ply blocks (3: 33.4, 1: 36.1; two rounds, one box,
// profiles/r06/blocks/)
__device__ __forceinline__ int pc_nblocks(int plies, int R) {
  return plies <= 1 ? 1 : 1 + (plies - 1 + R - 1) / R;
}
__device__ __forceinline__ void pc_block(int b, int plies, int R, int& p0, int& np) {
  p0 = b == 0 ? 0 : 1 + (b - 1) * R;
  const int sz = b == 0 ? 1 : R;
  np = max(0, min(sz, plies - p0));
}
constexpr int kPcRShort = 2;
constexpr int kPcShortPlies = 32;

struct PcLds {
  // 64 unused bytes ahead of the rings: with the rings at the start of the
  // workgroup's LDS a 20-ply launch ran ~1 us slower (back-to-back 31.2 ->
  // 30.2 us, sustained 0.156 -> 0.151 ms per 100 plies at 20 plies, 0.126 ->
  // 0.125 at 1,000; any lead of 16-512 bytes alike, one box, two rounds,
  // profiles/r06/lds_lead/)
  uint4 lead_[4];
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

// obs quad qq (points 4qq .. 4qq + 3) of workgroup-local env le from the ply
// results in LDS: only the two words it needs -- own word wi is dword wi of
// nib0, opponent word wi is dword 3 of nib0 or wi - 1 of nib1
template <class Lds>
__device__ __forceinline__ int4 pc_obs_quad(const Lds& L, int slot, int k, int le, int qq) {
  const int wi = qq >> 1, sh = (qq & 1) * 16;
  const uint32_t* n0w = reinterpret_cast<const uint32_t*>(&L.nib0[slot][k][le]);
  const uint32_t* n1w = reinterpret_cast<const uint32_t*>(&L.nib1[slot][k][le]);
  const uint32_t own = n0w[wi];
  const uint32_t opp = wi == 0 ? n0w[3] : n1w[wi - 1];
  int4 v;
  v.x = nib_at(own, sh) - nib_at(opp, sh);
  v.y = nib_at(own, sh + 4) - nib_at(opp, sh + 4);
  v.z = nib_at(own, sh + 8) - nib_at(opp, sh + 8);
  v.w = nib_at(own, sh + 12) - nib_at(opp, sh + 12);
  return v;
}

// Raw buffer stores for the rollouts' consumers: a
// scalar resource (base, extent) per output and ply, built by SALU, and a
// 32-bit per-lane byte offset -- the 64-bit address arithmetic of global
// stores (two VALU per store and ply) leaves the VALU that the SIMD's rule
// and consumer waves share.  The policy: kPcStorePolicy below.  Dword 3 =
// 0x00020000, the
// gfx9 raw-buffer word (/opt/rocm/include/ck/ck.hpp).
typedef int pc_v4i __attribute__((ext_vector_type(4)));
typedef unsigned pc_v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pc_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// pc_rsrc with the base and extent passed through v_readfirstlane: both are
// wave-uniform, but where the compiler cannot prove it (k_rollout_pp_full's
// consumer) it keeps the resource in VGPRs and wraps every store in a
// readfirstlane / compare / exec loop (11 per ply there, ~80 VALU of the
// kernel); k_rollout_pc's consumer needs no help (its form would add VALU)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pc_rsrc_u(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  void* ub = reinterpret_cast<void*>((uint64_t)lo | ((uint64_t)hi << 32));
  return __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
// The stores' cache policy (gfx950 CPol bits: sc0 = 1, nt = 2, sc1 = 16):
// sc1 | nt -- non-temporal at device scope, so the lines are written
// through the XCD's L2 instead of left dirty in it for the end-of-kernel
// write-back of a short launch (and no slower in long ones, pc_emit_ply).
// One 20-ply launch after an idle GPU
// (tools/diag/single_launch.py, medians of 30, two rounds, one box,
// profiles/r06/store_policy/): REF2 event span 34.8 -> 33.3 us, host round
// trip 49.6 -> 48.1 us, FULL4 74.8 -> 73.5 us; nt alone (round 5's policy)
// 34.8, nt | sc0 34.9, sc1 36.4, plain 38.6, sc0 38.8, sc0 | sc1 36.3,
// sc0 | sc1 | nt 33.4.
constexpr int kPcStorePolicy = 16 | 2;
__device__ __forceinline__ void pc_st16(__amdgpu_buffer_rsrc_t r, uint32_t off, int4 v) {
  const pc_v4i x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)off, 0, kPcStorePolicy);
}
__device__ __forceinline__ void pc_st8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint64_t v) {
  const pc_v2u x = {(unsigned)v, (unsigned)(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(x, r, (int)off, 0, kPcStorePolicy);
}
__device__ __forceinline__ void pc_st4(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, kPcStorePolicy);
}
__device__ __forceinline__ void pc_st1(__amdgpu_buffer_rsrc_t r, uint32_t off, uint8_t v) {
  __builtin_amdgcn_raw_buffer_store_b8(v, r, (int)off, 0, kPcStorePolicy);
}

// consumer: outputs of ply p (block slot `slot`, index k) for the 64 envs of
// consumer wave cw: raw buffer stores with a wave-uniform resource per output
// and ply, no per-lane bounds branch (the resource's extent drops the stores
// past n), policy kPcStorePolicy.  Round 5 kept a second form for launches
// of more than 32 plies (global stores with the bounds branches, plain
// policy, env_ply): with the sc1 | nt policy this one is as fast or faster at
// every length (tools/gpu_r06.sh libab / sus, two rounds, one box,
// profiles/r06/blocks/): bench.py's 1,000-ply line 5.15 -> 5.22 / 5.23e10,
// sustained 100-ply launches 0.1376 -> 0.1315 ms per 100 plies, 1,000-ply
// 0.1273 -> 0.1253 / 0.1260; FULL4 (pp_emit_ply) 100: 0.279 -> 0.277, 1,000:
// 0.249 either way.
__device__ __forceinline__ void pc_emit_ply(const PcLds& L, int slot, int k, int p, int n, int wg_env0, int cw,
                                            int lane, const Outs& out) {
  const int e0 = cw * 64;  // first env of this wave, workgroup-local (LDS index)
  const int g0 = wg_env0 + __builtin_amdgcn_readfirstlane(cw) * 64;  // global, wave-uniform
  const size_t row0 = (size_t)p * n + g0;                              // wave-uniform
  const uint32_t nw = (uint32_t)max(0, min(64, n - g0));              // envs of this wave
  if (out.obs) {
    // the wave's 64 obs rows are 384 contiguous int4 quads: lane takes
    // quads lane + 64 q, so every store instruction covers 1 KiB
    const __amdgpu_buffer_rsrc_t r = pc_rsrc(out.obs + row0 * 24, nw * 96u);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int j = lane + 64 * q;
      const int el = j / 6, qq = j - 6 * el;
      pc_st16(r, (uint32_t)j * 16u, pc_obs_quad(L, slot, k, e0 + el, qq));
    }
  }
  const uint2 lg = L.legal[slot][k][e0 + lane];
  const uint2 c = L.cf[slot][k][e0 + lane];
  const uint32_t l = (uint32_t)lane;
  if (out.reward) pc_st4(pc_rsrc(out.reward + row0, nw * 4u), 4u * l, c.y & 0xFFu);
  if (out.term) pc_st1(pc_rsrc(out.term + row0, nw), l, (uint8_t)((c.y >> 8) & 1u));
  if (out.trunc) pc_st1(pc_rsrc(out.trunc + row0, nw), l, (uint8_t)((c.y >> 16) & 1u));
  if (out.legal) pc_st8(pc_rsrc(out.legal + row0, nw * 8u), 8u * l, (uint64_t)lg.x | ((uint64_t)lg.y << 32));
  if (out.act_out) pc_st4(pc_rsrc(reinterpret_cast<uint32_t*>(out.act_out) + row0, nw * 4u), 4u * l, c.x);
}

// consumer: outputs of plies p0 .. p0+np-1
__device__ __forceinline__ void pc_emit(const PcLds& L, int slot, int np, int p0, int n, int wg_env0, int cw,
                                        int lane, const Outs& out) {
  for (int k = 0; k < np; ++k) pc_emit_ply(L, slot, k, p0 + k, n, wg_env0, cw, lane, out);
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
  const int R = plies <= kPcShortPlies ? kPcRShort : kPcR;  // plies per full block
  const int nb = pc_nblocks(plies, R);

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
    pc_block(b, plies, R, p0, np);
    uint32_t w[4];
    for (int k = 0; k < np; ++k) {
      const uint32_t t = t0 + (uint32_t)(p0 + k);
      if (k == 0 || (t & 1u) == 0u) ply_block(t, g.env0 + (uint32_t)i, g.k0, g.k1, w);
      const bool odd = (t & 1u) != 0u;
      L.draw[b % kPcSlots][k][le] = odd ? make_uint2(w[2], w[3]) : make_uint2(w[0], w[1]);
    }
  };
  // one ply of the rule wave: block b's draw k, results into b's slot
  auto one_ply = [&](int b, int k) {
    const uint2 rv = L.draw[b % kPcSlots][k][le];
    uint32_t r[4];
    ply_words(rv.x, rv.y, g.dice_mode, r);
    StepOut o;
    int term, trunc;
    // with outputs: the straight-line ply (0.1605 -> 0.1592 ms per 100
    // plies of 20-ply launches, tools/diag/gpu_ab_sl.sh; at 1,000 plies it
    // lost to env_ply with round 5's store forms, not with this round's --
    // pc_emit_ply); self-play alone keeps env_ply
    if constexpr (kOut) env_ply_policy_sl(s, st, r, g.dice_mode, max_steps, o, term, trunc);
    else env_ply(s, st, r, false, 0, 0, g.dice_mode, true, 0, 0, max_steps, true, o, term, trunc);
    if (kOut) pc_put(L, b % kPcSlots, k, le, s, o, term, trunc);
  };
  if (!producer) draw_block(0);
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    int p0, np;
    pc_block(b, plies, R, p0, np);
    if (producer) {
      if (valid)
        for (int k = 0; k < np; ++k) one_ply(b, k);
    } else {
      if (b + 1 < nb) draw_block(b + 1);
      if (kOut && b > 0) {
        int q0, nq;
        pc_block(b - 1, plies, R, q0, nq);
        pc_emit(L, (b - 1) % kPcSlots, nq, q0, n, wg_env0, cw, lane, out);
      }
    }
    __syncthreads();
  }
  if (kOut && !producer && nb > 0) {
    int p0, np;
    pc_block(nb - 1, plies, R, p0, np);
    pc_emit(L, (nb - 1) % kPcSlots, np, p0, n, wg_env0, cw, lane, out);
  }
  int4 cum = make_int4(0, 0, 0, 0);
  if (producer && valid) {
    uint4 ra, rb;
    side_to_record(s, ra, rb);
    pl.p0[i] = ra;
    pl.p1[i] = rb;
    cum = stats_after(pl.stats, i, st, out.totals != nullptr);
  }
  if (out.totals) wg_totals(cum, out.totals);
}


// ---------------------------------------------------------------------------
// k_rollout_pp_full: the FULL4 rollout with a pairwise hand-over.  Each
// producer wave (waves 0-3) has its own consumer wave (waves 4-7) and a ring
// of kPpR ply slots in LDS (draws and results); the pair hands plies over
// through three LDS counters instead of workgroup barriers, so a producer
// never waits for the other producers of its workgroup (REF2 stays with
// k_rollout_pc: its plies are short and even, and the same pairwise kernel
// playing REF2 plies ran 0.196 / 0.140 against k_rollout_pc's 0.160 / 0.126
// ms per 100 plies at 20 / 1,000 plies, 44.1 against 37.6 us at the
// driver's shape, profiles/r05/ab/*ref2_pc_vs_pairwise*) -- FULL4's turns vary
// several-fold in cost from ply to ply (block-bound plies, DESIGN.md
// section 10), and k_rollout_pc's one barrier per block of plies made every
// producer wait for the slowest of four (the same kernel with barrier
// blocks: 0.412 / 0.307 ms per 100 plies at 20 / 1,000 plies against the
// one-wave kernel's 0.405 / 0.290 and this one's 0.382 / 0.268,
// profiles/r05/ab/sus_wave_pc_pp.log).  Round 4's one-wave kernel
// (k_rollout_wave: each wave drew its own words and stored its own rows
// at a 96-B lane stride) is retired; git history has it.
//   producer, ply p: wait until drawn > p and emitted + kPpR > p, play the
//     turn with the words of draw slot p % kPpR, leave the results in result
//     slot p % kPpR; produced = p + 1 is published early in ply p + 1 (and
//     after the last ply);
//   consumer: draws plies 0 .. kPpR - 1 ahead; for each ply p: wait until
//     produced > p, store ply p's outputs, then emitted = p + 1 (the result
//     slot is free), draw ply p + kPpR into the draw slot ply p used (read
//     before ply p was produced), then drawn = p + kPpR + 1.  A draw is the
//     Philox words and what the turn takes from them (ply_dice_word: the
//     dice, the pick words, the auto-reset side), so that work is off the
//     producer's stream (20 plies 0.371 -> 0.364, 1,000 plies 0.259 -> 0.254
//     ms per 100 plies).
// (Measured and not kept: the consumer running each ply's block test
// (turn_block_set_sl on the masks the previous ply left) while the
// producer computes C_0 -- the producer then waits for it: 20-ply launches
// 0.382 -> 0.408, 1,000 plies 0.268 -> 0.287 ms per 100 plies,
// profiles/r05/ab/.)
// Counters are wave-uniform LDS words; a release fence (workgroup scope)
// orders each side's slot accesses before its counter store, an acquire
// fence after the counter load orders the other side's.
constexpr int kPpR = 8;  // ring depth in plies

// (the draw rings behind the result rings: sustained 0.352 -> 0.350 ms per
// 100 plies at 20 plies, 0.252 -> 0.251 at 1,000, two rounds, one box,
// profiles/r06/lds_lead/sus_full4_layouts.log)
struct PpLds {
  uint4 nib0[kPcGroups][kPpR][64];
  uint2 nib1[kPcGroups][kPpR][64];
  uint2 legal[kPcGroups][kPpR][64];
  uint2 played[kPcGroups][kPpR][64];
  uint32_t rtt[kPcGroups][kPpR][64];
  uint4 draw_w[kPcGroups][kPpR][64];   // the ply's pick words (turn_words)
  uint32_t draw_d[kPcGroups][kPpR][64];  // ply_dice_word: dh | dl << 4 | reset side << 8
  uint32_t drawn[kPcGroups], produced[kPcGroups], emitted[kPcGroups];
};
// gfx950 has 160 KiB of LDS per CU: a k_rollout_pp_full workgroup holds
// PpLds and wg_totals' reduction buffer (long long[16][3]); a deeper ring or
// another per-slot array must still fit in it
static_assert(sizeof(PpLds) + sizeof(long long) * 16 * 3 <= 160 * 1024, "PpLds exceeds the CU's LDS");
// the producer publishes ply p - 1's `produced` only after ply p's drawn /
// emitted waits, so the consumer must be able to draw ply p while ply p - 1
// is unemitted: one slot would deadlock the pair
static_assert(kPpR >= 2, "k_rollout_pp_full's hand-over needs at least two ring slots");

__device__ __forceinline__ uint32_t pp_load(const uint32_t* c) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void pp_publish(uint32_t* c, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_store(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// spin until f(counter value) holds (wave-uniform), then acquire; returns
// the value seen.  kSleep: s_sleep units (64 cycles) between polls -- 1 for
// the producer, longer for the consumer, whose polls would otherwise take
// the producer's issue slots (both waves share a SIMD) while it waits a
// whole turn
template <int kSleep, class F>
__device__ __forceinline__ uint32_t pp_wait(const uint32_t* c, F ok) {
  uint32_t v;
  while (!ok(v = pp_load(c))) __builtin_amdgcn_s_sleep(kSleep);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return v;
}

// obs quad qq of env el of pair cw, ring slot sl (pc_obs_quad's layout)
__device__ __forceinline__ int4 pp_obs_quad(const PpLds& L, int cw, int sl, int el, int qq) {
  const int wi = qq >> 1, sh = (qq & 1) * 16;
  const uint32_t* n0w = reinterpret_cast<const uint32_t*>(&L.nib0[cw][sl][el]);
  const uint32_t* n1w = reinterpret_cast<const uint32_t*>(&L.nib1[cw][sl][el]);
  const uint32_t own = n0w[wi];
  const uint32_t opp = wi == 0 ? n0w[3] : n1w[wi - 1];
  int4 v;
  v.x = nib_at(own, sh) - nib_at(opp, sh);
  v.y = nib_at(own, sh + 4) - nib_at(opp, sh + 4);
  v.z = nib_at(own, sh + 8) - nib_at(opp, sh + 8);
  v.w = nib_at(own, sh + 12) - nib_at(opp, sh + 12);
  return v;
}

// consumer: ply p's outputs of pair cw's 64 envs from ring slot sl
// (pc_emit_ply's store form)
__device__ __forceinline__ void pp_emit_ply(const PpLds& L, int cw, int sl, int p, int n, int g0, int lane,
                                            const Outs& out) {
  const size_t row0 = (size_t)p * n + g0;
  const uint32_t nw = (uint32_t)max(0, min(64, n - g0));
  if (out.obs) {
    const __amdgpu_buffer_rsrc_t r = pc_rsrc_u(out.obs + row0 * 24, nw * 96u);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int j = lane + 64 * q;
      const int el = j / 6, qq = j - 6 * el;
      pc_st16(r, (uint32_t)j * 16u, pp_obs_quad(L, cw, sl, el, qq));
    }
  }
  const uint32_t c = L.rtt[cw][sl][lane];
  const uint32_t l = (uint32_t)lane;
  if (out.reward) pc_st4(pc_rsrc_u(out.reward + row0, nw * 4u), 4u * l, c & 0xFFu);
  if (out.term) pc_st1(pc_rsrc_u(out.term + row0, nw), l, (uint8_t)((c >> 8) & 1u));
  if (out.trunc) pc_st1(pc_rsrc_u(out.trunc + row0, nw), l, (uint8_t)((c >> 16) & 1u));
  if (out.legal) {
    const uint2 lg = L.legal[cw][sl][lane];
    pc_st8(pc_rsrc_u(out.legal + row0, nw * 8u), 8u * l, (uint64_t)lg.x | ((uint64_t)lg.y << 32));
  }
  if (out.played) {
    const uint2 pw = L.played[cw][sl][lane];
    pc_st8(pc_rsrc_u(out.played + row0, nw * 8u), 8u * l, (uint64_t)pw.x | ((uint64_t)pw.y << 32));
  }
}

template <bool kOut>
__global__ void __launch_bounds__(kPcThreads) k_rollout_pp_full(Planes pl, int n, Rng g, int plies,
                                                                int max_steps, Outs out) {
  __shared__ PpLds L;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool producer = wave < kPcGroups;
  const int cw = __builtin_amdgcn_readfirstlane(wave % kPcGroups);
  const int g0 = blockIdx.x * kPcEnvs + cw * 64;  // the pair's first env (global)
  const int i = g0 + lane;
  const bool valid = i < n;
  if (threadIdx.x < kPcGroups) {
    L.drawn[threadIdx.x] = 0u;
    L.produced[threadIdx.x] = 0u;
    L.emitted[threadIdx.x] = 0u;
  }
  __syncthreads();
  int4 st = make_int4(0, 0, 0, 0), pre = make_int4(0, 0, 0, 0);
  if (producer) {
    Side s = valid ? side_from_record(pl.p0[i], pl.p1[i]) : side_start(0u);
    pre = stats_read(pl.stats, i, valid);
    // the counters as last seen: a poll (an LDS round trip) only when ply p
    // is past them -- the consumer runs up to kPpR plies ahead
    uint32_t dk = 0u, ek = 0u;
    for (int p = 0; p < plies; ++p) {
      const uint32_t up = (uint32_t)p;
      const int sl = p % kPpR;
      if (up >= dk) dk = pp_wait<1>(&L.drawn[cw], [&](uint32_t v) { return v > up; });
      if (kOut && up >= ek + (uint32_t)kPpR)
        ek = pp_wait<1>(&L.emitted[cw], [&](uint32_t v) { return v + (uint32_t)kPpR > up; });
      const uint4 wv = L.draw_w[cw][sl][lane];
      const uint32_t dw = L.draw_d[cw][sl][lane];
      const uint32_t w[4] = {wv.x, wv.y, wv.z, wv.w};
      // ply p - 1's results, published here: its LDS writes are long done
      // and the release's wait covers only this ply's draw reads, which the
      // turn needs at once anyway
      if (p > 0) pp_publish(&L.produced[cw], up);
      TurnOut o;
      int term, trunc;
      ply_full_dice(s, st, (int)(dw & 15u), (int)((dw >> 4) & 15u), w, dw >> 8, max_steps, true, o, term, trunc);
      if (kOut) {
        L.nib0[cw][sl][lane] = make_uint4(s.own.w[0], s.own.w[1], s.own.w[2], s.opp.w[0]);
        L.nib1[cw][sl][lane] = make_uint2(s.opp.w[1], s.opp.w[2]);
        L.legal[cw][sl][lane] = make_uint2((uint32_t)o.legal, (uint32_t)(o.legal >> 32));
        L.played[cw][sl][lane] = make_uint2((uint32_t)o.played, (uint32_t)(o.played >> 32));
        L.rtt[cw][sl][lane] = (uint32_t)o.reward | ((uint32_t)term << 8) | ((uint32_t)trunc << 16);
      }
    }
    pp_publish(&L.produced[cw], (uint32_t)plies);
    if (valid) {
      uint4 ra, rb;
      side_to_record(s, ra, rb);
      pl.p0[i] = ra;
      pl.p1[i] = rb;
    }
  } else {
    const uint32_t t0 = valid ? pl.p1[i].w : 0u;
    uint32_t R[4];  // the Philox block of the last ply drawn (one block per ply pair)
    // the words of ply p, and what the turn takes from them (ply_dice_word)
    auto draw = [&](int p) {
      const uint32_t t = t0 + (uint32_t)p;
      if (p == 0 || (t & 1u) == 0u) ply_block(t, g.env0 + (uint32_t)i, g.k0, g.k1, R);
      uint32_t r[4], w[4];
      ply_words_of(R, t, g.dice_mode, r);
      const uint32_t dw = ply_dice_word(r, g.dice_mode, w);
      L.draw_w[cw][p % kPpR][lane] = make_uint4(w[0], w[1], w[2], w[3]);
      L.draw_d[cw][p % kPpR][lane] = dw;
    };
    const int ahead = min(kPpR, plies);
    for (int p = 0; p < ahead; ++p) {  // each ply's words published as drawn: ply 0 starts at once
      draw(p);
      pp_publish(&L.drawn[cw], (uint32_t)p + 1u);
    }
    for (int p = 0; p < plies; ++p) {
      const uint32_t up = (uint32_t)p;
      pp_wait<8>(&L.produced[cw], [&](uint32_t v) { return v > up; });
      if (kOut) {
        pp_emit_ply(L, cw, p % kPpR, p, n, g0, lane, out);
        pp_publish(&L.emitted[cw], up + 1u);
      }
      if (p + kPpR < plies) {  // ply p's draw slot was read before ply p was produced
        draw(p + kPpR);
        pp_publish(&L.drawn[cw], up + (uint32_t)kPpR + 1u);
      }
    }
  }
  __syncthreads();
  int4 cum = make_int4(0, 0, 0, 0);
  if (producer && valid) cum = stats_after_pre(pl.stats, i, pre, st);
  if (out.totals) wg_totals(cum, out.totals);
}

}  // namespace
