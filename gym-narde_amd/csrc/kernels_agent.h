// kernels_agent.h -- what agents read and write: observations, move masks, the policy kernel and the DQN transition
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

namespace {

// obs i32[n][24] (get_perspective_board of the mover), one env per thread;
// a whole wave stages its 64 rows in LDS and stores them as contiguous
// 1-KiB pieces (store_obs_wave; a partial wave stores per lane)
__global__ void __launch_bounds__(kBlock) k_observe(Planes pl, int n, int32_t* __restrict__ obs) {
  OBS_LDS_DECL
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const int w0 = i - (int)(threadIdx.x & 63);
  if (w0 + 64 <= n) {  // wave-uniform
    store_obs_wave(obs, (size_t)i, side_from_record(pl.p0[i], pl.p1[i]), wave_lds);
  } else if (i < n) {
    store_obs(obs, (size_t)i, side_from_record(pl.p0[i], pl.p1[i]));
  }
}

// One DQN transition for every env, fused (config 4, gym_narde/dqn.py
// BatchedDQNDriver): the 198-float observation of the post-step record
// (k_observe's encoding), the reference trainer's reward shaping
// (train_deepq_pytorch.py:885-912), the prioritized-replay write of
// (a, r', done) with the running max priority, and s <- s'.
//
// Replay ring layout (DeviceReplay): row j holds transition j's s; its s'
// is row (j + n) % capacity -- the s of the same env's next transition, so
// each observation is stored once.  This step's rows are (pos + i) %
// capacity (their s is already there: written as s' by the previous step,
// or by DeviceReplay.seed); s' goes to row (pos + n + i) % capacity, whose
// priority drops to 0 until the next step completes it (never sampled).
// One thread per 4 observation floats (coalesced rows; the 32-B record is an
// L1 hit for the row's threads); the thread holding column 0 of a row also
// writes the env's scalars.  HBM per env: 2 x 792 B written (ring row, s').
struct TransArgs {
  Planes pl;
  int n;
  int shaping;
  float* state;                 // (n,198) out: s'
  const int64_t* actions;       // (n,2)
  const int32_t* reward;        // (n,)
  const uint8_t* term;          // (n,)
  const uint8_t* trunc;         // (n,)
  const uint64_t* legal;        // (n,) compact list #1 of the step; NULL = every env could move
  int32_t* misc;                // (n,) off_w | off_b << 4 | black << 10: in before the step, out after
  float* off_seen;              // (n,2) borne-off trackers, white/black
  float* r_obs;                 // replay ring (capacity,198)
  int64_t* r_action;            // replay (capacity,2)
  float* r_reward;              // replay (capacity,)
  float* r_done;                // replay (capacity,)
  float* r_prio;                // replay (capacity,)
  const float* max_prio;        // device scalar
  const int64_t* pos;           // device scalar: ring write cursor
  int64_t capacity;
};

// value of column col of the 198-float observation of a record (k_observe's
// layout), branch-free: the 64 lanes of a wave hold 64 consecutive columns,
// so per-column branches would run every case on every wave
__device__ __forceinline__ float tes_value(uint4 a, uint4 b, int col) {
  const bool black = (b.z >> 10) & 1u;
  const float player = (col == 196) != black ? 1.0f : 0.0f;
  const int side = col >= 98 ? 1 : 0;
  const int cc = col - 98 * side;
  const float offv = (float)(side ? ((b.z >> 4) & 15u) : (b.z & 15u)) / 15.0f;
  const int pt = cc < 96 ? (cc >> 2) : 0;
  const uint32_t w0 = side ? a.z : a.x, w1 = side ? a.w : a.y, w2 = side ? b.y : b.x;
  const int k = pt >> 3;
  const uint32_t word = k == 0 ? w0 : (k == 1 ? w1 : w2);
  const uint32_t v = (word >> (4 * (pt & 7))) & 15u;
  const int j = cc & 3;
  const float thr = v >= (uint32_t)(j + 1) ? 1.0f : 0.0f;  // j = 0, 1, 2: v >= 1, 2, 3
  const float over = v >= 3u ? (float)(v - 3u) / 2.0f : 0.0f;
  const float board = j == 3 ? over : thr;
  const float pv = cc == 96 ? 0.0f : (cc == 97 ? offv : board);
  return col >= 196 ? player : pv;
}

// The 198-float observation, a wave per 16 envs: lane l computes a quarter
// of env (l & 15)'s row -- quarter q = l >> 4: white points 0-11 (columns
// 0-47), white points 12-23 + bar + off (48-97), black points 0-11
// (98-145), black points 12-23 + bar + off + player one-hot (146-197) --
// from the record's nibbles with one bit-field extract per point (v, then
// the four floats [v >= 1, v >= 2, v >= 3, (v - 3) / 2 if v >= 3]: the
// values of tes_value, bit for bit), stages it in LDS, and the wave stores
// its 16 contiguous rows (12,672 B) as 1-KiB pieces.  Layout (README.md:42-102,
// absolute points): [white 24 x 4, bar, off, black 24 x 4, bar, off, player
// one-hot].  (Round 3's kernel -- one thread per 4 output floats, each float
// evaluated generically by tes_value, ~25 VALU per float -- was issue-bound:
// 19.3 us for 54 MB.)
constexpr int kTesEnvs = 16;                       // envs per wave
constexpr int kTesRowB = 198 * 4;                  // bytes per row
constexpr int kTesWaveB = kTesEnvs * kTesRowB;     // 12,672 B per wave
static_assert(kTesWaveB % 16 == 0, "16-B pieces");

__device__ __forceinline__ void tes_point4(uint32_t v, float* f) {
  f[0] = v >= 1u ? 1.0f : 0.0f;
  f[1] = v >= 2u ? 1.0f : 0.0f;
  f[2] = v >= 3u ? 1.0f : 0.0f;
  f[3] = v >= 3u ? (float)(v - 3u) / 2.0f : 0.0f;
}

// the wave's 16 rows (envs e0 .. e0 + 15, those below n) into wave_rows
// (LDS, 16 x 198 floats); the caller hands them over with wave_lds_handoff
__device__ __forceinline__ void tes_stage_rows(const Planes& pl, int n, int e0, float* wave_rows) {
  const int lane = threadIdx.x & 63;
  const int le = lane & 15, q = lane >> 4;
  const int i = e0 + le;
  float* row = wave_rows + le * 198;
  if (i < n) {
    const uint4 a = pl.p0[i], b = pl.p1[i];
    const int side = q >> 1, upper = q & 1;
    const uint32_t w0 = side ? a.z : a.x, w1 = side ? a.w : a.y, w2 = side ? b.y : b.x;
    // points 12q' .. 12q' + 11 of the side: 8 nibbles in X, 4 in Y
    const uint32_t X = upper ? ((w1 >> 16) | (w2 << 16)) : w0;
    const uint32_t Y = upper ? (w2 >> 16) : (w1 & 0xFFFFu);
    float f[52];
#pragma unroll
    for (int k = 0; k < 8; ++k) tes_point4(__builtin_amdgcn_ubfe(X, 4u * k, 4u), f + 4 * k);
#pragma unroll
    for (int k = 0; k < 4; ++k) tes_point4(__builtin_amdgcn_ubfe(Y, 4u * k, 4u), f + 32 + 4 * k);
    const uint32_t misc = b.z;
    const float offv = (float)(side ? ((misc >> 4) & 15u) : (misc & 15u)) / 15.0f;
    const bool black = (misc >> 10) & 1u;
    f[48] = 0.0f;   // bar (always empty in Narde)
    f[49] = offv;
    f[50] = black ? 0.0f : 1.0f;  // player one-hot (quarter 3 only)
    f[51] = black ? 1.0f : 0.0f;
    // columns of the quarter: 0, 48, 98, 146 (8-B aligned: ds_write_b64)
    const int c0 = q == 0 ? 0 : (q == 1 ? 48 : (q == 2 ? 98 : 146));
    const int nf = q == 0 || q == 2 ? 48 : (q == 1 ? 50 : 52);
#pragma unroll
    for (int k = 0; k < 26; ++k)
      if (2 * k < nf) *reinterpret_cast<float2*>(row + c0 + 2 * k) = make_float2(f[2 * k], f[2 * k + 1]);
  }
}

__global__ void __launch_bounds__(kBlock) k_tesauro198_rows(Planes pl, int n, float* __restrict__ tes) {
  __shared__ __attribute__((aligned(16))) float rows[kBlock / 64][kTesEnvs * 198];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e0 = (blockIdx.x * (kBlock / 64) + wave) * kTesEnvs;  // first env of the wave
  tes_stage_rows(pl, n, e0, rows[wave]);
  wave_lds_handoff();  // the wave reads only its own rows
  // the wave's rows: [e0, min(e0 + 16, n)) -> 16-B pieces, lane-major
  const int rows_here = max(0, min(kTesEnvs, n - e0));
  const uint32_t bytes = (uint32_t)rows_here * kTesRowB;
  const float4* src = reinterpret_cast<const float4*>(rows[wave]);
  float4* dst = reinterpret_cast<float4*>(tes + (size_t)e0 * 198);
  for (uint32_t k = (uint32_t)lane; 16u * k < bytes; k += 64u) {
    if (16u * k + 16u <= bytes) {
      dst[k] = src[k];
    } else {  // the row set ends inside this piece (an odd number of rows): its 8-B half
      *reinterpret_cast<float2*>(reinterpret_cast<float*>(dst + k)) = *reinterpret_cast<const float2*>(src + k);
    }
  }
}

// The reward shaping of train_deepq_pytorch.py:892-912 for one env: the
// trainer reads env.unwrapped.current_player AFTER the step and that
// player's borne-off count: +1 per checker newly borne off since its
// tracker and +0.1 x the count.  With auto-reset the record already holds
// the next game at a step that ends one, so the player and count come from
// the pre-step misc word there: a terminal step names the mover (the winner,
// 15 off, the player is not flipped), a truncated one the other player (the
// mover's checkers cannot change its count).  No legal move (list #1
// empty): no shaping, as the reference skips it (:869-873).  The trackers
// restart at 0 with a new episode.  Same fp32 ops as the torch restatement
// (BatchedDQNDriver._transition_torch).
__device__ __forceinline__ void trans_scalars(const TransArgs& t, int i, int64_t slot, int64_t nslot,
                                              uint4 b) {
  const bool term = t.term[i] != 0, trunc = t.trunc[i] != 0;
  const float done = (term || trunc) ? 1.0f : 0.0f;
  const uint32_t post = b.z;
  float r = (float)t.reward[i];
  if (t.shaping) {
    const uint32_t pre = (uint32_t)t.misc[i];
    const bool moved = !t.legal || (t.legal[i] & 0xFFFFFFFFFFFFull) != 0ull;
    const uint32_t pre_black = (pre >> 10) & 1u;
    const int black = (int)(term ? pre_black : (trunc ? (pre_black ^ 1u) : ((post >> 10) & 1u)));
    const uint32_t src = (term || trunc) ? pre : post;
    const float now = term ? 15.0f : (float)(black ? ((src >> 4) & 15u) : (src & 15u));
    const float before = t.off_seen[2 * i + black];
    if (moved) {
#pragma clang fp contract(off)  // torch rounds the product and the sum separately: no FMA
      r = (r + fmaxf(now - before, 0.0f)) + 0.1f * now;
    }
    const float keep = 1.0f - done;
    const float o0 = (moved && !black) ? now : t.off_seen[2 * i];
    const float o1 = (moved && black) ? now : t.off_seen[2 * i + 1];
    t.off_seen[2 * i] = o0 * keep;
    t.off_seen[2 * i + 1] = o1 * keep;
  }
  t.misc[i] = (int32_t)(post & 0x4FFu);  // off_w | off_b << 4 | black_to_move << 10
  t.r_action[2 * slot] = t.actions[2 * i];
  t.r_action[2 * slot + 1] = t.actions[2 * i + 1];
  t.r_reward[slot] = r;
  t.r_done[slot] = done;
  t.r_prio[slot] = *t.max_prio;
  t.r_prio[nslot] = 0.0f;
}

// Two kinds of block in one launch.  Blocks below obs_blocks: each thread
// owns 4 consecutive floats of the flat (n, 198) arrays, so s' goes out 16 B
// per lane (1 KiB per wave instruction; the ring row is written once and
// read only when sampled: non-temporal) when this step's s' rows
// (pos + n .. pos + 2n - 1) % capacity are contiguous and 16-B aligned (the
// steady state when the capacity is a multiple of n); otherwise each float
// goes on its own.  The blocks after them: one thread per env for the
// replay row's scalars and the shaping trackers, so those narrow arrays are
// written coalesced (a thread per env, not the one thread of each 198-float
// row that owns its column 0: those writes were scattered over partial
// lines).
__global__ void __launch_bounds__(kBlock) k_dqn_transition(TransArgs t, int obs_blocks) {
  const int64_t pos = *t.pos;  // pos < capacity, capacity >= 2n: one wrap at most
  int64_t q0 = pos + t.n;
  if (q0 >= t.capacity) q0 -= t.capacity;
  if ((int)blockIdx.x >= obs_blocks) {
    const int i = ((int)blockIdx.x - obs_blocks) * kBlock + (int)threadIdx.x;
    if (i >= t.n) return;
    int64_t slot = pos + i;
    if (slot >= t.capacity) slot -= t.capacity;
    int64_t nslot = q0 + i;
    if (nslot >= t.capacity) nslot -= t.capacity;
    trans_scalars(t, i, slot, nslot, t.pl.p1[i]);
    return;
  }
  // s' of the wave's 16 envs, staged once in LDS (tes_stage_rows, as
  // k_tesauro198_rows), then stored twice: the state rows (contiguous) and
  // the ring rows (q0 + e0 + r) % capacity, non-temporally (read only when
  // sampled) -- 8-byte pieces, as a ring row starts 8-byte aligned
  __shared__ __attribute__((aligned(16))) float rows[kBlock / 64][kTesEnvs * 198];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e0 = (blockIdx.x * (kBlock / 64) + wave) * kTesEnvs;
  tes_stage_rows(t.pl, t.n, e0, rows[wave]);
  wave_lds_handoff();
  const int rows_here = max(0, min(kTesEnvs, t.n - e0));
  const uint32_t bytes = (uint32_t)rows_here * kTesRowB;
  const float4* src = reinterpret_cast<const float4*>(rows[wave]);
  float4* dst = reinterpret_cast<float4*>(t.state + (size_t)e0 * 198);
  for (uint32_t k = (uint32_t)lane; 16u * k < bytes; k += 64u) {
    if (16u * k + 16u <= bytes) {
      dst[k] = src[k];
    } else {
      *reinterpret_cast<float2*>(reinterpret_cast<float*>(dst + k)) = *reinterpret_cast<const float2*>(src + k);
    }
  }
  int64_t r0 = q0 + e0;
  if (r0 >= t.capacity) r0 -= t.capacity;
  const float2* src2 = reinterpret_cast<const float2*>(rows[wave]);
  typedef float v2f __attribute__((ext_vector_type(2)));
  if (r0 + rows_here <= t.capacity) {  // no wrap inside the wave's rows: one run
    v2f* d2 = reinterpret_cast<v2f*>(t.r_obs + (size_t)r0 * 198);
    for (uint32_t k = (uint32_t)lane; 8u * k < bytes; k += 64u) {
      const float2 v = src2[k];
      const v2f x = {v.x, v.y};
      __builtin_nontemporal_store(x, d2 + k);
    }
  } else {  // the ring wraps inside them: row by row
    for (int r = 0; r < rows_here; ++r) {
      int64_t rr = r0 + r;
      if (rr >= t.capacity) rr -= t.capacity;
      v2f* d2 = reinterpret_cast<v2f*>(t.r_obs + (size_t)rr * 198);
      for (int k = lane; k < 99; k += 64) {
        const float2 v = src2[r * 99 + k];
        const v2f x = {v.x, v.y};
        __builtin_nontemporal_store(x, d2 + k);
      }
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_mask576(Planes pl, int n, Rng g,
                                                    uint64_t* __restrict__ mask) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Side s = side_from_record(pl.p0[i], pl.p1[i]);
  uint32_t r[4];
  ply_draw(g, s.t, (uint32_t)i, r);
  int d0, d1;
  dice_from(r[0], g.dice_mode, d0, d1);
  Legal l;
  legal2(s, d0, d1, l);
  uint64_t m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < l.n; ++k) {
    uint32_t b = l.L[k];
    while (b) {
      const int f = __builtin_ctz(b);
      b &= b - 1u;
      const int to = f - l.d[k] < 0 ? OFF : f - l.d[k];
      if (to == 0 && f <= 5) continue;  // (f, 0) cannot be requested by a code
      const int c = encode_move(f, to);
      m[c >> 6] |= 1ull << (c & 63);
    }
  }
  for (int q = 0; q < 9; ++q) mask[(size_t)i * 9 + q] = m[q];
}

// move-2 acceptance mask given each env's move-1 code, for the next step's
// device dice: what NardeEnv.step would accept as move2 after move1
// (narde_env.py:56-93: move1 must be in list #1 with >= 2 entries; the die
// bookkeeping picks the second die; list #2 = get_valid_moves([die]) on the
// post-move1 board; the decode quirk makes (f, 0), f <= 5, unrequestable).
// All zero when move1 would not be played.
__global__ void __launch_bounds__(kBlock) k_mask576_move2(Planes pl, int n, Rng g,
                                                          const int16_t* __restrict__ move1,
                                                          const uint8_t* __restrict__ dice,
                                                          uint64_t* __restrict__ mask) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Side s = side_from_record(pl.p0[i], pl.p1[i]);
  int d0, d1;
  if (dice) {
    d0 = dice[2 * i];
    d1 = dice[2 * i + 1];
  } else {
    uint32_t r[4];
    ply_draw(g, s.t, (uint32_t)i, r);
    dice_from(r[0], g.dice_mode, d0, d1);
  }
  // a given die outside 1..6: no legal move, nothing is accepted
  const bool bad = (uint32_t)(d0 - 1) > 5u || (uint32_t)(d1 - 1) > 5u;
  if (bad) d0 = d1 = 1;
  Legal l;
  legal2(s, d0, d1, l);
  uint64_t m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int f1, t1;
  decode_action(move1[i], f1, t1);
  if (!bad && l.count >= 2 && legal_contains(l, f1, t1)) {
    apply_move(s, f1, t1);
    const int dist = t1 == OFF ? f1 + 1 : (f1 > t1 ? f1 - t1 : t1 - f1);
    const int rem = (d0 == dist) ? d1 : ((d1 == dist) ? d0 : d1);
    uint32_t L2 = die_filter(s.O, s.S1o, block_info(s.O, s.P), die_candidates(s.O, s.P, rem), rem);
    while (L2) {
      const int f = __builtin_ctz(L2);
      L2 &= L2 - 1u;
      const int to = f - rem < 0 ? OFF : f - rem;
      if (to == 0 && f <= 5) continue;  // (f, 0) cannot be requested by a code
      const int c = encode_move(f, to);
      m[c >> 6] |= 1ull << (c & 63);
    }
  }
  for (int q = 0; q < 9; ++q) mask[(size_t)i * 9 + q] = m[q];
}

// Masked epsilon-greedy over the 576 action codes for a Q-value row per env
// (the policy half of train_deepq_pytorch.py:411-600, batched): one wave per
// row, lane l reads codes l + 64 j (coalesced), the legal ones are compared
// and a wave reduction keeps the largest value, lowest code on ties
// (torch.argmax's first maximum).  With probability epsilon the code is
// uniform over the legal ones instead; 0 where none is legal (the
// reference's "no move" code, :504-505).  Draws: Philox4x32-10({tag, row, 0,
// 5}, seed): r0 < epsilon * 2^32 explores, one shared decision for both
// heads of a step (same tag); the pick is mulhi(r1 or r2 by head, count).
// a move-1 code used as an index (the one-hot column / table row), kept in
// [0, 576) whatever the caller's buffer holds
__device__ __forceinline__ int64_t clamp_code(int64_t c) { return c < 0 ? 0 : (c > 575 ? 575 : c); }

// torch.argmax's order for (value, code) candidates: a NaN beats every
// number (the lowest code among NaNs), else the larger value, the lower
// code on ties; oi < 0 is "no candidate"
__device__ __forceinline__ bool argmax_takes(float ov, int oi, float best, int bi) {
  if (oi < 0) return false;
  if (bi < 0) return true;
  const bool on = __builtin_isnan(ov), bn = __builtin_isnan(best);
  if (on || bn) return on && (!bn || oi < bi);
  return ov > best || (ov == best && oi < bi);
}

__host__ __device__ inline uint64_t eps_to_q32(float epsilon) {
  const double e = epsilon <= 0.0f ? 0.0 : (epsilon >= 1.0f ? 1.0 : (double)epsilon);
  return (uint64_t)(e * 4294967296.0);
}

// the roll of env i for the play-set kernels: given (roll order) or the
// next step's device dice; false for a given die outside 1..6 (no play)
__device__ __forceinline__ bool play_dice(const Side& s, const Rng& g, int i, const uint8_t* __restrict__ dice,
                                          int& d0, int& d1) {
  if (dice) {
    d0 = dice[2 * i];
    d1 = dice[2 * i + 1];
  } else {
    uint32_t r[4];
    ply_draw(g, s.t, (uint32_t)i, r);
    dice_from(r[0], g.dice_mode, d0, d1);
  }
  return (uint32_t)(d0 - 1) <= 5u && (uint32_t)(d1 - 1) <= 5u;
}

// The play set per env (narde_rules.h play_walk): list #1 compact, the word
// of every list-#1 entry at table[i][k][p] (k = 0 the higher die's list, 1
// the lower's; 0 where (k, p) is no entry) and the play count.  One lane
// per env; the 192-B table row is zeroed, then the entries written.
__global__ void __launch_bounds__(kBlock) k_play_set(Planes pl, int n, Rng g, const uint8_t* __restrict__ dice,
                                                     int kind, uint64_t* __restrict__ legal,
                                                     uint32_t* __restrict__ table, int32_t* __restrict__ count) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Side s = side_from_record(pl.p0[i], pl.p1[i]);
  uint32_t* row = table + (size_t)i * 48;
  uint4* row4 = reinterpret_cast<uint4*>(row);
#pragma unroll
  for (int q = 0; q < 12; ++q) row4[q] = make_uint4(0u, 0u, 0u, 0u);
  int d0, d1;
  if (!play_dice(s, g, i, dice, d0, d1)) {
    if (legal) legal[i] = 0ull;
    count[i] = 0;
    return;
  }
  Legal l;
  legal2(s, d0, d1, l);
  if (legal) legal[i] = compact_legal(l);
  count[i] = play_walk(s, d0, d1, kind, l, [&](int k, int p, int, uint32_t w, bool) { row[k * 24 + p] = w; });
}

// act()'s greedy candidate masks per env (narde_rules.h act_masks): move1
// NULL -- the move-1 codes of list #1; else the move-2 codes act() offers
// after each env's move1[i] (pre-move lists).  u64[n][9].
__global__ void __launch_bounds__(kBlock) k_act_masks(Planes pl, int n, Rng g, const uint8_t* __restrict__ dice,
                                                      const int64_t* __restrict__ move1, int64_t ld_move1,
                                                      uint64_t* __restrict__ mask) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Side s = side_from_record(pl.p0[i], pl.p1[i]);
  uint64_t m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int d0, d1;
  if (play_dice(s, g, i, dice, d0, d1)) {
    Legal l;
    legal2(s, d0, d1, l);
    const int64_t c = move1 ? move1[(size_t)i * (size_t)ld_move1] : -1;
    act_masks(s, d0, d1, l, c < 0 ? -1 : (c > 575 ? 576 : (int)c), m);
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) mask[(size_t)i * 9 + q] = m[q];
}

// The batched driver's exploration (train_deepq_pytorch.py:514-515:
// np.random.rand() <= epsilon, then random.choice(valid_move_combinations)):
// the rows whose shared explore draw (Philox4x32-10({tag, row, 0, 5}, seed)
// r0 < epsilon * 2^32, the policy kernels' decision) takes the ε-branch
// get play mulhi(r1, count) of act()'s combination list -- uniform over
// (move 1, move 2) combinations, duplicates included -- as the two codes of
// their (B, 2) action row; other rows are left as the heads wrote them.  A
// row with no play keeps the heads' 0.
__global__ void __launch_bounds__(kBlock) k_explore_plays(Planes pl, int n, Rng g,
                                                          const uint8_t* __restrict__ dice,
                                                          const float* __restrict__ eps_p,
                                                          const int64_t* __restrict__ tag_p, uint32_t k0,
                                                          uint32_t k1, int64_t* __restrict__ out, int64_t ld_out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t r[4];
  philox4x32_10((uint32_t)*tag_p, (uint32_t)i, 0u, 5u, k0, k1, r);
  if (!((uint64_t)r[0] < eps_to_q32(*eps_p))) return;
  const Side s = side_from_record(pl.p0[i], pl.p1[i]);
  int d0, d1;
  if (!play_dice(s, g, i, dice, d0, d1)) return;
  Legal l;
  legal2(s, d0, d1, l);
  const int cnt = play_walk(s, d0, d1, kPlayAct, l, [](int, int, int, uint32_t, bool) {});
  if (cnt == 0) return;
  int c1, c2;
  play_codes_act(s, d0, d1, l, (int)mulhi_u32(r[1], (uint32_t)cnt), c1, c2);
  out[(size_t)i * (size_t)ld_out] = c1;
  out[(size_t)i * (size_t)ld_out + 1] = c2;
}

// k_head_policy576: k_policy576 with the head's Q-values computed in the
// kernel, only for the legal codes: q_c = sum_k f[k] W[c][k] + b[c]
// (+ addcol[c * ld_w + add_row[row]]: the move-2 head's one-hot column), the
// masked argmax over them (the first maximum in code order, as
// torch.argmax).  One wave per env: lane l holds f[4l .. 4l + 3] (F = 256),
// each legal code costs one coalesced 1-KiB row of W (L2-resident: 576 rows)
// and a 64-lane sum in a fixed tree order.  The dense head GEMM computes all
// 576 codes of every env (2 x 65536 x 256 x 576 flop per head); an env has
// ~6-30 legal codes.  The sums round differently from hipBLASLt's, so a
// greedy pick can differ from the dense one only between codes whose
// Q-values tie to fp32 rounding (tests/test_gpu_dqn.py checks the gap).
// Exploration is k_policy576's, draw for draw.
constexpr int kHeadF = 256;
__global__ void __launch_bounds__(256) k_head_policy576(const float* __restrict__ f, int64_t ldf,
                                                        const float* __restrict__ w, int64_t ldw,
                                                        const float* __restrict__ bias,
                                                        const uint64_t* __restrict__ mask, int n, uint32_t k0,
                                                        uint32_t k1, int head, int64_t* __restrict__ out,
                                                        int64_t ld_out, int16_t* __restrict__ out16,
                                                        int64_t ld_out16, const float* __restrict__ eps_p,
                                                        const int64_t* __restrict__ tag_p,
                                                        const float* __restrict__ addcol,
                                                        const int64_t* __restrict__ add_row, int64_t ld_row) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (row >= n) return;  // whole waves: the row is uniform over the wave
  const uint64_t eps_q32 = eps_to_q32(*eps_p);
  const uint32_t tag = (uint32_t)*tag_p;
  uint64_t mw[9];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    mw[j] = mask[(size_t)row * 9 + j];
    cnt += __builtin_popcountll(mw[j]);
  }
  uint32_t r[4];
  philox4x32_10(tag, (uint32_t)row, 0u, 5u, k0, k1, r);
  const bool explore = (uint64_t)r[0] < eps_q32;
  int code = 0;
  if (cnt > 0 && explore) {
    int k = (int)mulhi_u32(head ? r[2] : r[1], (uint32_t)cnt);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int c = __builtin_popcountll(mw[j]);
      if (k >= 0 && k < c) {
        uint64_t m = mw[j];
        for (int t = 0; t < k; ++t) m &= m - 1ull;
        code = 64 * j + __builtin_ctzll(m);
      }
      k -= c;
    }
  } else if (cnt > 0) {
    const float4 fv = reinterpret_cast<const float4*>(f + (size_t)row * (size_t)ldf)[lane];
    // the one-hot column's index is a move-1 code: kept inside [0, 576)
    const int64_t ar = addcol ? clamp_code(add_row[(size_t)row * (size_t)ld_row]) : 0;
    float best = 0.0f;
    int bi = -1;  // cnt > 0: the first legal code always takes it
    for (int j = 0; j < 9; ++j) {
      uint64_t m = mw[j];
      while (m) {  // the legal codes of this word, ascending (wave-uniform)
        const int c = 64 * j + __builtin_ctzll(m);
        m &= m - 1ull;
        const float4 wv = reinterpret_cast<const float4*>(w + (size_t)c * (size_t)ldw)[lane];
        float v = fmaf(fv.w, wv.w, fmaf(fv.z, wv.z, fmaf(fv.y, wv.y, fv.x * wv.x)));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        v += bias[c];
        if (addcol) v += addcol[(size_t)c * (size_t)ldw + ar];
        // ascending codes: the first maximum is kept, a NaN beats every
        // number and the first NaN is kept (torch.argmax's rule)
        if (bi < 0 || v > best || (__builtin_isnan(v) && !__builtin_isnan(best))) { best = v; bi = c; }
      }
    }
    code = bi;
  }
  if (lane == 0) {  // strided: straight into a column of the (B, 2) action rows
    out[(size_t)row * (size_t)ld_out] = code;
    if (out16) out16[(size_t)row * (size_t)ld_out16] = (int16_t)code;
  }
}

__global__ void __launch_bounds__(256) k_policy576(const float* __restrict__ q, int64_t ldq,
                                                   const uint64_t* __restrict__ mask, int n,
                                                   uint64_t eps_q32, uint32_t k0, uint32_t k1,
                                                   uint32_t tag, int head, int64_t* __restrict__ out,
                                                   const float* __restrict__ eps_p,
                                                   const int64_t* __restrict__ tag_p,
                                                   const float* __restrict__ add_tab, int64_t ld_add,
                                                   const int64_t* __restrict__ add_row) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (row >= n) return;  // whole waves: the row is uniform over the wave
  if (eps_p) eps_q32 = eps_to_q32(*eps_p);  // device-resident epsilon / tag (graph replays)
  if (tag_p) tag = (uint32_t)*tag_p;
  uint64_t mw[9];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    mw[j] = mask[(size_t)row * 9 + j];
    cnt += __builtin_popcountll(mw[j]);
  }
  uint32_t r[4];
  philox4x32_10(tag, (uint32_t)row, 0u, 5u, k0, k1, r);
  const bool explore = (uint64_t)r[0] < eps_q32;
  int code = 0;
  if (cnt > 0 && explore) {
    int k = (int)mulhi_u32(head ? r[2] : r[1], (uint32_t)cnt);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int c = __builtin_popcountll(mw[j]);
      if (k >= 0 && k < c) {
        uint64_t m = mw[j];
        for (int t = 0; t < k; ++t) m &= m - 1ull;
        code = 64 * j + __builtin_ctzll(m);
      }
      k -= c;
    }
  } else if (cnt > 0) {
    const float* qr = q + (size_t)row * (size_t)ldq;
    // optional addend row (the move-2 head's one-hot column, DecomposedDQN):
    // v = q[row][c] + add_tab[add_row[row]][c], the same single fp32 add
    // (the table has one row per move-1 code: the row index kept in [0, 576))
    const float* ar = add_tab ? add_tab + (size_t)clamp_code(add_row[row]) * (size_t)ld_add : nullptr;
    float best = 0.0f;
    int bi = -1;  // -1: no legal code in this lane
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      if ((mw[j] >> lane) & 1ull) {
        const float v = ar ? qr[64 * j + lane] + ar[64 * j + lane] : qr[64 * j + lane];
        // j ascending: the first maximum kept; a NaN beats every number
        if (bi < 0 || v > best || (__builtin_isnan(v) && !__builtin_isnan(best))) { best = v; bi = 64 * j + lane; }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (argmax_takes(ov, oi, best, bi)) { best = ov; bi = oi; }
    }
    code = bi;  // cnt > 0: some lane held a legal code
  }
  if (lane == 0) out[row] = code;
}

}  // namespace
