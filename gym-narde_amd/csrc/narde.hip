// narde.hip -- HIP kernels (gfx950) + the C ABI of libnarde (include/narde.h).
//
// One lane = one env.  Each env is a 32-byte record split into two planar
// 16-byte planes (narde_rules.h), so every wave-wide load/store of state is
// a single contiguous 1 KiB transaction.  The rules engine is branch-light
// bitmask arithmetic on 24-bit point masks held in VGPRs; nothing is staged
// through LDS because no data is shared between lanes (envs are independent).
//
// Kernels
//   k_step      NardeEnv.step for B envs (API step and the self-play ply):
//               Philox dice, list #1, policy or given actions, apply, list #2,
//               apply, end check, flip, TimeLimit, auto-reset, outputs.
//   k_rollout   the same step looped over K plies with the record in VGPRs,
//               streaming each ply's outputs to [ply][B] rollout buffers.
//   k_legal     Narde.get_valid_moves with 1..4 dice, expanded or compact.
//   k_reset / k_set_state / k_get_state / k_apply / k_observe / k_mask576 /
//   k_block / k_peek_dice   state management and the rest of the ABI.
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

constexpr int kBlock = 256;
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

struct Planes {
  uint4* p0;
  uint4* p1;
  int4* stats;
};

struct Rng {
  uint32_t env0, k0, k1;
  int dice_mode;
};

__device__ __forceinline__ void draw(const Rng& g, uint32_t t, uint32_t i, uint32_t stream,
                                     uint32_t r[4]) {
  philox4x32_10(t, g.env0 + i, 0u, stream, g.k0, g.k1, r);
}

// the four words of ply t of env i (narde_rules.h ply_words: one Philox
// block per two plies; a kernel that runs consecutive plies keeps the block)
__device__ __forceinline__ void ply_draw(const Rng& g, uint32_t t, uint32_t i, uint32_t r[4]) {
  uint32_t R[4];
  ply_block(t, g.env0 + i, g.k0, g.k1, R);
  ply_words_of(R, t, g.dice_mode, r);
}

// ------------------------------------------------------------------ kernels
// init_t >= 0: also set the RNG counter (create); < 0: keep each env's counter
__global__ void __launch_bounds__(kBlock) k_reset(Planes pl, int n, Rng g, uint32_t epoch,
                                                  const uint8_t* __restrict__ mask, int64_t init_t) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
  uint32_t r[4];
  draw(g, epoch, (uint32_t)i, 1u, r);
  Side s = side_reset(r[0]);
  s.t = init_t >= 0 ? (uint32_t)init_t : pl.p1[i].w;
  uint4 a, b;
  side_to_record(s, a, b);
  pl.p0[i] = a;
  pl.p1[i] = b;
  pl.stats[i] = make_int4(0, 0, 0, 0);
}

// keep_t: preserve each env's RNG counter (device state); else set it to 0
__global__ void __launch_bounds__(kBlock) k_set_state(Planes pl, int n, const int8_t* __restrict__ board,
                                                      const uint8_t* __restrict__ off,
                                                      const uint8_t* __restrict__ ft,
                                                      const int8_t* __restrict__ player,
                                                      const uint16_t* __restrict__ elapsed, int keep_t) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t t = keep_t ? pl.p1[i].w : 0u;
  uint4 a, b;
  record_from_board(board + (size_t)i * 24, off[2 * i], off[2 * i + 1], ft[2 * i], ft[2 * i + 1],
                    player[i], elapsed ? elapsed[i] : 0u, t, a, b);
  pl.p0[i] = a;
  pl.p1[i] = b;
}

__global__ void __launch_bounds__(kBlock) k_get_state(Planes pl, int n, int8_t* __restrict__ board,
                                                      uint8_t* __restrict__ off, uint8_t* __restrict__ ft,
                                                      int8_t* __restrict__ player,
                                                      uint16_t* __restrict__ elapsed) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  board_from_record(pl.p0[i], pl.p1[i], board ? board + (size_t)i * 24 : nullptr,
                    off ? off + 2 * i : nullptr, ft ? ft + 2 * i : nullptr,
                    player ? player + i : nullptr, elapsed ? elapsed + i : nullptr);
}

__global__ void __launch_bounds__(kBlock) k_set_ply(Planes pl, int n, uint32_t t) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  pl.p1[i].w = t;
}

__global__ void __launch_bounds__(kBlock) k_peek_dice(Planes pl, int n, Rng g, uint8_t* __restrict__ dice) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t r[4];
  ply_draw(g, pl.p1[i].w, (uint32_t)i, r);
  int d0, d1;
  dice_from(r[0], g.dice_mode, d0, d1);
  dice[2 * i] = (uint8_t)d0;
  dice[2 * i + 1] = (uint8_t)d1;
}

__device__ __forceinline__ uint64_t compact_legal(const Legal& l) {
  return (uint64_t)l.L[0] | ((uint64_t)l.L[1] << 24) | ((uint64_t)l.d[0] << 48) |
         ((uint64_t)l.d[1] << 52);
}

__global__ void __launch_bounds__(kBlock) k_legal(Planes pl, int n, Rng g,
                                                  const uint8_t* __restrict__ dice4,
                                                  int16_t* __restrict__ out_count,
                                                  int8_t* __restrict__ out_moves,
                                                  uint64_t* __restrict__ out_compact) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Side s = side_from_record(pl.p0[i], pl.p1[i]);
  Legal l;
  if (dice4) {
    legal_roll(s, dice4 + 4 * i, l);
  } else {
    uint32_t r[4];
    ply_draw(g, s.t, (uint32_t)i, r);
    int d0, d1;
    dice_from(r[0], g.dice_mode, d0, d1);
    legal2(s, d0, d1, l);
  }
  const int nd = l.n;
  out_count[i] = (int16_t)l.count;
  if (out_compact) out_compact[i] = nd <= 2 ? compact_legal(l) : 0ull;
  if (out_moves) {
    int4* row = reinterpret_cast<int4*>(out_moves + (size_t)i * NARDE_MAX_MOVES * 2);
    const int4 neg = make_int4(-1, -1, -1, -1);
#pragma unroll
    for (int q = 0; q < 8; ++q) row[q] = neg;
    int e = 0;
    uint16_t* pairs = reinterpret_cast<uint16_t*>(out_moves + (size_t)i * NARDE_MAX_MOVES * 2);
    for (int k = 0; k < nd; ++k) {
      uint32_t m = l.L[k];
      while (m) {
        const int f = __builtin_ctz(m);
        m &= m - 1u;
        const int to = f - l.d[k] < 0 ? OFF : f - l.d[k];
        pairs[e++] = (uint16_t)((uint32_t)f | ((uint32_t)to << 8));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Wave-cooperative FULL4 turn (device only).
//
// Same rule and result as env_turn_full (narde_rules.h, which the host check
// runs; the GPU parity tests hold this one to the oracle), organised for
// SIMT.  The expensive part of a turn is per source: "after this first
// sub-move, can the other die still move" (two dice) and "after this
// sub-move, are M-k-1 more still playable" (doubles, a depth-first search).
// Run per lane, a wave loops as long as its busiest lane while the others
// idle: on a typical ply ~10 of the 64 lanes roll doubles, and the rest wait.
// Here every lane publishes its (lane, source) checks; a wave prefix sum of
// the per-lane counts places them in one task list in LDS, and all 64 lanes
// take tasks 64 at a time (the owner's state is read back from LDS, results
// are OR-ed into the owner's mask with ds_or).  Every call is made with the
// whole wave converged: the turn below is straight-line code with per-lane
// masks instead of rule branches around the calls.
struct CoopLds {
  uint4 snap[64][2];          // owner state: {own w0..w2, O}, {S1, P, low, params}
  uint32_t task[64 * 32];     // (lane << 8) | (which << 7) | source; 2 masks x <= 15 sources
  uint32_t res[64][3];
};

// exclusive prefix sum of x (0 <= x < 64) over the wave, and the total, from
// one ballot per bit of x: lane l's prefix adds 2^b for every lower lane with
// bit b set (v_mbcnt counts them) -- no LDS round trips, unlike shuffles
__device__ __forceinline__ int wave_prefix(int x, int lane, int& total) {
  (void)lane;
  int excl = 0;
  total = 0;
#pragma unroll
  for (int b = 0; b < 6; ++b) {
    const uint64_t m = __ballot((x >> b) & 1);
    excl += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    total += __builtin_popcountll(m) << b;
  }
  return excl;
}

// One cooperative pass over every lane's per-source checks.  Per lane:
//   mode 1 (pair, two dice a = d_hi, b = d_lo): m0 = first moves with a,
//     kept (res 0) iff b still has a move after them; m1 = first moves with
//     b, kept (res 1) iff a still does.
//   mode 0 (depth, doubles a): m0 = sources; res j gets the sources after
//     which at least j + 1 more sub-moves are playable (searched up to
//     `need`; block-free lanes try the chain bound first).
__device__ void coop_run(CoopLds& W, const Side& s, uint32_t low, int a, int b, int hl, uint32_t m0,
                         uint32_t m1, int need, bool bf, int mode, int lane, uint32_t out[3]) {
  out[0] = out[1] = out[2] = 0u;
  if (__ballot((m0 | m1) != 0u) == 0ull) return;  // wave-uniform: nothing to check
  const int c0 = __builtin_popcount(m0), cnt = c0 + __builtin_popcount(m1);
  int total;
  const int off = wave_prefix(cnt, lane, total);
  W.res[lane][0] = W.res[lane][1] = W.res[lane][2] = 0u;
  if (cnt) {
    W.snap[lane][0] = make_uint4(s.own.w[0], s.own.w[1], s.own.w[2], s.O);
    W.snap[lane][1] = make_uint4(s.S1o, s.P, low,
                                 (uint32_t)a | ((uint32_t)b << 4) | ((uint32_t)(hl + 1) << 8) |
                                     ((uint32_t)need << 12) | ((uint32_t)bf << 16) |
                                     ((uint32_t)mode << 17) | (s.off_own << 20));
    int k = off;
    for (int which = 0; which < 2; ++which) {
      uint32_t m = which ? m1 : m0;
      while (m) {
        const int p = __builtin_ctz(m);
        m &= m - 1u;
        W.task[k++] = ((uint32_t)lane << 8) | ((uint32_t)which << 7) | (uint32_t)p;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();  // a wave's LDS operations retire in issue order
  for (int base = 0; base < total; base += 64) {
    const int t = base + lane;
    if (t < total) {
      const uint32_t tk = W.task[t];
      const int ow = (int)(tk >> 8), which = (int)((tk >> 7) & 1u), p = (int)(tk & 0x7Fu);
      const uint4 x = W.snap[ow][0], y = W.snap[ow][1];
      Side c;
      c.own.w[0] = x.x; c.own.w[1] = x.y; c.own.w[2] = x.z;
      c.O = x.w; c.S1o = y.x; c.P = y.y;
      c.opp.w[0] = c.opp.w[1] = c.opp.w[2] = 0u;
      c.S1p = 0u; c.off_opp = 0u; c.ft_own = 0u; c.ft_opp = 0u; c.black = 0u; c.elapsed = 0u; c.t = 0u;
      const uint32_t lw = y.z, prm = y.w;
      c.off_own = prm >> 20;
      const int pa = (int)(prm & 15u), pb = (int)((prm >> 4) & 15u);
      const int thl = (int)((prm >> 8) & 15u) - 1, tneed = (int)((prm >> 12) & 15u);
      const bool tbf = (prm >> 16) & 1u;
      if ((prm >> 17) & 1u) {
        const int ta = which ? pb : pa, tb = which ? pa : pb;
        uint32_t O2, S2;
        child_masks(c, p, ta, O2, S2);
        uint32_t L2 = die_candidates(O2, c.P, tb);
        if (!tbf) L2 = die_filter(O2, S2, block_info_low(O2, lw), L2, tb);
        if (p == 23) L2 &= ~HEAD;
        if (L2) atomicOr(&W.res[ow][which], 1u << p);
      } else {
        const int hl2 = thl - (p == 23 ? 1 : 0);
        int dep = 0;
        if (tbf) {
          uint32_t O2, S2;
          child_masks(c, p, pa, O2, S2);
          const int lb = f4_chain_bound(O2, S2, c.P, pa, hl2);
          dep = lb >= tneed ? tneed : 0;
        }
        if (dep < tneed) {
          apply_die(c, p, pa);
          dep = tneed == 1 ? f4_depth<1>(c, lw, pa, hl2, tbf)
                           : (tneed == 2 ? f4_depth<2>(c, lw, pa, hl2, tbf) : f4_depth<3>(c, lw, pa, hl2, tbf));
        }
        for (int j = 0; j < dep; ++j) atomicOr(&W.res[ow][j], 1u << p);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  out[0] = W.res[lane][0];
  out[1] = W.res[lane][1];
  out[2] = W.res[lane][2];
}

// env_turn_full with the per-source checks done cooperatively (see above)
__device__ void coop_turn_full(Side& s, int d0, int d1, bool play, uint64_t pw, const uint32_t w[4],
                               TurnOut& o, CoopLds& W, int lane) {
  const uint32_t low = block_lowmask(s.P);
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  const bool dbl = dh == dl;
#if NARDE_DIAG_ABLATE & 4
  const bool bf = true;  // DIAGNOSTIC timing only: wrong results
#else
  const bool bf = turn_block_free(s.O, s.P, low, dh, dl);
#endif
  // first sub-move: the lists, the shortcuts, then every lane's checks at once
  const uint32_t Lh = legal1(s, low, dh, bf);
  const uint32_t Ll = dbl ? 0u : legal1(s, low, dl, bf);
  const bool all_h = !dbl && bf && f4_lower_bound(s.O, s.S1o, s.P, dl, 1) >= 2;
  const bool all_l = !dbl && bf && f4_lower_bound(s.O, s.S1o, s.P, dh, 1) >= 2;
  const int hl0 = (dbl && s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1;
  const bool fast = dbl && bf && f4_lower_bound(s.O, s.S1o, s.P, dh, hl0) >= 4;
  // not fast: a chain bound >= 7 still keeps every first sub-move (one
  // sub-move lowers it by <= 4) with M = 4
  const int cb0 = (dbl && bf && !fast) ? f4_chain_bound(s.O, s.S1o, s.P, dh, hl0) : 0;
  // block-free with bear-off fixed: M exactly from the chains and every
  // C_k = L_k (f4_exact_moves) -- ~3/4 of the doubles turns the bounds miss
  const bool exact = dbl && bf && !fast && cb0 < 7 && Lh != 0u && f4_bearoff_fixed(s);
  const int Mx = exact ? f4_exact_moves(s, dh, hl0) : 0;
  const bool srch = dbl && !fast && Lh != 0u && cb0 < 7 && !exact;
  // one cooperative pass for every lane's first-sub-move checks
  uint32_t r0[3];
  {
    const bool pair = !dbl;
    const uint32_t m0 = pair ? (all_h ? 0u : Lh) : (srch ? Lh : 0u);
    const uint32_t m1 = pair ? (all_l ? 0u : Ll) : 0u;
#if NARDE_DIAG_ABLATE & 3
    r0[0] = Lh; r0[1] = Ll; r0[2] = Lh;  // DIAGNOSTIC timing only: wrong results
    (void)m0; (void)m1; (void)pair;
#else
    coop_run(W, s, low, dh, dl, pair ? 1 : hl0, m0, m1, 3, bf, pair ? 1 : 0, lane, r0);
#endif
  }
  uint32_t Ch, Cl;
  int M;
  if (!dbl) {
    Ch = all_h ? Lh : r0[0];
    Cl = all_l ? Ll : r0[1];
    if (Ch | Cl) {
      M = 2;
    } else {
      M = (Lh | Ll) ? 1 : 0;
      Ch = Lh;  // only one die playable: the higher one if it can
      Cl = Lh ? 0u : Ll;
    }
  } else {
    Cl = 0u;
    if (fast || (cb0 >= 7 && Lh)) { Ch = Lh; M = 4; }
    else if (!Lh) { Ch = 0u; M = 0; }
    else if (exact) { Ch = Lh; M = Mx; }
    else if (r0[2]) { Ch = r0[2]; M = 4; }  // some source leaves 3 more
    else if (r0[1]) { Ch = r0[1]; M = 3; }
    else if (r0[0]) { Ch = r0[0]; M = 2; }
    else { Ch = Lh; M = 1; }
  }
  o.legal = (uint64_t)Ch | ((uint64_t)Cl << 24) | ((uint64_t)dh << 48) | ((uint64_t)dl << 52) |
            ((uint64_t)M << 56);
  uint64_t played = ~0ull;
  int hl = hl0;
  bool go = M >= 1;
  int d = dh;
  if (go) {
    const int nh = __builtin_popcount(Ch), n = nh + __builtin_popcount(Cl);
    int p;
    if (play) {
      p = play_byte(pw, 0);
      d = play_byte(pw, 1);
      go = p >= 0 && p < 24 && ((d == dh && ((Ch >> p) & 1u)) || (!dbl && d == dl && ((Cl >> p) & 1u)));
    } else {
      const int idx = (int)mulhi_u32(w[0], (uint32_t)n);
      const bool hi = idx < nh;
      d = hi ? dh : dl;
      p = select_bit(hi ? Ch : Cl, hi ? idx : idx - nh);
    }
    if (go) {
      apply_die(s, p, d);
      played = played_set(played, 0, p, d);
      hl -= p == 23 ? 1 : 0;
    }
  }
  // sub-moves 1..3 (two dice: only k = 1, with the other die)
  for (int k = 1; k < 4; ++k) {
    const bool act = go && k < M;
    if (__ballot(act) == 0ull) break;  // wave-uniform: no lane has sub-move k
    const int dk = dbl ? dh : (d == dh ? dl : dh);
    uint32_t Lk = act ? legal1(s, low, dk, bf) : 0u;
    if (hl <= 0) Lk &= ~HEAD;
    const int need = M - k - 1;
    const bool direct = !dbl || fast || exact || need <= 0 ||
                        (act && bf && (f4_bearoff_fixed(s, need + 1) ||
                                       f4_chain_bound(s.O, s.S1o, s.P, dk, hl) >= need + 4));
    uint32_t rk[3];
#if NARDE_DIAG_ABLATE & 2
    rk[0] = rk[1] = rk[2] = Lk;
#else
    coop_run(W, s, low, dk, 0, hl, (act && !direct) ? Lk : 0u, 0u, need > 0 ? need : 1, bf, 0, lane, rk);
#endif
    const uint32_t C = direct ? Lk : (need >= 2 ? rk[1] : rk[0]);
    if (act) {
      int p;
      bool ok = true;
      if (play) {
        p = play_byte(pw, 2 * k);
        ok = play_byte(pw, 2 * k + 1) == dk && p >= 0 && p < 24 && ((C >> p) & 1u);
      } else {
        const uint32_t wk = k == 1 ? w[1] : (k == 2 ? w[2] : w[3]);
        p = select_bit(C, (int)mulhi_u32(wk, (uint32_t)__builtin_popcount(C)));
      }
      if (ok) {
        apply_die(s, p, dk);
        played = played_set(played, k, p, dk);
        hl -= p == 23 ? 1 : 0;
      } else {
        go = false;
      }
    }
  }
  o.played = played;
  o.max_dice = M;
  o.term = s.off_own == 15u;
  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
  if (!o.term) side_flip(s);
}

// this wave's slice of the block's cooperative scratch
#define COOP_LDS_DECL                                  \
  __shared__ CoopLds coop_lds[kBlock / 64];           \
  CoopLds& wave_coop = coop_lds[threadIdx.x >> 6];

// FULL4 first-sub-move set C_0 and max dice M for the given (or the next
// device) dice: the turn engine run on a copy with a play whose first
// sub-move is invalid, so nothing is applied.
__global__ void __launch_bounds__(kBlock) k_legal_full(Planes pl, int n, Rng g,
                                                       const uint8_t* __restrict__ dice2,
                                                       uint64_t* __restrict__ out) {
  COOP_LDS_DECL
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < n;  // no early exit: the turn is wave-cooperative
  Side s = valid ? side_from_record(pl.p0[i], pl.p1[i]) : side_start(0u);
  int d0 = 1, d1 = 2;
  if (dice2) {
    if (valid) {
      d0 = dice2[2 * i];
      d1 = dice2[2 * i + 1];
    }
  } else {
    uint32_t r[4];
    ply_draw(g, s.t, (uint32_t)i, r);
    dice_from(r[0], g.dice_mode, d0, d1);
  }
  const uint32_t w[4] = {0u, 0u, 0u, 0u};
  TurnOut o;
  // play word of -1s: nothing is applied
  coop_turn_full(s, d0, d1, true, ~0ull, w, o, wave_coop, (int)(threadIdx.x & 63));
  if (valid) out[i] = o.legal;
}

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

// Output store strategy (tuning knob, tools/diag/variants.sh):
//   0: each lane stores its own 96-B obs row (6 x 16 B at a 96-B lane stride:
//      every wave-instruction touches ~48 partial 128-B lines);
//   1: the wave transposes its 64 rows (6 KiB) through LDS so each
//      wave-instruction stores one contiguous 1 KiB (8 whole lines);
//   2: as 1 with non-temporal (streaming) stores for every per-ply output.
// REF2 rollout kernel: 1 = producer/consumer k_rollout_pc (default),
// 0 = one wave per 64 envs (k_rollout; A/B diagnostic builds only)
#ifndef NARDE_ROLLOUT_PC
#define NARDE_ROLLOUT_PC 1
#endif

// DIAGNOSTIC ablations of the cooperative FULL4 turn (timing only; results
// are wrong): 1 no two-dice checks, 2 no doubles searches, 4 all turns
// treated as block-free
#ifndef NARDE_DIAG_ABLATE
#define NARDE_DIAG_ABLATE 0
#endif

// wave priority in k_rollout_pc (diagnostic knob): 0 none (age decides),
// 1 consumers first, 2 producers first
#ifndef NARDE_PC_PRIO
#define NARDE_PC_PRIO 0
#endif

#ifndef NARDE_OBS_STORE
#define NARDE_OBS_STORE 2
#endif

template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
#if NARDE_OBS_STORE == 2
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void st_out(int4* p, int4 v) {
#if NARDE_OBS_STORE == 2
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

__device__ __forceinline__ void store_common(const Outs& out, size_t ix, const Side& s, int reward,
                                             int term, int trunc, int4* lds, bool wave_full) {
  if (out.obs) {
    if (NARDE_OBS_STORE != 0 && wave_full) store_obs_wave(out.obs, ix, s, lds);
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
  store_common(out, ix, s, o.reward, term, trunc, lds, wave_full);
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
__global__ void __launch_bounds__(kBlock) k_rollout(Planes pl, int n, Rng g, int plies, int max_steps,
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
// Plies go in blocks of kPcR with one workgroup barrier per block; LDS holds
// two slots of each ring (draws and results), 16 + 96 KiB.
// Equivalent, bit for bit, to `plies` narde_step(NULL, NULL, autoreset=1).
#ifndef NARDE_PC_SETS
#define NARDE_PC_SETS 1
#endif
constexpr int kPcEnvs = 256;                  // envs per workgroup
constexpr int kPcSets = NARDE_PC_SETS;        // consumer waves per producer wave
constexpr int kPcThreads = (1 + kPcSets) * kPcEnvs;  // producers + consumers
// plies per barrier block (tuning knob: 3, 4 and 5 time the same)
#ifndef NARDE_PC_R
#define NARDE_PC_R 4
#endif
constexpr int kPcR = NARDE_PC_R;                       // plies per barrier block

struct PcLds {
  uint2 draw[2][kPcR][kPcEnvs];               // the ply's (wa, wb) per env and ply
  uint4 res[2][kPcR][3][kPcEnvs];             // ply results (kOut only)
};

// results of one ply of one env, as the consumers read them:
//   res[.][.][0] = {own w0, own w1, own w2, opp w0}  (next mover's view)
//   res[.][.][1] = {opp w1, opp w2, legal lo, legal hi}
//   res[.][.][2] = {code1 | code2 << 16, reward | term << 8 | trunc << 16, 0, 0}
__device__ __forceinline__ void pc_put(PcLds& L, int slot, int k, int le, const Side& s,
                                       const StepOut& o, int term, int trunc) {
  const uint64_t lg = compact_legal(o.l1);
  L.res[slot][k][0][le] = make_uint4(s.own.w[0], s.own.w[1], s.own.w[2], s.opp.w[0]);
  L.res[slot][k][1][le] = make_uint4(s.opp.w[1], s.opp.w[2], (uint32_t)lg, (uint32_t)(lg >> 32));
  L.res[slot][k][2][le] =
      make_uint4(((uint32_t)(uint16_t)o.code1) | ((uint32_t)(uint16_t)o.code2 << 16),
                 (uint32_t)o.reward | ((uint32_t)term << 8) | ((uint32_t)trunc << 16), 0u, 0u);
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
        // of group 0, opponent word wi is dword 3 of group 0 or wi - 1 of
        // group 1 (2 x ds_read_b32 instead of 2 x ds_read_b128)
        const uint32_t* g0w = reinterpret_cast<const uint32_t*>(&L.res[slot][k][0][e0 + el]);
        const uint32_t* g1w = reinterpret_cast<const uint32_t*>(&L.res[slot][k][1][e0 + el]);
        const uint32_t own = g0w[wi];
        const uint32_t opp = wi == 0 ? g0w[3] : g1w[wi - 1];
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
    if (mine) {
      const uint4 b = L.res[slot][k][1][e0 + lane];
      const uint4 c = L.res[slot][k][2][e0 + lane];
      const size_t ix = row0 + lane;
      if (out.reward) st_out(out.reward + ix, (int32_t)(c.y & 0xFFu));
      if (out.term) st_out(out.term + ix, (uint8_t)((c.y >> 8) & 1u));
      if (out.trunc) st_out(out.trunc + ix, (uint8_t)((c.y >> 16) & 1u));
      if (out.legal) st_out(out.legal + ix, (uint64_t)b.z | ((uint64_t)b.w << 32));
      if (out.act_out) st_out(reinterpret_cast<uint32_t*>(out.act_out) + ix, c.x);
    }
  }
}

template <bool kOut>
__global__ void __launch_bounds__(kPcThreads) k_rollout_pc(Planes pl, int n, Rng g, int plies,
                                                           int max_steps, Outs out) {
  __shared__ PcLds L;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool producer = wave < 4;
#if NARDE_PC_PRIO == 1
  if (!producer) __builtin_amdgcn_s_setprio(1);
#elif NARDE_PC_PRIO == 2
  if (producer) __builtin_amdgcn_s_setprio(1);
#endif
  const int le = (wave & 3) * 64 + lane;            // workgroup-local env
  // consumer set: with kPcSets > 1 the consumer waves of one env group split
  // the plies of each block (set c takes plies k = c, c + kPcSets, ...)
  const int cset = producer ? 0 : (wave - 4) >> 2;
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
      L.draw[b & 1][k][le] = odd ? make_uint2(R[2], R[3]) : make_uint2(R[0], R[1]);
    }
  };
  if (!producer) draw_block(0);
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    const int p0 = b * kPcR;
    const int np = min(kPcR, plies - p0);
    if (producer) {
      if (valid) {
        for (int k = 0; k < np; ++k) {
          const uint2 rv = L.draw[b & 1][k][le];
          uint32_t r[4];
          ply_words(rv.x, rv.y, g.dice_mode, r);
          StepOut o;
          int term, trunc;
          env_ply(s, st, r, false, 0, 0, g.dice_mode, true, 0, 0, max_steps, true, o, term, trunc);
          if (kOut) pc_put(L, b & 1, k, le, s, o, term, trunc);
        }
      }
    } else {
      if (b + 1 < nb) draw_block(b + 1);
      if (kOut && b > 0)
        pc_emit(L, (b - 1) & 1, kPcR, p0 - kPcR, n, wg_env0, wave & 3, lane, out, cset, kPcSets);
    }
    __syncthreads();
  }
  if (kOut && !producer && nb > 0) {
    const int p0 = (nb - 1) * kPcR;
    pc_emit(L, (nb - 1) & 1, plies - p0, p0, n, wg_env0, wave & 3, lane, out, cset, kPcSets);
  }
  if (producer && valid) {
    uint4 ra, rb;
    side_to_record(s, ra, rb);
    pl.p0[i] = ra;
    pl.p1[i] = rb;
    add_stats(pl.stats, i, st);
  }
}

__global__ void __launch_bounds__(kBlock) k_get_stats(Planes pl, int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int4 s = pl.stats[i];
  out[3 * i] = s.x; out[3 * i + 1] = s.y; out[3 * i + 2] = s.z;
}

__global__ void __launch_bounds__(kBlock) k_apply(Planes pl, int n, const int8_t* __restrict__ moves,
                                                  const int8_t* __restrict__ player) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int f = moves[2 * i], t = moves[2 * i + 1];
  if (f < 0 || f > 23 || t < 0 || t > OFF) return;
  Side s = side_from_record(pl.p0[i], pl.p1[i]);
  const uint32_t want_black = player ? (player[i] == -1 ? 1u : 0u) : s.black;
  const bool flip = want_black != s.black;
  if (flip) side_flip(s);
  apply_move(s, f, t);
  if (flip) side_flip(s);
  uint4 a, b;
  side_to_record(s, a, b);
  pl.p0[i] = a;
  pl.p1[i] = b;
}

__global__ void __launch_bounds__(kBlock) k_observe(Planes pl, int n, int32_t* __restrict__ obs,
                                                    float* __restrict__ tes) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint4 a = pl.p0[i], b = pl.p1[i];
  if (obs) {
    const Side s = side_from_record(a, b);
    store_obs(obs, i, s);
  }
  if (tes) {
    // README.md:42-102 layout, absolute points: [white 24x4, bar, off,
    // black 24x4, bar, off, player one-hot]
    const Nib w{{a.x, a.y, b.x}};
    const Nib k{{a.z, a.w, b.y}};
    float2* o = reinterpret_cast<float2*>(tes + (size_t)i * 198);
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const Nib& c = side == 0 ? w : k;
#pragma unroll
      for (int p = 0; p < 24; ++p) {
        const uint32_t v = nib_get(c, p);
        const int base = side * 49 + p * 2;  // in float2 units
        o[base] = make_float2(v >= 1u ? 1.0f : 0.0f, v >= 2u ? 1.0f : 0.0f);
        o[base + 1] = make_float2(v >= 3u ? 1.0f : 0.0f, v >= 3u ? (float)(v - 3u) / 2.0f : 0.0f);
      }
      const uint32_t offc = side == 0 ? (b.z & 15u) : ((b.z >> 4) & 15u);
      o[side * 49 + 48] = make_float2(0.0f, (float)offc / 15.0f);
    }
    const bool black = (b.z >> 10) & 1u;
    o[98] = make_float2(black ? 0.0f : 1.0f, black ? 1.0f : 0.0f);
  }
}

// One DQN transition for every env, fused (config 4, gym_narde/dqn.py
// BatchedDQNDriver): the 198-float observation of the post-step record
// (k_observe's encoding), the reference trainer's reward shaping
// (train_deepq_pytorch.py:885-908), the prioritized-replay write of
// (s, a, r', s', done) at ring slot (pos + i) % capacity with the running max
// priority, and s <- s'.  One thread per observation float (coalesced rows;
// the 32 B record is an L1 hit for the row's 198 threads); column 0 also
// writes the env's scalars.  HBM per env: 792 B read (s) + 3 x 792 B written.
struct TransArgs {
  Planes pl;
  int n;
  int shaping;
  float* state;                 // (n,198) in: s, out: s'
  const int64_t* actions;       // (n,2)
  const int32_t* reward;        // (n,)
  const uint8_t* term;          // (n,)
  const uint8_t* trunc;         // (n,)
  float* off_seen;              // (n,2) borne-off trackers, white/black
  float* r_obs;                 // replay (capacity,198)
  float* r_next;                // replay (capacity,198)
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

// the env scalars of one transition (the thread holding column 0 of row i)
__device__ __forceinline__ void trans_scalars(const TransArgs& t, int i, int64_t slot, uint4 b) {
  const float done = (t.term[i] | t.trunc[i]) ? 1.0f : 0.0f;
  float r = (float)t.reward[i];
  if (t.shaping) {
    // +1 per checker newly borne off and +0.1 x total off, for the player
    // to move AFTER the step (the reference reads the post-flip player);
    // the trackers restart at 0 with a new episode.  Same fp32 ops as the
    // torch restatement (BatchedDQNDriver._transition_torch).
    const int black = (int)((b.z >> 10) & 1u);
    const float now = (float)(black ? ((b.z >> 4) & 15u) : (b.z & 15u));
    const float before = t.off_seen[2 * i + black];
    {
#pragma clang fp contract(off)  // torch rounds the product and the sum separately: no FMA
      r = (r + fmaxf(now - before, 0.0f)) + 0.1f * now;
    }
    const float keep = 1.0f - done;
    const float o0 = black ? t.off_seen[2 * i] : now;
    const float o1 = black ? now : t.off_seen[2 * i + 1];
    t.off_seen[2 * i] = o0 * keep;
    t.off_seen[2 * i + 1] = o1 * keep;
  }
  t.r_action[2 * slot] = t.actions[2 * i];
  t.r_action[2 * slot + 1] = t.actions[2 * i + 1];
  t.r_reward[slot] = r;
  t.r_done[slot] = done;
  t.r_prio[slot] = *t.max_prio;
}

// Each thread owns 4 consecutive floats of the flat (n, 198) arrays, so the
// state load and the three row stores are 16 B per lane (1 KiB per wave
// instruction; the two replay rows are written once and read only when
// sampled: non-temporal).  That needs the ring rows pos .. pos + n - 1
// contiguous and 16-B aligned (pos * 198 % 4 == 0, no wrap -- the steady
// state when the capacity is a multiple of n); otherwise each float goes
// on its own.
__global__ void __launch_bounds__(kBlock) k_dqn_transition(TransArgs t) {
  const uint32_t total = (uint32_t)t.n * 198u;  // n * 198 < 2^31 (checked on the host)
  const uint32_t e0 = 4u * (blockIdx.x * kBlock + threadIdx.x);
  if (e0 >= total) return;
  const int64_t pos = *t.pos;  // pos < capacity and i < n <= capacity: one wrap at most
  const bool vec = (pos * 198) % 4 == 0 && pos + t.n <= t.capacity && e0 + 4u <= total;
  const int i0 = (int)(e0 / 198u);
  const int c0 = (int)(e0 - (uint32_t)i0 * 198u);
  const uint4 a0 = t.pl.p0[i0], b0 = t.pl.p1[i0];
  // the 4 floats span rows i0 and (if c0 > 194) i0 + 1
  const bool split = c0 > 194 && i0 + 1 < t.n;
  uint4 a1 = a0, b1 = b0;
  if (split) { a1 = t.pl.p0[i0 + 1]; b1 = t.pl.p1[i0 + 1]; }
  float nv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + q;
    nv[q] = c < 198 ? tes_value(a0, b0, c) : tes_value(a1, b1, c - 198);
  }
  if (vec) {
    float4* st4 = reinterpret_cast<float4*>(t.state + e0);
    const float4 ov = *st4;
    const size_t d = (size_t)pos * 198 + e0;
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f o = {ov.x, ov.y, ov.z, ov.w};
    const v4f nn = {nv[0], nv[1], nv[2], nv[3]};
    __builtin_nontemporal_store(o, reinterpret_cast<v4f*>(t.r_obs + d));
    __builtin_nontemporal_store(nn, reinterpret_cast<v4f*>(t.r_next + d));
    *st4 = make_float4(nv[0], nv[1], nv[2], nv[3]);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t e = e0 + (uint32_t)q;
      if (e >= total) break;
      const int i = (int)(e / 198u);
      const int col = (int)(e - (uint32_t)i * 198u);
      int64_t slot = pos + i;
      if (slot >= t.capacity) slot -= t.capacity;
      t.r_obs[slot * 198 + col] = t.state[e];
      t.r_next[slot * 198 + col] = nv[q];
      t.state[e] = nv[q];
    }
  }
  // column 0 of a row lies in at most one thread's 4 floats
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t e = e0 + (uint32_t)q;
    if (e >= total) break;
    const int i = (int)(e / 198u);
    if (e - (uint32_t)i * 198u != 0u) continue;
    int64_t slot = pos + i;
    if (slot >= t.capacity) slot -= t.capacity;
    trans_scalars(t, i, slot, i == i0 ? b0 : b1);
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
  Legal l;
  legal2(s, d0, d1, l);
  uint64_t m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int f1, t1;
  decode_action(move1[i], f1, t1);
  if (l.count >= 2 && legal_contains(l, f1, t1)) {
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
__host__ __device__ inline uint64_t eps_to_q32(float epsilon) {
  const double e = epsilon <= 0.0f ? 0.0 : (epsilon >= 1.0f ? 1.0 : (double)epsilon);
  return (uint64_t)(e * 4294967296.0);
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
    const float* ar = add_tab ? add_tab + (size_t)add_row[row] * (size_t)ld_add : nullptr;
    float best = -__builtin_inff();
    int bi = 0x7FFFFFFF;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      if ((mw[j] >> lane) & 1ull) {
        const float v = ar ? qr[64 * j + lane] + ar[64 * j + lane] : qr[64 * j + lane];
        if (v > best) { best = v; bi = 64 * j + lane; }  // j ascending: first max kept
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    code = bi;
  }
  if (lane == 0) out[row] = code;
}

__global__ void __launch_bounds__(kBlock) k_block(const int8_t* __restrict__ boards, int n,
                                                  uint8_t* __restrict__ out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t O = 0, P = 0;
  for (int p = 0; p < 24; ++p) {
    const int v = boards[i * 24 + p];
    O |= (v > 0 ? 1u : 0u) << p;
    P |= (v < 0 ? 1u : 0u) << p;
  }
  out[i] = (runs6(O) & block_lowmask(P)) ? 1 : 0;
}

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

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
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

int narde_version(void) { return 1; }
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
                                                     (int64_t)0);
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
  k_set_ply<<<grid(e->n), kBlock, 0, e->hstream>>>(e->pl, (int)e->n, t);
  int rc = check_launch("k_set_ply");
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(e->hstream));
  return NARDE_OK;
}

int narde_reset(narde_env* e, const uint8_t* mask, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  DeviceGuard dg(e->device);
  k_reset<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), e->epoch, mask,
                                                           (int64_t)-1);
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

int narde_rollout(narde_env* e, int plies, int32_t* obs, int32_t* reward, uint8_t* terminated,
                  uint8_t* truncated, uint64_t* legal_compact, int16_t* actions_out, void* stream) {
  if (!e || plies < 0) return fail(NARDE_EINVAL, "bad argument");
  if (plies == 0) return NARDE_OK;
  DeviceGuard dg(e->device);
  const Outs out{obs, reward, terminated, truncated, legal_compact, actions_out, nullptr};
  const bool any = obs || reward || terminated || truncated || legal_compact || actions_out;
  const int pc_grid = (int)((e->n + kPcEnvs - 1) / kPcEnvs);
#if NARDE_ROLLOUT_PC
  if (any)
    k_rollout_pc<true><<<pc_grid, kPcThreads, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e), plies,
                                                                      e->max_steps, out);
  else
    k_rollout_pc<false><<<pc_grid, kPcThreads, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e),
                                                                       plies, e->max_steps, out);
#else
  (void)pc_grid;
  if (any)
    k_rollout<true, false><<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e),
                                                                          plies, e->max_steps, out);
  else
    k_rollout<false, false><<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e),
                                                                           plies, e->max_steps, out);
#endif
  return check_launch("k_rollout");
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
  if (any)
    k_rollout<true, true><<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e),
                                                                         plies, e->max_steps, out);
  else
    k_rollout<false, true><<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, rng_of(e),
                                                                          plies, e->max_steps, out);
  return check_launch("k_rollout<full>");
}

int narde_selfplay_full(narde_env* e, int plies, void* stream) {
  return narde_rollout_full(e, plies, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
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

int narde_apply_moves(narde_env* e, const int8_t* moves, const int8_t* player, void* stream) {
  if (!e || !moves) return fail(NARDE_EINVAL, "NULL argument");
  DeviceGuard dg(e->device);
  k_apply<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, moves, player);
  return check_launch("k_apply");
}

int narde_observe(narde_env* e, int32_t* obs, float* tes, void* stream) {
  if (!e) return fail(NARDE_EINVAL, "NULL handle");
  if (!obs && !tes) return NARDE_OK;
  DeviceGuard dg(e->device);
  k_observe<<<grid(e->n), kBlock, 0, (hipStream_t)stream>>>(e->pl, (int)e->n, obs, tes);
  return check_launch("k_observe");
}

int narde_dqn_transition(narde_env* e, float* state, const int64_t* actions, const int32_t* reward,
                         const uint8_t* terminated, const uint8_t* truncated, float* off_seen, int shaping,
                         float* r_obs, float* r_next, int64_t* r_action, float* r_reward, float* r_done,
                         float* r_prio, const float* max_prio, const int64_t* pos, int64_t capacity,
                         void* stream) {
  if (!e || !state || !actions || !reward || !terminated || !truncated || !r_obs || !r_next || !r_action ||
      !r_reward || !r_done || !r_prio || !max_prio || !pos || (shaping && !off_seen))
    return fail(NARDE_EINVAL, "NULL argument");
  if (capacity < e->n) return fail(NARDE_EINVAL, "replay capacity below the env count");
  if (e->n * 198 >= (int64_t(1) << 31)) return fail(NARDE_EINVAL, "too many envs for one transition launch");
  DeviceGuard dg(e->device);
  TransArgs t{e->pl, (int)e->n, shaping, state, actions, reward, terminated, truncated, off_seen,
              r_obs, r_next, r_action, r_reward, r_done, r_prio, max_prio, pos, capacity};
  const int64_t quads = (e->n * 198 + 3) / 4;
  k_dqn_transition<<<(unsigned)((quads + kBlock - 1) / kBlock), kBlock, 0, (hipStream_t)stream>>>(t);
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
  HIP_TRY(hipMemcpyAsync(e->d_in, e->h_in, hi.off, hipMemcpyHostToDevice, e->hstream));
  k_set_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db, doff, dft, dp, nullptr, 0);
  k_apply<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, dm, dp);
  k_get_state<<<grid(n), kBlock, 0, e->hstream>>>(e->hpl, (int)n, db2, doff2, dft2, nullptr, nullptr);
  if ((rc = check_launch("host apply"))) return rc;
  HIP_TRY(hipMemcpyAsync(e->h_out, e->d_out, dq.off, hipMemcpyDeviceToHost, e->hstream));
  if ((rc = host_sync(e))) return rc;
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
