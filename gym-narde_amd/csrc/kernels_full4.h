// kernels_full4.h -- the wave-cooperative FULL4 turn and its list query
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

namespace {

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

// The same pass transposed (for at most NARDE_COOP_XPOSE owners): no task list.
// The wave walks the lanes that have checks (a scalar loop over a ballot);
// for each such owner its state is broadcast with v_readlane and every lane
// takes one source of the owner's masks (lanes 0-23: m0 bit `lane`, lanes
// 32-55: m1 bit `lane - 32`); the results come back as ballots.  No LDS,
// no prefix sums, no per-bit task-writing loop: a wave with few owners --
// ~2 on a ply, often none in the later sub-moves -- pays per owner, not a
// fixed pass.
// levels of a pass's block-bound doubles search that first test whether
// the node is block-free for the sub-moves it has left (f4_depth's CUT)
#ifndef NARDE_F4_CUT
#define NARDE_F4_CUT 0
#endif
// later sub-moves of a block-bound doubles turn: 0 always search, 2 stop at
// a node block-free for the sub-moves left, 3 stop where the root's safe
// bound (f4_safe_bound) covers the sub-moves left (2 and 3 measured slower,
// code in this loop runs in every wave, the searches in few)
#ifndef NARDE_F4_LATE
#define NARDE_F4_LATE 0
#endif
// owners up to which a pass is transposed (above: the packed LDS task list).
// 2 was best while ~2.4 block-bound lanes per wave had checks; with the
// block-bound lanes down to ~0.7 per wave the transposed walk wins for every
// wave (64: the packed list is compiled out and the kernel needs no LDS):
// 0.4218 against 0.4266 ms per 100 plies (1 / 3: 0.4238 / 0.4267)
#ifndef NARDE_COOP_XPOSE
#define NARDE_COOP_XPOSE 64
#endif
__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ void coop_run_x(const Side& s, uint32_t low, int a, int b, int hl, uint32_t m0, uint32_t m1,
                           int need, bool bf, int mode, int lane, uint32_t out[3]) {
  out[0] = out[1] = out[2] = 0u;
  uint64_t owners = __ballot((m0 | m1) != 0u);
  const int which = lane >> 5, p = lane & 31;
  while (owners) {
    const int ow = (int)__builtin_ctzll(owners);
    owners &= owners - 1ull;
    // the owner's state and parameters (wave-uniform from here on)
    Side c;
    c.own.w[0] = rl(s.own.w[0], ow); c.own.w[1] = rl(s.own.w[1], ow); c.own.w[2] = rl(s.own.w[2], ow);
    c.O = rl(s.O, ow); c.S1o = rl(s.S1o, ow); c.P = rl(s.P, ow);
    c.off_own = rl(s.off_own, ow);
    c.opp.w[0] = c.opp.w[1] = c.opp.w[2] = 0u;
    c.S1p = 0u; c.off_opp = 0u; c.ft_own = 0u; c.ft_opp = 0u; c.black = 0u; c.elapsed = 0u; c.t = 0u;
    const uint32_t lw = rl(low, ow), om0 = rl(m0, ow), om1 = rl(m1, ow);
    const int pa = (int)rl((uint32_t)a, ow), pb = (int)rl((uint32_t)b, ow);
    const int thl = (int)rl((uint32_t)hl, ow), tneed = (int)rl((uint32_t)need, ow);
    const bool tbf = rl(bf ? 1u : 0u, ow) != 0u;
    const bool pair = rl((uint32_t)mode, ow) != 0u;
    const uint32_t m = which == 0 ? om0 : (which == 1 ? om1 : 0u);
    const bool has = p < 24 && ((m >> p) & 1u);
    bool k0 = false, k1 = false, k2 = false;
    if (pair) {
      if (has) {
        const int ta = which ? pb : pa, tb = which ? pa : pb;
        uint32_t O2, S2;
        child_masks(c, p, ta, O2, S2);
        uint32_t L2 = die_candidates(O2, c.P, tb);
        if (!tbf) L2 = die_filter(O2, S2, block_info_low(O2, lw), L2, tb);
        if (p == 23) L2 &= ~HEAD;
        k0 = L2 != 0u;
      }
      const uint64_t r = __ballot(k0);
      const uint32_t r0 = (uint32_t)r & MASK24, r1 = (uint32_t)(r >> 32) & MASK24;
      out[0] = lane == ow ? r0 : out[0];
      out[1] = lane == ow ? r1 : out[1];
    } else {
      if (has) {
        const int hl2 = thl - (p == 23 ? 1 : 0);
        int dep = 0;  // (only block-bound lanes publish doubles tasks)
#if NARDE_DIAG_ABLATE & 128
        dep = tneed;  // DIAGNOSTIC timing only: no doubles search in the passes
#endif
        if (dep < tneed) {
          Side cc = c;
          apply_die(cc, p, pa);
          dep = tneed == 1 ? f4_depth<1, NARDE_F4_CUT>(cc, lw, pa, hl2, tbf)
                           : (tneed == 2 ? f4_depth<2, NARDE_F4_CUT>(cc, lw, pa, hl2, tbf) : f4_depth<3, NARDE_F4_CUT>(cc, lw, pa, hl2, tbf));
        }
        k0 = dep >= 1; k1 = dep >= 2; k2 = dep >= 3;
      }
      const uint32_t r0 = (uint32_t)__ballot(k0), r1 = (uint32_t)__ballot(k1), r2 = (uint32_t)__ballot(k2);
      out[0] = lane == ow ? r0 : out[0];
      out[1] = lane == ow ? r1 : out[1];
      out[2] = lane == ow ? r2 : out[2];
    }
  }
}

// One cooperative pass over every lane's per-source checks.  Per lane:
//   mode 1 (pair, two dice a = d_hi, b = d_lo): m0 = first moves with a,
//     kept (res 0) iff b still has a move after them; m1 = first moves with
//     b, kept (res 1) iff a still does.
//   mode 0 (depth, doubles a): m0 = sources; res j gets the sources after
//     which at least j + 1 more sub-moves are playable (searched up to
//     `need`; only block-bound lanes have such tasks).
__device__ void coop_run(CoopLds& W, const Side& s, uint32_t low, int a, int b, int hl, uint32_t m0,
                         uint32_t m1, int need, bool bf, int mode, int lane, uint32_t out[3]) {
  out[0] = out[1] = out[2] = 0u;
  const uint64_t any = __ballot((m0 | m1) != 0u);
  if (any == 0ull) return;  // wave-uniform: nothing to check
#if NARDE_COOP_XPOSE
  // few owners: the transposed walk; many: one packed task list
  if (__builtin_popcountll(any) <= NARDE_COOP_XPOSE) {
    coop_run_x(s, low, a, b, hl, m0, m1, need, bf, mode, lane, out);
    return;
  }
#endif
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
#if NARDE_DIAG_ABLATE & 256
        if (true) { atomicOr(&W.res[ow][which], 1u << p); continue; }  // DIAGNOSTIC: no pair checks
#endif
        const int ta = which ? pb : pa, tb = which ? pa : pb;
        uint32_t O2, S2;
        child_masks(c, p, ta, O2, S2);
        uint32_t L2 = die_candidates(O2, c.P, tb);
        if (!tbf) L2 = die_filter(O2, S2, block_info_low(O2, lw), L2, tb);
        if (p == 23) L2 &= ~HEAD;
        if (L2) atomicOr(&W.res[ow][which], 1u << p);
      } else {
        const int hl2 = thl - (p == 23 ? 1 : 0);
        int dep = 0;  // (only block-bound lanes publish doubles tasks)
#if NARDE_DIAG_ABLATE & 128
        dep = tneed;  // DIAGNOSTIC timing only: no doubles search in the passes
#endif
        if (dep < tneed) {
          apply_die(c, p, pa);
          dep = tneed == 1 ? f4_depth<1, NARDE_F4_CUT>(c, lw, pa, hl2, tbf)
                           : (tneed == 2 ? f4_depth<2, NARDE_F4_CUT>(c, lw, pa, hl2, tbf) : f4_depth<3, NARDE_F4_CUT>(c, lw, pa, hl2, tbf));
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
#elif NARDE_DIAG_ABLATE & 1024
  const bool bf = dbl ? turn_block_free(s.O, s.S1o, s.P, low, dh, dl) : true;  // DIAGNOSTIC
#elif NARDE_DIAG_ABLATE & 2048
  const bool bf = dbl ? true : turn_block_free(s.O, s.S1o, s.P, low, dh, dl);  // DIAGNOSTIC
#else
  // one block test for both kinds of turn (turn_block_set)
  const uint32_t bs = turn_block_set(s.O, s.S1o, s.P, low, dh, dl);
  const bool bf = bs == 0u;
  const uint32_t hs = dbl ? 0u : bs, ws = dbl ? bs : 0u;
#endif
  // first sub-move: the lists, the shortcuts, then every lane's checks at once
  // (both dice's lists from one block-info of the root: legal1 twice would
  // compute it twice in the block-bound lanes)
  uint32_t Lh = die_candidates(s.O, s.P, dh);
  uint32_t Ll = dbl ? 0u : die_candidates(s.O, s.P, dl);
  if (!bf) {
    const Blocks bl = block_info_low(s.O, low);
    Lh = die_filter(s.O, s.S1o, bl, Lh, dh);
    Ll = die_filter(s.O, s.S1o, bl, Ll, dl);
  }
  // two dice, block-free: the pair checks of every source from the masks
  // (f4_keep_pair_bf) -- only non-block-free lanes publish pair tasks
  const bool pbf = !dbl && bf;
  const uint32_t kh = pbf ? f4_keep_pair_bf(s.O, s.S1o, s.P, dh, dl, Lh) : 0u;
  const uint32_t kl = pbf ? f4_keep_pair_bf(s.O, s.S1o, s.P, dl, dh, Ll) : 0u;
  // block-bound two dice: the sources sure from the masks (f4_sure_pair)
  // need no task -- ~3/4 of these lanes have no task left
#if NARDE_DIAG_ABLATE & (4 | 1024 | 2048)
  const uint32_t hs = 0u;  // DIAGNOSTIC builds
#endif
  const bool nbf2 = !dbl && !bf;
  uint32_t sh = 0u, sl = 0u;
  if (__ballot(nbf2) != 0ull) {  // wave-uniform: only waves with such a lane
    sh = nbf2 ? f4_sure_pair(s.O, s.P, dl, Lh, hs) : 0u;
    sl = nbf2 ? f4_sure_pair(s.O, s.P, dh, Ll, hs) : 0u;
  }
  const int hl0 = (dbl && s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1;
#if NARDE_DIAG_ABLATE & (4 | 1024 | 2048)
  const uint32_t ws = 0u;  // DIAGNOSTIC builds
#endif
  // block-free doubles: M exactly from the chains (f4_exact_moves, bear-off
  // fixed) or from the chains and the bear-offs they can open
  // (f4_open_moves), every C_k = L_k -- no bound, no search
  const bool xbf = dbl && bf;
  const int T0 = xbf ? f4_exact_moves(s, dh, hl0) : 0;
  const int Mx = (xbf && !f4_bearoff_fixed(s)) ? f4_open_moves(s, dh, hl0, T0) : T0;
  // block-bound doubles: M = 4 and every C_k = L_k when the moves that can
  // never be rejected give >= 4 (f4_safe_bound); else the search
  bool fast = false;
  if (__ballot(dbl && !bf) != 0ull) fast = dbl && !bf && f4_safe_bound(s, dh, hl0, ws) >= 4;
  const bool srch = dbl && !bf && !fast && Lh != 0u;
  // one cooperative pass for every lane's first-sub-move checks
  uint32_t r0[3];
  {
    const bool pair = !dbl;
    const uint32_t m0 = pair ? (bf ? 0u : Lh & ~sh) : (srch ? Lh : 0u);
    const uint32_t m1 = pair ? (bf ? 0u : Ll & ~sl) : 0u;
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
    Ch = bf ? kh : (sh | r0[0]);
    Cl = bf ? kl : (sl | r0[1]);
    if (Ch | Cl) {
      M = 2;
    } else {
      M = (Lh | Ll) ? 1 : 0;
      Ch = Lh;  // only one die playable: the higher one if it can
      Cl = Lh ? 0u : Ll;
    }
  } else {
    Cl = 0u;
    if (xbf) { Ch = Lh; M = Lh ? Mx : 0; }
    else if (fast) { Ch = Lh; M = 4; }
    else if (!Lh) { Ch = 0u; M = 0; }
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
    // block-free doubles and 'fast' block-bound ones: every C_k = L_k
    bool direct = !dbl || bf || fast || need <= 0;
#if NARDE_F4_LATE == 2
    // A block-bound lane stops searching once its node is block-free for the
    // need + 1 sub-moves it has left (env_turn_full): the test only in waves
    // that have one
    const bool maybe = act && !direct;
    if (__ballot(maybe) != 0ull)
      direct = direct || (maybe && dbl_block_free(s.O, s.S1o, s.P, low, dk, need + 1));
#elif NARDE_F4_LATE == 3
    // A block-bound lane stops searching once the moves that can never be
    // rejected (the root's failing windows, f4_safe_bound) leave >= need + 1
    // at its node: on an M-path a sub-move lowers that bound by at most one,
    // so every source keeps need more
    const bool maybe = act && !direct;
    if (__ballot(maybe) != 0ull)
      direct = direct || (maybe && f4_safe_bound(s, dk, hl, ws) >= need + 1);
#endif
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
  bool bad = false;  // a given die outside 1..6: no legal move
  if (dice2) {
    if (valid) {
      d0 = dice2[2 * i];
      d1 = dice2[2 * i + 1];
      bad = (uint32_t)(d0 - 1) > 5u || (uint32_t)(d1 - 1) > 5u;
      if (bad) { d0 = 1; d1 = 2; }
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
  if (valid) out[i] = bad ? 0ull : o.legal;
}

}  // namespace
