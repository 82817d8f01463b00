// full4_wave.h -- the wave-cooperative FULL4 turn:
// coop_turn_full (explicit plays, given dice), coop_depth_w, coop_pair_w
// and ply_bound_turn (the rollout's waves with a block-bound doubles lane).
// Device functions only, every lane of a wave converged at each call; the
// cross-lane operations are __ballot and __builtin_amdgcn_readlane and
// nothing else (no LDS, no thread indices), so tests/hostcheck compiles this
// header for the CPU with those two emulated over 64 host threads (the host
// check of ply_bound_turn against env_turn_full).  Included by
// kernels_full4.h (narde.hip's one translation unit).
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
// idle.  Here a lane with such checks only publishes them; the pass below
// runs them with the whole wave.  Every call is made with the whole wave
// converged: the turn is straight-line code with per-lane masks instead of
// rule branches around the calls.
//
// The pass (transposed): the wave walks the lanes that have checks (a scalar
// loop over a ballot); for each such owner its state is broadcast with
// v_readlane and every lane takes one source of the owner's masks (lanes
// 0-23: m0 bit `lane`, lanes 32-55: m1 bit `lane - 32`); the results come
// back as ballots.  No LDS, no prefix sums: a wave pays per owner -- a few
// per wave at most, since only block-bound lanes publish checks.
//   mode 1 (pair, two dice a = d_hi, b = d_lo): m0 = first moves with a,
//     kept (out 0) iff b still has a move after them; m1 = first moves with
//     b, kept (out 1) iff a still does.
//   mode 0 (depth, doubles a): m0 = sources; out j gets the sources after
//     which at least j + 1 more sub-moves are playable (searched up to
//     `need`).
// (A packed LDS task list instead of the walk -- a wave prefix sum placing
// every lane's checks, all 64 lanes taking tasks -- won while ~2.4 lanes per
// wave had checks; with the block-free tests below ~0.7 per wave have any,
// and the walk was faster: 0.4218 against 0.4266 ms per 100 plies.)
__device__ __forceinline__ uint32_t rl(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ void coop_run(const Side& s, uint32_t low, int a, int b, int hl, uint32_t m0, uint32_t m1,
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
        Side cc = c;
        apply_die(cc, p, pa);
        // (no block-free cut inside the device search: the test inlined into
        // every level cost more than the searches it saved)
        const int dep = tneed == 1 ? f4_depth<1, 0>(cc, lw, pa, hl2, tbf)
                                   : (tneed == 2 ? f4_depth<2, 0>(cc, lw, pa, hl2, tbf)
                                                 : f4_depth<3, 0>(cc, lw, pa, hl2, tbf));
        k0 = dep >= 1; k1 = dep >= 2; k2 = dep >= 3;
      }
      const uint32_t r0 = (uint32_t)__ballot(k0), r1 = (uint32_t)__ballot(k1), r2 = (uint32_t)__ballot(k2);
      out[0] = lane == ow ? r0 : out[0];
      out[1] = lane == ow ? r1 : out[1];
      out[2] = lane == ow ? r2 : out[2];
    }
  }
}

// The sub-moves of a turn once C_0 and M are known (shared by the general and
// the block-free turn): sub-move 0 from C_0 = (Ch, Cl), sub-moves 1..3
// (two dice: only k = 1, with the other die) from the list of their node,
// filtered through `later(k, dk, need, act, hl, Lk)` -- the general turn's
// cooperative depth check, or nothing on a block-free turn (every C_k = L_k).
// Then _check_game_ended and the flip.
template <class Later>
__device__ __forceinline__ void turn_play(Side& s, int dh, int dl, uint32_t Ch, uint32_t Cl, int M, int hl,
                                          bool play, uint64_t pw, const uint32_t w[4], TurnOut& o,
                                          Later&& later) {
  const bool dbl = dh == dl;
  o.legal = (uint64_t)Ch | ((uint64_t)Cl << 24) | ((uint64_t)dh << 48) | ((uint64_t)dl << 52) |
            ((uint64_t)M << 56);
  uint64_t played = ~0ull;
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
  // unrolled: with the general turn's cooperative check inside `later` the
  // compiler keeps a rolled loop, whose per-iteration control cost a short
  // FULL4 launch (k_rollout_wave, 20 plies) 6 % (0.519 -> 0.487 ms per 100
  // plies, profiles/r03/session3/wave_clock/wc9)
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const bool act = go && k < M;
    if (__ballot(act) == 0ull) break;  // wave-uniform: no lane has sub-move k
    const int dk = dbl ? dh : (d == dh ? dl : dh);
    uint32_t Lk = act ? die_candidates(s.O, s.P, dk) : 0u;
    const uint32_t C = later(k, dk, M - k - 1, act, hl, Lk);
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

// env_turn_full with the per-source checks done cooperatively (see above):
// the device turn for explicit plays and given dice (k_step<true>) and the
// FULL4 list query (k_legal_full); the rollouts' policy turn is
// ply_policy_full's straight-line one (kernels_rollout.h)
__device__ void coop_turn_full(Side& s, int d0, int d1, bool play, uint64_t pw, const uint32_t w[4],
                               TurnOut& o, int lane) {
  const uint32_t low = block_lowmask(s.P);
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  const bool dbl = dh == dl;
  // one block test for both kinds of turn (turn_block_set)
  const uint32_t bs = turn_block_set(s.O, s.S1o, s.P, low, dh, dl);
  const bool bf = bs == 0u;
  const uint32_t hs = dbl ? 0u : bs, ws = dbl ? bs : 0u;
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
  const bool nbf2 = !dbl && !bf;
  uint32_t sh = 0u, sl = 0u;
  if (__ballot(nbf2) != 0ull) {  // wave-uniform: only waves with such a lane
    sh = nbf2 ? f4_sure_pair(s.O, s.P, dl, Lh, hs) : 0u;
    sl = nbf2 ? f4_sure_pair(s.O, s.P, dh, Ll, hs) : 0u;
  }
  const int hl0 = (dbl && s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1;
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
    coop_run(s, low, dh, dl, pair ? 1 : hl0, m0, m1, 3, bf, pair ? 1 : 0, lane, r0);
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
  // later sub-moves: the node's list (block filter unless block-free), and
  // for a block-bound doubles turn that is not `fast` the cooperative check
  // that M - k - 1 more stay playable
  turn_play(s, dh, dl, Ch, Cl, M, hl0, play, pw, w, o,
            [&](int k, int dk, int need, bool act, int hl, uint32_t Lk) -> uint32_t {
              (void)k;
              if (act && !bf) Lk = die_filter(s.O, s.S1o, block_info_low(s.O, low), Lk, dk);
              if (hl <= 0) Lk &= ~HEAD;
              const bool direct = !dbl || bf || fast || need <= 0;
              uint32_t rk[3];
              coop_run(s, low, dk, 0, hl, (act && !direct) ? Lk : 0u, 0u, need > 0 ? need : 1, bf, 0, lane,
                       rk);
              return direct ? Lk : (need >= 2 ? rk[1] : rk[0]);
            });
}

// ---------------------------------------------------------------------------
// Round 4: waves with a block-bound doubles lane.  Every lane's turn goes
// the straight-line way (turn_c0_free, turn_c0_pair_bound_w), and only the
// block-bound doubles lanes that f4_safe_bound does not settle search --
// cooperatively, over lists filtered by the turn's failing windows
// (block_reject_w, f4_depth_w: no block_info / die_filter loop at the nodes):
// the root and sub-move 1 in one pass over (source, next source) pairs
// (coop_pair_w, round 5), sub-move 2 in a pass of its own (coop_depth_w).
// Same result as coop_turn_full (the host check: env_turn_full against
// f4_depth_w, hc_dbl_bound_w_random).

// coop_run's depth mode over the failing-window lists: for each owner lane
// (m0 != 0) in turn, every lane takes one source of its m0 (lanes 0-23) and
// searches f4_depth_w<need> below it; out[j] (owner lane) = the sources
// with depth >= j + 1 after them
__device__ void coop_depth_w(const Side& s, uint32_t fw, int d, int hl, uint32_t m0, int need, int lane,
                             uint32_t out[3]) {
  out[0] = out[1] = out[2] = 0u;
  uint64_t owners = __ballot(m0 != 0u);
  while (owners) {
    const int ow = (int)__builtin_ctzll(owners);
    owners &= owners - 1ull;
    Side c;
    c.own.w[0] = rl(s.own.w[0], ow); c.own.w[1] = rl(s.own.w[1], ow); c.own.w[2] = rl(s.own.w[2], ow);
    c.O = rl(s.O, ow); c.S1o = rl(s.S1o, ow); c.P = rl(s.P, ow);
    c.off_own = rl(s.off_own, ow);
    c.opp.w[0] = c.opp.w[1] = c.opp.w[2] = 0u;
    c.S1p = 0u; c.off_opp = 0u; c.ft_own = 0u; c.ft_opp = 0u; c.black = 0u; c.elapsed = 0u; c.t = 0u;
    const uint32_t ofw = rl(fw, ow), om = rl(m0, ow);
    const int od = (int)rl((uint32_t)d, ow), ohl = (int)rl((uint32_t)hl, ow), oneed = (int)rl((uint32_t)need, ow);
    const bool has = lane < 24 && ((om >> lane) & 1u);
    // below each source: the search's first path straight-line
    // (f4_probe_w), the search itself only where that path falls short
    const int src = has ? lane : 0;
    Side cc = c;
    apply_die_if(cc, src, od, has);
    const int hl2 = ohl - ((has && src == 23) ? 1 : 0);
    int dep = oneed == 1 ? f4_probe_w<1>(cc, ofw, od, hl2)
                         : (oneed == 2 ? f4_probe_w<2>(cc, ofw, od, hl2) : f4_probe_w<3>(cc, ofw, od, hl2));
    const bool miss = has && dep < oneed;
    if (__ballot(miss) != 0ull) {  // wave-uniform
      if (miss)
        dep = oneed == 1 ? f4_depth_w<1>(cc, ofw, od, hl2)
                         : (oneed == 2 ? f4_depth_w<2>(cc, ofw, od, hl2) : f4_depth_w<3>(cc, ofw, od, hl2));
    }
    const bool k0 = has && dep >= 1, k1 = has && dep >= 2, k2 = has && dep >= 3;
    const uint32_t r0 = (uint32_t)__ballot(k0), r1 = (uint32_t)__ballot(k1), r2 = (uint32_t)__ballot(k2);
    out[0] = lane == ow ? r0 : out[0];
    out[1] = lane == ow ? r1 : out[1];
    out[2] = lane == ow ? r2 : out[2];
  }
}

// The root search and the check of sub-move 1 in one pass (round 5): for
// each owner lane (m0 != 0: its filtered root list) in turn, lane j takes
// the pair (s0, s1) = (source r = j / 8 of m0, entry j % 8 of L1(s0), the
// list after s0 -- the failing windows' filter, the head rule) and finds
// whether one / two more sub-moves follow them (f4_probe_w<2>, the search
// where the probe stops at one).  From the pairs: r0[j] (owner lane) = the
// sources after which j + 1 more follow (coop_depth_w's out at need 3:
// after s0, 1 more iff L1(s0) is not empty, 2 / 3 more iff some pair leaves
// 1 / 2), and c1 = the check of sub-move 1 after the source p0 the turn will
// pick (w0 over C_0 as turn code does it): the entries s1 of L1(p0) after
// which M - 2 more follow -- so that sub-move needs no pass of its own.  ok
// (owner lane): done here; an owner with more than 8 root sources or an
// L1 of more than 8 entries is left to coop_depth_w.  (Host-checked with
// the rest of ply_bound_turn, tests/hostcheck hc_ply_bound_turn_random.)
__device__ void coop_pair_w(const Side& s, uint32_t fw, int d, int hl, uint32_t m0, uint32_t w0, int lane,
                            uint32_t r0[3], uint32_t& c1, bool& ok) {
  r0[0] = r0[1] = r0[2] = 0u;
  c1 = 0u;
  ok = false;
  uint64_t owners = __ballot(m0 != 0u);
  while (owners) {
    const int ow = (int)__builtin_ctzll(owners);
    owners &= owners - 1ull;
    Side c;
    c.own.w[0] = rl(s.own.w[0], ow); c.own.w[1] = rl(s.own.w[1], ow); c.own.w[2] = rl(s.own.w[2], ow);
    c.O = rl(s.O, ow); c.S1o = rl(s.S1o, ow); c.P = rl(s.P, ow);
    c.off_own = rl(s.off_own, ow);
    c.opp.w[0] = c.opp.w[1] = c.opp.w[2] = 0u;
    c.S1p = 0u; c.off_opp = 0u; c.ft_own = 0u; c.ft_opp = 0u; c.black = 0u; c.elapsed = 0u; c.t = 0u;
    const uint32_t ofw = rl(fw, ow), om = rl(m0, ow), ow0 = rl(w0, ow);
    const int od = (int)rl((uint32_t)d, ow), ohl = (int)rl((uint32_t)hl, ow);
    const int nsrc = __builtin_popcount(om);
    // lane j: source rank r, entry k
    const int r = lane >> 3, k = lane & 7;
    const bool hs = r < nsrc;
    const int s0 = select_bit(om, hs ? r : 0);
    Side ca = c;
    apply_die_if(ca, s0, od, hs);
    const int hla = ohl - ((hs && s0 == 23) ? 1 : 0);
    uint32_t L1 = die_candidates_sl(ca.O, ca.P, od);
    L1 &= ~block_reject_w(ca.O, ca.S1o, ofw, L1, od);
    L1 &= hla <= 0 ? ~HEAD : ~0u;
    L1 = hs ? L1 : 0u;
    const int cnt = __builtin_popcount(L1);
    if (nsrc > 8 || __ballot(k == 0 && cnt > 8) != 0ull) continue;  // wave-uniform: coop_depth_w's
    const bool hp = k < cnt;
    const int s1 = select_bit(L1, hp ? k : 0);
    Side cp = ca;
    apply_die_if(cp, s1, od, hp);
    const int hlp = hla - ((hp && s1 == 23) ? 1 : 0);
    int dep = f4_probe_w<2>(cp, ofw, od, hlp);
    const bool miss = hp && dep == 1;  // one more follows the pair; does a second?
    if (__ballot(miss) != 0ull) {     // wave-uniform
      if (miss) dep = f4_depth_w<2>(cp, ofw, od, hlp);
    }
    const uint64_t B0 = __ballot(k == 0 && cnt > 0), B1 = __ballot(hp && dep >= 1), B2 = __ballot(hp && dep >= 2);
    // the root sets as coop_depth_w's out: lane t < 24 (a source point) looks
    // at its source's group of 8 pair lanes
    const bool src = lane < 24 && ((om >> lane) & 1u);
    const int rt = __builtin_popcount(om & ((1u << (lane & 31)) - 1u));  // its rank
    const int sh = src ? 8 * rt : 0;
    const uint32_t a0 = (uint32_t)__ballot(src && ((B0 >> sh) & 1ull) != 0ull);
    const uint32_t a1 = (uint32_t)__ballot(src && ((B1 >> sh) & 0xFFull) != 0ull);
    const uint32_t a2 = (uint32_t)__ballot(src && ((B2 >> sh) & 0xFFull) != 0ull);
    // M, C_0 and the turn's first source as ply_bound_turn_c0 takes them
    const int M = a2 ? 4 : (a1 ? 3 : (a0 ? 2 : 1));
    const uint32_t Cs = a2 ? a2 : (a1 ? a1 : (a0 ? a0 : om));
    const int p0 = select_bit(Cs, (int)mulhi_u32(ow0, (uint32_t)__builtin_popcount(Cs)));
    const int r0p = __builtin_popcount(om & ((1u << p0) - 1u));
    const uint32_t Lp = rl(L1, 8 * r0p);  // L1(p0)
    const uint32_t G = (uint32_t)(((M >= 4 ? B2 : B1) >> (8 * r0p)) & 0xFFull);
    // entry e of L1(p0) (in order) is kept iff bit e of G: lane t < 24 is point t
    const bool inl = lane < 24 && ((Lp >> lane) & 1u);
    const int e = __builtin_popcount(Lp & ((1u << (lane & 31)) - 1u));
    const uint32_t cv = (uint32_t)__ballot(inl && ((G >> e) & 1u));
    r0[0] = lane == ow ? a0 : r0[0];
    r0[1] = lane == ow ? a1 : r0[1];
    r0[2] = lane == ow ? a2 : r0[2];
    c1 = lane == ow ? cv : c1;
    ok = lane == ow ? true : ok;
  }
}

// The turn of every lane of a wave holding a block-bound doubles lane (bs,
// fw: turn_block_set_sl): C_0 / M from the masks (turn_c0_free);
// block-bound two-dice lanes from the failing windows
// (turn_c0_pair_bound_w); block-bound doubles lanes: the filtered root
// list, M = 4 with every C_k = L_k when the moves that can never be
// rejected give >= 4 (f4_safe_bound), else the cooperative search; then the
// sub-moves, the bound lanes' lists filtered (block_reject_w) and the
// searching lanes' checks (coop_depth_w).  The rare blocks sit behind
// wave-uniform ballots.  Every lane must call it.  (Round 3's
// coop_turn_full here, per-lane branches and the die_filter search: 20-ply
// launches 0.454 -> 0.437 ms per 100 plies.)
// (ply_bound_turn_c0: with turn_c0_free's results given, c)
__device__ __forceinline__ void ply_bound_turn_c0(Side& s, int dh, int dl, uint32_t bs, uint32_t fw,
                                                  const uint32_t w[4], bool flip_always, TurnOut& o, int lane,
                                                  const TurnC0& c) {
  uint32_t Lh = c.Lh, Ll = c.Ll, Ch = c.Ch, Cl = c.Cl;
  int M = c.M;
  const int hl0 = c.hl0;
  const bool dbl = dh == dl;
  const bool b2 = bs != 0u && !dbl, bd = bs != 0u && dbl;
  if (__ballot(b2) != 0ull) {
    if (b2) turn_c0_pair_bound_w(s, dh, dl, bs, fw, Lh, Ll, Ch, Cl, M);
  }
  bool srch = false, pairs = false;
  uint32_t c1p = 0u;  // sub-move 1's checked list, when the pair pass made it (pairs)
  if (__ballot(bd) != 0ull) {
    // block-bound doubles: the filtered root list; M = 4 with every C_k =
    // L_k when the never-rejected moves give >= 4; else the search
    const uint32_t Lb = Lh & ~block_reject_w(s.O, s.S1o, bd ? fw : 0u, Lh, dh);
    const bool fast = bd && f4_safe_bound(s, dh, hl0, bs) >= 4;
    srch = bd && !fast && Lb != 0u;
    uint32_t r0[3];
    coop_pair_w(s, fw, dh, hl0, srch ? Lb : 0u, w[0], lane, r0, c1p, pairs);
    if (__ballot(srch && !pairs) != 0ull) {  // wave-uniform: owners too wide for the pairs
      uint32_t rd[3];
      coop_depth_w(s, fw, dh, hl0, (srch && !pairs) ? Lb : 0u, 3, lane, rd);
      if (srch && !pairs) { r0[0] = rd[0]; r0[1] = rd[1]; r0[2] = rd[2]; }
    }
    const int Ms = r0[2] ? 4 : (r0[1] ? 3 : (r0[0] ? 2 : 1));
    const uint32_t Cs = r0[2] ? r0[2] : (r0[1] ? r0[1] : (r0[0] ? r0[0] : Lb));
    Ch = bd ? (fast ? Lb : (Lb ? Cs : 0u)) : Ch;
    M = bd ? (fast ? 4 : (Lb ? Ms : 0)) : M;
  }
  o.legal = (uint64_t)Ch | ((uint64_t)Cl << 24) | ((uint64_t)dh << 48) | ((uint64_t)dl << 52) |
            ((uint64_t)M << 56);
  const int nh = __builtin_popcount(Ch), n = nh + __builtin_popcount(Cl);
  const int idx = (int)mulhi_u32(w[0], (uint32_t)n);
  const bool hi = idx < nh;
  const int d0 = hi ? dh : dl;
  const int p0 = select_bit(hi ? Ch : Cl, hi ? idx : idx - nh);
  const bool go = M >= 1;
  apply_die_if(s, p0, d0, go);
  uint32_t pl0 = go ? (0xFFFF0000u | ((uint32_t)d0 << 8) | (uint32_t)p0) : 0xFFFFFFFFu, pl1 = 0xFFFFFFFFu;
  int hl = hl0 - ((go && p0 == 23) ? 1 : 0);
  const int d1 = dbl ? dh : (d0 == dh ? dl : dh);
  const bool anyb = __ballot(bs != 0u) != 0ull;  // wave-uniform
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const int dk = k == 1 ? d1 : dh;
    const bool act = k < M;
    uint32_t Lk = die_candidates_sl(s.O, s.P, dk);
    if (anyb) {
      const bool filt = bd || (k == 1 && b2);
      Lk &= ~block_reject_w(s.O, s.S1o, filt ? fw : 0u, Lk, dk);
    }
    Lk &= hl <= 0 ? ~HEAD : ~0u;
    const int need = M - k - 1;
    const bool byp = k == 1 && pairs && need > 0;  // from the pair pass
    Lk = (srch && act && byp) ? c1p : Lk;
    const bool chk = srch && act && need > 0 && !byp;
    if (__ballot(chk) != 0ull) {  // wave-uniform
      uint32_t rk[3];
      coop_depth_w(s, fw, dk, hl, chk ? Lk : 0u, need, lane, rk);
      Lk = chk ? (need >= 2 ? rk[1] : rk[0]) : Lk;
    }
    const uint32_t wk = k == 1 ? w[1] : (k == 2 ? w[2] : w[3]);
    const int p = select_bit(Lk, (int)mulhi_u32(wk, (uint32_t)__builtin_popcount(Lk)));
    apply_die_if(s, p, dk, act);
    const uint32_t v = ((uint32_t)dk << 8) | (uint32_t)p;
    if (k == 1) pl0 = act ? ((pl0 & 0xFFFFu) | (v << 16)) : pl0;
    if (k == 2) pl1 = act ? ((pl1 & 0xFFFF0000u) | v) : pl1;
    if (k == 3) pl1 = act ? ((pl1 & 0xFFFFu) | (v << 16)) : pl1;
    hl -= (act && p == 23) ? 1 : 0;
  }
  o.played = (uint64_t)pl0 | ((uint64_t)pl1 << 32);
  o.max_dice = M;
  o.term = s.off_own == 15u;
  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
  if (flip_always) side_flip(s);
  else side_flip_if(s, !o.term);
}

__device__ __forceinline__ void ply_bound_turn(Side& s, int dh, int dl, uint32_t bs, uint32_t fw, const uint32_t w[4],
                                               bool flip_always, TurnOut& o, int lane) {
  TurnC0 c;
  turn_c0_free(s, dh, dl, c.Lh, c.Ll, c.Ch, c.Cl, c.M, c.hl0);
  ply_bound_turn_c0(s, dh, dl, bs, fw, w, flip_always, o, lane, c);
}

}  // namespace
