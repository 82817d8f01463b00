// DIAGNOSTIC (host): the per-window loop of turn_block_set over random
// self-play, by 64-lane wave: how many lanes enter it and how many window
// iterations the wave runs (the most of any lane), with the current window
// filter and with a sharper branch-free prefilter (win_prefilter below);
// checks that the prefilter keeps every window the exact test fails
// (unsound: must be 0).
//   hipcc -O2 -std=c++17 -o /tmp/win_stats tools/diag/win_stats.cpp && /tmp/win_stats
#include <cstdio>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

// the candidate windows of turn_block_set as they stand
static uint32_t win_current(uint32_t O, uint32_t P, uint32_t low, int dh, int dl) {
  const bool dbl = dh == dl;
  const uint32_t A = O | land_step(O, P, dh) | land_step(O, P, dl);
  uint32_t U = A | land_step(A, P, dh) | land_step(A, P, dl);
  const uint32_t V = land_step(U, P, dh);
  U |= dbl ? (V | land_step(V, P, dh)) : 0u;
  return runs6(U) & low & windows_few_holes(O, dbl ? 4 : 2);
}

// the windows turn_block_set's exact per-window test fails (~0u: a full one)
static uint32_t win_failing(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  const bool dbl = dh == dl;
  uint32_t win = win_current(O, P, low, dh, dl), out = 0u;
  while (win) {
    const int i = __builtin_ctz(win);
    win &= win - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    if (!H) return ~0u;
    const uint32_t src = O & ~(W & S1);
    bool fail;
    if (dbl) {
      uint32_t T = src, seen = 0u;
      int cost = 0;
      for (int j = 1; j <= 4; ++j) {
        T = land_step(T, P, dh);
        const uint32_t nw = H & T & ~seen;
        cost += j * __builtin_popcount(nw);
        seen |= nw;
      }
      fail = seen == H && cost <= 4;
    } else {
      const uint32_t Lh = land_step(src, P, dh), Ll = land_step(src, P, dl);
      const uint32_t h1 = H & (0u - H), h2 = H ^ h1;
      fail = !h2 ? (H & (Lh | Ll | land_step(Lh, P, dl) | land_step(Ll, P, dh))) != 0u
                 : (((h1 & Lh) && (h2 & Ll)) || ((h1 & Ll) && (h2 & Lh)));
    }
    out |= fail ? (1u << i) : 0u;
  }
  return out;
}

// 3-bit bit-sliced add with an overflow mask
struct B3 {
  uint32_t b0, b1, b2, ov;
};
static B3 add3(const B3& a, const B3& b) {
  B3 s;
  const uint32_t x0 = a.b0 ^ b.b0, c0 = a.b0 & b.b0;
  const uint32_t x1 = a.b1 ^ b.b1;
  s.b0 = x0;
  s.b1 = x1 ^ c0;
  const uint32_t c1 = (a.b1 & b.b1) | (c0 & x1);
  const uint32_t x2 = a.b2 ^ b.b2;
  s.b2 = x2 ^ c1;
  s.ov = a.ov | b.ov | (a.b2 & b.b2) | (c1 & x2);
  return s;
}
static B3 shr3(const B3& a, int k) { return B3{a.b0 >> k, a.b1 >> k, a.b2 >> k, a.ov >> k}; }

// sharper candidate windows, no loop: two dice -- a 1-hole window's hole is a
// landing of one die or of both in turn, a 2-hole window's holes are
// single-die landings (sources unrestricted: a superset of the exact test);
// doubles -- every hole reachable within 4 steps and the holes' fewest
// steps summing to <= 4
static uint32_t win_prefilter(uint32_t O, uint32_t P, uint32_t low, int dh, int dl) {
  if (dh != dl) {
    const uint32_t Rh = land_step(O, P, dh), Rl = land_step(O, P, dl);
    const uint32_t X1 = O | Rh | Rl;
    const uint32_t X2 = X1 | land_step(Rh, P, dl) | land_step(Rl, P, dh);
    const uint32_t h = ~O & MASK24;
    uint32_t s0 = 0u, s1 = 0u, s2 = 0u;
    for (int j = 0; j < 6; ++j) {
      const uint32_t x = h >> j;
      const uint32_t c0 = s0 & x;
      s0 ^= x;
      const uint32_t c1 = s1 & c0;
      s1 ^= c0;
      s2 |= c1;
    }
    const uint32_t le1 = ~s2 & ~s1, eq2 = ~s2 & s1 & ~s0;
    return low & runs6(X2) & (le1 | (eq2 & runs6(X1)));
  }
  const int d = dh;
  const uint32_t T1 = land_step(O, P, d), T2 = land_step(T1, P, d), T3 = land_step(T2, P, d),
                 T4 = land_step(T3, P, d);
  const uint32_t E1 = T1 & ~O, E2 = T2 & ~(O | T1), E3 = T3 & ~(O | T1 | T2), E4 = T4 & ~(O | T1 | T2 | T3);
  const uint32_t reach = O | T1 | T2 | T3 | T4;
  const B3 c{E1 | E3, E2 | E3, E4, 0u};
  const B3 s2 = add3(c, shr3(c, 1));
  const B3 s4 = add3(s2, shr3(s2, 2));
  const B3 s6 = add3(s4, shr3(s2, 4));
  const uint32_t le4 = ~s6.ov & (~s6.b2 | (~s6.b1 & ~s6.b0));
  return low & runs6(reach) & le4;
}

int main() {
  const int n = 64 * 128, plies = 400;
  long lanes = 0, lanes_cur = 0, lanes_new = 0, lanes_fail = 0, unsound = 0;
  long waves = 0, waves_cur = 0, waves_new = 0, waves_fail = 0, it_cur = 0, it_new = 0;
  long dlanes = 0, dlanes_cur = 0, dlanes_new = 0;
  static Side S[64 * 128];
  static int4 ST[64 * 128];
  for (int e = 0; e < n; ++e) {
    S[e] = side_start(e & 1);
    S[e].t = 0;
    ST[e] = make_int4(0, 0, 0, 0);
  }
  for (int p = 0; p < plies; ++p) {
    for (int w = 0; w < n / 64; ++w) {
      int mc = 0, mn = 0;
      bool ac = false, an = false, af = false;
      for (int l = 0; l < 64; ++l) {
        const int e = w * 64 + l;
        Side& s = S[e];
        uint32_t R[4], r[4];
        ply_block(s.t, (uint32_t)e, 1u, 2u, R);
        ply_words_of(R, s.t, 0, r);
        int d0, d1;
        dice_from(r[0], 0, d0, d1);
        const uint32_t low = block_lowmask(s.P);
        const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
        const uint32_t wc = win_current(s.O, s.P, low, dh, dl);
        const uint32_t wn = win_prefilter(s.O, s.P, low, dh, dl);
        const uint32_t wf = win_failing(s.O, s.S1o, s.P, low, dh, dl);
        ++lanes;
        lanes_cur += wc != 0u;
        lanes_new += wn != 0u;
        lanes_fail += wf != 0u;
        if (dh == dl) {
          ++dlanes;
          dlanes_cur += wc != 0u;
          dlanes_new += wn != 0u;
        }
        if (wf != ~0u && (wf & ~wn)) ++unsound;
        if (wf == ~0u && !(wn & wc)) ++unsound;  // a full window must stay a candidate
        mc = mc > __builtin_popcount(wc) ? mc : __builtin_popcount(wc);
        mn = mn > __builtin_popcount(wn) ? mn : __builtin_popcount(wn);
        ac |= wc != 0u;
        an |= wn != 0u;
        af |= wf != 0u;
        TurnOut o;
        int tm, tr;
        env_ply_full(s, ST[e], r, (uint32_t)e, 1u, 2u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
      }
      ++waves;
      waves_cur += ac;
      waves_new += an;
      waves_fail += af;
      it_cur += mc;
      it_new += mn;
    }
  }
  printf("lanes %ld: current filter %.4f, prefilter %.4f, exact fail %.4f (doubles %ld: %.4f / %.4f)\n", lanes,
         (double)lanes_cur / lanes, (double)lanes_new / lanes, (double)lanes_fail / lanes, dlanes,
         (double)dlanes_cur / dlanes, (double)dlanes_new / dlanes);
  printf("waves %ld with a looping lane: current %.4f, prefilter %.4f, exact fail %.4f\n", waves,
         (double)waves_cur / waves, (double)waves_new / waves, (double)waves_fail / waves);
  printf("window iterations per wave-ply (max lane): current %.3f, prefilter %.3f\n", (double)it_cur / waves,
         (double)it_new / waves);
  printf("unsound: %ld\n", unsound);
  return 0;
}
