// DIAGNOSTIC (host): a branch-free body for turn_block_set's per-window loop
// (tbs_bf: both kinds of turn computed, selects instead of branches, a full
// window as a sticky ~0u instead of an early return) against the product
// turn_block_set, over FULL4 self-play and over random positions.  Must print
// 0 mismatches.
//   hipcc -O2 -std=c++17 -o /tmp/tbs_check tools/diag/tbs_check.cpp && /tmp/tbs_check
#include <cstdio>
#include <random>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

static uint32_t tbs_bf(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  const bool dbl = dh == dl;
  const uint32_t A = O | land_step(O, P, dh) | land_step(O, P, dl);
  uint32_t U = A | land_step(A, P, dh) | land_step(A, P, dl);
  const uint32_t V = land_step(U, P, dh);
  U |= dbl ? (V | land_step(V, P, dh)) : 0u;
  uint32_t win = runs6(U) & low & windows_few_holes(O, dbl ? 4 : 2), out = 0u;
  while (win) {
    const int i = __builtin_ctz(win);
    win &= win - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    const uint32_t src = O & ~(W & S1);
    uint32_t T = src, seen = 0u, cost = 0u;
    for (int j = 1; j <= 4; ++j) {
      T = land_step(T, P, dh);
      const uint32_t nw = H & T & ~seen;
      cost += (uint32_t)j * (uint32_t)__builtin_popcount(nw);
      seen |= nw;
    }
    const uint32_t fd = (seen == H && cost <= 4u) ? W : 0u;
    const uint32_t Lh = land_step(src, P, dh), Ll = land_step(src, P, dl);
    const uint32_t h1 = H & (0u - H), h2 = H ^ h1;
    const int i1 = __builtin_ctz(H | 0x80000000u), i2 = __builtin_ctz(h2 | 0x80000000u);
    const uint32_t a1 = (Lh >> i1) & (Ll >> i2), a2 = (Ll >> i1) & (Lh >> i2);
    const uint32_t reach = Lh | Ll | land_step(Lh, P, dl) | land_step(Ll, P, dh);
    const uint32_t f1 = (H & reach) ? H : 0u, f2 = ((a1 | a2) & 1u) ? H : 0u;
    const uint32_t ft = h2 ? f2 : f1;
    out |= H == 0u ? ~0u : (dbl ? fd : ft);
  }
  return out;
}

int main() {
  long checked = 0, bad = 0, nonzero = 0;
  // FULL4 self-play
  const int n = 64 * 64, plies = 600;
  static Side S[64 * 64];
  static int4 ST[64 * 64];
  for (int e = 0; e < n; ++e) {
    S[e] = side_start(e & 1);
    ST[e] = make_int4(0, 0, 0, 0);
  }
  for (int p = 0; p < plies; ++p)
    for (int e = 0; e < n; ++e) {
      Side& s = S[e];
      uint32_t R[4], r[4];
      ply_block(s.t, (uint32_t)e, 7u, 9u, R);
      ply_words_of(R, s.t, 0, r);
      const uint32_t low = block_lowmask(s.P);
      for (int dh = 1; dh <= 6; ++dh)
        for (int dl = 1; dl <= dh; ++dl) {
          const uint32_t a = turn_block_set(s.O, s.S1o, s.P, low, dh, dl), b = tbs_bf(s.O, s.S1o, s.P, low, dh, dl);
          ++checked;
          nonzero += a != 0u;
          bad += a != b;
        }
      TurnOut o;
      int tm, tr;
      env_ply_full(s, ST[e], r, (uint32_t)e, 7u, 9u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
    }
  // random positions: own and opponent checkers on disjoint random points
  std::mt19937 rng(12345);
  for (int k = 0; k < 2000000; ++k) {
    uint32_t own[24] = {0}, opp[24] = {0};
    const int no = 15 - (int)(rng() % 4), np = 15;
    for (int c = 0; c < no; ++c) own[rng() % 24]++;
    for (int c = 0; c < np; ++c) {
      int q = (int)(rng() % 24);
      while (own[q]) q = (int)(rng() % 24);
      opp[q]++;
    }
    uint32_t O = 0, P = 0, S1 = 0;
    for (int q = 0; q < 24; ++q) {
      O |= own[q] ? 1u << q : 0u;
      P |= opp[q] ? 1u << q : 0u;
      S1 |= own[q] == 1 ? 1u << q : 0u;
    }
    const int dh = 1 + (int)(rng() % 6), dl = 1 + (int)(rng() % dh);
    const uint32_t low = block_lowmask(P);
    const uint32_t a = turn_block_set(O, S1, P, low, dh, dl), b = tbs_bf(O, S1, P, low, dh, dl);
    ++checked;
    nonzero += a != 0u;
    bad += a != b;
  }
  printf("checked %ld (block-bound %ld), mismatches %ld\n", checked, nonzero, bad);
  return bad != 0;
}
