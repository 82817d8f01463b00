// DIAGNOSTIC (host): narde_rules.h's die_filter and a loop-free form of it
// (die_filter_x below: measured slower on both rules, also when used only
// in block-bound turns -- DESIGN.md 10) against the per-candidate loop
// (restated here as
// filter_loop: every single-checker source whose move may complete a
// window tested by runs6 of its child board), for every die, on FULL4
// self-play positions and on random positions rich in 6-runs.  Must print 0
// mismatches.
//   hipcc -O2 -std=c++17 -o /tmp/filter_check tools/diag/filter_check.cpp && /tmp/filter_check
#include <cstdio>
#include <random>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

// Q as round 2 computed it (block_info_low before the suffix ORs)
static uint32_t q_round2(uint32_t O, uint32_t low) {
  const uint32_t r2 = O & (O >> 1);
  const uint32_t r3 = r2 & (O >> 2);
  const uint32_t r4 = r2 & (r2 >> 2);
  const uint32_t r5 = r4 & (O >> 4);
  const uint32_t lp = low + 1u;
  uint32_t q = (r5 >> 1) & low;
  q |= (O << 1) & (r4 >> 1) & ((lp << 1) - 1u);
  q |= (r2 << 2) & (r3 >> 1) & ((lp << 2) - 1u);
  q |= (r3 << 3) & (r2 >> 1) & ((lp << 3) - 1u);
  q |= (r4 << 4) & (O >> 1) & ((lp << 4) - 1u);
  q |= (r5 << 5) & ((lp << 5) - 1u);
  return q & ~O & MASK24;
}

// the round-2 filter: a multi-checker source violates iff a full window
// exists or its landing completes one; a single-checker source that may
// violate is tested on its child board
static uint32_t filter_loop(uint32_t O, uint32_t S1, uint32_t low, uint32_t C, int d) {
  const uint32_t F = runs6(O) & low;
  const uint32_t hit = F ? MASK24 : (q_round2(O, low) << d);
  uint32_t L = C & ~(hit & ~S1);
  uint32_t m = C & hit & S1;
  while (m) {
    const int p = __builtin_ctz(m);
    m &= m - 1u;
    const uint32_t bp = 1u << p;
    const uint32_t Op = (O & ~bp) | (p >= d ? (1u << (p - d)) : 0u);
    if (runs6(Op) & low) L &= ~bp;
  }
  return L;
}

// After a single-checker source p moves to q = p - d, an allowed window
// violates iff it does not hold p and is either already full (a bit of F
// outside [p-5, p]) or completed by q with its other five points own --
// window [q-a, q-a+5] misses p iff a >= 6 - d.
static uint32_t die_filter_x(uint32_t O, uint32_t S1, uint32_t low, uint32_t C, int d) {
  const uint32_t r2 = O & (O >> 1);
  const uint32_t r3 = r2 & (O >> 2);
  const uint32_t r4 = r2 & (r2 >> 2);
  const uint32_t r5 = r4 & (O >> 4);
  const uint32_t F = r4 & (r2 >> 4) & low;
  const uint32_t lp = low + 1u;
  const uint32_t t0 = (r5 >> 1) & low;
  const uint32_t t1 = (O << 1) & (r4 >> 1) & ((lp << 1) - 1u);
  const uint32_t t2 = (r2 << 2) & (r3 >> 1) & ((lp << 2) - 1u);
  const uint32_t t3 = (r3 << 3) & (r2 >> 1) & ((lp << 3) - 1u);
  const uint32_t t4 = (r4 << 4) & (O >> 1) & ((lp << 4) - 1u);
  const uint32_t t5 = (r5 << 5) & ((lp << 5) - 1u);
  const uint32_t Q = (t0 | t1 | t2 | t3 | t4 | t5) & ~O & MASK24;
  const uint32_t Qd = (t5 | (d >= 2 ? t4 : 0u) | (d >= 3 ? t3 : 0u) | (d >= 4 ? t2 : 0u) | (d >= 5 ? t1 : 0u) |
                       (d >= 6 ? t0 : 0u)) & ~O & MASK24;
  const int fmin = __builtin_ctz(F | (1u << 31)), fmax = 31 - __builtin_clz(F | 1u);
  const uint32_t v1 = F ? ((~0u << (fmin + 6)) | ((1u << fmax) - 1u)) : 0u;
  const uint32_t hit = F ? MASK24 : (Q << d);
  return C & ~(hit & ~S1) & ~(S1 & (v1 | (Qd << d)));
}

static long checked = 0, bad = 0, differs = 0;

static void check(uint32_t O, uint32_t S1, uint32_t P) {
  const uint32_t low = block_lowmask(P);
  const Blocks bl = block_info_low(O, low);
  for (int d = 1; d <= 6; ++d) {
    const uint32_t C = die_candidates(O, P, d);
    const uint32_t a = filter_loop(O, S1, low, C, d), b = die_filter(O, S1, bl, C, d);
    const uint32_t x = die_filter_x(O, S1, low, C, d);
    ++checked;
    differs += a != C;
    if (a != b || a != x) {
      if (bad < 10) printf("  loop-free %06x\n", x);
      if (bad < 10) printf("O %06x S1 %06x P %06x d %d: loop %06x new %06x\n", O, S1, P, d, a, b);
      ++bad;
    }
  }
}

int main() {
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
      ply_block(s.t, (uint32_t)e, 3u, 5u, R);
      ply_words_of(R, s.t, 0, r);
      check(s.O, s.S1o, s.P);
      TurnOut o;
      int tm, tr;
      env_ply_full(s, ST[e], r, (uint32_t)e, 3u, 5u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
    }
  // random positions: own checkers mostly in runs (so that full and
  // one-hole windows are common), the opponent on other points
  std::mt19937 rng(777);
  for (int k = 0; k < 4000000; ++k) {
    uint32_t own[24] = {0}, opp[24] = {0};
    int left = 15 - (int)(rng() % 6);
    const int start = (int)(rng() % 24), len = 4 + (int)(rng() % 6);
    for (int j = 0; j < len && left > 0; ++j) {
      const int q = (start + j) % 24;
      if (rng() % 8 == 0) continue;  // a hole
      own[q]++;
      --left;
    }
    while (left-- > 0) own[rng() % 24]++;
    for (int c = 0; c < 15; ++c) {
      int q = (int)(rng() % 24);
      for (int t = 0; t < 48 && own[q]; ++t) q = (int)(rng() % 24);
      if (!own[q]) opp[q]++;
    }
    uint32_t O = 0, P = 0, S1 = 0;
    for (int q = 0; q < 24; ++q) {
      O |= own[q] ? 1u << q : 0u;
      P |= opp[q] ? 1u << q : 0u;
      S1 |= own[q] == 1 ? 1u << q : 0u;
    }
    check(O, S1, P);
  }
  printf("checked %ld (filter removes a candidate in %ld), mismatches %ld\n", checked, differs, bad);
  return bad != 0;
}
