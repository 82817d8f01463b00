// DIAGNOSTIC (host): how many turns of random self-play the block-free test
// (turn_block_free) calls block-bound although the block rule never removes
// a candidate anywhere in the turn, and whether it ever calls a turn
// block-free in which the rule does bind (unsound: must be 0).
// Ground truth: a depth-first walk over every sub-move sequence of the turn
// (head rule ignored: a superset) that compares die_filter with
// die_candidates at every node.
//   hipcc -O2 -std=c++17 -o /tmp/bf_stats tools/diag/bf_stats.cpp && /tmp/bf_stats
#include <cstdio>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

static bool binds_at(const Side& s, uint32_t low, int d) {
  const uint32_t C = die_candidates(s.O, s.P, d);
  return die_filter(s.O, s.S1o, block_info_low(s.O, low), C, d) != C;
}

// does the block rule remove a candidate anywhere below this node?
// dice: remaining dice (two-dice: the other die; doubles: k copies)
static bool binds_dbl(const Side& s, uint32_t low, int d, int left) {
  if (left == 0) return false;
  if (binds_at(s, low, d)) return true;
  uint32_t L = die_candidates(s.O, s.P, d);
  while (L) {
    const int p = __builtin_ctz(L);
    L &= L - 1u;
    Side c = s;
    apply_die(c, p, d);
    if (binds_dbl(c, low, d, left - 1)) return true;
  }
  return false;
}

static bool binds_two(const Side& s, uint32_t low, int a, int b) {
  if (binds_at(s, low, a) || binds_at(s, low, b)) return true;
  for (int k = 0; k < 2; ++k) {
    const int x = k ? b : a, y = k ? a : b;
    uint32_t L = die_candidates(s.O, s.P, x);
    while (L) {
      const int p = __builtin_ctz(L);
      L &= L - 1u;
      Side c = s;
      apply_die(c, p, x);
      if (binds_at(c, low, y)) return true;
    }
  }
  return false;
}

int main() {
  const int n = 4096, plies = 400;
  long two = 0, two_nobf = 0, two_binds = 0, bad = 0;
  long new_bf = 0, dbl = 0, dbl_nobf = 0, dbl_binds = 0;
  for (int e = 0; e < n; ++e) {
    Side s = side_start(e & 1);
    s.t = 0;
    int4 st = make_int4(0, 0, 0, 0);
    for (int p = 0; p < plies; ++p) {
      uint32_t R[4], r[4];
      ply_block(s.t, (uint32_t)e, 1u, 2u, R);
      ply_words_of(R, s.t, 0, r);
      int d0, d1;
      dice_from(r[0], 0, d0, d1);
      const uint32_t low = block_lowmask(s.P);
      const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
      const bool bf = turn_block_free(s.O, s.S1o, s.P, low, dh, dl);
      new_bf += bf;
      if (dh != dl) {
        ++two;
        const bool b = binds_two(s, low, dh, dl);
        two_nobf += !bf;
        two_binds += b;
        bad += bf && b;
      } else {
        ++dbl;
        const bool b = binds_dbl(s, low, dh, 4);
        dbl_nobf += !bf;
        dbl_binds += b;
        bad += bf && b;
      }
      TurnOut o;
      int tm, tr;
      env_ply_full(s, st, r, (uint32_t)e, 1u, 2u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
    }
  }
  printf("two-dice turns %ld: block-bound by the test %ld, rule really binds %ld\n", two, two_nobf, two_binds);
  printf("doubles turns %ld: block-bound by the test %ld, rule really binds %ld\n", dbl, dbl_nobf, dbl_binds);
  printf("unsound (called block-free, the rule binds): %ld\n", bad);
  printf("turns block-free by turn_block_free: %ld of %ld\n", new_bf, two + dbl);
  return 0;
}
