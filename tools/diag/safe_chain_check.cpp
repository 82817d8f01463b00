// DIAGNOSTIC (host): f4_safe_bound (narde_rules.h) in its chain form against
// its first form (restated here as safe_single).  The first form counted the
// sub-moves whose landing can never fill a failing window (min(count, 2) per
// such source, the head at most hl); the chain form also counts each
// checker's further steps over such landings, as f4_chain_bound does for
// block-free turns.  Claim: >= 4 at the root gives
// M = 4 and every C_k = L_k (a legal sub-move lowers it by at most one: the
// moved checker keeps the rest of its chain).  Checked here on every legal
// path of the turn (each node at depth k must still reach 4 - k), on FULL4
// self-play and on random block-prone positions; prints how many of the
// searched turns (block-bound doubles, f4_safe_bound < 4) it would settle.
//   hipcc -O2 -std=c++17 -o /tmp/safe_chain_check tools/diag/safe_chain_check.cpp && /tmp/safe_chain_check
#include <cstdio>
#include <random>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

static int safe_single(const Side& s, int d, int hl, uint32_t ws) {
  if (ws == ~0u) return 0;
  const uint32_t C = die_candidates(s.O, s.P, d);
  const uint32_t opens = f4_bearoff_fixed(s) ? 0u : ((1u << d) - 1u);
  const uint32_t bad = ws & (~s.O | C | opens);
  uint32_t L = C & ~(bad << d);
  if (hl <= 0) L &= ~HEAD;
  const uint32_t body = L & ~HEAD;
  const int head = (L & HEAD) ? ((hl >= 2 && !(s.S1o & HEAD)) ? 2 : 1) : 0;
  return __builtin_popcount(body) + __builtin_popcount(body & ~s.S1o) + head;
}

static int depth_n(const Side& s, uint32_t low, int d, int hl, int n) {
  switch (n) {
    case 1: return f4_depth<1>(s, low, d, hl, false);
    case 2: return f4_depth<2>(s, low, d, hl, false);
    case 3: return f4_depth<3>(s, low, d, hl, false);
    case 4: return f4_depth<4>(s, low, d, hl, false);
    default: return 0;
  }
}

// every legal path from this node (k sub-moves played) still reaches 4
static long verify(const Side& s, uint32_t low, int d, int hl, int k) {
  if (k == 4) return 0;
  if (depth_n(s, low, d, hl, 4 - k) < 4 - k) return 1;
  uint32_t L = legal1(s, low, d, false);
  if (hl <= 0) L &= ~HEAD;
  long bad = 0;
  while (L) {
    const int p = __builtin_ctz(L);
    L &= L - 1u;
    Side c = s;
    apply_die(c, p, d);
    bad += verify(c, low, d, hl - (p == 23 ? 1 : 0), k + 1);
  }
  return bad;
}

static long turns = 0, bound = 0, fast_old = 0, fast_new = 0, violations = 0;

static void check(const Side& s, int d, int hl) {
  const uint32_t low = block_lowmask(s.P);
  if (turn_block_free(s.O, s.S1o, s.P, low, d, d)) return;
  ++bound;
  const uint32_t ws = dbl_block_windows(s.O, s.S1o, s.P, low, d, 4);
  const bool old = safe_single(s, d, hl, ws) >= 4;
  const bool neu = f4_safe_bound(s, d, hl, ws) >= 4;
  fast_old += old;
  if (old && !neu) ++violations;  // the chain form must not lose a settled turn
  if (neu) {
    fast_new += 1;
    violations += verify(s, low, d, hl, 0);
  }
}

int main() {
  // FULL4 self-play: every doubles roll of every position reached
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
      for (int d = 1; d <= 6; ++d) {
        ++turns;
        check(s, d, (s.ft_own && (d == 3 || d == 4 || d == 6)) ? 2 : 1);
      }
      TurnOut o;
      int tm, tr;
      env_ply_full(s, ST[e], r, (uint32_t)e, 7u, 9u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
    }
  const long sp_turns = turns, sp_bound = bound, sp_old = fast_old, sp_new = fast_new;
  // random block-prone positions: an own 6-window with 0-4 holes, the
  // opponent mostly above it (so the rule applies)
  std::mt19937 rng(4242);
  for (int k = 0; k < 400000; ++k) {
    Side s = side_start(0u);
    for (int j = 0; j < 3; ++j) { s.own.w[j] = 0u; s.opp.w[j] = 0u; }
    const int i0 = (int)(rng() % 19);
    uint32_t Hm = 0u;
    const int holes = (int)(rng() % 5);
    while (__builtin_popcount(Hm) < holes) Hm |= 1u << (i0 + (int)(rng() % 6));
    int left = 15;
    for (int p = i0; p < i0 + 6 && left > 0; ++p)
      if (!((Hm >> p) & 1u)) {
        const int c = 1 + (rng() % 3 == 0 ? 1 : 0);
        for (int j = 0; j < c && left > 0; ++j, --left) nib_inc(s.own, p);
      }
    while (left > 0) {
      const int p = (int)(rng() % 24);
      if (((Hm >> p) & 1u) && (rng() & 1u)) continue;
      nib_inc(s.own, p);
      --left;
    }
    uint32_t used = 0u;
    for (int p = 0; p < 24; ++p) used |= nib_get(s.own, p) ? (1u << p) : 0u;
    const int lo_min = rng() % 4 == 0 ? 0 : i0 + 1;
    int placed = 0;
    for (int t = 0; t < 400 && placed < 15; ++t) {
      const int p = lo_min + (int)(rng() % (uint32_t)(24 - lo_min));
      if ((used >> p) & 1u) continue;
      nib_inc(s.opp, p);
      ++placed;
    }
    s.ft_own = rng() % 8 == 0 ? 1u : 0u;
    side_masks(s);
    const int d = 1 + (int)(rng() % 6);
    ++turns;
    check(s, d, (s.ft_own && (d == 3 || d == 4 || d == 6)) ? 2 : 1);
  }
  printf("self-play: doubles turns %ld, block-bound %ld, settled by the first form %ld, by the chain form %ld\n",
         sp_turns, sp_bound, sp_old, sp_new);
  printf("random: block-bound %ld, settled by the first form %ld, by the chain form %ld\n", bound - sp_bound,
         fast_old - sp_old, fast_new - sp_new);
  printf("violations %ld\n", violations);
  return violations != 0;
}
