// DIAGNOSTIC (host): the cost of the device's doubles depth searches
// (coop_run mode 0: per first-sub-move source, f4_depth<3> on its child with
// no block-free cut) over FULL4 self-play, and what an upper bound from the
// block-rule-free relaxation (f4_exact_moves / f4_open_moves of the child:
// the block rule only removes options, so their count bounds the true one)
// would prune.  Per searched turn: nodes of the most expensive source (the
// wave waits for its slowest lane) and in total; must print 0 unsound prunes.
//   hipcc -O2 -std=c++17 -o /tmp/dsearch_stats tools/diag/dsearch_stats.cpp && /tmp/dsearch_stats
#include <cstdio>
#include <vector>
#include <algorithm>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

static long g_nodes;

// f4_depth<N, 0> with a node count
template <int N>
static int depth_count(const Side& s, uint32_t low, int d, int hl) {
  ++g_nodes;
  uint32_t L = legal1(s, low, d, false);
  if (hl <= 0) L &= ~HEAD;
  if (!L) return 0;
  if constexpr (N == 1) {
    return 1;
  } else {
    int best = 1;
    while (L && best < N) {
      const int p = __builtin_ctz(L);
      L &= L - 1u;
      Side c = s;
      apply_die(c, p, d);
      const int v = 1 + depth_count<N - 1>(c, low, d, hl - (p == 23 ? 1 : 0));
      best = v > best ? v : best;
    }
    return best;
  }
}

// the relaxed (no block rule) sub-move count of a doubles node, capped at k
static int relaxed(const Side& s, int d, int hl, int k) {
  const int T = f4_exact_moves(s, d, hl);
  const int M = f4_bearoff_fixed(s, k) ? T : f4_open_moves(s, d, hl, T);
  return M < k ? M : k;
}

static int depth_n(int n, const Side& s, uint32_t low, int d, int hl) {
  return n <= 0 ? 0 : (n == 1 ? depth_count<1>(s, low, d, hl) : (n == 2 ? depth_count<2>(s, low, d, hl) : depth_count<3>(s, low, d, hl)));
}

int main() {
  const int n = 64 * 64, plies = 600;
  static Side S[64 * 64];
  static int4 ST[64 * 64];
  for (int e = 0; e < n; ++e) {
    S[e] = side_start(e & 1);
    ST[e] = make_int4(0, 0, 0, 0);
  }
  long turns = 0, searched = 0, unsound = 0, later_need = 0, later_bf = 0, later_safe = 0, later_either = 0, later_root = 0, need2 = 0, later_root2 = 0;
  std::vector<long> maxn, maxp, sumn, sump;
  for (int p = 0; p < plies; ++p)
    for (int e = 0; e < n; ++e) {
      Side& s = S[e];
      uint32_t R[4], r[4];
      ply_block(s.t, (uint32_t)e, 11u, 13u, R);
      ply_words_of(R, s.t, 0, r);
      int d0, d1;
      dice_from(r[0], 0, d0, d1);
      ++turns;
      if (d0 == d1) {
        const int d = d0;
        const uint32_t low = block_lowmask(s.P);
        const uint32_t bs = turn_block_set(s.O, s.S1o, s.P, low, d, d);
        const int hl0 = (s.ft_own && (d == 3 || d == 4 || d == 6)) ? 2 : 1;
        const bool fast = bs != 0u && f4_safe_bound(s, d, hl0, bs) >= 4;
        uint32_t L = legal1(s, low, d, false);
        if (bs != 0u && !fast && L) {
          ++searched;
          long mx = 0, sm = 0, mxp = 0, smp = 0;
          uint32_t m = L;
          while (m) {
            const int q = __builtin_ctz(m);
            m &= m - 1u;
            const int hl2 = hl0 - (q == 23 ? 1 : 0);
            Side c = s;
            apply_die(c, q, d);
            g_nodes = 0;
            const int dep = depth_count<3>(c, low, d, hl2);
            mx = std::max(mx, g_nodes);
            sm += g_nodes;
            // pruned: search only as deep as the relaxed bound allows
            const int ub = relaxed(c, d, hl2, 3);
            g_nodes = 0;
            const int dep2 = depth_n(ub, c, low, d, hl2);
            mxp = std::max(mxp, g_nodes);
            smp += g_nodes;
            if (dep2 != dep) ++unsound;
          }
          maxn.push_back(mx); sumn.push_back(sm); maxp.push_back(mxp); sump.push_back(smp);
          // the later sub-moves of this turn, played as env_turn_full plays
          // them: how many need the search (need = M - k - 1 > 0) and how
          // many of those the block-free shortcut (dbl_block_free(node,
          // M - k)) settles
          {
            Side t = s;
            TurnOut o2;
            const uint32_t w[4] = {r[1], r[2], r[1] * 0x85EBCA6Bu, r[2] * 0xC2B2AE35u};
            // M and C_0 from the host turn on a copy with an invalid play (nothing applied)
            env_turn_full(t, d, d, true, ~0ull, w, o2);
            const int M = o2.max_dice;
            Side u = s;
            int hl = hl0;
            uint32_t C = (uint32_t)(o2.legal & 0xFFFFFFu);
            for (int k = 0; k < M; ++k) {
              if (k > 0) {
                uint32_t Lk = legal1(u, low, d, false);
                if (hl <= 0) Lk &= ~HEAD;
                const int need = M - k - 1;
                if (need > 0) {
                  ++later_need;
                  const bool bfk = dbl_block_free(u.O, u.S1o, u.P, low, d, M - k);
                  const bool sfk = f4_safe_bound(u, d, hl, dbl_block_windows(u.O, u.S1o, u.P, low, d, M - k)) >= M - k;
                  later_bf += bfk;
                  later_safe += sfk;
                  later_either += bfk || sfk;
                  // the same with the root's failing windows (no window test at the node)
                  const bool srk = f4_safe_bound(u, d, hl, bs) >= M - k;
                  later_root += srk;
                  if (srk && f4_keep_rt(u, low, d, hl, Lk, need, false) != Lk) ++unsound;
                  need2 += need == 2;
                  later_root2 += srk && need == 2;
                  // the safe bound settles the node: every source keeps M - k - 1
                  if (sfk && f4_keep_rt(u, low, d, hl, Lk, need, false) != Lk) ++unsound;
                }
                C = need > 0 ? f4_keep_rt(u, low, d, hl, Lk, need, false) : Lk;
              }
              if (!C) break;
              const uint32_t wk = k == 0 ? w[0] : (k == 1 ? w[1] : (k == 2 ? w[2] : w[3]));
              const int q = select_bit(C, (int)mulhi_u32(wk, (uint32_t)__builtin_popcount(C)));
              apply_die(u, q, d);
              hl -= q == 23 ? 1 : 0;
            }
          }
        }
      }
      TurnOut o;
      int tm, tr;
      env_ply_full(s, ST[e], r, (uint32_t)e, 11u, 13u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
    }
  auto pct = [](std::vector<long> v, double q) { std::sort(v.begin(), v.end()); return v.empty() ? 0L : v[(size_t)(q * (v.size() - 1))]; };
  auto mean = [](const std::vector<long>& v) { double t = 0; for (long x : v) t += x; return v.empty() ? 0.0 : t / v.size(); };
  printf("turns %ld, searched (block-bound doubles, not fast) %ld (%.3f %%)\n", turns, searched, 100.0 * searched / turns);
  printf("max nodes per turn (slowest source): mean %.1f p50 %ld p90 %ld p99 %ld max %ld\n", mean(maxn), pct(maxn, .5), pct(maxn, .9), pct(maxn, .99), pct(maxn, 1.0));
  printf("  with the relaxed bound:             mean %.1f p50 %ld p90 %ld p99 %ld max %ld\n", mean(maxp), pct(maxp, .5), pct(maxp, .9), pct(maxp, .99), pct(maxp, 1.0));
  printf("total nodes per turn: mean %.1f -> %.1f\n", mean(sumn), mean(sump));
  printf("later sub-moves that search: %ld, settled by the block-free shortcut: %ld, by f4_safe_bound: %ld, by either: %ld\n",
         later_need, later_bf, later_safe, later_either);
  printf("  by f4_safe_bound with the root's windows: %ld (need 2: %ld of %ld)\n", later_root, later_root2, need2);
  printf("unsound prunes (depth differs): %ld\n", unsound);
  return unsound != 0;
}
