// DIAGNOSTIC (host): how FULL4 doubles turns of random self-play split over
// the device turn's shortcuts -- which ones still need a search.
//   hipcc -O2 -std=c++17 -o /tmp/full4_stats tools/diag/full4_stats.cpp && /tmp/full4_stats
#include <cstdio>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

// windows i..i+5 (bit i) with at most 2 points missing from O (bit-sliced
// count of the holes over the 6 shifted masks)
static uint32_t windows_le2_holes(uint32_t O) {
  const uint32_t h = ~O & MASK24;
  uint32_t s0 = 0, s1 = 0, s2 = 0;  // 3-bit counter per window start
  for (int k = 0; k < 6; ++k) {
    const uint32_t x = (h >> k);
    const uint32_t c0 = s0 & x;
    s0 ^= x;
    const uint32_t c1 = s1 & c0;
    s1 ^= c0;
    s2 |= c1;
  }
  // count <= 2: s2 == 0 and not (s1 && s0)
  return ~s2 & ~(s1 & s0) & MASK24;
}

// exact own-checker count per point class: counts >= j masks
static uint32_t ge_mask(const Nib& b, uint32_t j) {
  uint32_t m = 0;
  for (int p = 0; p < 24; ++p) m |= (nib_get(b, p) >= j ? 1u : 0u) << p;
  return m;
}

// sum over checkers of their chain length (block-free, no bear-off change)
static int chain_total(const Side& s, int d, int hl) {
  int tot = 0;
  for (int p = 0; p < 24; ++p) {
    int c = nib_get(s.own, p);
    if (!c) continue;
    int ch = 0;
    for (int q = p - d; ch < 4; q -= d) {
      if (q < 0) {
        if ((s.O >> 6) == 0u) ++ch;  // bears off: only if all home already
        break;
      }
      if ((s.P >> q) & 1u) break;
      ++ch;
    }
    if (p == 23) c = c < hl ? c : hl;
    tot += c * ch;
  }
  return tot;
}

int main() {
  const int n = 4096, plies = 400;
  long dbl = 0, fast = 0, cb7 = 0, searched = 0, s_bf = 0, s_exact = 0, s_exact4 = 0, nobf = 0;
  long nobf2_all = 0, nobf_but_bf2 = 0, bad_fixed = 0, bad_exact = 0, two = 0, pair_tasks = 0, pair_nobf = 0, pair_n = 0;
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
      if (d0 != d1) {
        ++two;
        const uint32_t low = block_lowmask(s.P);
        const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
        const bool bf = turn_block_free(s.O, s.S1o, s.P, low, dh, dl);
        const uint32_t Lh = legal1(s, low, dh, bf), Ll = legal1(s, low, dl, bf);
        const bool all_h = bf && f4_lower_bound(s.O, s.S1o, s.P, dl, 1) >= 2;
        const bool all_l = bf && f4_lower_bound(s.O, s.S1o, s.P, dh, 1) >= 2;
        if (!bf) {
          ++nobf2_all;
          const uint32_t A = s.O | land_step(s.O, s.P, dh) | land_step(s.O, s.P, dl);
          const uint32_t U = A | land_step(A, s.P, dh) | land_step(A, s.P, dl);
          const bool bf2 = (runs6(U) & low & windows_le2_holes(s.O)) == 0u;
          if (bf2) ++nobf_but_bf2;
        }
        if ((!all_h && Lh) || (!all_l && Ll)) {
          ++pair_tasks;
          if (!bf) ++pair_nobf;
          pair_n += (!all_h ? __builtin_popcount(Lh) : 0) + (!all_l ? __builtin_popcount(Ll) : 0);
        }
      }
      if (d0 == d1) {
        ++dbl;
        const uint32_t low = block_lowmask(s.P);
        const bool bf = turn_block_free(s.O, s.S1o, s.P, low, d0, d0);
        const int hl0 = (s.ft_own && (d0 == 3 || d0 == 4 || d0 == 6)) ? 2 : 1;
        const bool f = bf && f4_lower_bound(s.O, s.S1o, s.P, d0, hl0) >= 4;
        const int cb0 = (bf && !f) ? f4_chain_bound(s.O, s.S1o, s.P, d0, hl0) : 0;
        const uint32_t L = legal1(s, low, d0, bf);
        if (!bf) ++nobf;
        if (f) ++fast;
        else if (cb0 >= 7 && L) ++cb7;
        else if (L) {
          ++searched;
          if (bf) {
            ++s_bf;
            // outside-home checkers (points >= 6)
            int outside = 0;
            for (int q = 6; q < 24; ++q) outside += nib_get(s.own, q);
            const bool nob = (s.O >> 6) == 0u || outside >= 4;
            if (nob != f4_bearoff_fixed(s)) ++bad_fixed;
            if (nob) {
              ++s_exact;
              const int T = chain_total(s, d0, hl0);
              if (T >= 4) ++s_exact4;
              // the search's M and C_0 against the exact count
              uint32_t C = f4_keep<3>(s, low, d0, hl0, L, bf);
              int M = 4;
              if (!C) { C = f4_keep<2>(s, low, d0, hl0, L, bf); M = 3; }
              if (!C) { C = f4_keep<1>(s, low, d0, hl0, L, bf); M = 2; }
              if (!C) { C = L; M = 1; }
              const int Me = f4_exact_moves(s, d0, hl0);
              if (Me != M || C != L || (T < 4 ? T : 4) != Me) ++bad_exact;
            }
          }
        }
      }
      TurnOut o;
      int tm, tr;
      env_ply_full(s, st, r, (uint32_t)e, 1u, 2u, false, 0, 0, 0, false, 0ull, 1000, true, o, tm, tr);
    }
  }
  printf("doubles turns %ld: fast %ld, chain>=7 %ld, searched %ld (non-bf lanes overall %ld)\n", dbl, fast, cb7,
         searched, nobf);
  printf("searched & block-free %ld: exact-chain applicable %ld, of which total>=4 %ld\n", s_bf, s_exact, s_exact4);
  printf("two-dice turns %ld: needing pair checks %ld (non-bf %ld), tasks %ld\n", two, pair_tasks, pair_nobf, pair_n);
  printf("two-dice non-bf %ld, of which block-free by the 2-hole window test %ld\n", nobf2_all, nobf_but_bf2);
  printf("mismatches: bearoff_fixed %ld, exact M/C vs search %ld\n", bad_fixed, bad_exact);
  return 0;
}
