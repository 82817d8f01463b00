// DIAGNOSTIC (round 5, host): the cooperative checks of block-bound doubles
// turns that search (ply_bound_turn_c0): per searching turn of random-legal
// FULL4 self-play at 65,536 envs, the later sub-moves' passes (k = 1, 2) and
// how many a safe bound at the node (f4_safe_bound >= need + 1) would settle,
// checked against the pass result (C_k == L_k).  Build:
//   g++ -O2 -std=c++17 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -x c++ tools/diag/search_pass_stats.cpp
#include <cstdio>
#include <vector>
#include "../../gym-narde_amd/csrc/narde_rules.h"
using namespace narde;
// one searching doubles lane's turn as ply_bound_turn_c0 plays it; counts the
// cooperative passes at k = 1, 2 and those a safe bound at the node settles
static long turns = 0, pass_k[4] = {0}, skip_k[4] = {0}, wrong = 0, mhist[5] = {0};
template <int N> static int dep_w(const Side& c, uint32_t fw, int d, int hl) { return f4_depth_w<N>(c, fw, d, hl); }
static int depth_need(const Side& c, uint32_t fw, int d, int hl, int need) {
  return need == 1 ? dep_w<1>(c, fw, d, hl) : (need == 2 ? dep_w<2>(c, fw, d, hl) : dep_w<3>(c, fw, d, hl));
}
static void search_turn(Side s, int dh, int hl0, uint32_t bs, uint32_t fw, const uint32_t w[4]) {
  uint32_t Lh = die_candidates(s.O, s.P, dh);
  const uint32_t Lb = Lh & ~block_reject_w(s.O, s.S1o, fw, Lh, dh);
  if (f4_safe_bound(s, dh, hl0, bs) >= 4 || !Lb) return;
  ++turns;
  uint32_t r0[3] = {0, 0, 0};
  for (uint32_t m = Lb; m; m &= m - 1) {
    const int p = __builtin_ctz(m);
    Side c = s; apply_die(c, p, dh);
    const int dep = dep_w<3>(c, fw, dh, hl0 - (p == 23));
    for (int j = 0; j < 3; ++j) if (dep >= j + 1) r0[j] |= 1u << p;
  }
  const int M = r0[2] ? 4 : (r0[1] ? 3 : (r0[0] ? 2 : 1));
  const uint32_t Ch = r0[2] ? r0[2] : (r0[1] ? r0[1] : (r0[0] ? r0[0] : Lb));
  ++mhist[M];
  const int n = __builtin_popcount(Ch);
  int p = select_bit(Ch, (int)mulhi_u32(w[0], (uint32_t)n));
  apply_die(s, p, dh);
  int hl = hl0 - (p == 23);
  for (int k = 1; k < 4; ++k) {
    if (k >= M) break;
    uint32_t Lk = die_candidates_sl(s.O, s.P, dh);
    Lk &= ~block_reject_w(s.O, s.S1o, fw, Lk, dh);
    if (hl <= 0) Lk &= ~HEAD;
    const int need = M - k - 1;
    if (need > 0) {
      ++pass_k[k];
      uint32_t C = 0;
      for (uint32_t m = Lk; m; m &= m - 1) {
        const int q = __builtin_ctz(m);
        Side c = s; apply_die(c, q, dh);
        if (depth_need(c, fw, dh, hl - (q == 23), need) >= need) C |= 1u << q;
      }
      if (f4_safe_bound(s, dh, hl, bs) >= need + 1) { ++skip_k[k]; if (C != Lk) ++wrong; }
      Lk = C;
    }
    const uint32_t wk = k == 1 ? w[1] : (k == 2 ? w[2] : w[3]);
    p = select_bit(Lk, (int)mulhi_u32(wk, (uint32_t)__builtin_popcount(Lk)));
    apply_die(s, p, dh);
    hl -= p == 23;
  }
}
int main(int argc, char** argv) {
  const int n = 65536, plies = argc > 1 ? atoi(argv[1]) : 300;
  std::vector<Side> S(n);
  for (int i = 0; i < n; ++i) { uint32_t r[4]; philox4x32_10(0,(uint32_t)i,0u,1u,0u,0u,r); S[i]=side_reset(r[0]); S[i].t=0; }
  for (int p = 0; p < plies; ++p) for (int i = 0; i < n; ++i) {
    Side& s = S[i];
    uint32_t R[4], r[4];
    ply_block(s.t, (uint32_t)i, 0u, 0u, R); ply_words_of(R, s.t, 0, r);
    int d0, d1; dice_from(r[0], 0, d0, d1);
    const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
    uint32_t fw; const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, block_lowmask(s.P), dh, dl, fw);
    uint32_t w[4]; turn_words(r, w);
    if (bs && dh == dl) search_turn(s, dh, (s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1, bs, fw, w);
    const uint32_t mb = s.black; TurnOut o;
    env_turn_full(s, d0, d1, false, 0ull, w, o);
    int4 st = make_int4(0,0,0,0); int tm, tr;
    ply_close(s, st, o.term, o.reward, mb, r[3], 1000, true, tm, tr);
  }
  printf("searching turns %ld  M hist 1:%ld 2:%ld 3:%ld 4:%ld\n", turns, mhist[1], mhist[2], mhist[3], mhist[4]);
  for (int k = 1; k < 3; ++k) printf("k=%d passes %ld  settled by the node's safe bound %ld\n", k, pass_k[k], skip_k[k]);
  printf("safe-bound settled but C != L: %ld\n", wrong);
}
