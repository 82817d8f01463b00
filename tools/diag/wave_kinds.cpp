// DIAGNOSTIC (round 4, host): what each 64-lane wave of the FULL4 rollout
// meets per ply -- the kinds of turn by game phase.  Plays N envs of
// random-legal FULL4 self-play from the start (the device's ply: Philox
// draws, turn_block_set_sl, env_turn_full) and, per ply, counts waves with
// a block-bound doubles lane (ply_bound_turn), waves with block-bound
// two-dice lanes only, free waves, and the block-bound doubles lanes that
// search (not settled by f4_safe_bound).
// Build: g++ -O2 -std=c++17 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -x c++ ... (see gpu_kinds notes)
#include <cstdio>
#include <vector>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384, plies = argc > 2 ? atoi(argv[2]) : 200;
  const uint64_t seed = 0;
  std::vector<Side> S(n);
  for (int i = 0; i < n; ++i) {
    uint32_t r[4];
    philox4x32_10(0, (uint32_t)i, 0u, 1u, (uint32_t)seed, (uint32_t)(seed >> 32), r);
    S[i] = side_reset(r[0]);
    S[i].t = 0;
  }
  printf("ply,waves,bound_dbl_waves,bound_two_only_waves,bound_dbl_lanes,search_lanes,bound_two_lanes\n");
  for (int p = 0; p < plies; ++p) {
    int wbd = 0, wb2 = 0, lbd = 0, lsr = 0, lb2 = 0;
    for (int w0 = 0; w0 < n; w0 += 64) {
      bool anyd = false, any2 = false;
      for (int i = w0; i < w0 + 64 && i < n; ++i) {
        Side& s = S[i];
        uint32_t R[4], r[4];
        ply_block(s.t, (uint32_t)i, (uint32_t)seed, (uint32_t)(seed >> 32), R);
        ply_words_of(R, s.t, 0, r);
        int d0, d1;
        dice_from(r[0], 0, d0, d1);
        const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
        uint32_t fw;
        const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, block_lowmask(s.P), dh, dl, fw);
        if (bs && dh == dl) {
          anyd = true;
          ++lbd;
          const int hl = (s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1;
          if (f4_safe_bound(s, dh, hl, bs) < 4) ++lsr;
        } else if (bs) {
          any2 = true;
          ++lb2;
        }
        uint32_t w[4];
        turn_words(r, w);
        const uint32_t mb = s.black;
        TurnOut o;
        env_turn_full(s, d0, d1, false, 0ull, w, o);
        int4 st = make_int4(0, 0, 0, 0);
        int tm, tr;
        ply_close(s, st, o.term, o.reward, mb, r[3], 1000, true, tm, tr);
      }
      wbd += anyd;
      wb2 += !anyd && any2;
    }
    printf("%d,%d,%d,%d,%d,%d,%d\n", p, (n + 63) / 64, wbd, wb2, lbd, lsr, lb2);
  }
  return 0;
}
