#!/bin/bash
# DIAGNOSTIC (round 5): k_step<true> builds with per-wave clocks
# (tools/diag/kstep_full_clock.py): kclk (the product turn), kclk_nolate
# (the later sub-moves' cooperative checks skipped), kclk_noroot (the root
# search skipped: M = 4 from the filtered list) -- the last two give wrong
# turns, timing only.
set -euo pipefail
cd "$(dirname "$0")/../.."
OLD1='  uint32_t R[4];
  if constexpr (kFull)
    ply(s, st, a.g, (uint32_t)i, valid, a.play, a.dice, a.max_steps, a.autoreset != 0, o, term, trunc, R,
        true);'
NEW1='  uint32_t R[4];
  int kd_bd = 0, kd_b2 = 0, kd_sr = 0;
  if constexpr (kFull) {
    uint32_t R0[4], r0[4];
    ply_block(s.t, a.g.env0 + (uint32_t)i, a.g.k0, a.g.k1, R0);
    ply_words_of(R0, s.t, a.g.dice_mode, r0);
    int e0, e1;
    dice_from(r0[0], a.g.dice_mode, e0, e1);
    const int eh = e0 > e1 ? e0 : e1, el = e0 > e1 ? e1 : e0;
    uint32_t fw0;
    const uint32_t bs0 = turn_block_set_sl(s.O, s.S1o, s.P, block_lowmask(s.P), eh, el, fw0);
    bool sr = false;
    if (valid && bs0 && eh == el) {
      const int hl = (s.ft_own && (eh == 3 || eh == 4 || eh == 6)) ? 2 : 1;
      const uint32_t Lh = die_candidates(s.O, s.P, eh);
      const uint32_t Lb = Lh & ~block_reject_w(s.O, s.S1o, fw0, Lh, eh);
      sr = f4_safe_bound(s, eh, hl, bs0) < 4 && Lb != 0u;
    }
    kd_bd = __builtin_popcountll(__ballot(valid && bs0 && eh == el));
    kd_b2 = __builtin_popcountll(__ballot(valid && bs0 && eh != el));
    kd_sr = __builtin_popcountll(__ballot(sr));
  }
  const uint64_t kc0 = __builtin_amdgcn_s_memtime();
  if constexpr (kFull)
    ply(s, st, a.g, (uint32_t)i, valid, a.play, a.dice, a.max_steps, a.autoreset != 0, o, term, trunc, R,
        true);'
OLD2='  store_outs(a.out, (size_t)i, s, o, term, trunc, wave_lds, i - (int)(threadIdx.x & 63) + 64 <= a.n);
}'
NEW2='  store_outs(a.out, (size_t)i, s, o, term, trunc, wave_lds, i - (int)(threadIdx.x & 63) + 64 <= a.n);
  if constexpr (kFull) {
    const uint64_t kc1 = __builtin_amdgcn_s_memtime();
    const int ln = (int)(threadIdx.x & 63);
    if (a.out.reward && ln < 4)
      a.out.reward[i] = ln == 0 ? (int32_t)(kc1 - kc0) : (ln == 1 ? kd_bd : (ln == 2 ? kd_b2 : kd_sr));
  }
}'
bash tools/diag/build_patch.sh kclk kernels_rollout.h "$OLD1" "$NEW1" kernels_rollout.h "$OLD2" "$NEW2"
bash tools/diag/build_patch.sh kclk_nolate kernels_rollout.h "$OLD1" "$NEW1" kernels_rollout.h "$OLD2" "$NEW2" \
  full4_wave.h '    if (__ballot(chk) != 0ull) {  // wave-uniform' '    if (false && __ballot(chk) != 0ull) {'
bash tools/diag/build_patch.sh kclk_noroot kernels_rollout.h "$OLD1" "$NEW1" kernels_rollout.h "$OLD2" "$NEW2" \
  full4_wave.h '    coop_depth_w(s, fw, dh, hl0, srch ? Lb : 0u, 3, lane, r0);' '    r0[0] = r0[1] = r0[2] = Lb;'
