// kernels_full4.h -- the FULL4 list query k_legal_full (DESIGN.md section
// 10); the wave-cooperative turn itself is full4_wave.h.
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

#include "full4_wave.h"

namespace {

// FULL4 first-sub-move set C_0 and max dice M for the given (or the next
// device) dice: the turn engine run on a copy with a play whose first
// sub-move is invalid, so nothing is applied.
__global__ void __launch_bounds__(kBlock) k_legal_full(Planes pl, int n, Rng g,
                                                       const uint8_t* __restrict__ dice2,
                                                       uint64_t* __restrict__ out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < n;  // no early exit: the turn is wave-cooperative
  Side s = valid ? side_from_record(pl.p0[i], pl.p1[i]) : side_start(0u);
  int d0 = 1, d1 = 2;
  bool bad = false;  // a given die outside 1..6: no legal move
  if (dice2) {
    if (valid) {
      d0 = dice2[2 * i];
      d1 = dice2[2 * i + 1];
      bad = (uint32_t)(d0 - 1) > 5u || (uint32_t)(d1 - 1) > 5u;
      if (bad) { d0 = 1; d1 = 2; }
    }
  } else {
    uint32_t r[4];
    ply_draw(g, s.t, (uint32_t)i, r);
    dice_from(r[0], g.dice_mode, d0, d1);
  }
  const uint32_t w[4] = {0u, 0u, 0u, 0u};
  TurnOut o;
  // play word of -1s: nothing is applied
  coop_turn_full(s, d0, d1, true, ~0ull, w, o, (int)(threadIdx.x & 63));
  if (valid) out[i] = bad ? 0ull : o.legal;
}

}  // namespace
