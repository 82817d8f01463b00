// kernels_state.h -- state management and the list queries: reset, set/get state, peek dice, get_valid_moves, apply, statistics, block rule
// Part of the one translation unit narde.hip (included there, in order);
// not a standalone header.
#pragma once

namespace {

// ------------------------------------------------------------------ kernels
// init_t >= 0: also set the RNG counter (create); < 0: keep each env's counter.
// opening (optional) u8[n][pairs][2]: each env's opening draws (white roll,
// black roll) in draw order; as narde_env.py:111-117 the first pair of
// different dice decides (higher roll moves first), pairs with a die outside
// 1..6 are padding, and a row with no deciding pair takes the device draw.
__global__ void __launch_bounds__(kBlock) k_reset(Planes pl, int n, Rng g, uint32_t epoch,
                                                  const uint8_t* __restrict__ mask, int64_t init_t,
                                                  const uint8_t* __restrict__ opening, int pairs) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
  uint32_t r[4];
  draw(g, epoch, (uint32_t)i, 1u, r);
  Side s = side_reset(r[0]);
  if (opening) {
    const uint8_t* row = opening + (size_t)i * (size_t)pairs * 2;
    for (int k = 0; k < pairs; ++k) {
      const int w = row[2 * k], b = row[2 * k + 1];
      if ((uint32_t)(w - 1) <= 5u && (uint32_t)(b - 1) <= 5u && w != b) {
        s = side_start(w > b ? 0u : 1u);
        break;
      }
    }
  }
  s.t = init_t >= 0 ? (uint32_t)init_t : pl.p1[i].w;
  uint4 a, b;
  side_to_record(s, a, b);
  pl.p0[i] = a;
  pl.p1[i] = b;
  pl.stats[i] = make_int4(0, 0, 0, 0);
}

// keep_t: preserve each env's RNG counter (device state); else set it to 0
__global__ void __launch_bounds__(kBlock) k_set_state(Planes pl, int n, const int8_t* __restrict__ board,
                                                      const uint8_t* __restrict__ off,
                                                      const uint8_t* __restrict__ ft,
                                                      const int8_t* __restrict__ player,
                                                      const uint16_t* __restrict__ elapsed, int keep_t) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t t = keep_t ? pl.p1[i].w : 0u;
  uint4 a, b;
  record_from_board(board + (size_t)i * 24, off[2 * i], off[2 * i + 1], ft[2 * i], ft[2 * i + 1],
                    player[i], elapsed ? elapsed[i] : 0u, t, a, b);
  pl.p0[i] = a;
  pl.p1[i] = b;
}

__global__ void __launch_bounds__(kBlock) k_get_state(Planes pl, int n, int8_t* __restrict__ board,
                                                      uint8_t* __restrict__ off, uint8_t* __restrict__ ft,
                                                      int8_t* __restrict__ player,
                                                      uint16_t* __restrict__ elapsed) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  board_from_record(pl.p0[i], pl.p1[i], board ? board + (size_t)i * 24 : nullptr,
                    off ? off + 2 * i : nullptr, ft ? ft + 2 * i : nullptr,
                    player ? player + i : nullptr, elapsed ? elapsed + i : nullptr);
}

__global__ void __launch_bounds__(kBlock) k_set_ply(Planes pl, int n, uint32_t t) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  pl.p1[i].w = t;
}

__global__ void __launch_bounds__(kBlock) k_peek_dice(Planes pl, int n, Rng g, uint8_t* __restrict__ dice) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t r[4];
  ply_draw(g, pl.p1[i].w, (uint32_t)i, r);
  int d0, d1;
  dice_from(r[0], g.dice_mode, d0, d1);
  dice[2 * i] = (uint8_t)d0;
  dice[2 * i + 1] = (uint8_t)d1;
}

__device__ __forceinline__ uint64_t compact_legal(const Legal& l) {
  return (uint64_t)l.L[0] | ((uint64_t)l.L[1] << 24) | ((uint64_t)l.d[0] << 48) |
         ((uint64_t)l.d[1] << 52);
}

__global__ void __launch_bounds__(kBlock) k_legal(Planes pl, int n, Rng g,
                                                  const uint8_t* __restrict__ dice4,
                                                  int16_t* __restrict__ out_count,
                                                  int8_t* __restrict__ out_moves,
                                                  uint64_t* __restrict__ out_compact) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Side s = side_from_record(pl.p0[i], pl.p1[i]);
  Legal l;
  if (dice4) {
    legal_roll(s, dice4 + 4 * i, l);
  } else {
    uint32_t r[4];
    ply_draw(g, s.t, (uint32_t)i, r);
    int d0, d1;
    dice_from(r[0], g.dice_mode, d0, d1);
    legal2(s, d0, d1, l);
  }
  const int nd = l.n;
  out_count[i] = (int16_t)l.count;
  if (out_compact) out_compact[i] = nd <= 2 ? compact_legal(l) : 0ull;
  if (out_moves) {
    int4* row = reinterpret_cast<int4*>(out_moves + (size_t)i * NARDE_MAX_MOVES * 2);
    const int4 neg = make_int4(-1, -1, -1, -1);
#pragma unroll
    for (int q = 0; q < 8; ++q) row[q] = neg;
    int e = 0;
    uint16_t* pairs = reinterpret_cast<uint16_t*>(out_moves + (size_t)i * NARDE_MAX_MOVES * 2);
    for (int k = 0; k < nd; ++k) {
      uint32_t m = l.L[k];
      while (m) {
        const int f = __builtin_ctz(m);
        m &= m - 1u;
        const int to = f - l.d[k] < 0 ? OFF : f - l.d[k];
        pairs[e++] = (uint16_t)((uint32_t)f | ((uint32_t)to << 8));
      }
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_get_stats(Planes pl, int n, int32_t* __restrict__ out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int4 s = pl.stats[i];
  out[3 * i] = s.x; out[3 * i + 1] = s.y; out[3 * i + 2] = s.z;
}

// Per-rank totals of the statistics as kTotalRows partial rows (row b: the
// envs of the b-th contiguous range), int64: one launch, no cross-block
// combine (a last-block combine needs a device-scope fence per block, which
// writes back the XCD's L2); the reader adds the rows.
__global__ void __launch_bounds__(kBlock) k_get_totals(Planes pl, int n, int64_t* __restrict__ rows) {
  __shared__ long long red[kBlock / 64][3];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = (n + kTotalRows - 1) / kTotalRows;
  const int i0 = b * per, i1 = min(n, i0 + per);
  long long e = 0, w = 0, k = 0;
  for (int i = i0 + (int)threadIdx.x; i < i1; i += kBlock) {
    const int4 s = pl.stats[i];
    e += s.x; w += s.y; k += s.z;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    e += __shfl_xor(e, o, 64);
    w += __shfl_xor(w, o, 64);
    k += __shfl_xor(k, o, 64);
  }
  if (lane == 0) { red[wave][0] = e; red[wave][1] = w; red[wave][2] = k; }
  __syncthreads();
  if (threadIdx.x < 3) {
    long long t = 0;
#pragma unroll
    for (int q = 0; q < kBlock / 64; ++q) t += red[q][threadIdx.x];
    rows[3 * b + threadIdx.x] = (int64_t)t;
  }
}

// execute_rotated_move (narde.py:36-56,108-125) of one move per env.  The
// reference executes any (from, to) it is handed; the moves this record can
// hold are those whose source has one of the mover's checkers and whose
// target is not an opponent point (every listed move is one).  Others -- an
// empty source makes narde.py:123-125 conjure a checker of the other colour,
// an opponent target cancels one checker of each -- leave the env unchanged
// and set status[i] = 1 (status optional; from < 0 skips the env, status 0).
__global__ void __launch_bounds__(kBlock) k_apply(Planes pl, int n, const int8_t* __restrict__ moves,
                                                  const int8_t* __restrict__ player,
                                                  uint8_t* __restrict__ status) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int f = moves[2 * i], t = moves[2 * i + 1];
  if (status) status[i] = (f >= 0 && (f > 23 || t < 0 || t > OFF)) ? 1 : 0;
  if (f < 0 || f > 23 || t < 0 || t > OFF) return;
  Side s = side_from_record(pl.p0[i], pl.p1[i]);
  const uint32_t want_black = player ? (player[i] == -1 ? 1u : 0u) : s.black;
  const bool flip = want_black != s.black;
  if (flip) side_flip(s);
  if (nib_get(s.own, f) == 0u || (t != OFF && nib_get(s.opp, t) != 0u)) {
    if (status) status[i] = 1;
    return;
  }
  apply_move(s, f, t);
  if (flip) side_flip(s);
  uint4 a, b;
  side_to_record(s, a, b);
  pl.p0[i] = a;
  pl.p1[i] = b;
}

__global__ void __launch_bounds__(kBlock) k_block(const int8_t* __restrict__ boards, int n,
                                                  uint8_t* __restrict__ out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t O = 0, P = 0;
  for (int p = 0; p < 24; ++p) {
    const int v = boards[i * 24 + p];
    O |= (v > 0 ? 1u : 0u) << p;
    P |= (v < 0 ? 1u : 0u) << p;
  }
  out[i] = (runs6(O) & block_lowmask(P)) ? 1 : 0;
}

}  // namespace
