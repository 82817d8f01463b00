// narde_rules.h -- branch-light bitmask Narde rules engine, one env per lane.
//
// MI355X-native restatement of the reference hot path (cites are
// /root/reference/<path>:<line>):
//   Narde.get_valid_moves        gym_narde/envs/narde.py:58-92
//   Narde._violates_block_rule   gym_narde/envs/narde.py:139-184
//   Narde._filter_head_moves     gym_narde/envs/narde.py:94-106,127-137
//   Narde.execute_rotated_move   gym_narde/envs/narde.py:36-56,108-125
//   NardeEnv.step                gym_narde/envs/narde_env.py:27-103
//   NardeEnv._check_game_ended   gym_narde/envs/narde_env.py:134-141
//
// Representation (all in the MOVER's perspective, mover checkers move toward
// lower indices, head = 23, home = 0..5, 'off' encoded as to = 24):
//   * counts: 24 points x 4-bit nibbles per side in three u32 words
//     (w[0] = points 0..7, w[1] = 8..15, w[2] = 16..23); a side never has
//     more than 15 checkers.  A perspective flip is a 48-bit rotation of the
//     96-bit word triple = three v_alignbit_b32.
//   * masks: O (own occupied), P (opponent occupied), S1o/S1p (count == 1).
//   * a legal-move list is a list of per-die 24-bit source masks L[k] with
//     dice d[k] sorted descending: entry order = die-major, source ascending,
//     which is exactly the reference's list order (duplicates included).
// The whole engine is __host__ __device__ so the same code runs on the GPU
// and in the test-only host build (tests/hostcheck).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NARDE_FN __host__ __device__ __forceinline__

namespace narde {

constexpr uint32_t MASK24 = 0xFFFFFFu;
constexpr int OFF = 24;

// ---------------------------------------------------------------- nibbles
struct Nib {
  uint32_t w[3];  // points 0..7, 8..15, 16..23
};

// (hi:lo) >> 16, low 32 bits: one v_alignbit_b32 on gfx950
NARDE_FN uint32_t funnel16(uint32_t hi, uint32_t lo) { return (lo >> 16) | (hi << 16); }

// (value selects, never an address computed from p: a select between the
// words' addresses would keep the record out of VGPRs, in scratch)
NARDE_FN uint32_t nib_word(const Nib& b, int p) {
  const uint32_t w0 = b.w[0], w1 = b.w[1], w2 = b.w[2];
  const int k = p >> 3;
  return (k == 0 ? w0 : 0u) | (k == 1 ? w1 : 0u) | (k == 2 ? w2 : 0u);
}
NARDE_FN uint32_t nib_get(const Nib& b, int p) { return (nib_word(b, p) >> (4 * (p & 7))) & 15u; }
NARDE_FN void nib_add(Nib& b, int p, uint32_t delta /* +1 or 0xFFFFFFFF */) {
  const uint32_t v = delta << (4 * (p & 7));
  const int k = p >> 3;
  b.w[0] += k == 0 ? v : 0u;
  b.w[1] += k == 1 ? v : 0u;
  b.w[2] += k == 2 ? v : 0u;
}
NARDE_FN void nib_inc(Nib& b, int p) { nib_add(b, p, 1u); }
NARDE_FN void nib_dec(Nib& b, int p) { nib_add(b, p, 0xFFFFFFFFu); }
// perspective flip: new[p] = old[(p + 12) % 24]  (narde.py:16-17 without the sign)
NARDE_FN Nib nib_rot12(const Nib& b) {
  Nib r;
  r.w[0] = funnel16(b.w[2], b.w[1]);
  r.w[1] = funnel16(b.w[0], b.w[2]);
  r.w[2] = funnel16(b.w[1], b.w[0]);
  return r;
}
NARDE_FN uint32_t rot12(uint32_t m) { return ((m >> 12) | (m << 12)) & MASK24; }

// gather bit 4k of x (k = 0..7) into bit k
NARDE_FN uint32_t compact4(uint32_t x) {
  x = (x | (x >> 3)) & 0x03030303u;
  x = (x | (x >> 6)) & 0x000F000Fu;
  x = (x | (x >> 12)) & 0x000000FFu;
  return x;
}
NARDE_FN uint32_t fold_nz(uint32_t x) {
  x |= x >> 1;
  x |= x >> 2;
  return x & 0x11111111u;
}
NARDE_FN uint32_t nz_mask(const Nib& b) {
  return compact4(fold_nz(b.w[0])) | (compact4(fold_nz(b.w[1])) << 8) |
         (compact4(fold_nz(b.w[2])) << 16);
}
NARDE_FN uint32_t eq1_mask(const Nib& b) {
  const uint32_t k = 0x11111111u;
  return compact4(~fold_nz(b.w[0] ^ k) & k) | (compact4(~fold_nz(b.w[1] ^ k) & k) << 8) |
         (compact4(~fold_nz(b.w[2] ^ k) & k) << 16);
}

// ------------------------------------------------------------ env record
// HBM record = two 16-byte planes per env (planar => every load/store of a
// wave is one contiguous 1 KiB):
//   plane0 = {white w0, white w1, black w0, black w1}   absolute coords
//   plane1 = {white w2, black w2, misc, t}
//   misc   = off_w[0:4) | off_b[4:8) | ft_w<<8 | ft_b<<9 | black_to_move<<10
//            | elapsed[16:32)
//   t      = the env's RNG ply counter (Philox counter word 0): the dice and
//            policy draws of the env's next step; +1 per step, kept across
//            episodes.  Living in the record (not a launch argument) makes a
//            step launch replayable from a hipGraph.
struct Side {
  Nib own, opp;
  uint32_t O, P, S1o, S1p;
  uint32_t off_own, off_opp;
  uint32_t ft_own, ft_opp;
  uint32_t black;    // 1 if the mover is black (current_player == -1)
  uint32_t elapsed;  // steps taken in this episode (TimeLimit)
  uint32_t t;        // RNG ply counter
};

NARDE_FN void side_masks(Side& s) {
  s.O = nz_mask(s.own);
  s.P = nz_mask(s.opp);
  s.S1o = eq1_mask(s.own);
  s.S1p = eq1_mask(s.opp);
}

NARDE_FN Side side_from_record(const uint4& a, const uint4& b) {
  const Nib w{{a.x, a.y, b.x}};
  const Nib k{{a.z, a.w, b.y}};
  const uint32_t misc = b.z;
  Side s;
  s.black = (misc >> 10) & 1u;
  const uint32_t offw = misc & 15u, offb = (misc >> 4) & 15u;
  const uint32_t ftw = (misc >> 8) & 1u, ftb = (misc >> 9) & 1u;
  if (s.black) {
    s.own = nib_rot12(k); s.opp = nib_rot12(w);
    s.off_own = offb; s.off_opp = offw; s.ft_own = ftb; s.ft_opp = ftw;
  } else {
    s.own = w; s.opp = k;
    s.off_own = offw; s.off_opp = offb; s.ft_own = ftw; s.ft_opp = ftb;
  }
  s.elapsed = misc >> 16;
  s.t = b.w;
  side_masks(s);
  return s;
}

NARDE_FN void side_to_record(const Side& s, uint4& a, uint4& b) {
  Nib w, k;
  uint32_t offw, offb, ftw, ftb;
  if (s.black) {
    w = nib_rot12(s.opp); k = nib_rot12(s.own);
    offw = s.off_opp; offb = s.off_own; ftw = s.ft_opp; ftb = s.ft_own;
  } else {
    w = s.own; k = s.opp;
    offw = s.off_own; offb = s.off_opp; ftw = s.ft_own; ftb = s.ft_opp;
  }
  a.x = w.w[0]; a.y = w.w[1];
  a.z = k.w[0]; a.w = k.w[1];
  b.x = w.w[2]; b.y = k.w[2];
  b.z = offw | (offb << 4) | (ftw << 8) | (ftb << 9) | (s.black << 10) | (s.elapsed << 16);
  b.w = s.t;
}

// reference layout (int8 board[24] absolute, off {w,b}, first_turn {w,b},
// player +1/-1) <-> record.  Counts must be in 0..15 (checked by callers).
NARDE_FN void record_from_board(const int8_t* board, uint32_t offw, uint32_t offb, uint32_t ftw,
                                uint32_t ftb, int player, uint32_t elapsed, uint32_t t, uint4& a,
                                uint4& b) {
  Nib w{{0, 0, 0}}, k{{0, 0, 0}};
  for (int p = 0; p < 24; ++p) {
    const int v = board[p];
    const uint32_t cw = v > 0 ? (uint32_t)v : 0u, ck = v < 0 ? (uint32_t)(-v) : 0u;
    w.w[p >> 3] |= (cw & 15u) << (4 * (p & 7));
    k.w[p >> 3] |= (ck & 15u) << (4 * (p & 7));
  }
  a.x = w.w[0]; a.y = w.w[1];
  a.z = k.w[0]; a.w = k.w[1];
  b.x = w.w[2]; b.y = k.w[2];
  b.z = (offw & 15u) | ((offb & 15u) << 4) | ((ftw ? 1u : 0u) << 8) | ((ftb ? 1u : 0u) << 9) |
        ((player == -1 ? 1u : 0u) << 10) | (elapsed << 16);
  b.w = t;
}

NARDE_FN void board_from_record(const uint4& a, const uint4& b, int8_t* board, uint8_t* off,
                                uint8_t* ft, int8_t* player, uint16_t* elapsed) {
  const Nib w{{a.x, a.y, b.x}};
  const Nib k{{a.z, a.w, b.y}};
  if (board)
    for (int p = 0; p < 24; ++p) board[p] = (int8_t)((int)nib_get(w, p) - (int)nib_get(k, p));
  if (off) { off[0] = b.z & 15u; off[1] = (b.z >> 4) & 15u; }
  if (ft) { ft[0] = (b.z >> 8) & 1u; ft[1] = (b.z >> 9) & 1u; }
  if (player) *player = ((b.z >> 10) & 1u) ? -1 : 1;
  if (elapsed) *elapsed = (uint16_t)(b.z >> 16);
}

// start position (narde.py:21-29): white 15 on abs 23, black 15 on abs 11
NARDE_FN Side side_start(uint32_t black_first) {
  Side s;
  // in either perspective the mover has 15 on 23 and the opponent 15 on 11
  s.own.w[0] = 0; s.own.w[1] = 0; s.own.w[2] = 15u << 28;
  s.opp.w[0] = 0; s.opp.w[1] = 15u << 12; s.opp.w[2] = 0;
  s.off_own = s.off_opp = 0;
  s.ft_own = s.ft_opp = 1;
  s.black = black_first;
  s.elapsed = 0;
  s.t = 0;
  s.O = 1u << 23; s.P = 1u << 11; s.S1o = 0; s.S1p = 0;
  return s;
}

// mover change (narde_env.py:99-100)
NARDE_FN void side_flip(Side& s) {
  const Nib t = s.own;
  s.own = nib_rot12(s.opp);
  s.opp = nib_rot12(t);
  uint32_t m = s.O; s.O = rot12(s.P); s.P = rot12(m);
  m = s.S1o; s.S1o = rot12(s.S1p); s.S1p = rot12(m);
  m = s.off_own; s.off_own = s.off_opp; s.off_opp = m;
  m = s.ft_own; s.ft_own = s.ft_opp; s.ft_opp = m;
  s.black ^= 1u;
}

// --------------------------------------------------------- move generation
// bit i set iff points i..i+5 are all own (a 6-block starting at i)
NARDE_FN uint32_t runs6(uint32_t m) {
  const uint32_t a = m & (m >> 1);
  const uint32_t b = a & (a >> 2);
  return b & (a >> 4);
}

// Block rule (narde.py:139-184) as a mask test: a maximal own run of >= 6
// violates iff no opponent checker sits below its start, i.e. iff some
// 6-window start i <= lo = lowest opponent point (all 24 if none).
NARDE_FN uint32_t block_lowmask(uint32_t P) {
  return P ? ((2u << __builtin_ctz(P)) - 1u) : MASK24;
}

// What a single move can do to the block rule on this board, for any die:
//   F = allowed 6-windows already full of own checkers (they violate unless
//       the move breaks them);
//   Q = empty/opponent points q whose filling completes an allowed window:
//       window [q-a, q-a+5] (a = 0..5) needs own q-a..q-1 and q+1..q+5-a and
//       its start q-a <= lo.
struct Blocks {
  uint32_t low, F, Q;
};

NARDE_FN Blocks block_info_low(uint32_t O, uint32_t low) {
  Blocks b;
  b.low = low;
  const uint32_t r2 = O & (O >> 1);
  const uint32_t r3 = r2 & (O >> 2);
  const uint32_t r4 = r2 & (r2 >> 2);
  const uint32_t r5 = r4 & (O >> 4);
  b.F = r4 & (r2 >> 4) & b.low;
  const uint32_t lp = b.low + 1u;  // 1 << (lo + 1)
  // q <= lo + a  <=>  bit q of (lp << a) - 1
  uint32_t q = (r5 >> 1) & b.low;                               // a = 0
  q |= (O << 1) & (r4 >> 1) & ((lp << 1) - 1u);                 // a = 1
  q |= (r2 << 2) & (r3 >> 1) & ((lp << 2) - 1u);                // a = 2
  q |= (r3 << 3) & (r2 >> 1) & ((lp << 3) - 1u);                // a = 3
  q |= (r4 << 4) & (O >> 1) & ((lp << 4) - 1u);                 // a = 4
  q |= (r5 << 5) & ((lp << 5) - 1u);                            // a = 5
  b.Q = q & ~O & MASK24;
  return b;
}
NARDE_FN Blocks block_info(uint32_t O, uint32_t P) { return block_info_low(O, block_lowmask(P)); }

// narde.py:64-77 for one die: sources with a legal single move
NARDE_FN uint32_t die_candidates(uint32_t O, uint32_t P, int d) {
  const uint32_t normal = O & ~(P << d) & (MASK24 << d) & MASK24;
  const uint32_t off = ((O >> 6) == 0u) ? (O & ((1u << d) - 1u)) : 0u;  // bear-off, :73-77
  return normal | off;
}

// narde.py:78-89 block filter of one die's candidates C.  A source with >= 2
// checkers keeps O' = O | {q}: it violates iff F != 0 or q in Q.  Only a
// single-checker source that would complete (or keep) a window needs the
// exact per-candidate test, which is rare.
NARDE_FN uint32_t die_filter(uint32_t O, uint32_t S1, const Blocks& bl, uint32_t C, int d) {
  const uint32_t hit = bl.F ? MASK24 : (bl.Q << d);
  uint32_t L = C & ~(hit & ~S1);
  uint32_t m = C & hit & S1;
  while (m) {
    const int p = __builtin_ctz(m);
    m &= m - 1u;
    const uint32_t bp = 1u << p;
    const uint32_t Op = (O & ~bp) | (p >= d ? (1u << (p - d)) : 0u);
    if (runs6(Op) & bl.low) L &= ~bp;
  }
  return L;
}

struct Legal {
  uint32_t L[4];
  int d[4];
  int n;
  int count;
};

// Narde.get_valid_moves(roll, mover) for n <= 4 dice already sorted descending.
NARDE_FN void legal_sorted(const Side& s, const int* dd, int n, Legal& l) {
  const Blocks bl = block_info(s.O, s.P);
  l.n = n;
  for (int k = 0; k < 4; ++k) { l.L[k] = 0u; l.d[k] = 0; }
  for (int k = 0; k < n; ++k) {
    l.d[k] = dd[k];
    if (k > 0 && dd[k] == dd[k - 1]) { l.L[k] = l.L[k - 1]; continue; }
    l.L[k] = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, dd[k]), dd[k]);
  }
  // head rule (narde.py:94-106,127-137): keep the first max_head entries from 23
  const int max_head =
      (s.ft_own && n == 2 && dd[0] == dd[1] && (dd[0] == 3 || dd[0] == 4 || dd[0] == 6)) ? 2 : 1;
  int seen = 0;
  int count = 0;
  for (int k = 0; k < n; ++k) {
    if (l.L[k] >> 23) {
      if (seen < max_head) ++seen;
      else l.L[k] &= ~(1u << 23);
    }
    count += __builtin_popcount(l.L[k]);
  }
  l.count = count;
}

// the two-dice list of NardeEnv.step (roll in any order); low =
// block_lowmask(s.P)
NARDE_FN void legal2_low(const Side& s, int d0, int d1, uint32_t low, Legal& l) {
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  const Blocks bl = block_info_low(s.O, low);
  l.n = 2;
  l.d[0] = dh; l.d[1] = dl; l.d[2] = 0; l.d[3] = 0;
  l.L[2] = 0u; l.L[3] = 0u;
  uint32_t Lh = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, dh), dh);
  uint32_t Ll = dl == dh ? Lh : die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, dl), dl);
  // head rule: the second head entry survives only on a first-turn 3-3/4-4/6-6
  const bool two_heads = s.ft_own && dh == dl && (dh == 3 || dh == 4 || dh == 6);
  if ((Lh >> 23) && !two_heads) Ll &= ~(1u << 23);
  l.L[0] = Lh;
  l.L[1] = Ll;
  l.count = __builtin_popcount(Lh) + __builtin_popcount(Ll);
}
NARDE_FN void legal2(const Side& s, int d0, int d1, Legal& l) { legal2_low(s, d0, d1, block_lowmask(s.P), l); }

// get_valid_moves for an explicit roll of up to 4 dice (0 = unused slot)
NARDE_FN void legal_roll(const Side& s, const uint8_t* d4, Legal& l) {
  int dd[4] = {0, 0, 0, 0};
  int nd = 0;
  for (int k = 0; k < 4; ++k) {
    const int v = d4[k];
    if (v >= 1 && v <= 6) dd[nd++] = v;
  }
  // roll = sorted(roll, reverse=True), narde.py:59
  for (int a = 1; a < 4; ++a)
    for (int b = a; b > 0; --b)
      if (dd[b] > dd[b - 1]) { const int x = dd[b]; dd[b] = dd[b - 1]; dd[b - 1] = x; }
  legal_sorted(s, dd, nd, l);
}

// j-th (0-based) set bit of a 24-bit m (j < popcount(m)), branch-free: the
// byte from the two cumulative byte counts, then a 4 / 2 / 1 search inside
// it, every step a bit-field extract at the position found so far (round 2:
// a 12 / 6 / 3 / 1 / 1 search, ~10 more VALU per call)
NARDE_FN int select_bit(uint32_t m, int j) {
  const uint32_t u = (uint32_t)j;
  const uint32_t c0 = __builtin_popcount(m & 0xFFu), c1 = __builtin_popcount(m & 0xFFFFu);
  const bool b2 = u >= c1, b1 = u >= c0;
  uint32_t pos = b2 ? 16u : (b1 ? 8u : 0u);
  uint32_t r = u - (b2 ? c1 : (b1 ? c0 : 0u));
  uint32_t c = __builtin_popcount((m >> pos) & 0xFu);
  if (r >= c) { r -= c; pos += 4u; }
  c = __builtin_popcount((m >> pos) & 0x3u);
  if (r >= c) { r -= c; pos += 2u; }
  c = (m >> pos) & 1u;
  if (r >= c) pos += 1u;
  return (int)pos;
}

// list entry i -> (from, to); to = OFF for bear-off
NARDE_FN void legal_entry(const Legal& l, int i, int& f, int& t) {
  int k = 0;
  for (; k < l.n - 1; ++k) {
    const int c = __builtin_popcount(l.L[k]);
    if (i < c) break;
    i -= c;
  }
  f = select_bit(l.L[k], i);
  t = f - l.d[k] < 0 ? OFF : f - l.d[k];
}

// entry i of a two-dice list -> (from, to, die)
NARDE_FN void legal2_entry(const Legal& l, int i, int& f, int& t) {
  const int c0 = __builtin_popcount(l.L[0]);
  const bool second = i >= c0;
  const uint32_t m = second ? l.L[1] : l.L[0];
  const int d = second ? l.d[1] : l.d[0];
  f = select_bit(m, second ? i - c0 : i);
  t = f - d < 0 ? OFF : f - d;
}

// `move in valid_moves` (narde_env.py:63 for move 1, :89 for move 2) in O(n)
NARDE_FN bool legal_contains(const Legal& l, int f, int t) {
  if (f < 0 || f > 23) return false;
  const uint32_t bf = 1u << f;
  bool hit = false;
  for (int k = 0; k < l.n; ++k)
    hit |= (l.L[k] & bf) != 0u && (t == OFF ? (f < l.d[k]) : (f - t == l.d[k]));
  return hit;
}

NARDE_FN int encode_move(int f, int t) { return f * 24 + (t == OFF ? 0 : t); }

// narde_env.py:45-62 action decode (the 'off' quirk: to==0 & from<=5)
NARDE_FN void decode_action(int code, int& f, int& t) {
  if (code < 0 || code >= 576) { f = -1; t = -1; return; }
  f = code / 24;
  t = code % 24;
  if (t == 0 && f <= 5) t = OFF;
}

// execute_rotated_move in mover perspective (narde.py:36-56,108-125)
// Straight-line (no divergent branch around the bear-off case): a bear-off
// adds nothing to the board (delta 0, empty target bit) and one to off_own.
// count==1 mask: the source's bit flips iff it held 1 or 2 checkers, the
// target's iff it held 0 or 1 (it can never hold the source's checkers:
// t < f).  Needs O and S1o to match the own nibbles (every Side does).
NARDE_FN void apply_move(Side& s, int f, int t) {
  const bool off = t == OFF;
  const int tq = off ? 0 : t;
  const uint32_t cf = nib_get(s.own, f);
  const uint32_t bf = 1u << f;
  const uint32_t bt = off ? 0u : (1u << tq);
  const uint32_t vf = 0xFFFFFFFFu << (4 * (f & 7));
  const uint32_t vt = (off ? 0u : 1u) << (4 * (tq & 7));
  const int kf = f >> 3, kt = tq >> 3;
  s.own.w[0] += (kf == 0 ? vf : 0u) + (kt == 0 ? vt : 0u);
  s.own.w[1] += (kf == 1 ? vf : 0u) + (kt == 1 ? vt : 0u);
  s.own.w[2] += (kf == 2 ? vf : 0u) + (kt == 2 ? vt : 0u);
  // the target held 0 or 1 checkers iff it is not an own point or a
  // count-1 one (from the masks: no second nibble read; t != f)
  const uint32_t t01 = bt & (~s.O | s.S1o);
  s.O = (s.O & (cf == 1u ? ~bf : ~0u)) | bt;
  s.S1o ^= (cf - 1u < 2u ? bf : 0u) ^ t01;
  s.off_own += off ? 1u : 0u;
  s.ft_own = 0u;
}

NARDE_FN uint32_t mulhi_u32(uint32_t r, uint32_t n) { return (uint32_t)(((uint64_t)r * n) >> 32); }

struct StepOut {
  Legal l1;
  uint32_t L2;
  int d2;
  int count2;  // -1 when no second list was generated
  int code1, code2;
  int reward;
  int term;
};

// NardeEnv.step (narde_env.py:27-103) with dice (d0, d1) in roll order.
// policy: draw code1 from list1 with r1 and code2 from the env's own second
// list with r2 (the build's random-legal policy); otherwise use code1/code2.
// flip_always: flip even after the game ended -- for callers that reset a
// terminated env in the same ply anyway (auto-reset), where it saves the
// divergent branch around the flip
// nomove: the roll has no legal move whatever the board (a caller-given die
// outside 1..6, see env_ply): list #1 is empty.
NARDE_FN void env_step(Side& s, int d0, int d1, int code1, int code2, bool policy, uint32_t r1,
                       uint32_t r2, StepOut& o, bool flip_always = false, bool nomove = false) {
  // the mover's moves never change the opponent's points: one low mask
  // serves both lists
  const uint32_t low = block_lowmask(s.P);
  legal2_low(s, d0, d1, low, o.l1);
  if (nomove) {
    o.l1.L[0] = o.l1.L[1] = 0u;
    o.l1.count = 0;
  }
  o.L2 = 0u; o.d2 = 0; o.count2 = -1;
  const int n1 = o.l1.count;
  int f1 = -1, t1 = -1;
  bool play1;
  if (policy) {
    // the drawn entry is its own code; decode(encode(f, t)) differs from (f, t)
    // only for a normal move (f, 0) with f <= 5, which decodes to (f, 'off')
    // (mulhi(r1, n1) is 0 for n1 <= 1: no branch around it)
    legal2_entry(o.l1, (int)mulhi_u32(r1, (uint32_t)n1), f1, t1);
    code1 = n1 >= 2 ? encode_move(f1, t1) : 0;
    code2 = 0;
    play1 = n1 >= 1;
    if (n1 >= 2 && t1 == 0 && f1 <= 5) {
      t1 = OFF;
      play1 = legal_contains(o.l1, f1, t1);
    }
  } else if (n1 == 1) {
    legal2_entry(o.l1, 0, f1, t1);  // narde_env.py:41-43, action ignored
    play1 = true;
  } else {
    decode_action(code1, f1, t1);
    play1 = n1 >= 2 && legal_contains(o.l1, f1, t1);
  }
  if (play1) apply_move(s, f1, t1);
  if (n1 >= 2 && play1) {
    // die bookkeeping, narde_env.py:63-83: remove dist if rolled, else pop(0)
    // (a played move is a listed one: t1 = f1 - die < f1, so |f1 - t1| = f1 - t1)
    const int dist = t1 == OFF ? f1 + 1 : f1 - t1;
    const int rem = (d0 == dist) ? d1 : ((d1 == dist) ? d0 : d1);
    // second get_valid_moves([rem]) (:88): one die, first_turn already cleared
    const Blocks bl = block_info_low(s.O, low);
    const uint32_t L2 = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, rem), rem);
    o.L2 = L2;
    o.d2 = rem;
    o.count2 = __builtin_popcount(L2);
    int f2, t2;
    bool play2;
    if (policy) {
      f2 = select_bit(L2, (int)mulhi_u32(r2, (uint32_t)o.count2));
      t2 = f2 - rem < 0 ? OFF : f2 - rem;
      code2 = o.count2 > 0 ? encode_move(f2, t2) : 0;
      // a drawn (f, 0) with f <= 5 decodes to (f, 'off'), never in a one-die
      // list (it needs f < rem = f); code 0 = (0, 'off') on an empty list
      play2 = o.count2 > 0 && !(t2 == 0 && f2 <= 5);
    } else {
      decode_action(code2, f2, t2);
      play2 = f2 >= 0 && ((L2 >> f2) & 1u) && (t2 == OFF ? (f2 < rem) : (f2 - t2 == rem));
    }
    if (play2) apply_move(s, f2, t2);
  }
  o.code1 = code1;
  o.code2 = code2;
  // _check_game_ended (narde_env.py:134-141): only the mover is checked
  o.term = s.off_own == 15u;
  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
  if (flip_always || !o.term) side_flip(s);
}

// ============================================================ play sets
// The plays of a two-dice roll (the README's get_valid_actions,
// README.md:156-165; VecNardeEnv.play_set), per entry of list #1 in list
// order (the higher die's sources ascending, then the lower die's; doubles:
// the same die twice, NardeEnv's list with its duplicates) -- the second
// moves that follow it:
//   kPlayAct  DQNAgent.act's valid_move_combinations
//             (train_deepq_pytorch.py:430-507): the remaining die is the
//             roll less the die act() matches to move 1 -- the first die in
//             roll order equal to the distance, for a bear-off from p the
//             first one >= p + 1 -- and its list is get_valid_moves([rem])
//             on the PRE-move board (:486); an empty one gives (move 1, 0);
//   kPlayStep what NardeEnv.step carries out (narde_env.py:45-93): move 1
//             applied, rem = the roll less its distance (else pop(0)),
//             get_valid_moves([rem]) on the POST-move board; a one-entry
//             list #1 is played alone whatever the action.
// Entry word: second-move sources (24 bits) | rem << 24 | kPlayValid.
// Plays counted: kPlayAct every entry (duplicates included) times
// max(1, |second list|) -- len(valid_move_combinations); kPlayStep the
// distinct plays (a move listed under both dice -- doubles, or a bear-off
// both dice reach -- once), 1 for a one-entry list.
constexpr int kPlayAct = 0;
constexpr int kPlayStep = 1;
constexpr uint32_t kPlayValid = 1u << 27;

// visit(k, p, die, word, dup) for every entry of list #1 in list order;
// returns the play count.  l: legal2(s, d0, d1) (dice in roll order).
template <class F>
NARDE_FN int play_walk(const Side& s, int d0, int d1, int kind, const Legal& l, F&& visit) {
  const int n1 = l.count;
  const Blocks bl = block_info(s.O, s.P);
  // act: the two one-die lists of the pre-move board (rem is d0 or d1)
  const uint32_t M0 = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, d0), d0);
  const uint32_t M1 = d1 == d0 ? M0 : die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, d1), d1);
  int count = 0;
  for (int k = 0; k < 2; ++k) {
    const int die = l.d[k];
    uint32_t m = l.L[k];
    while (m) {
      const int p = __builtin_ctz(m);
      m &= m - 1u;
      const bool off = p < die;
      const bool dup = k == 1 && ((l.L[0] >> p) & 1u) && (l.d[0] == l.d[1] || off);
      uint32_t word;
      if (kind == kPlayAct) {
        const bool first = off ? d0 >= p + 1 : d0 == die;  // act() matched roll[0]
        const int rem = first ? d1 : d0;
        word = (first ? M1 : M0) | ((uint32_t)rem << 24) | kPlayValid;
        const int c2 = __builtin_popcount(word & 0xFFFFFFu);
        count += c2 > 0 ? c2 : 1;
      } else if (n1 == 1) {
        word = kPlayValid;  // narde_env.py:41-43: played alone
        count = 1;
      } else {
        Side c = s;
        apply_move(c, p, off ? OFF : p - die);
        const int dist = off ? p + 1 : die;
        const int rem = (d0 == dist) ? d1 : ((d1 == dist) ? d0 : d1);
        const uint32_t L2 = die_filter(c.O, c.S1o, block_info(c.O, c.P), die_candidates(c.O, c.P, rem), rem);
        word = L2 | ((uint32_t)rem << 24) | kPlayValid;
        if (!dup) {
          const int c2 = __builtin_popcount(L2);
          count += c2 > 0 ? c2 : 1;
        }
      }
      visit(k, p, die, word, dup);
    }
  }
  return count;
}

// the play of act-kind index j (0 <= j < count) -> (move-1 code, move-2
// code) as act() writes them (from * 24 + to, 'off' -> to 0; no second
// move -> 0)
NARDE_FN void play_codes_act(const Side& s, int d0, int d1, const Legal& l, int j, int& c1, int& c2) {
  c1 = 0;
  c2 = 0;
  int left = j;
  bool found = false;
  play_walk(s, d0, d1, kPlayAct, l, [&](int, int p, int die, uint32_t word, bool) {
    if (found) return;
    const uint32_t m2 = word & 0xFFFFFFu;
    const int w = m2 ? __builtin_popcount(m2) : 1;
    if (left >= w) { left -= w; return; }
    found = true;
    c1 = encode_move(p, p < die ? OFF : p - die);
    if (m2) {
      const int rem = (int)((word >> 24) & 7u);
      const int q = select_bit(m2, left);
      c2 = encode_move(q, q < rem ? OFF : q - rem);
    }
  });
}

// DQNAgent.act's greedy candidate sets (train_deepq_pytorch.py:520-560) as
// 576-bit masks m[9]: move1 < 0 -- the codes of list #1's entries
// (valid_first_moves' keys, :526); else valid_first_moves[move1]: the move-2
// codes act() listed for the LAST list-#1 entry coded move1 (the dict entry
// is reset at every occurrence, :474), {0} when that list is empty, nothing
// when no entry has that code.
NARDE_FN void act_masks(const Side& s, int d0, int d1, const Legal& l, int move1, uint64_t m[9]) {
  for (int q = 0; q < 9; ++q) m[q] = 0ull;
  uint32_t last = 0u;
  play_walk(s, d0, d1, kPlayAct, l, [&](int, int p, int die, uint32_t word, bool) {
    const int c = encode_move(p, p < die ? OFF : p - die);
    if (move1 < 0) m[c >> 6] |= 1ull << (c & 63);
    else if (c == move1) last = word;
  });
  if (move1 < 0 || !last) return;
  uint32_t src = last & 0xFFFFFFu;
  const int rem = (int)((last >> 24) & 7u);
  if (!src) m[0] |= 1ull;  // (move 1, 0)
  while (src) {
    const int q = __builtin_ctz(src);
    src &= src - 1u;
    const int c = encode_move(q, q < rem ? OFF : q - rem);
    m[c >> 6] |= 1ull << (c & 63);
  }
}

// ============================================================ FULL4 turns
// Build extension: one
// step = the mover's WHOLE turn -- four sub-moves on doubles, the
// max-dice-used rule (README.md:27-30), the higher die when only one of two
// can be played.  Every sub-move is the reference's single-die primitive
// (get_valid_moves([d]) = legal1 below, execute_rotated_move = apply_die);
// the composition is restated independently in oracle/narde_oracle.c
// (or_full4_turn) and pinned to tests/golden/full4.npz.
//   H = 2 head moves on a first-turn 3-3/4-4/6-6 (narde.py:94-106's
//   condition), else 1, for the whole turn.
//   M = the longest playable sequence; C_k = the sub-moves that keep M
//   reachable; list order die-descending, source-ascending.
// The opponent never changes during a turn, so the block rule's low mask is
// computed once per turn.
constexpr uint32_t HEAD = 1u << 23;

// Block-free turns.  The opponent is fixed for the whole turn and a
// sub-move never lands on an opponent point, so every own-occupied mask the
// turn can produce lies inside U = O plus up to n landings from it.  If U
// holds no 6-window the block rule may reject (runs6(U) & low == 0; runs6 is
// monotone), no die_filter can ever remove a candidate this turn: the
// single-die lists are then the plain candidate masks, and sub-moves from
// different sources cannot interfere.  That holds on ~97 % of two-dice and
// ~80 % of doubles turns of random self-play.
NARDE_FN uint32_t land_step(uint32_t S, uint32_t P, int d) { return (S >> d) & ~P; }

// 6-windows (bit i = points i..i+5) holding at most k (2 or 4) points that
// are not own: a bit-sliced count of the holes over the six shifted masks
// the hole count of every 6-window (bit i = points i..i+5) bit-sliced, s2 s1
// s0: the six shifted hole masks through two carry-save adders (xor3 /
// majority: one v_bitop3 each)
NARDE_FN void window_hole_count(uint32_t O, uint32_t& s0, uint32_t& s1, uint32_t& s2) {
  const uint32_t h = ~O & MASK24;
  const uint32_t x0 = h, x1 = h >> 1, x2 = h >> 2, x3 = h >> 3, x4 = h >> 4, x5 = h >> 5;
  const uint32_t sa = x0 ^ x1 ^ x2, ca = (x0 & x1) | (x2 & (x0 ^ x1));
  const uint32_t sb = x3 ^ x4 ^ x5, cb = (x3 & x4) | (x5 & (x3 ^ x4));
  const uint32_t c0 = sa & sb;
  s0 = sa ^ sb;
  s1 = ca ^ cb ^ c0;
  s2 = (ca & cb) | (c0 & (ca ^ cb));
}
NARDE_FN uint32_t windows_few_holes(uint32_t O, int k) {
  uint32_t s0, s1, s2;
  window_hole_count(O, s0, s1, s2);
  return k >= 4 ? ~(s2 & (s1 | s0)) : ~s2 & ~(s1 & s0);
}

// A window can only fill during the turn if the turn's landings can cover
// its holes: each sub-move adds at most one new own point, so a window the
// block rule could see full has at most 2 (two dice) or 4 (doubles) holes
// in O.  The few windows that pass this count (usually none) get a sharper
// per-window test; the window is harmless unless:
//   * it is full already (no holes);
//   * two dice, one hole: the hole is a landing of one die or of both in
//     turn from a source the window can spare -- outside it, or a point of
//     >= 2 checkers (a single checker leaving a window point leaves a hole
//     no other sub-move is left to refill);
//   * two dice, two holes: each hole is a single-die landing from such a
//     source, with different dice (each sub-move fills one hole; a checker
//     moving on from the first hole empties it again);
//   * doubles: the holes' fewest steps from such sources sum to <= 4 (each
//     hole's final checker walks its own steps; a single checker that
//     leaves a window point must be replaced along the same d-chain, which
//     reaches the hole from the replacement's origin in the same number of
//     steps).
// Checked against a depth-first walk of every sub-move sequence
// (tools/diag/bf_stats.cpp, tests/hostcheck hc_block_free_random): it frees
// ~2/3 of the two-dice and ~3/5 of the doubles turns the count alone calls
// block-bound, and never a turn in which the rule removes a candidate.
// doubles, the next k (1..4) sub-moves of die d: the points of the windows
// that fail the per-window test (~0u if one is full already; 0: block-free)
// -- the same test with k landings and a step budget of k (a node inside a
// block-bound turn is often block-free for the sub-moves it has left)
NARDE_FN uint32_t dbl_block_windows(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int d, int k) {
  uint32_t S = O, U = O;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    S = land_step(S, P, d);
    U |= j < k ? S : 0u;
  }
  uint32_t win = runs6(U) & low & windows_few_holes(O, k > 2 ? 4 : 2), ws = 0u;
  while (win) {
    const int i = __builtin_ctz(win);
    win &= win - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    if (!H) return ~0u;
    uint32_t T = O & ~(W & S1), seen = 0u;
    int cost = 0;
#pragma unroll
    for (int j = 1; j <= 4; ++j) {
      T = land_step(T, P, d);
      const uint32_t nw = j <= k ? (H & T & ~seen) : 0u;
      cost += j * __builtin_popcount(nw);
      seen |= nw;
    }
    ws |= (seen == H && cost <= k) ? W : 0u;
  }
  return ws;
}
NARDE_FN bool dbl_block_free(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int d, int k) {
  return dbl_block_windows(O, S1, P, low, d, k) == 0u;
}

// two dice: the per-window test; returns the holes (in O) of the windows
// that fail it -- the only windows that can ever be full at a node of the
// turn -- and sets `bound` if there is one (~0u: one of them is full already)
NARDE_FN uint32_t two_block_holes(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl,
                                  bool& bound) {
  const uint32_t A = O | land_step(O, P, dh) | land_step(O, P, dl);
  const uint32_t U = A | land_step(A, P, dh) | land_step(A, P, dl);
  uint32_t win = runs6(U) & low & windows_few_holes(O, 2), hs = 0u;
  bound = false;
  while (win) {
    const int i = __builtin_ctz(win);
    win &= win - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    const uint32_t src = O & ~(W & S1);
    const uint32_t Lh = land_step(src, P, dh), Ll = land_step(src, P, dl);
    const uint32_t h1 = H & (0u - H), h2 = H ^ h1;
    const bool fail = !H || (!h2 ? (H & (Lh | Ll | land_step(Lh, P, dl) | land_step(Ll, P, dh))) != 0u
                                 : (((h1 & Lh) && (h2 & Ll)) || ((h1 & Ll) && (h2 & Lh))));
    bound = bound || fail;
    hs |= fail ? (H ? H : ~0u) : 0u;
  }
  return hs;
}

// Both kinds of turn in one pass (a wave holds both: one reachable set, one
// hole count, one window loop instead of two of each): 0 if the turn is
// block-free; else two_block_holes' holes (two dice) or
// dbl_block_windows' points (doubles, k = 4), ~0u if a failing window is
// full already.  The doubles reachable set is a superset here (two more
// steps of O..S2 cover S3, S4), which only lets more windows into the
// exact per-window test.
NARDE_FN uint32_t turn_block_set(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  const bool dbl = dh == dl;
  const uint32_t A = O | land_step(O, P, dh) | land_step(O, P, dl);
  uint32_t U = A | land_step(A, P, dh) | land_step(A, P, dl);
  const uint32_t V = land_step(U, P, dh);
  U |= dbl ? (V | land_step(V, P, dh)) : 0u;
  uint32_t win = runs6(U) & low & windows_few_holes(O, dbl ? 4 : 2), out = 0u;
  while (win) {
    const int i = __builtin_ctz(win);
    win &= win - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    if (!H) return ~0u;
    const uint32_t src = O & ~(W & S1);
    if (dbl) {
      uint32_t T = src, seen = 0u;
      int cost = 0;
#pragma unroll
      for (int j = 1; j <= 4; ++j) {
        T = land_step(T, P, dh);
        const uint32_t nw = H & T & ~seen;
        cost += j * __builtin_popcount(nw);
        seen |= nw;
      }
      out |= (seen == H && cost <= 4) ? W : 0u;
    } else {
      const uint32_t Lh = land_step(src, P, dh), Ll = land_step(src, P, dl);
      const uint32_t h1 = H & (0u - H), h2 = H ^ h1;
      const bool fail = !h2 ? (H & (Lh | Ll | land_step(Lh, P, dl) | land_step(Ll, P, dh))) != 0u
                            : (((h1 & Lh) && (h2 & Ll)) || ((h1 & Ll) && (h2 & Lh)));
      out |= fail ? H : 0u;
    }
  }
  return out;
}

NARDE_FN bool turn_block_free(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  return turn_block_set(O, S1, P, low, dh, dl) == 0u;
}

// Block-bound two dice: the first moves p of die a (in La) sure to leave die
// b a move, from the masks.  hs = two_block_holes.  A root candidate x of b
// stays a candidate after p unless x = p; the rule can only reject a move
// that fills the last hole of a failing window, i.e. lands on a hole in hs
// or on p itself (a single checker leaving a window point); the head rule
// drops x = 23 after p = 23 (x = p again).  So the candidates landing
// outside hs ("safe") other than p and p + b survive: p is sure if one is
// left.  On random self-play 73 % of the block-bound two-dice turns have
// every first move sure (tools/diag/bf_stats.cpp-style count; checked
// against f4_keep_pair in tests/hostcheck hc_sure_pair_random).
NARDE_FN uint32_t f4_sure_pair(uint32_t O, uint32_t P, int b, uint32_t La, uint32_t hs) {
  if (hs == ~0u) return 0u;
  const uint32_t safe = die_candidates(O, P, b) & ~(hs << b);
  const int c = __builtin_popcount(safe);
  const uint32_t ok = c >= 3 ? ~0u : (c == 2 ? ~(safe & (safe >> b)) : (c == 1 ? ~(safe | (safe >> b)) : 0u));
  return La & ok;
}

// get_valid_moves([d], mover) (narde.py:58-92 with one die: the head filter
// is a no-op, a one-die list has at most one head entry); bf = block-free turn
NARDE_FN uint32_t legal1(const Side& s, uint32_t low, int d, bool bf) {
  const uint32_t C = die_candidates(s.O, s.P, d);
  return bf ? C : die_filter(s.O, s.S1o, block_info_low(s.O, low), C, d);
}

NARDE_FN void apply_die(Side& s, int p, int d) { apply_move(s, p, p - d < 0 ? OFF : p - d); }

// the own masks (O, count==1) after sub-move p -> p-d, without the nibbles
NARDE_FN void child_masks(const Side& s, int p, int d, uint32_t& O2, uint32_t& S2) {
  const uint32_t bp = 1u << p;
  const uint32_t cp = nib_get(s.own, p);
  O2 = cp == 1u ? (s.O & ~bp) : s.O;
  S2 = cp == 1u ? (s.S1o & ~bp) : (cp == 2u ? (s.S1o | bp) : s.S1o);
  if (p - d >= 0) {
    const uint32_t bq = 1u << (p - d);
    // empty -> 1 (set); 1 -> 2 (clear); >= 2 stays (bit already clear)
    S2 = (O2 & bq) ? (S2 & ~bq) : (S2 | bq);
    O2 |= bq;
  }
}

// Block-free lower bound on the sub-moves of die d playable from a node with
// own masks (O, S1): every checker of a listed source can make the same move
// (its landing stays free of the opponent, bear-off stays allowed), sources
// do not interfere, so each source gives min(count, 2) and the head at most
// hl.  A sub-move lowers it by at most one.
NARDE_FN int f4_lower_bound(uint32_t O, uint32_t S1, uint32_t P, int d, int hl) {
  uint32_t L = die_candidates(O, P, d);
  if (hl <= 0) L &= ~HEAD;
  const uint32_t body = L & ~HEAD;
  const int head = (L & HEAD) ? ((hl >= 2 && !(S1 & HEAD)) ? 2 : 1) : 0;
  return __builtin_popcount(body) + __builtin_popcount(body & ~S1) + head;
}

// The same with chains: a checker also walks on from its landing while the
// next landing is free of the opponent (and bears off at the end when all
// are home -- only counted if all are home already, which a turn never
// undoes).  Chains of different checkers do not interfere, so
//   sum over sources x of min(count, 2) * chain(x)   (head: min(hl, 2))
// sub-moves are playable (block-free turns).  One sub-move lowers it by at
// most chain <= 4.
NARDE_FN int f4_chain_bound(uint32_t O, uint32_t S1, uint32_t P, int d, int hl) {
  const uint32_t gn = (~P << d) & (MASK24 << d) & MASK24;       // y: y - d on the board, free
  const uint32_t go = ((O >> 6) == 0u) ? ((1u << d) - 1u) : 0u;  // y: bears off
  const uint32_t a = gn | go;
  const uint32_t keep = hl > 0 ? O : (O & ~HEAD);
  const uint32_t g1 = gn & (gn << d), g2 = g1 & (gn << (2 * d));
  const uint32_t c1 = keep & a;
  const uint32_t c2 = keep & gn & (a << d);
  const uint32_t c3 = keep & g1 & (a << (2 * d));
  const uint32_t c4 = keep & g2 & (a << (3 * d));
  const uint32_t multi = ~S1 & ~HEAD;
  const int hm = (hl >= 2 && !(S1 & HEAD)) ? 2 : 1;
  int lb = __builtin_popcount(c1 & ~HEAD) + __builtin_popcount(c2 & ~HEAD) +
           __builtin_popcount(c3 & ~HEAD) + __builtin_popcount(c4 & ~HEAD) +
           __builtin_popcount(c1 & multi) + __builtin_popcount(c2 & multi) +
           __builtin_popcount(c3 & multi) + __builtin_popcount(c4 & multi);
  lb += hm * (int)(((c1 >> 23) & 1u) + ((c2 >> 23) & 1u) + ((c3 >> 23) & 1u) + ((c4 >> 23) & 1u));
  return lb;
}

// own points holding >= 3 / >= 4 checkers (24-bit masks from the nibbles)
NARDE_FN uint32_t nib_ge3_ge4(const Nib& b, uint32_t& ge4) {
  uint32_t m3 = 0u, m4 = 0u;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint32_t w = b.w[k];
    const uint32_t hi = ((w >> 2) | (w >> 3)) & 0x11111111u;  // v >= 4
    const uint32_t lo = w & (w >> 1) & 0x11111111u;          // bits 0 and 1 set
    m4 |= compact4(hi) << (8 * k);
    m3 |= compact4(hi | lo) << (8 * k);
  }
  ge4 = m4;
  return m3;
}

// Can bear-off change within the next `rem` sub-moves of a doubles turn?
// Not if every own checker is home already (it stays allowed) or at least
// rem are outside (each sub-move brings at most one home, so one stays out
// until the last of them).
NARDE_FN bool f4_bearoff_fixed(const Side& s, int rem = 4) {
  if ((s.O >> 6) == 0u) return true;
  uint32_t x = s.own.w[0] & 0xFFFFFFu;  // points 0..5
  x = (x & 0x0F0F0Fu) + ((x >> 4) & 0x0F0F0Fu);
  const uint32_t home = ((x * 0x010101u) >> 16) & 0xFFu;
  return (int)(15u - s.off_own - home) >= rem;
}

// f4_chain_bound for a block-bound doubles turn, from ws = dbl_block_windows
// (its failing windows: no other window can ever fill this turn).  Only
// steps whose landing cannot fill a failing window count: not a hole of
// one, not a window point some sub-move may vacate (a source now, or a
// bear-off source once bear-off opens, if it can this turn).  Such steps are
// never rejected, in any order; a checker walks on over them (its chain).
// The count (min(count, 2) checkers per point) is at most E = the sum over
// checkers of their chain lengths, a legal sub-move lowers E by at most one
// (the mover keeps the rest of its chain, the others theirs; the window set
// stays that of the root), and min(4, E) sub-moves stay playable -- so, as
// for the block-free bounds, >= 4 at the root gives M = 4 and every C_k = L_k.
// ws = 0 (block-free) gives f4_chain_bound itself.  Settles 38 % of the
// block-bound doubles turns of random self-play (the single steps alone,
// the first form: 23 %); every legal path of each settled turn checked in
// tools/diag/safe_chain_check.cpp.
NARDE_FN int f4_safe_bound(const Side& s, int d, int hl, uint32_t ws) {
  if (ws == ~0u) return 0;
  const uint32_t O = s.O, P = s.P;
  const uint32_t C = die_candidates(O, P, d);
  const uint32_t opens = f4_bearoff_fixed(s) ? 0u : ((1u << d) - 1u);
  const uint32_t bad = ws & (~O | C | opens);
  const uint32_t gn = (~(P | bad) << d) & (MASK24 << d) & MASK24;  // y: y - d free, safe
  const uint32_t go = ((O >> 6) == 0u) ? ((1u << d) - 1u) : 0u;    // y: bears off
  const uint32_t a = gn | go;
  const uint32_t keep = hl > 0 ? O : (O & ~HEAD);
  const uint32_t g1 = gn & (gn << d), g2 = g1 & (gn << (2 * d));
  const uint32_t c1 = keep & a;
  const uint32_t c2 = keep & gn & (a << d);
  const uint32_t c3 = keep & g1 & (a << (2 * d));
  const uint32_t c4 = keep & g2 & (a << (3 * d));
  const uint32_t multi = ~s.S1o & ~HEAD;
  const int hm = (hl >= 2 && !(s.S1o & HEAD)) ? 2 : 1;
  int lb = __builtin_popcount(c1 & ~HEAD) + __builtin_popcount(c2 & ~HEAD) +
           __builtin_popcount(c3 & ~HEAD) + __builtin_popcount(c4 & ~HEAD) +
           __builtin_popcount(c1 & multi) + __builtin_popcount(c2 & multi) +
           __builtin_popcount(c3 & multi) + __builtin_popcount(c4 & multi);
  lb += hm * (int)(((c1 >> 23) & 1u) + ((c2 >> 23) & 1u) + ((c3 >> 23) & 1u) + ((c4 >> 23) & 1u));
  return lb;
}

// Exact sub-move count of a block-free doubles turn whose bear-off status
// is fixed (f4_bearoff_fixed): each checker walks its own chain of die-d
// steps (free landings, and a final bear-off when all are home), chains of
// different checkers never interact, and only hl checkers may leave the
// head.  So M = min(4, sum over checkers of their chain lengths), and any
// legal sub-move lowers that sum by exactly one: every C_k = L_k.
NARDE_FN int f4_exact_moves(const Side& s, int d, int hl) {
  const uint32_t O = s.O, P = s.P;
  const uint32_t gn = (~P << d) & (MASK24 << d) & MASK24;       // y: y - d on the board, free
  const uint32_t go = ((O >> 6) == 0u) ? ((1u << d) - 1u) : 0u;  // y: bears off
  const uint32_t a = gn | go;
  const uint32_t keep = hl > 0 ? O : (O & ~HEAD);
  const uint32_t g1 = gn & (gn << d), g2 = g1 & (gn << (2 * d));
  const uint32_t c1 = keep & a;                   // chain >= 1
  const uint32_t c2 = keep & gn & (a << d);       // >= 2
  const uint32_t c3 = keep & g1 & (a << (2 * d)); // >= 3
  const uint32_t c4 = keep & g2 & (a << (3 * d)); // >= 4
  uint32_t ge4;
  const uint32_t ge3 = nib_ge3_ge4(s.own, ge4) & ~HEAD;
  ge4 &= ~HEAD;
  const uint32_t ge1 = O & ~HEAD, ge2 = O & ~s.S1o & ~HEAD;
  int t = 0;
  const uint32_t cs[4] = {c1, c2, c3, c4};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    t += __builtin_popcount(cs[j] & ge1) + __builtin_popcount(cs[j] & ge2) + __builtin_popcount(cs[j] & ge3) +
         __builtin_popcount(cs[j] & ge4);
  const int hm = (hl >= 2 && !(s.S1o & HEAD)) ? 2 : 1;  // head leavers (keep drops the head at hl <= 0)
  t += hm * (int)(((c1 >> 23) & 1u) + ((c2 >> 23) & 1u) + ((c3 >> 23) & 1u) + ((c4 >> 23) & 1u));
  return t < 4 ? t : 4;
}

// Exact sub-move count of a block-free doubles turn whose bear-off is not
// open yet (not f4_bearoff_fixed), given T = f4_exact_moves (its normal
// steps, as bear-off is closed).  Block-free, the checkers never interact:
// each walks its own chain of die-d steps over free landings; a chain that
// walks below d ends with a bear-off -- but only once every own checker is
// home, which the turn can bring about iff each outside checker's chain
// reaches home (and every head checker may leave).  The longest turn then
// makes all T normal steps and then the B bear-offs: M = min(4, T + B);
// else M = min(4, T).  A sub-move lowers T + B (or T) by at most one, so
// every C_k = L_k.  (At T >= 4, M = 4; below, every chain that matters is
// at most 3 steps long.)
NARDE_FN int f4_open_moves(const Side& s, int d, int hl, int T) {
  if (T >= 4) return 4;
  const uint32_t O = s.O, fr = ~s.P & MASK24;
  // chains that end off the board: R0 = below d, R(k+1) = x whose landing
  // x - d is free and in Rk
  const uint32_t r0 = (1u << d) - 1u;
  const uint32_t r1 = ((r0 & fr) << d) & MASK24;
  const uint32_t r2 = ((r1 & fr) << d) & MASK24;
  const uint32_t r3 = ((r2 & fr) << d) & MASK24;
  const uint32_t R = (r0 | r1 | r2 | r3) & O;
  // chains that reach home (points 0..5) within 3 steps
  const uint32_t h1 = ((0x3Fu & fr) << d) & MASK24;
  const uint32_t h2 = ((h1 & fr) << d) & MASK24;
  const uint32_t h3 = ((h2 & fr) << d) & MASK24;
  const uint32_t X = O & ~0x3Fu;  // points of the checkers outside home
  const int head = (int)nib_get(s.own, 23);
  if ((X & ~(h1 | h2 | h3)) != 0u || ((X & HEAD) && head > hl)) return T;
  uint32_t ge4;
  const uint32_t ge3 = nib_ge3_ge4(s.own, ge4);
  const uint32_t Rb = R & ~HEAD;
  int B = __builtin_popcount(Rb) + __builtin_popcount(Rb & ~s.S1o) + __builtin_popcount(Rb & ge3) +
          __builtin_popcount(Rb & ge4);
  if (R & HEAD) B += head;  // every head checker leaves (checked above)
  const int t = T + B;
  return t < 4 ? t : 4;
}

// Exact sub-move count of a doubles node block-free for its k remaining
// sub-moves (dbl_block_free): the exact counts above, capped at k.  (Bear-off
// fixed for k sub-moves: the chains alone; else f4_open_moves -- if the
// outside checkers cannot all get home with a move to spare, T >= k already.)
NARDE_FN int f4_bf_moves(const Side& s, int d, int hl, int k) {
  const int T = f4_exact_moves(s, d, hl);
  const int M = f4_bearoff_fixed(s, k) ? T : f4_open_moves(s, d, hl, T);
  return M < k ? M : k;
}

// can N more sub-moves of die d be played (hl head moves still allowed)?
// A block-bound search stops at the first node that is block-free for the
// N sub-moves it has left: the exact count decides there.  (Tested on the
// top CUT levels: a device search inlines every level, and the test at all
// of them costs more registers than it saves.)
template <int N, int CUT = N>
NARDE_FN bool f4_reach(const Side& s, uint32_t low, int d, int hl, bool bf) {
  if constexpr (CUT > 0)
    if (!bf && dbl_block_free(s.O, s.S1o, s.P, low, d, N)) return f4_bf_moves(s, d, hl, N) >= N;
  uint32_t L = legal1(s, low, d, bf);
  if (hl <= 0) L &= ~HEAD;
  if constexpr (N == 1) {
    return L != 0u;
  } else {
    while (L) {
      const int p = __builtin_ctz(L);
      L &= L - 1u;
      Side c = s;
      apply_die(c, p, d);
      if (f4_reach<N - 1, (CUT > 0 ? CUT - 1 : 0)>(c, low, d, hl - (p == 23 ? 1 : 0), bf)) return true;
    }
    return false;
  }
}

// the most sub-moves of die d (up to N) playable from s: depth-first with
// early exit at N (hl head moves still allowed); block-bound searches stop
// at block-free nodes as f4_reach does
template <int N, int CUT = N>
NARDE_FN int f4_depth(const Side& s, uint32_t low, int d, int hl, bool bf) {
  if constexpr (CUT > 0)
    if (!bf && dbl_block_free(s.O, s.S1o, s.P, low, d, N)) return f4_bf_moves(s, d, hl, N);
  uint32_t L = legal1(s, low, d, bf);
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
      const int v = 1 + f4_depth<N - 1, (CUT > 0 ? CUT - 1 : 0)>(c, low, d, hl - (p == 23 ? 1 : 0), bf);
      best = v > best ? v : best;
    }
    return best;
  }
}

// the sources of L (die d) after which NEED more sub-moves stay playable:
// block-free turns try the lower bound first, the exact search only where
// it falls short
template <int NEED>
NARDE_FN uint32_t f4_keep(const Side& s, uint32_t low, int d, int hl, uint32_t L, bool bf) {
  if constexpr (NEED == 0) {
    return L;
  } else {
    uint32_t C = 0u, m = L;
    while (m) {
      const int p = __builtin_ctz(m);
      m &= m - 1u;
      const int hl2 = hl - (p == 23 ? 1 : 0);
      bool ok = false;
      if (bf) {
        uint32_t O2, S2;
        child_masks(s, p, d, O2, S2);
        ok = f4_lower_bound(O2, S2, s.P, d, hl2) >= NEED;
      }
      if (!ok) {
        Side c = s;
        apply_die(c, p, d);
        ok = f4_reach<NEED>(c, low, d, hl2, bf);
      }
      C |= ok ? (1u << p) : 0u;
    }
    return C;
  }
}

NARDE_FN uint32_t f4_keep_rt(const Side& s, uint32_t low, int d, int hl, uint32_t L, int need,
                             bool bf) {
  switch (need) {
    case 1: return f4_keep<1>(s, low, d, hl, L, bf);
    case 2: return f4_keep<2>(s, low, d, hl, L, bf);
    case 3: return f4_keep<3>(s, low, d, hl, L, bf);
    default: return L;
  }
}

// two different dice: the first sub-move's options of die a whose child can
// still play die b (a head move used up the turn's single head move);
// block-free: exact from the child's masks alone
NARDE_FN uint32_t f4_keep_pair(const Side& s, uint32_t low, int a, int b, uint32_t L, bool bf) {
  uint32_t C = 0u, m = L;
  while (m) {
    const int p = __builtin_ctz(m);
    m &= m - 1u;
    // the child's own masks are all the second list needs (no nibble update)
    uint32_t O2, S2;
    child_masks(s, p, a, O2, S2);
    uint32_t L2 = die_candidates(O2, s.P, b);
    if (!bf) L2 = die_filter(O2, S2, block_info_low(O2, low), L2, b);
    if (p == 23) L2 &= ~HEAD;
    C |= L2 ? (1u << p) : 0u;
  }
  return C;
}

// f4_keep_pair for a block-free turn, all sources at once (no per-source
// loop).  After first move p -> q = p - a (a bear-off if q < 0), the
// child's die-b list (get_valid_moves([b]) on it: no block filter can bite)
// is non-empty iff one of:
//   E1  a die-b normal source of the current board survives: X = O's normal
//       b-sources; p leaves X only if it held one checker (S1), and after a
//       head move (p = 23) the head cannot move again (one head move a turn);
//   E2  the landed checker moves on: q >= b and q - b is not an opponent
//       point (q is own after the move whatever it held);
//   E3  a bear-off with b: bear-off is allowed on the child (all own
//       checkers home: already so, or p was the single checker outside and
//       lands home) and some own checker sits below b -- one from the
//       current board (p only if it held >= 2) or the landed one (q < b).
// `nz1(Y, S1)`: the sources p for which Y minus {p if S1(p)} is non-empty.
NARDE_FN uint32_t nz1(uint32_t Y, uint32_t S1) {
  const int c = __builtin_popcount(Y);
  return c >= 2 ? MASK24 : (c == 1 ? (~(Y & S1) & MASK24) : 0u);
}
NARDE_FN uint32_t f4_keep_pair_bf(uint32_t O, uint32_t S1, uint32_t P, int a, int b, uint32_t L) {
  const uint32_t G = ~(P << b) & (MASK24 << b) & MASK24;  // y: y - b on the board, not an opponent point
  const uint32_t X = O & G;
  const uint32_t e1 = (nz1(X, S1) & ~HEAD) | (((X & ~HEAD) != 0u) ? HEAD : 0u);
  const uint32_t e2 = (G << a) & MASK24;                  // p: q = p - a in G (so q >= b >= 1)
  const uint32_t LB = (1u << b) - 1u;
  const uint32_t out = O & ~0x3Fu;
  // home after the move: already home, or p = the lone outside checker landing home
  const uint32_t homep = out == 0u ? MASK24
                         : ((out & (out - 1u)) == 0u && (out & S1) != 0u && __builtin_ctz(out) - a < 6 ? out : 0u);
  const uint32_t e3 = homep & (nz1(O & LB, S1) | ((LB << a) & MASK24));  // own below b, or q in [0, b)
  return L & (e1 | e2 | e3);
}

struct TurnOut {
  uint64_t legal;   // C_0: C_hi | C_lo<<24 | d_hi<<48 | d_lo<<52 | M<<56
  uint64_t played;  // byte 2k = from, 2k+1 = die of sub-move k; 0xFF = none
  int max_dice;
  int reward;
  int term;
};

NARDE_FN uint64_t played_set(uint64_t pl, int k, int p, int d) {
  const int sh = 16 * k;
  return (pl & ~(0xFFFFull << sh)) | ((uint64_t)(((uint32_t)d << 8) | (uint32_t)p) << sh);
}

// byte j of a play word, sign-extended (plays are int8 (from, die)[4])
NARDE_FN int play_byte(uint64_t pw, int j) { return (int)(int8_t)(uint8_t)(pw >> (8 * j)); }

// One FULL4 turn with dice (d0, d1).  !play: sub-move k is entry
// mulhi(w[k], |C_k|) of C_k (the random-legal policy); else pw holds the
// caller's int8 (from, die)[4] little-endian and sub-moves are applied while
// each is in C_k (the first one that is not ends the turn -- illegal actions
// are ignored, as in narde_env.py:56-93).  Then _check_game_ended and the
// flip (narde_env.py:95-103, 134-141).
NARDE_FN void env_turn_full(Side& s, int d0, int d1, bool play, uint64_t pw, const uint32_t w[4],
                            TurnOut& o) {
  const uint32_t low = block_lowmask(s.P);
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  const bool bf = turn_block_free(s.O, s.S1o, s.P, low, dh, dl);
  uint64_t played = ~0ull;
  int M = 0;
  if (dh != dl) {
    const uint32_t Lh = legal1(s, low, dh, bf), Ll = legal1(s, low, dl, bf);
    // block-free: every source at once from the masks (f4_keep_pair_bf);
    // else the per-source loop (lanes that skip pass an empty mask: the
    // wave's loop runs only as long as the lanes that need it)
    // block-bound: the sources sure from the masks (f4_sure_pair), the
    // per-source check for the rest
    bool bound;
    const uint32_t hs = bf ? 0u : two_block_holes(s.O, s.S1o, s.P, low, dh, dl, bound);
    const uint32_t sh = bf ? 0u : f4_sure_pair(s.O, s.P, dl, Lh, hs);
    const uint32_t sl = bf ? 0u : f4_sure_pair(s.O, s.P, dh, Ll, hs);
    uint32_t Ch = bf ? f4_keep_pair_bf(s.O, s.S1o, s.P, dh, dl, Lh) : (sh | f4_keep_pair(s, low, dh, dl, Lh & ~sh, bf));
    uint32_t Cl = bf ? f4_keep_pair_bf(s.O, s.S1o, s.P, dl, dh, Ll) : (sl | f4_keep_pair(s, low, dl, dh, Ll & ~sl, bf));
    if (Ch | Cl) {
      M = 2;
    } else {
      M = (Lh | Ll) ? 1 : 0;
      Ch = Lh;              // only one die playable: the higher one if it can
      Cl = Lh ? 0u : Ll;
    }
    o.legal = (uint64_t)Ch | ((uint64_t)Cl << 24) | ((uint64_t)dh << 48) | ((uint64_t)dl << 52) |
              ((uint64_t)M << 56);
    if (M >= 1) {
      const int nh = __builtin_popcount(Ch), n = nh + __builtin_popcount(Cl);
      int p, d;
      bool ok;
      if (play) {
        p = play_byte(pw, 0);
        d = play_byte(pw, 1);
        ok = p >= 0 && p < 24 && ((d == dh && ((Ch >> p) & 1u)) || (d == dl && ((Cl >> p) & 1u)));
      } else {
        const int idx = (int)mulhi_u32(w[0], (uint32_t)n);
        const bool hi = idx < nh;
        d = hi ? dh : dl;
        p = select_bit(hi ? Ch : Cl, hi ? idx : idx - nh);
        ok = true;
      }
      if (ok) {
        apply_die(s, p, d);
        played = played_set(played, 0, p, d);
        if (M == 2) {
          const int d2 = d == dh ? dl : dh;
          uint32_t L2 = legal1(s, low, d2, bf);
          if (p == 23) L2 &= ~HEAD;
          int p2;
          bool ok2;
          if (play) {
            p2 = play_byte(pw, 2);
            ok2 = play_byte(pw, 3) == d2 && p2 >= 0 && p2 < 24 && ((L2 >> p2) & 1u);
          } else {
            p2 = select_bit(L2, (int)mulhi_u32(w[1], (uint32_t)__builtin_popcount(L2)));
            ok2 = true;
          }
          if (ok2) {
            apply_die(s, p2, d2);
            played = played_set(played, 1, p2, d2);
          }
        }
      }
    }
  } else {
    const int d = dh;
    int hl = (s.ft_own && (d == 3 || d == 4 || d == 6)) ? 2 : 1;
    uint32_t L = legal1(s, low, d, bf);
    uint32_t C = 0u;
    // block-free: M exactly from the chains and the bear-offs they can open
    // (f4_bf_moves), and as a sub-move lowers that count by at most one,
    // every C_k = L_k (no search).  Block-bound: the same M = 4 and C_k = L_k
    // when the moves that can never be rejected give >= 4 (f4_safe_bound);
    // else the search.
    const bool fast = !bf && f4_safe_bound(s, d, hl, dbl_block_windows(s.O, s.S1o, s.P, low, d, 4)) >= 4;
    if (bf) {
      C = L;
      M = L ? f4_bf_moves(s, d, hl, 4) : 0;
    } else if (fast) {
      C = L;
      M = 4;
    } else if (L) {
      C = f4_keep<3>(s, low, d, hl, L, bf);
      M = 4;
      if (!C) { C = f4_keep<2>(s, low, d, hl, L, bf); M = 3; }
      if (!C) { C = f4_keep<1>(s, low, d, hl, L, bf); M = 2; }
      if (!C) { C = L; M = 1; }
    }
    o.legal = (uint64_t)C | ((uint64_t)d << 48) | ((uint64_t)d << 52) | ((uint64_t)M << 56);
    for (int k = 0; k < M; ++k) {
      if (k > 0) {
        L = legal1(s, low, d, bf);
        if (hl <= 0) L &= ~HEAD;
        // block-free turns never search; a block-bound one stops searching
        // once the node is block-free for the M - k sub-moves it has left:
        // on an M-path its exact count (f4_bf_moves) is >= M - k and a
        // sub-move lowers it by at most one, so every C_k = L_k
        const bool direct = bf || fast || dbl_block_free(s.O, s.S1o, s.P, low, d, M - k);
        C = direct ? L : f4_keep_rt(s, low, d, hl, L, M - k - 1, bf);
      }
      int p;
      if (play) {
        p = play_byte(pw, 2 * k);
        if (!(play_byte(pw, 2 * k + 1) == d && p >= 0 && p < 24 && ((C >> p) & 1u))) break;
      } else {
        // w[k] with a runtime k as selects (a dynamic index would put w in scratch)
        const uint32_t wk = k == 0 ? w[0] : (k == 1 ? w[1] : (k == 2 ? w[2] : w[3]));
        p = select_bit(C, (int)mulhi_u32(wk, (uint32_t)__builtin_popcount(C)));
      }
      apply_die(s, p, d);
      hl -= p == 23 ? 1 : 0;
      played = played_set(played, k, p, d);
    }
  }
  o.played = played;
  o.max_dice = M;
  o.term = s.off_own == 15u;
  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
  if (!o.term) side_flip(s);
}

// ================================================ FULL4, straight-line forms
// The device plays a ply in lockstep waves of 64 envs, one wave per SIMD.
// There a branch whose condition differs between lanes costs its VALU ->
// SALU turnaround (~30 cycles) plus ~3 scalar issue slots, whether or not a
// lane skips its body (tools/diag/issue_probe.hip: 59 cycles per divergent
// if-region around 2 VALU, 45 per ballot branch; one VALU ~4.6 cycles), and
// in a wave that holds both kinds of turn every side runs anyway.  So the
// block-free turn below computes every side and selects -- no branch but the
// loop of the block filter, which only block-bound two-dice lanes take.
// Same results as env_turn_full (tests/hostcheck: hc_turn_sl_random,
// hc_selfplay_full_sl; the GPU parity tests).

// all ones iff c (selects written as masks: the compiler turns a select
// between two computed values into a branch when one side is costly)
NARDE_FN uint32_t msk(bool c) { return 0u - (uint32_t)c; }

// die_candidates with the bear-off condition as a mask (no select the
// compiler may turn into a branch)
NARDE_FN uint32_t die_candidates_sl(uint32_t O, uint32_t P, int d) {
  const uint32_t normal = O & ~(P << d) & (MASK24 << d) & MASK24;
  const uint32_t home = 0u - (uint32_t)((O >> 6) == 0u);  // all ones iff every own checker is home
  return normal | (O & ((1u << d) - 1u) & home);
}

// apply_move when `en`, else nothing (every update masked)
NARDE_FN void apply_move_if(Side& s, int f, int t, bool en) {
  const bool off = t == OFF;
  const int tq = off ? 0 : t;
  const uint32_t cf = nib_get(s.own, f);
  const bool land = en && !off;
  const uint32_t bf = en ? (1u << f) : 0u;
  const uint32_t bt = land ? (1u << tq) : 0u;
  const uint32_t vf = en ? (0xFFFFFFFFu << (4 * (f & 7))) : 0u;
  const uint32_t vt = (land ? 1u : 0u) << (4 * (tq & 7));
  const int kf = f >> 3, kt = tq >> 3;
  s.own.w[0] += (kf == 0 ? vf : 0u) + (kt == 0 ? vt : 0u);
  s.own.w[1] += (kf == 1 ? vf : 0u) + (kt == 1 ? vt : 0u);
  s.own.w[2] += (kf == 2 ? vf : 0u) + (kt == 2 ? vt : 0u);
  const uint32_t t01 = bt & (~s.O | s.S1o);
  s.O = (s.O & (cf == 1u ? ~bf : ~0u)) | bt;
  s.S1o ^= (cf - 1u < 2u ? bf : 0u) ^ t01;
  s.off_own += (en && off) ? 1u : 0u;
  s.ft_own = en ? 0u : s.ft_own;
}

// apply_move_if(s, p, p - d < 0 ? OFF : p - d, en) with the landing as
// max(p - d, 0) and the bear-off test as its sign (no OFF round trip)
NARDE_FN void apply_die_if(Side& s, int p, int d, bool en) {
  const int t = p - d;
  const bool off = t < 0;
  const int tq = t > 0 ? t : 0;
  const uint32_t cf = nib_get(s.own, p);
  const bool land = en && !off;
  const uint32_t bf = en ? (1u << p) : 0u;
  const uint32_t bt = land ? (1u << tq) : 0u;
  const uint32_t vf = en ? (0xFFFFFFFFu << (4 * (p & 7))) : 0u;
  const uint32_t vt = (land ? 1u : 0u) << (4 * (tq & 7));
  const int kf = p >> 3, kt = tq >> 3;
  s.own.w[0] += (kf == 0 ? vf : 0u) + (kt == 0 ? vt : 0u);
  s.own.w[1] += (kf == 1 ? vf : 0u) + (kt == 1 ? vt : 0u);
  s.own.w[2] += (kf == 2 ? vf : 0u) + (kt == 2 ? vt : 0u);
  const uint32_t t01 = bt & (~s.O | s.S1o);
  s.O = (s.O & (cf == 1u ? ~bf : ~0u)) | bt;
  s.S1o ^= (cf - 1u < 2u ? bf : 0u) ^ t01;
  s.off_own += (en && off) ? 1u : 0u;
  s.ft_own = en ? 0u : s.ft_own;
}

// f4_keep_pair_bf with the home test as masks
NARDE_FN uint32_t f4_keep_pair_bf_sl(uint32_t O, uint32_t S1, uint32_t P, int a, int b, uint32_t L) {
  const uint32_t G = ~(P << b) & (MASK24 << b) & MASK24;
  const uint32_t X = O & G;
  const uint32_t e1 = (nz1(X, S1) & ~HEAD) | (((X & ~HEAD) != 0u) ? HEAD : 0u);
  const uint32_t e2 = (G << a) & MASK24;
  const uint32_t LB = (1u << b) - 1u;
  const uint32_t out = O & ~0x3Fu;
  const bool lone = (out & (out - 1u)) == 0u && (out & S1) != 0u &&
                    (int)__builtin_ctz(out | 0x80000000u) - a < 6;
  const uint32_t homep = (out == 0u ? MASK24 : 0u) | (lone ? out : 0u);
  const uint32_t e3 = homep & (nz1(O & LB, S1) | ((LB << a) & MASK24));
  return L & (e1 | e2 | e3);
}

NARDE_FN bool f4_bearoff_fixed_sl(const Side& s, int rem) {
  uint32_t x = s.own.w[0] & 0xFFFFFFu;  // points 0..5
  x = (x & 0x0F0F0Fu) + ((x >> 4) & 0x0F0F0Fu);
  const uint32_t home = ((x * 0x010101u) >> 16) & 0xFFu;
  return ((s.O >> 6) == 0u) | ((int)(15u - s.off_own - home) >= rem);
}

// f4_open_moves without its early returns
NARDE_FN int f4_open_moves_sl(const Side& s, int d, int hl, int T) {
  const uint32_t O = s.O, fr = ~s.P & MASK24;
  const uint32_t r0 = (1u << d) - 1u;
  const uint32_t r1 = ((r0 & fr) << d) & MASK24;
  const uint32_t r2 = ((r1 & fr) << d) & MASK24;
  const uint32_t r3 = ((r2 & fr) << d) & MASK24;
  const uint32_t R = (r0 | r1 | r2 | r3) & O;
  const uint32_t h1 = ((0x3Fu & fr) << d) & MASK24;
  const uint32_t h2 = ((h1 & fr) << d) & MASK24;
  const uint32_t h3 = ((h2 & fr) << d) & MASK24;
  const uint32_t X = O & ~0x3Fu;
  const int head = (int)nib_get(s.own, 23);
  const bool reach = (X & ~(h1 | h2 | h3)) == 0u && !((X & HEAD) && head > hl);
  uint32_t ge4;
  const uint32_t ge3 = nib_ge3_ge4(s.own, ge4);
  const uint32_t Rb = R & ~HEAD;
  const int B = __builtin_popcount(Rb) + __builtin_popcount(Rb & ~s.S1o) + __builtin_popcount(Rb & ge3) +
                __builtin_popcount(Rb & ge4) + ((R & HEAD) ? head : 0);
  const int t = T + (reach ? B : 0);
  return t < 4 ? t : 4;
}

// C_0 and M of a block-free turn, from the masks (env_turn_full's bf
// branches): two dice from the pair checks (f4_keep_pair_bf), doubles from
// the exact counts (f4_exact_moves, f4_open_moves).  Lh / Ll: the root
// candidates; hl0: the turn's head allowance.
NARDE_FN void turn_c0_free(const Side& s, int dh, int dl, uint32_t& Lh, uint32_t& Ll, uint32_t& Ch, uint32_t& Cl,
                           int& M, int& hl0) {
  const bool dbl = dh == dl;
  Lh = die_candidates_sl(s.O, s.P, dh);
  Ll = die_candidates_sl(s.O, s.P, dl) & msk(!dbl);
  const uint32_t kh = f4_keep_pair_bf_sl(s.O, s.S1o, s.P, dh, dl, Lh);
  const uint32_t kl = f4_keep_pair_bf_sl(s.O, s.S1o, s.P, dl, dh, Ll);
  hl0 = (dbl && s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1;
  const int T0 = f4_exact_moves(s, dh, hl0);
  const int Mo = f4_open_moves_sl(s, dh, hl0, T0);
  const int Mx = f4_bearoff_fixed_sl(s, 4) ? T0 : Mo;
  const bool pair = (kh | kl) != 0u;
  const bool two = !dbl && pair;  // two dice, both playable in some order
  Ch = (kh & msk(two)) | (Lh & msk(!two));
  Cl = (kl & msk(two)) | (Ll & msk(!dbl && !pair && Lh == 0u));
  const int M2 = two ? 2 : ((Lh | Ll) != 0u ? 1 : 0);
  M = dbl ? (Lh != 0u ? Mx : 0) : M2;
}

// turn_c0_free's results (a block-free turn's C_0 and M, the root lists,
// the head allowance), for callers that compute them before the block test
// is known (k_rollout_pp_full: the consumer wave runs the block test)
struct TurnC0 {
  uint32_t Lh, Ll, Ch, Cl;
  int M, hl0;
};

// the mover change as selects (no branch): when `flip`
NARDE_FN void side_flip_if(Side& s, bool flip) {
  Side f = s;
  side_flip(f);
  s.own.w[0] = flip ? f.own.w[0] : s.own.w[0];
  s.own.w[1] = flip ? f.own.w[1] : s.own.w[1];
  s.own.w[2] = flip ? f.own.w[2] : s.own.w[2];
  s.opp.w[0] = flip ? f.opp.w[0] : s.opp.w[0];
  s.opp.w[1] = flip ? f.opp.w[1] : s.opp.w[1];
  s.opp.w[2] = flip ? f.opp.w[2] : s.opp.w[2];
  s.O = flip ? f.O : s.O;
  s.P = flip ? f.P : s.P;
  s.S1o = flip ? f.S1o : s.S1o;
  s.S1p = flip ? f.S1p : s.S1p;
  s.off_own = flip ? f.off_own : s.off_own;
  s.off_opp = flip ? f.off_opp : s.off_opp;
  s.ft_own = flip ? f.ft_own : s.ft_own;
  s.ft_opp = flip ? f.ft_opp : s.ft_opp;
  s.black = flip ? f.black : s.black;
}

// The sub-moves of a turn whose C_0 = (Ch, Cl) and M are known, straight-
// line (all three later sub-moves computed, applied where k < M), the
// random-legal policy (w).  filt: the lane's lists are block-filtered (a
// block-bound two-dice turn with failing windows fw; its only later sub-move
// is k = 1) -- block_reject_w's loop over fw, the only loop.  Then _check_game_ended and
// the flip (every lane when flip_always: callers that auto-reset a finished
// env in the same ply).
NARDE_FN uint32_t block_reject_w(uint32_t O, uint32_t S1, uint32_t fw, uint32_t C, int d);
NARDE_FN void turn_moves_sl(Side& s, int dh, int dl, uint32_t Ch, uint32_t Cl, int M, int hl, const uint32_t w[4],
                            bool filt, uint32_t fw, bool flip_always, TurnOut& o) {
  const bool dbl = dh == dl;
  o.legal = (uint64_t)Ch | ((uint64_t)Cl << 24) | ((uint64_t)dh << 48) | ((uint64_t)dl << 52) |
            ((uint64_t)M << 56);
  const int nh = __builtin_popcount(Ch), n = nh + __builtin_popcount(Cl);
  const int idx = (int)mulhi_u32(w[0], (uint32_t)n);
  const bool hi = idx < nh;
  const int d0 = hi ? dh : dl;
  const int p0 = select_bit(hi ? Ch : Cl, hi ? idx : idx - nh);
  const bool go = M >= 1;
  apply_die_if(s, p0, d0, go);
  // the played word as two 32-bit halves (sub-moves 0-1, 2-3)
  uint32_t pl0 = go ? (0xFFFF0000u | ((uint32_t)d0 << 8) | (uint32_t)p0) : 0xFFFFFFFFu, pl1 = 0xFFFFFFFFu;
  hl -= (go && p0 == 23) ? 1 : 0;
  const int d1 = dbl ? dh : (d0 == dh ? dl : dh);
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const int dk = k == 1 ? d1 : dh;
    const bool act = k < M;
    uint32_t Lk = die_candidates_sl(s.O, s.P, dk);
    if (k == 1 && filt) Lk &= ~block_reject_w(s.O, s.S1o, fw, Lk, dk);
    Lk &= hl <= 0 ? ~HEAD : ~0u;
    const uint32_t wk = k == 1 ? w[1] : (k == 2 ? w[2] : w[3]);
    const int p = select_bit(Lk, (int)mulhi_u32(wk, (uint32_t)__builtin_popcount(Lk)));
    apply_die_if(s, p, dk, act);
    const uint32_t v = ((uint32_t)dk << 8) | (uint32_t)p;
    if (k == 1) pl0 = act ? ((pl0 & 0xFFFFu) | (v << 16)) : pl0;
    if (k == 2) pl1 = act ? ((pl1 & 0xFFFF0000u) | v) : pl1;
    if (k == 3) pl1 = act ? ((pl1 & 0xFFFFu) | (v << 16)) : pl1;
    hl -= (act && p == 23) ? 1 : 0;
  }
  o.played = (uint64_t)pl0 | ((uint64_t)pl1 << 32);
  o.max_dice = M;
  o.term = s.off_own == 15u;
  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
  if (flip_always) side_flip(s);
  else side_flip_if(s, !o.term);
}

// The block-free turn, straight-line (env_turn_full when turn_block_set is 0).
NARDE_FN void turn_free_sl(Side& s, int dh, int dl, const uint32_t w[4], bool flip_always, TurnOut& o) {
  uint32_t Lh, Ll, Ch, Cl;
  int M, hl0;
  turn_c0_free(s, dh, dl, Lh, Ll, Ch, Cl, M, hl0);
  turn_moves_sl(s, dh, dl, Ch, Cl, M, hl0, w, false, 0u, flip_always, o);
}

// ============================================== REF2, straight-line forms
// NardeEnv.step with the random-legal policy (env_step, policy = true) for
// the device's lockstep waves: the same arithmetic with every branch whose
// condition differs between lanes turned into masks, and the three block
// filters' loops merged into two (the root's two dice in one loop).  Equal
// to env_step (tests/hostcheck hc_selfplay_sl).

// die_filter of two dice on one board, one loop over both dice's risky
// single-checker sources
NARDE_FN void die_filter2(uint32_t O, uint32_t S1, const Blocks& bl, uint32_t Ca, int a, uint32_t Cb, int b,
                          uint32_t& La, uint32_t& Lb) {
  const uint32_t hitA = bl.F ? MASK24 : (bl.Q << a);
  const uint32_t hitB = bl.F ? MASK24 : (bl.Q << b);
  La = Ca & ~(hitA & ~S1);
  Lb = Cb & ~(hitB & ~S1);
  uint32_t ma = Ca & hitA & S1, mb = Cb & hitB & S1;
  while (ma | mb) {
    const bool fa = ma != 0u;
    const uint32_t m = fa ? ma : mb;
    const int d = fa ? a : b;
    const int p = __builtin_ctz(m);
    const uint32_t bp = 1u << p;
    ma &= fa ? ~bp : ~0u;
    mb &= fa ? ~0u : ~bp;
    const uint32_t Op = (O & ~bp) | (p >= d ? (1u << (p - d)) : 0u);
    const uint32_t rej = (runs6(Op) & bl.low) ? bp : 0u;
    La &= fa ? ~rej : ~0u;
    Lb &= fa ? ~0u : ~rej;
  }
}

// legal2_low (the step's list #1), straight-line but for the filter loop
NARDE_FN void legal2_low_sl(const Side& s, int d0, int d1, uint32_t low, Legal& l) {
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  const bool dbl = dh == dl;
  const Blocks bl = block_info_low(s.O, low);
  uint32_t Lh, Ll;
  die_filter2(s.O, s.S1o, bl, die_candidates_sl(s.O, s.P, dh), dh,
              die_candidates_sl(s.O, s.P, dl) & msk(!dbl), dl, Lh, Ll);
  Ll = dbl ? Lh : Ll;
  const bool two_heads = s.ft_own && dbl && (dh == 3 || dh == 4 || dh == 6);
  Ll &= ((Lh >> 23) != 0u && !two_heads) ? ~HEAD : ~0u;
  l.n = 2;
  l.d[0] = dh; l.d[1] = dl; l.d[2] = 0; l.d[3] = 0;
  l.L[0] = Lh; l.L[1] = Ll; l.L[2] = 0u; l.L[3] = 0u;
  l.count = __builtin_popcount(Lh) + __builtin_popcount(Ll);
}

// env_step(s, d0, d1, -, -, policy = true, r1, r2, o, flip_always = true)
NARDE_FN void env_step_policy_sl(Side& s, int d0, int d1, uint32_t r1, uint32_t r2, StepOut& o) {
  const uint32_t low = block_lowmask(s.P);
  legal2_low_sl(s, d0, d1, low, o.l1);
  const int n1 = o.l1.count;
  int f1, t1;
  legal2_entry(o.l1, (int)mulhi_u32(r1, (uint32_t)n1), f1, t1);
  const int code1 = n1 >= 2 ? encode_move(f1, t1) : 0;
  // the 'off' quirk: a drawn normal move (f, 0), f <= 5, decodes to (f, 'off')
  const bool quirk = n1 >= 2 && t1 == 0 && f1 <= 5;
  const uint32_t bf1 = 1u << f1;
  const bool listed_off = (((o.l1.L[0] & bf1) != 0u) & (f1 < o.l1.d[0])) | (((o.l1.L[1] & bf1) != 0u) & (f1 < o.l1.d[1]));
  t1 = quirk ? OFF : t1;
  const bool play1 = quirk ? listed_off : n1 >= 1;
  apply_move_if(s, f1, t1, play1);
  // the second list (narde_env.py:63-89): one die, the post-move board
  const bool has2 = n1 >= 2 && play1;
  const int dist = t1 == OFF ? f1 + 1 : f1 - t1;
  const int rem = (d0 == dist) ? d1 : ((d1 == dist) ? d0 : d1);
  const Blocks bl = block_info_low(s.O, low);
  uint32_t L2, unused;
  die_filter2(s.O, s.S1o, bl, die_candidates_sl(s.O, s.P, rem) & msk(has2), rem, 0u, 1, L2, unused);
  const int c2 = __builtin_popcount(L2);
  const int f2 = select_bit(L2, (int)mulhi_u32(r2, (uint32_t)c2));
  const int t2 = f2 - rem < 0 ? OFF : f2 - rem;
  const bool play2 = c2 > 0 && !(t2 == 0 && f2 <= 5);
  apply_move_if(s, f2, t2, play2);
  o.L2 = L2;
  o.d2 = has2 ? rem : 0;
  o.count2 = has2 ? c2 : -1;
  o.code1 = code1;
  o.code2 = c2 > 0 ? encode_move(f2, t2) : 0;
  o.term = s.off_own == 15u;
  o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
  side_flip(s);
}

// f4_depth<N, 0> of a block-bound doubles node with the lists filtered by
// the turn's failing windows (block_reject_w: a loop over the windows,
// usually one, instead of block_info_low + die_filter's per-source loop at
// every node of the search)
template <int N>
NARDE_FN int f4_depth_w(const Side& s, uint32_t fw, int d, int hl) {
  uint32_t L = die_candidates_sl(s.O, s.P, d);
  L &= ~block_reject_w(s.O, s.S1o, fw, L, d);
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
      const int v = 1 + f4_depth_w<N - 1>(c, fw, d, hl - (p == 23 ? 1 : 0));
      best = v > best ? v : best;
    }
    return best;
  }
}

// The first path f4_depth_w<N> walks (the lowest listed source at every
// node), straight-line: its depth, which is f4_depth_w's whenever it reaches
// N (the search stops there) -- so only a lane whose probe falls short needs
// the search.  (Doubles searches end at depth N along this path in ~90 % of
// the block-bound turns that f4_safe_bound leaves)
template <int N>
NARDE_FN int f4_probe_w(Side c, uint32_t fw, int d, int hl) {
  int dep = 0;
  bool alive = true;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    uint32_t L = die_candidates_sl(c.O, c.P, d);
    L &= ~block_reject_w(c.O, c.S1o, fw, L, d);
    L &= hl <= 0 ? ~HEAD : ~0u;
    alive = alive && L != 0u;
    dep += alive ? 1 : 0;
    if (k + 1 < N) {
      const int p = (int)__builtin_ctz(L | 0x800000u);  // 23 when L is empty (nothing applied then)
      apply_die_if(c, p, d, alive);
      hl -= (alive && p == 23) ? 1 : 0;
    }
  }
  return dep;
}

// turn_block_set without its early exit, straight-line over the kinds of
// turn (a wave holds both): the windows that can fill, then one loop per
// kind over its lanes' windows (a wave pays a kind's loop only where a lane
// of that kind has a window; round 3's single loop computed both kinds'
// tests in every iteration).  Windows whose holes are too far from the own
// points for the turn's steps never enter a loop: 1.46 -> 0.94 + 0.36
// iterations per wave-ply (host statistics of random self-play).
// fw (out): the failing windows' start points (bit i = points i..i+5): the
// only windows that can be full at a node of the turn (block_reject_w)
NARDE_FN uint32_t turn_block_set_sl(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl,
                                    uint32_t& fw) {
  const bool dbl = dh == dl;
  const uint32_t A = O | land_step(O, P, dh) | land_step(O, P, dl);  // one step
  const uint32_t U2 = A | land_step(A, P, dh) | land_step(A, P, dl);  // two
  const uint32_t V = land_step(U2, P, dh);
  const uint32_t U = U2 | (dbl ? (V | land_step(V, P, dh)) : 0u);     // doubles: four
  uint32_t s0, s1, s2;
  window_hole_count(O, s0, s1, s2);
  const uint32_t le1 = ~s2 & ~s1, le2 = ~s2 & ~(s1 & s0), eq2 = s1 & ~s0 & ~s2;
  const uint32_t eq3 = s1 & s0 & ~s2, eq4 = s2 & ~s1 & ~s0;
  const uint32_t rU = runs6(U) & low, rA = runs6(A) & low;
  // the landings' steps to a window's holes sum to at most 4 (doubles) or
  // each hole takes one sub-move (two dice): three or four holes need every
  // hole within two / one steps, two holes with two dice one step each
  uint32_t win2 = dbl ? 0u : ((le1 & rU) | (eq2 & rA));
  uint32_t wind = dbl ? ((le2 & rU) | (eq3 & runs6(U2) & low) | (eq4 & rA)) : 0u;
  uint32_t out = 0u;
  bool full = false;
  fw = 0u;
  while (win2) {  // two dice
    const int i = __builtin_ctz(win2);
    win2 &= win2 - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    full = full || H == 0u;
    const uint32_t src = O & ~(W & S1);
    const uint32_t Lh = land_step(src, P, dh), Ll = land_step(src, P, dl);
    const uint32_t h1 = H & (0u - H), h2 = H ^ h1;
    // (bitwise: && / || would branch)
    const bool one = (H & (Lh | Ll | land_step(Lh, P, dl) | land_step(Ll, P, dh))) != 0u;
    const bool two = (((h1 & Lh) != 0u) & ((h2 & Ll) != 0u)) | (((h1 & Ll) != 0u) & ((h2 & Lh) != 0u));
    const bool tfail = h2 == 0u ? one : two;
    out |= H & msk(tfail);
    fw |= (H == 0u || tfail) ? (1u << i) : 0u;
  }
  while (wind) {  // doubles
    const int i = __builtin_ctz(wind);
    wind &= wind - 1u;
    const uint32_t W = 0x3Fu << i;
    const uint32_t H = W & ~O;
    full = full || H == 0u;
    uint32_t T = O & ~(W & S1), seen = 0u;
    int cost = 0;
#pragma unroll
    for (int j = 1; j <= 4; ++j) {
      T = land_step(T, P, dh);
      const uint32_t nw = H & T & ~seen;
      cost += j * __builtin_popcount(nw);
      seen |= nw;
    }
    const bool dfail = seen == H && cost <= 4;
    out |= W & msk(dfail);
    fw |= (H == 0u || dfail) ? (1u << i) : 0u;
  }
  return full ? ~0u : out;
}
NARDE_FN uint32_t turn_block_set_sl(uint32_t O, uint32_t S1, uint32_t P, uint32_t low, int dh, int dl) {
  uint32_t fw;
  return turn_block_set_sl(O, S1, P, low, dh, dl, fw);
}

// The block filter of one die from a turn's failing windows fw, masks only
// (die_filter's result at any node of the turn, whose full windows can only
// be failing ones): a candidate x -> x - d is rejected iff it leaves some
// failing window W full -- W full already (no hole) and x not a single
// checker of W, or W's one hole is the landing and x not a single checker of
// W.  A loop over the failing windows (usually one), no per-source loop.
NARDE_FN uint32_t block_reject_w1(uint32_t O, uint32_t S1, uint32_t W, uint32_t C, int d) {
  const uint32_t H = W & ~O;
  const uint32_t stay = C & ~(W & S1);  // moving it does not open a hole in W
  const uint32_t one = (H & (H - 1u)) == 0u ? (H << d) : 0u;  // landing on the one hole
  return H == 0u ? stay : (stay & one & MASK24);
}
NARDE_FN uint32_t block_reject_w(uint32_t O, uint32_t S1, uint32_t fw, uint32_t C, int d) {
  // the lowest window outside the loop (usually the only one): no loop
  // iteration's branches when there is one window
  uint32_t rej = block_reject_w1(O, S1, (0x3Fu << (__builtin_ctz(fw | 0x80000000u) & 31)) & MASK24, C, d);
  rej &= msk(fw != 0u);
  for (uint32_t f = fw & (fw - 1u); f; f &= f - 1u) rej |= block_reject_w1(O, S1, 0x3Fu << __builtin_ctz(f), C, d);
  return rej;
}

// after first move p of die a (a two-dice turn with failing windows fw):
// does die b still have a move (head rule: not a second head move)?
NARDE_FN bool pair_child_ok_w(const Side& s, uint32_t fw, int p, int a, int b) {
  uint32_t O2, S2;
  child_masks(s, p, a, O2, S2);
  const uint32_t Cb = die_candidates_sl(O2, s.P, b) & (p == 23 ? ~HEAD : ~0u);
  return (Cb & ~block_reject_w(O2, S2, fw, Cb, b)) != 0u;
}

// turn_c0_pair_bound from the failing windows (hs: their holes, fw: their
// starts; turn_block_set_sl): the lists filtered by block_reject_w, the sure
// first moves from the masks (f4_sure_pair), the child check for the rest in
// one loop over both dice's unsure sources (usually none)
NARDE_FN void turn_c0_pair_bound_w(const Side& s, int dh, int dl, uint32_t hs, uint32_t fw, uint32_t& Lh,
                                   uint32_t& Ll, uint32_t& Ch, uint32_t& Cl, int& M) {
  const uint32_t Chc = die_candidates_sl(s.O, s.P, dh), Clc = die_candidates_sl(s.O, s.P, dl);
  // both dice's lists through one loop over the failing windows
  // (block_reject_w twice, the window masks shared)
  uint32_t rh = 0u, rl = 0u;
  for (uint32_t f = fw; f; f &= f - 1u) {
    const uint32_t W = 0x3Fu << __builtin_ctz(f);
    const uint32_t H = W & ~s.O;
    const bool one = (H & (H - 1u)) == 0u;
    const uint32_t keep = ~(W & s.S1o);
    rh |= H == 0u ? (Chc & keep) : (Chc & keep & (one ? (H << dh) : 0u) & MASK24);
    rl |= H == 0u ? (Clc & keep) : (Clc & keep & (one ? (H << dl) : 0u) & MASK24);
  }
  Lh = Chc & ~rh;
  Ll = Clc & ~rl;
  uint32_t kh = f4_sure_pair(s.O, s.P, dl, Lh, hs), kl = f4_sure_pair(s.O, s.P, dh, Ll, hs);
  uint32_t mh = Lh & ~kh, ml = Ll & ~kl;
  while (mh | ml) {
    const bool hi = mh != 0u;
    const int p = __builtin_ctz(hi ? mh : ml);
    const uint32_t bp = 1u << p;
    mh &= hi ? ~bp : ~0u;
    ml &= hi ? ~0u : ~bp;
    const bool ok = pair_child_ok_w(s, fw, p, hi ? dh : dl, hi ? dl : dh);
    kh |= (hi && ok) ? bp : 0u;
    kl |= (!hi && ok) ? bp : 0u;
  }
  const bool pair = (kh | kl) != 0u;
  Ch = pair ? kh : Lh;
  Cl = pair ? kl : (Lh ? 0u : Ll);
  M = pair ? 2 : ((Lh | Ll) ? 1 : 0);
}

// obs = get_perspective_board(current_player) (narde.py:31-34): int32[24]
NARDE_FN int obs_point(const Side& s, int p) { return (int)nib_get(s.own, p) - (int)nib_get(s.opp, p); }

// ------------------------------------------------------------- Philox4x32-10
NARDE_FN void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                            uint32_t k1, uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// dice_mode 0: 36 ordered pairs; 1: the 30 ordered non-double pairs
NARDE_FN void dice_from(uint32_t r, int dice_mode, int& d0, int& d1) {
  if (dice_mode == 1) {
    const uint32_t k = mulhi_u32(r, 30u);
    const uint32_t q = (k * 205u) >> 10;  // k / 5 for k < 30
    const int a = (int)q + 1, j = (int)(k - 5u * q);
    d0 = a;
    d1 = j < a - 1 ? j + 1 : j + 2;
  } else {
    const uint32_t k = mulhi_u32(r, 36u);
    const uint32_t q = (k * 43u) >> 8;  // k / 6 for k < 36, a full-rate 24-bit multiply
    d0 = (int)q + 1;
    d1 = (int)(k - 6u * q) + 1;
  }
}

// opening roll (narde_env.py:111-117): uniform over the 30 unequal ordered
// pairs (same law as the reference's redraw loop); higher roll = white moves
// first.  reset_black: the side to move of the new episode (1 = black)
NARDE_FN uint32_t reset_black(uint32_t r) {
  int w, b;
  dice_from(r, 1, w, b);
  return w > b ? 0u : 1u;
}
NARDE_FN Side side_reset(uint32_t r) { return side_start(reset_black(r)); }

// The ply stream.  One Philox4x32-10 block serves two
// consecutive plies of an env: R = Philox(ctr = {t >> 1, env, 0, 0}); ply t
// takes (wa, wb) = (R0, R1) if t is even, (R2, R3) if odd, and derives the
// four words it consumes:
//   r0 = wa                 dice (mulhi(r0, 36), or 30 non-double pairs)
//   r1 = wa * m mod 2^32    policy pick 1: the low part the dice draw leaves
//                           (m = 36, or 30), uniform and independent of it
//   r2 = wb                 policy pick 2
//   r3 = wb * 0x9E3779B9    opening roll of the next episode (odd multiplier)
NARDE_FN void ply_words(uint32_t wa, uint32_t wb, int dice_mode, uint32_t r[4]) {
  r[0] = wa;
  r[1] = wa * (dice_mode == 1 ? 30u : 36u);
  r[2] = wb;
  r[3] = wb * 0x9E3779B9u;
}

// the Philox block of ply t (shared by plies 2j and 2j + 1)
NARDE_FN void ply_block(uint32_t t, uint32_t env, uint32_t k0, uint32_t k1, uint32_t R[4]) {
  philox4x32_10(t >> 1, env, 0u, 0u, k0, k1, R);
}

NARDE_FN void ply_words_of(const uint32_t R[4], uint32_t t, int dice_mode, uint32_t r[4]) {
  const bool odd = (t & 1u) != 0u;
  ply_words(odd ? R[2] : R[0], odd ? R[3] : R[1], dice_mode, r);
}

// The end of every ply after its turn (narde_env.py:95-103 done, then the
// gymnasium TimeLimit and the auto-reset): elapsed, terminated/truncated,
// the statistics at an episode end, the next episode's opening roll from
// r3, and t += 1.
NARDE_FN void ply_close(Side& s, int4& st, int o_term, int o_reward, uint32_t mover_black, uint32_t r3,
                        int max_steps, bool autoreset, int& term, int& trunc) {
  s.elapsed += 1u;
  term = o_term;
  trunc = max_steps > 0 && s.elapsed >= (uint32_t)max_steps;
  if (term | trunc) {
    st.x += 1;
    if (term) {
      if (mover_black) st.z += o_reward;
      else st.y += o_reward;
    }
    if (autoreset) {
      const uint32_t t = s.t;
      s = side_reset(r3);
      s.t = t;
    }
  }
  s.t += 1u;
}

// ply_close with auto-reset as selects (the reset state is mostly constants);
// rb = reset_black(r3) of the ply's words
NARDE_FN void ply_close_sl_b(Side& s, int4& st, int o_term, int o_reward, uint32_t mover_black, uint32_t rb,
                             int max_steps, int& term, int& trunc) {
  s.elapsed += 1u;
  term = o_term;
  trunc = max_steps > 0 && s.elapsed >= (uint32_t)max_steps;
  const bool end = (term | trunc) != 0;
  st.x += end ? 1 : 0;
  st.y += (term && !mover_black) ? o_reward : 0;
  st.z += (term && mover_black) ? o_reward : 0;
  const Side r = side_start(rb);
  s.own.w[0] = end ? r.own.w[0] : s.own.w[0];
  s.own.w[1] = end ? r.own.w[1] : s.own.w[1];
  s.own.w[2] = end ? r.own.w[2] : s.own.w[2];
  s.opp.w[0] = end ? r.opp.w[0] : s.opp.w[0];
  s.opp.w[1] = end ? r.opp.w[1] : s.opp.w[1];
  s.opp.w[2] = end ? r.opp.w[2] : s.opp.w[2];
  s.O = end ? r.O : s.O;
  s.P = end ? r.P : s.P;
  s.S1o = end ? r.S1o : s.S1o;
  s.S1p = end ? r.S1p : s.S1p;
  s.off_own = end ? r.off_own : s.off_own;
  s.off_opp = end ? r.off_opp : s.off_opp;
  s.ft_own = end ? r.ft_own : s.ft_own;
  s.ft_opp = end ? r.ft_opp : s.ft_opp;
  s.black = end ? r.black : s.black;
  s.elapsed = end ? 0u : s.elapsed;
  s.t += 1u;
}
NARDE_FN void ply_close_sl(Side& s, int4& st, int o_term, int o_reward, uint32_t mover_black, uint32_t r3,
                           int max_steps, int& term, int& trunc) {
  ply_close_sl_b(s, st, o_term, o_reward, mover_black, reset_black(r3), max_steps, term, trunc);
}

// the four pick words of a FULL4 turn (see env_ply_full_with)
NARDE_FN void turn_words(const uint32_t r[4], uint32_t w[4]) {
  w[0] = r[1];
  w[1] = r[2];
  w[2] = r[1] * 0x85EBCA6Bu;
  w[3] = r[2] * 0xC2B2AE35u;
}

// One ply for one env: NardeEnv.step + gymnasium TimeLimit
// (max_episode_steps, gym_narde/__init__.py:3-7) + optional auto-reset,
// then t += 1.
// r = the ply's words (ply_words above): r0 dice (unless given), r1/r2
// policy picks, r3 opening roll of the next episode.  st = {episodes,
// white points, black points} increments.
NARDE_FN void env_ply(Side& s, int4& st, const uint32_t r[4], bool have_dice, int d0, int d1,
                      int dice_mode, bool policy, int c1, int c2, int max_steps, bool autoreset,
                      StepOut& o, int& term, int& trunc) {
  if (!have_dice) dice_from(r[0], dice_mode, d0, d1);
  // a caller-given die outside 1..6 (no roll has one; the reference would
  // scan with it, narde.py:64-77): a ply with no legal move
  const bool bad = have_dice && ((uint32_t)(d0 - 1) > 5u || (uint32_t)(d1 - 1) > 5u);
  if (bad) d0 = d1 = 1;
  const uint32_t mover_black = s.black;
  env_step(s, d0, d1, c1, c2, policy, r[1], r[2], o, autoreset, bad);
  ply_close(s, st, o.term, o.reward, mover_black, r[3], max_steps, autoreset, term, trunc);
}

// env_ply with device dice, the random-legal policy and auto-reset,
// straight-line (env_step_policy_sl, ply_close_sl): the rollouts' ply
NARDE_FN void env_ply_policy_sl(Side& s, int4& st, const uint32_t r[4], int dice_mode, int max_steps, StepOut& o,
                                int& term, int& trunc) {
  int d0, d1;
  dice_from(r[0], dice_mode, d0, d1);
  const uint32_t mover_black = s.black;
  env_step_policy_sl(s, d0, d1, r[1], r[2], o);
  ply_close_sl(s, st, o.term, o.reward, mover_black, r[3], max_steps, term, trunc);
}

// One FULL4 ply: env_ply with a whole turn per step.  Pick words w = {r1,
// r2, r1 * 0x85EBCA6B, r2 * 0xC2B2AE35} (mod 2^32): sub-moves 2 and 3 of a
// doubles turn take the high bits of odd multiples of the first two words
// (a multiplicative hash of independent Philox outputs) instead of a second
// Philox block -- every wave rolls a double on nearly every ply, so that
// block cost a whole Philox per ply.
// Turn = the function that plays the turn (env_turn_full, or the device's
// wave-cooperative equivalent), called as turn(s, d0, d1, play, pw, w, o)
// with every lane converged.
template <class Turn>
NARDE_FN void env_ply_full_with(Side& s, int4& st, const uint32_t r[4], uint32_t env, uint32_t k0,
                                uint32_t k1, bool have_dice, int d0, int d1, int dice_mode, bool play,
                                uint64_t pw, int max_steps, bool autoreset, TurnOut& o, int& term,
                                int& trunc, Turn&& turn) {
  if (!have_dice) dice_from(r[0], dice_mode, d0, d1);
  // a caller-given die outside 1..6: a turn with no legal move (the turn
  // still runs on valid dice -- the device turn is wave-cooperative -- and
  // its result is dropped)
  const bool bad = have_dice && ((uint32_t)(d0 - 1) > 5u || (uint32_t)(d1 - 1) > 5u);
  if (bad) { d0 = 1; d1 = 2; }
  uint32_t w[4];
  turn_words(r, w);
  (void)env; (void)k0; (void)k1;
  const uint32_t mover_black = s.black;
  const Side before = s;
  turn(s, d0, d1, play, pw, w, o);
  if (bad) {
    s = before;
    o.legal = 0ull;
    o.played = ~0ull;
    o.max_dice = 0;
    o.term = s.off_own == 15u;
    o.reward = o.term ? (s.off_opp > 0u ? 1 : 2) : 0;
    if (!o.term) side_flip(s);
  }
  ply_close(s, st, o.term, o.reward, mover_black, r[3], max_steps, autoreset, term, trunc);
}

NARDE_FN void env_ply_full(Side& s, int4& st, const uint32_t r[4], uint32_t env, uint32_t k0,
                           uint32_t k1, bool have_dice, int d0, int d1, int dice_mode, bool play,
                           uint64_t pw, int max_steps, bool autoreset, TurnOut& o, int& term,
                           int& trunc) {
  env_ply_full_with(s, st, r, env, k0, k1, have_dice, d0, d1, dice_mode, play, pw, max_steps,
                    autoreset, o, term, trunc,
                    [](Side& s2, int a, int b, bool pl, uint64_t pw2, const uint32_t* w2, TurnOut& o2) {
                      env_turn_full(s2, a, b, pl, pw2, w2, o2);
                    });
}

}  // namespace narde
