// hostcheck.cpp -- TEST-ONLY host build of the device rules engine.
//
// Compiles gym-narde_amd/csrc/narde_rules.h (__host__ __device__) for the
// CPU so the bitmask formulation can be diffed against the oracle and the
// golden vectors in a container without a GPU.  It mirrors the per-lane
// bodies of k_legal / k_step / k_selfplay / k_reset.  Never loaded by the
// product: the product path is libnarde.so on the GPU and fails loudly
// without it.  The GPU tests (tests/test_gpu_*.py) are the parity tests.
#include <cstring>

#include "../../gym-narde_amd/csrc/narde_rules.h"

using namespace narde;

static void draw(uint64_t seed, uint32_t t, uint32_t env, uint32_t stream, uint32_t r[4]) {
  philox4x32_10(t, env, 0u, stream, (uint32_t)seed, (uint32_t)(seed >> 32), r);
}

// the words of ply t (narde_rules.h ply_words), a fresh Philox block per ply
static void ply_draw(uint64_t seed, uint32_t t, uint32_t env, int dice_mode, uint32_t r[4]) {
  uint32_t R[4];
  ply_block(t, env, (uint32_t)seed, (uint32_t)(seed >> 32), R);
  ply_words_of(R, t, dice_mode, r);
}

static Side load(const int8_t* board, const uint8_t* off, const uint8_t* ft, int player,
                 uint32_t elapsed) {
  uint4 a, b;
  record_from_board(board, off[0], off[1], ft[0], ft[1], player, elapsed, 0u, a, b);
  return side_from_record(a, b);
}

static void store(const Side& s, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                  uint16_t* elapsed) {
  uint4 a, b;
  side_to_record(s, a, b);
  board_from_record(a, b, board, off, ft, player, elapsed);
}

static void expand(const Legal& l, int8_t* out /*[64][2]*/) {
  memset(out, -1, 128);
  int e = 0;
  for (int k = 0; k < l.n; ++k) {
    uint32_t m = l.L[k];
    while (m) {
      const int f = __builtin_ctz(m);
      m &= m - 1u;
      out[2 * e] = (int8_t)f;
      out[2 * e + 1] = (int8_t)(f - l.d[k] < 0 ? OFF : f - l.d[k]);
      ++e;
    }
  }
}

extern "C" {

void hc_legal_batch(int64_t n, const int8_t* board, const uint8_t* off, const uint8_t* ft,
                    const int8_t* player, const uint8_t* roll4, int8_t* moves, int16_t* count) {
  for (int64_t i = 0; i < n; ++i) {
    const Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    Legal l;
    legal_roll(s, roll4 + 4 * i, l);
    count[i] = (int16_t)l.count;
    expand(l, moves + i * 128);
  }
}

void hc_step_batch(int64_t n, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                   const uint8_t* dice, const int16_t* action, int8_t* obs, int8_t* reward,
                   uint8_t* term, int8_t* list1, int16_t* count1, int8_t* list2, int16_t* count2) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    StepOut o;
    env_step(s, dice[2 * i], dice[2 * i + 1], action[2 * i], action[2 * i + 1], false, 0, 0, o);
    for (int p = 0; p < 24; ++p) obs[i * 24 + p] = (int8_t)obs_point(s, p);
    reward[i] = (int8_t)o.reward;
    term[i] = (uint8_t)o.term;
    count1[i] = (int16_t)o.l1.count;
    expand(o.l1, list1 + i * 128);
    count2[i] = (int16_t)o.count2;
    Legal l2;
    l2.n = 1; l2.L[0] = o.L2; l2.d[0] = o.d2; l2.count = o.count2;
    if (o.count2 >= 0) expand(l2, list2 + i * 128);
    else memset(list2 + i * 128, -1, 128);
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, player + i, nullptr);
  }
}

// k_play_set's per-lane body (narde_rules.h play_walk); dice in roll order
void hc_play_set(int64_t n, const int8_t* board, const uint8_t* off, const uint8_t* ft, const int8_t* player,
                 const uint8_t* dice, int kind, uint64_t* legal, uint32_t* table, int32_t* count) {
  for (int64_t i = 0; i < n; ++i) {
    const Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    uint32_t* row = table + i * 48;
    memset(row, 0, 48 * sizeof(uint32_t));
    const int d0 = dice[2 * i], d1 = dice[2 * i + 1];
    if (d0 < 1 || d0 > 6 || d1 < 1 || d1 > 6) {
      legal[i] = 0;
      count[i] = 0;
      continue;
    }
    Legal l;
    legal2(s, d0, d1, l);
    legal[i] = (uint64_t)l.L[0] | ((uint64_t)l.L[1] << 24) | ((uint64_t)l.d[0] << 48) | ((uint64_t)l.d[1] << 52);
    count[i] = play_walk(s, d0, d1, kind, l, [&](int k, int p, int, uint32_t w, bool) { row[k * 24 + p] = w; });
  }
}

// play_codes_act for every play index j < count of env 0's roll (dice in
// roll order): codes[2 j], codes[2 j + 1]
int hc_play_codes_act(const int8_t* board, const uint8_t* off, const uint8_t* ft, int8_t player,
                      const uint8_t* dice, int16_t* codes, int cap) {
  const Side s = load(board, off, ft, player, 0);
  Legal l;
  legal2(s, dice[0], dice[1], l);
  const int cnt = play_walk(s, dice[0], dice[1], kPlayAct, l, [](int, int, int, uint32_t, bool) {});
  for (int j = 0; j < cnt && j < cap; ++j) {
    int c1, c2;
    play_codes_act(s, dice[0], dice[1], l, j, c1, c2);
    codes[2 * j] = (int16_t)c1;
    codes[2 * j + 1] = (int16_t)c2;
  }
  return cnt;
}

// k_act_masks' per-lane body; move1 < 0 = the move-1 mask
void hc_act_masks(int64_t n, const int8_t* board, const uint8_t* off, const uint8_t* ft, const int8_t* player,
                  const uint8_t* dice, const int16_t* move1, uint64_t* mask) {
  for (int64_t i = 0; i < n; ++i) {
    const Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    Legal l;
    legal2(s, dice[2 * i], dice[2 * i + 1], l);
    act_masks(s, dice[2 * i], dice[2 * i + 1], l, move1 ? move1[i] : -1, mask + 9 * i);
  }
}

void hc_reset_batch(int64_t n, int64_t env0, uint64_t seed, uint32_t epoch, int8_t* board,
                    uint8_t* off, uint8_t* ft, int8_t* player, uint16_t* elapsed) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t r[4];
    draw(seed, epoch, (uint32_t)(env0 + i), 1u, r);
    store(side_reset(r[0]), board + i * 24, off + 2 * i, ft + 2 * i, player + i, elapsed + i);
  }
}

// the compact list-#1 word the rollouts store (kernels_state.h compact_legal)
static uint64_t compact2(const Legal& l) {
  return (uint64_t)l.L[0] | ((uint64_t)l.L[1] << 24) | ((uint64_t)l.d[0] << 48) | ((uint64_t)l.d[1] << 52);
}

void hc_selfplay(int64_t n, int64_t env0, uint64_t seed, uint32_t t0, int plies, int dice_mode,
                 int max_steps, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                 uint16_t* elapsed, int32_t* stats, int8_t* obs, int8_t* reward, uint8_t* term,
                 uint8_t* trunc, uint8_t* dice_out, int16_t* action_out, int16_t* count1_out,
                 uint64_t* legal_out) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], elapsed[i]);
    int4 st = make_int4(0, 0, 0, 0);
    for (int p = 0; p < plies; ++p) {
      uint32_t r[4];
      ply_draw(seed, t0 + (uint32_t)p, (uint32_t)(env0 + i), dice_mode, r);
      int d0, d1;
      dice_from(r[0], dice_mode, d0, d1);
      StepOut o;
      int tm, tr;
      env_ply(s, st, r, true, d0, d1, dice_mode, true, 0, 0, max_steps, true, o, tm, tr);
      const int64_t ix = (int64_t)p * n + i;
      if (obs)
        for (int q = 0; q < 24; ++q) obs[ix * 24 + q] = (int8_t)obs_point(s, q);
      if (reward) reward[ix] = (int8_t)o.reward;
      if (term) term[ix] = (uint8_t)tm;
      if (trunc) trunc[ix] = (uint8_t)tr;
      if (dice_out) { dice_out[2 * ix] = (uint8_t)d0; dice_out[2 * ix + 1] = (uint8_t)d1; }
      if (action_out) { action_out[2 * ix] = (int16_t)o.code1; action_out[2 * ix + 1] = (int16_t)o.code2; }
      if (count1_out) count1_out[ix] = (int16_t)o.l1.count;
      if (legal_out) legal_out[ix] = compact2(o.l1);
    }
    stats[3 * i] += st.x;
    stats[3 * i + 1] += st.y;
    stats[3 * i + 2] += st.z;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, player + i, elapsed + i);
  }
}

// FULL4 turns with given dice and pick words (mirror of or_full4_batch):
// post-turn state without the flip, C_0 compact, played sub-moves.
void hc_full4_batch(int64_t n, int8_t* board, uint8_t* off, uint8_t* ft, const int8_t* player,
                    const uint8_t* dice, const uint32_t* words, uint64_t* legal, uint64_t* played,
                    int8_t* reward, uint8_t* done) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    TurnOut o;
    env_turn_full(s, dice[2 * i], dice[2 * i + 1], false, 0ull, words + 4 * i, o);
    if (!o.term) side_flip(s);  // undo the flip: compare the mover's post-turn board
    legal[i] = o.legal;
    played[i] = o.played;
    reward[i] = (int8_t)o.reward;
    done[i] = (uint8_t)o.term;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, nullptr, nullptr);
  }
}

// FULL4 turns with explicit plays int8 (from, die)[4] (the narde_step_full
// action path).
void hc_full4_play_batch(int64_t n, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                         const uint8_t* dice, const int8_t* play, uint64_t* played) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    TurnOut o;
    const uint32_t w[4] = {0, 0, 0, 0};
    uint64_t pw;
    memcpy(&pw, play + 8 * i, 8);
    env_turn_full(s, dice[2 * i], dice[2 * i + 1], true, pw, w, o);
    played[i] = o.played;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, player + i, nullptr);
  }
}

void hc_selfplay_full(int64_t n, int64_t env0, uint64_t seed, uint32_t t0, int plies, int dice_mode,
                      int max_steps, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                      uint16_t* elapsed, int32_t* stats, int8_t* obs, int8_t* reward, uint8_t* term,
                      uint8_t* trunc, uint64_t* legal_out, uint64_t* played_out) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], elapsed[i]);
    s.t = t0;
    int4 st = make_int4(0, 0, 0, 0);
    for (int p = 0; p < plies; ++p) {
      uint32_t r[4];
      ply_draw(seed, s.t, (uint32_t)(env0 + i), dice_mode, r);
      TurnOut o;
      int tm, tr;
      env_ply_full(s, st, r, (uint32_t)(env0 + i), (uint32_t)seed, (uint32_t)(seed >> 32), false, 0,
                   0, dice_mode, false, 0ull, max_steps, true, o, tm, tr);
      const int64_t ix = (int64_t)p * n + i;
      if (obs)
        for (int q = 0; q < 24; ++q) obs[ix * 24 + q] = (int8_t)obs_point(s, q);
      if (reward) reward[ix] = (int8_t)o.reward;
      if (term) term[ix] = (uint8_t)tm;
      if (trunc) trunc[ix] = (uint8_t)tr;
      if (legal_out) legal_out[ix] = o.legal;
      if (played_out) played_out[ix] = o.played;
    }
    stats[3 * i] += st.x;
    stats[3 * i + 1] += st.y;
    stats[3 * i + 2] += st.z;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, player + i, elapsed + i);
  }
}

// hc_selfplay through the rollouts' straight-line REF2 ply (env_ply_policy_sl)
void hc_selfplay_sl(int64_t n, int64_t env0, uint64_t seed, uint32_t t0, int plies, int dice_mode,
                    int max_steps, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                    uint16_t* elapsed, int32_t* stats, int8_t* obs, int8_t* reward, uint8_t* term,
                    uint8_t* trunc, uint8_t* dice_out, int16_t* action_out, int16_t* count1_out,
                    uint64_t* legal_out) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], elapsed[i]);
    int4 st = make_int4(0, 0, 0, 0);
    for (int p = 0; p < plies; ++p) {
      uint32_t r[4];
      ply_draw(seed, t0 + (uint32_t)p, (uint32_t)(env0 + i), dice_mode, r);
      int d0, d1;
      dice_from(r[0], dice_mode, d0, d1);
      StepOut o;
      int tm, tr;
      env_ply_policy_sl(s, st, r, dice_mode, max_steps, o, tm, tr);
      const int64_t ix = (int64_t)p * n + i;
      if (obs)
        for (int q = 0; q < 24; ++q) obs[ix * 24 + q] = (int8_t)obs_point(s, q);
      if (reward) reward[ix] = (int8_t)o.reward;
      if (term) term[ix] = (uint8_t)tm;
      if (trunc) trunc[ix] = (uint8_t)tr;
      if (dice_out) { dice_out[2 * ix] = (uint8_t)d0; dice_out[2 * ix + 1] = (uint8_t)d1; }
      if (action_out) { action_out[2 * ix] = (int16_t)o.code1; action_out[2 * ix + 1] = (int16_t)o.code2; }
      if (count1_out) count1_out[ix] = (int16_t)o.l1.count;
      if (legal_out) legal_out[ix] = compact2(o.l1);
    }
    stats[3 * i] += st.x;
    stats[3 * i + 1] += st.y;
    stats[3 * i + 2] += st.z;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, player + i, elapsed + i);
  }
}

// ---- the device's straight-line FULL4 turn (round 4) ----------------------
// kernels_rollout.h ply_policy_full per lane: turn_block_set_sl; a lane whose
// turn is not a block-bound double takes the straight-line forms
// (turn_c0_free, turn_c0_pair_bound for a block-bound two-dice turn,
// turn_moves_sl), a block-bound double the general turn (on the device the
// cooperative one, equal to env_turn_full).  flip_always as on the device's
// auto-resetting rollouts.
static void turn_device_sl(Side& s, int d0, int d1, const uint32_t w[4], bool flip_always, TurnOut& o) {
  const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
  const uint32_t low = block_lowmask(s.P);
  uint32_t fw;
  const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, low, dh, dl, fw);
  if (bs != 0u && dh == dl) {
    env_turn_full(s, d0, d1, false, 0ull, w, o);
    if (flip_always && o.term) side_flip(s);
    return;
  }
  uint32_t Lh, Ll, Ch, Cl;
  int M, hl0;
  turn_c0_free(s, dh, dl, Lh, Ll, Ch, Cl, M, hl0);
  if (bs != 0u) turn_c0_pair_bound_w(s, dh, dl, bs, fw, Lh, Ll, Ch, Cl, M);
  turn_moves_sl(s, dh, dl, Ch, Cl, M, hl0, w, bs != 0u, fw, flip_always, o);
}

// hc_full4_batch through turn_device_sl
void hc_full4_batch_sl(int64_t n, int8_t* board, uint8_t* off, uint8_t* ft, const int8_t* player,
                       const uint8_t* dice, const uint32_t* words, uint64_t* legal, uint64_t* played,
                       int8_t* reward, uint8_t* done) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], 0);
    TurnOut o;
    turn_device_sl(s, dice[2 * i], dice[2 * i + 1], words + 4 * i, false, o);
    if (!o.term) side_flip(s);
    legal[i] = o.legal;
    played[i] = o.played;
    reward[i] = (int8_t)o.reward;
    done[i] = (uint8_t)o.term;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, nullptr, nullptr);
  }
}

// hc_selfplay_full through the device's rollout ply: turn_device_sl with
// flip_always, then ply_close_sl (auto-reset as selects)
void hc_selfplay_full_sl(int64_t n, int64_t env0, uint64_t seed, uint32_t t0, int plies, int dice_mode,
                         int max_steps, int8_t* board, uint8_t* off, uint8_t* ft, int8_t* player,
                         uint16_t* elapsed, int32_t* stats, int8_t* obs, int8_t* reward, uint8_t* term,
                         uint8_t* trunc, uint64_t* legal_out, uint64_t* played_out) {
  for (int64_t i = 0; i < n; ++i) {
    Side s = load(board + i * 24, off + 2 * i, ft + 2 * i, player[i], elapsed[i]);
    s.t = t0;
    int4 st = make_int4(0, 0, 0, 0);
    for (int p = 0; p < plies; ++p) {
      uint32_t r[4];
      ply_draw(seed, s.t, (uint32_t)(env0 + i), dice_mode, r);
      int d0, d1;
      dice_from(r[0], dice_mode, d0, d1);
      uint32_t w[4];
      turn_words(r, w);
      const uint32_t mover_black = s.black;
      TurnOut o;
      turn_device_sl(s, d0, d1, w, true, o);
      int tm, tr;
      ply_close_sl(s, st, o.term, o.reward, mover_black, r[3], max_steps, tm, tr);
      const int64_t ix = (int64_t)p * n + i;
      if (obs)
        for (int q = 0; q < 24; ++q) obs[ix * 24 + q] = (int8_t)obs_point(s, q);
      if (reward) reward[ix] = (int8_t)o.reward;
      if (term) term[ix] = (uint8_t)tm;
      if (trunc) trunc[ix] = (uint8_t)tr;
      if (legal_out) legal_out[ix] = o.legal;
      if (played_out) played_out[ix] = o.played;
    }
    stats[3 * i] += st.x;
    stats[3 * i + 1] += st.y;
    stats[3 * i + 2] += st.z;
    store(s, board + i * 24, off + 2 * i, ft + 2 * i, player + i, elapsed + i);
  }
}

}  // extern "C"

// env_step_policy_sl against env_step (policy = true, flip_always) on n
// random positions (hc_block_set_sl_random's boards: run-heavy, head-heavy,
// endgames), random dice and words.  Returns mismatches of the state, list
// #1, list #2, codes, reward or end flag; *bound = lists the block rule cut.
extern "C" int64_t hc_step_sl_random(int64_t n, uint32_t seed, int64_t* bound) {
  uint64_t x = 0x9E3779B97F4A7C15ull ^ ((uint64_t)seed << 17);
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, nb = 0;
  for (int64_t done = 0; done < n; ++done) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const uint32_t mode = rnd(4);
    const int offc = mode == 3 ? (int)rnd(14) : 0;
    int left = 15 - offc;
    uint32_t used = 0u;
    while (left > 0) {
      int p = mode >= 2 ? (int)rnd(mode == 3 ? 6 : 12) : (int)rnd(24);
      if (mode == 1 && rnd(3) == 0) p = 23;
      const int c = 1 + (int)rnd(left < 3 ? left : 3);
      for (int j = 0; j < c; ++j) nib_inc(s.own, p);
      used |= 1u << p;
      left -= c;
    }
    for (int lo = 15 - (int)rnd(3); lo > 0;) {
      const int p = (int)rnd(24);
      if ((used >> p) & 1u) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    s.off_own = (uint32_t)offc;
    s.ft_own = rnd(4) == 0;
    side_masks(s);
    const int d0 = 1 + (int)rnd(6), d1 = rnd(4) == 0 ? d0 : 1 + (int)rnd(6);
    const uint32_t r1 = (uint32_t)(x >> 7), r2 = (uint32_t)(x >> 29) * 2654435761u;
    Side a = s, b = s;
    StepOut oa, ob;
    env_step(a, d0, d1, 0, 0, true, r1, r2, oa, true);
    env_step_policy_sl(b, d0, d1, r1, r2, ob);
    uint4 ra0, ra1, rb0, rb1;
    side_to_record(a, ra0, ra1);
    side_to_record(b, rb0, rb1);
    const bool same = ra0.x == rb0.x && ra0.y == rb0.y && ra0.z == rb0.z && ra0.w == rb0.w && ra1.x == rb1.x &&
                      ra1.y == rb1.y && ra1.z == rb1.z && a.O == b.O && a.P == b.P && a.S1o == b.S1o &&
                      a.S1p == b.S1p && oa.l1.L[0] == ob.l1.L[0] && oa.l1.L[1] == ob.l1.L[1] &&
                      oa.l1.count == ob.l1.count && oa.L2 == ob.L2 && oa.d2 == ob.d2 && oa.count2 == ob.count2 &&
                      oa.code1 == ob.code1 && oa.code2 == ob.code2 && oa.reward == ob.reward && oa.term == ob.term;
    bad += !same;
    Legal l;
    legal2(s, d0, d1, l);
    nb += (uint32_t)__builtin_popcount(die_candidates(s.O, s.P, d0 > d1 ? d0 : d1)) != (uint32_t)__builtin_popcount(l.L[0]);
  }
  *bound = nb;
  return bad;
}

// ---- block-bound two-dice turns from the failing windows (round 4) --------
// the reference: env_turn_full's bound two-dice branch (die_filter lists, the
// sure-pair masks, f4_keep_pair's child checks)
static void c0_pair_bound_ref(const Side& s, uint32_t low, int dh, int dl, uint32_t hs, uint32_t& Lh, uint32_t& Ll,
                              uint32_t& Ch, uint32_t& Cl, int& M) {
  const Blocks bl = block_info_low(s.O, low);
  Lh = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, dh), dh);
  Ll = die_filter(s.O, s.S1o, bl, die_candidates(s.O, s.P, dl), dl);
  const uint32_t sh = f4_sure_pair(s.O, s.P, dl, Lh, hs), sl = f4_sure_pair(s.O, s.P, dh, Ll, hs);
  const uint32_t kh = sh | f4_keep_pair(s, low, dh, dl, Lh & ~sh, false);
  const uint32_t kl = sl | f4_keep_pair(s, low, dl, dh, Ll & ~sl, false);
  const bool pair = (kh | kl) != 0u;
  Ch = pair ? kh : Lh;
  Cl = pair ? kl : (Lh ? 0u : Ll);
  M = pair ? 2 : ((Lh | Ll) ? 1 : 0);
}

// On n random block-bound two-dice positions (run-heavy boards, few
// opponent points below): turn_c0_pair_bound_w equals the reference, and at
// every child of the turn (each first move of either die) the other die's
// list filtered by block_reject_w equals die_filter's.  Returns mismatches;
// *cut = child lists the block rule shortened.
extern "C" int64_t hc_pair_bound_w_random(int64_t n, uint32_t seed, int64_t* cut) {
  uint64_t x = 0xA0761D6478BD642Full ^ ((uint64_t)seed << 20);
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, nc = 0;
  for (int64_t done = 0; done < n;) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    // a run of 4-7 own points somewhere, the rest scattered
    const int r0 = (int)rnd(18), rl = 4 + (int)rnd(4);
    int left = 15;
    uint32_t used = 0u;
    for (int p = r0; p < r0 + rl && p < 24 && left > 0; ++p) {
      const int c = 1 + (int)rnd(left < 3 ? left : 3);
      for (int j = 0; j < c; ++j) nib_inc(s.own, p);
      used |= 1u << p;
      left -= c;
    }
    while (left > 0) {
      const int p = (int)rnd(24);
      nib_inc(s.own, p);
      used |= 1u << p;
      --left;
    }
    int lo = 15;
    for (int tries = 0; lo > 0 && tries < 1000; ++tries) {  // opponent mostly above the run
      const int p = rnd(3) == 0 ? (int)rnd(24) : r0 + (int)rnd(24 - r0);
      if (p > 23 || ((used >> p) & 1u)) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    if (lo > 0) continue;
    s.ft_own = rnd(4) == 0;
    side_masks(s);
    const int a = 1 + (int)rnd(6), b = 1 + (int)rnd(6);
    if (a == b) continue;
    const int dh = a > b ? a : b, dl = a > b ? b : a;
    const uint32_t low = block_lowmask(s.P);
    uint32_t fw;
    const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, low, dh, dl, fw);
    if (bs == 0u) continue;
    ++done;
    uint32_t Lh, Ll, Ch, Cl, Lh2, Ll2, Ch2, Cl2;
    int M, M2;
    c0_pair_bound_ref(s, low, dh, dl, bs, Lh, Ll, Ch, Cl, M);
    turn_c0_pair_bound_w(s, dh, dl, bs, fw, Lh2, Ll2, Ch2, Cl2, M2);
    bad += Lh != Lh2 || Ll != Ll2 || Ch != Ch2 || Cl != Cl2 || M != M2;
    for (int w = 0; w < 2; ++w) {
      const int u = w ? dl : dh, v = w ? dh : dl;
      for (uint32_t m = w ? Ll : Lh; m; m &= m - 1u) {
        const int p = __builtin_ctz(m);
        Side c = s;
        apply_die(c, p, u);
        const uint32_t C = die_candidates(c.O, c.P, v);
        const uint32_t ref = die_filter(c.O, c.S1o, block_info_low(c.O, low), C, v);
        bad += ref != (C & ~block_reject_w(c.O, c.S1o, fw, C, v));
        nc += ref != C;
      }
    }
  }
  *cut = nc;
  return bad;
}

// On n random block-bound doubles positions: block_reject_w equals
// die_filter at every node of the turn up to depth 3 (the lists the search
// and the later sub-moves read), and f4_depth_w<3> equals f4_depth<3, 0> for
// every root source.  Returns mismatches; *cut = node lists the rule cut.
extern "C" int64_t hc_dbl_bound_w_random(int64_t n, uint32_t seed, int64_t* cut) {
  uint64_t x = 0xE7037ED1A0B428DBull ^ ((uint64_t)seed << 21);
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, nc = 0;
  for (int64_t done = 0; done < n;) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const int r0 = (int)rnd(18), rl = 3 + (int)rnd(5);
    int left = 15;
    uint32_t used = 0u;
    for (int p = r0; p < r0 + rl && p < 24 && left > 0; ++p) {
      const int c = 1 + (int)rnd(left < 3 ? left : 3);
      for (int j = 0; j < c; ++j) nib_inc(s.own, p);
      used |= 1u << p;
      left -= c;
    }
    while (left > 0) {
      const int p = (int)rnd(24);
      nib_inc(s.own, p);
      used |= 1u << p;
      --left;
    }
    int lo = 15;
    for (int tries = 0; lo > 0 && tries < 1000; ++tries) {
      const int p = rnd(3) == 0 ? (int)rnd(24) : r0 + (int)rnd(24 - r0);
      if (p > 23 || ((used >> p) & 1u)) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    if (lo > 0) continue;
    s.ft_own = rnd(3) == 0;
    side_masks(s);
    const int d = 1 + (int)rnd(6);
    const int hl = (s.ft_own && (d == 3 || d == 4 || d == 6)) ? 2 : 1;
    const uint32_t low = block_lowmask(s.P);
    uint32_t fw;
    if (turn_block_set_sl(s.O, s.S1o, s.P, low, d, d, fw) == 0u) continue;
    ++done;
    // every node to depth 3 (breadth-first over the plain search tree)
    Side q[1 + 24 + 576];
    int depth[1 + 24 + 576], hls[1 + 24 + 576], nq = 1, head = 0;
    q[0] = s; depth[0] = 0; hls[0] = hl;
    while (head < nq) {
      const Side c = q[head];
      const int dep = depth[head], h = hls[head];
      ++head;
      const uint32_t C = die_candidates(c.O, c.P, d);
      const uint32_t ref = die_filter(c.O, c.S1o, block_info_low(c.O, low), C, d);
      bad += ref != (C & ~block_reject_w(c.O, c.S1o, fw, C, d));
      nc += ref != C;
      if (dep >= 3) continue;
      uint32_t L = ref & (h <= 0 ? ~HEAD : ~0u);
      while (L && nq < (int)(sizeof(q) / sizeof(q[0]))) {
        const int p = __builtin_ctz(L);
        L &= L - 1u;
        q[nq] = c;
        apply_die(q[nq], p, d);
        depth[nq] = dep + 1;
        hls[nq] = h - (p == 23 ? 1 : 0);
        ++nq;
      }
    }
    uint32_t L = die_filter(s.O, s.S1o, block_info_low(s.O, low), die_candidates(s.O, s.P, d), d);
    if (hl <= 0) L &= ~HEAD;
    for (; L; L &= L - 1u) {
      const int p = __builtin_ctz(L);
      Side c = s;
      apply_die(c, p, d);
      const int h2 = hl - (p == 23 ? 1 : 0);
      bad += f4_depth<3, 0>(c, low, d, h2, false) != f4_depth_w<3>(c, fw, d, h2);
      // the straight-line probe: never deeper than the search, and equal to
      // it whenever it reaches the bound
      const int e1 = f4_depth_w<1>(c, fw, d, h2), e2 = f4_depth_w<2>(c, fw, d, h2), e3 = f4_depth_w<3>(c, fw, d, h2);
      const int q1 = f4_probe_w<1>(c, fw, d, h2), q2 = f4_probe_w<2>(c, fw, d, h2), q3 = f4_probe_w<3>(c, fw, d, h2);
      bad += q1 > e1 || q2 > e2 || q3 > e3 || (q1 == 1 && e1 != 1) || (q2 == 2 && e2 != 2) || (q3 == 3 && e3 != 3);
      bad += q1 != e1;  // depth 1: the probe is the search
    }
  }
  *cut = nc;
  return bad;
}

// turn_block_set_sl (no early exit, both kinds' window tests) against
// turn_block_set on n random positions (hc_pair_bf_random's boards, both
// kinds of roll).  Returns mismatches; *bound = block-bound cases.
extern "C" int64_t hc_block_set_sl_random(int64_t n, uint32_t seed, int64_t* bound) {
  uint64_t x = 0x2545F4914F6CDD1Dull ^ seed;
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, nb = 0;
  for (int64_t done = 0; done < n; ++done) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const uint32_t mode = rnd(4);
    int left = 15 - (mode == 3 ? (int)rnd(14) : 0);
    uint32_t used = 0u;
    while (left > 0) {
      int p = mode >= 2 ? (int)rnd(12) : (int)rnd(24);
      if (mode == 1 && rnd(3) == 0) p = 23;
      const int c = 1 + (int)rnd(left < 3 ? left : 3);
      for (int j = 0; j < c; ++j) nib_inc(s.own, p);
      used |= 1u << p;
      left -= c;
    }
    for (int lo = 15; lo > 0;) {
      const int p = (int)rnd(24);
      if ((used >> p) & 1u) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    side_masks(s);
    const int a = 1 + (int)rnd(6), b = rnd(3) == 0 ? a : 1 + (int)rnd(6);
    const int dh = a > b ? a : b, dl = a > b ? b : a;
    const uint32_t low = block_lowmask(s.P);
    const uint32_t ref = turn_block_set(s.O, s.S1o, s.P, low, dh, dl);
    bad += ref != turn_block_set_sl(s.O, s.S1o, s.P, low, dh, dl);
    nb += ref != 0u;
  }
  *bound = nb;
  return bad;
}

// f4_keep_pair_bf (all sources from the masks) against f4_keep_pair (the
// per-source child check) on n random block-free two-dice positions, both
// dice orders; random boards with a split-home / head-heavy / endgame mix.
// Returns the number of mismatches; *nontrivial = checks where C != L.
extern "C" int64_t hc_pair_bf_random(int64_t n, uint32_t seed, int64_t* nontrivial) {
  uint64_t x = 0x9E3779B97F4A7C15ull ^ seed;
  auto rnd = [&x](uint32_t m) {  // xorshift64*, value in [0, m)
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, nt = 0, done = 0;
  while (done < n) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const uint32_t mode = rnd(4);
    const int off = mode == 3 ? (int)rnd(14) : 0;
    int left = 15 - off;
    uint32_t used = 0u;
    while (left > 0) {
      int p = mode >= 2 ? (int)rnd(8) : (int)rnd(24);
      if (mode == 1 && rnd(3) == 0) p = 23;
      const int c = 1 + (int)rnd(left < 4 ? left : 4);
      for (int j = 0; j < c; ++j) nib_inc(s.own, p);
      used |= 1u << p;
      left -= c;
    }
    for (int lo = 15; lo > 0;) {
      const int p = (int)rnd(24);
      if ((used >> p) & 1u) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    s.off_own = (uint32_t)off;
    side_masks(s);
    const int a = 1 + (int)rnd(6), b = 1 + (int)rnd(6);
    if (a == b) continue;
    const uint32_t low = block_lowmask(s.P);
    if (!turn_block_free(s.O, s.S1o, s.P, low, a > b ? a : b, a > b ? b : a)) continue;
    ++done;
    for (int w = 0; w < 2; ++w) {
      const int u = w ? b : a, v = w ? a : b;
      const uint32_t L = legal1(s, low, u, true);
      const uint32_t ref = f4_keep_pair(s, low, u, v, L, true);
      bad += ref != f4_keep_pair_bf(s.O, s.S1o, s.P, u, v, L);
      nt += ref != L;
    }
  }
  *nontrivial = nt;
  return bad;
}

// f4_open_moves (exact count of a block-free doubles turn whose bear-off may
// open mid-turn, every C_k = L_k) against the depth-first search (f4_keep
// with NEED 3, 2, 1) on n random such positions: bear-off endgames with
// 1-3 stragglers outside home.  Returns mismatches; *raised = positions
// where the opening bear-off raises M above the normal steps.
extern "C" int64_t hc_open_moves_random(int64_t n, uint32_t seed, int64_t* raised) {
  uint64_t x = 0xD1B54A32D192ED03ull ^ seed;
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, up = 0, done = 0;
  while (done < n) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const int off = (int)rnd(14);
    int strag = 1 + (int)rnd(3);
    for (int left = 15 - off; left > 0; --left) {
      const int p = strag > 0 ? 6 + (int)rnd(18) : (int)rnd(6);
      if (strag > 0) --strag;
      nib_inc(s.own, p);
    }
    uint32_t used = 0u;
    for (int p = 0; p < 24; ++p) used |= nib_get(s.own, p) ? (1u << p) : 0u;
    for (int lo = 15; lo > 0;) {
      const int p = (int)rnd(24);
      if ((used >> p) & 1u) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    s.off_own = (uint32_t)off;
    s.ft_own = rnd(2);
    side_masks(s);
    const int d = 1 + (int)rnd(6);
    const int hl = (s.ft_own && (d == 3 || d == 4 || d == 6)) ? 2 : 1;
    const uint32_t low = block_lowmask(s.P);
    if (!turn_block_free(s.O, s.S1o, s.P, low, d, d) || f4_bearoff_fixed(s)) continue;
    const uint32_t L = legal1(s, low, d, true);
    if (!L) continue;
    ++done;
    uint32_t C = f4_keep<3>(s, low, d, hl, L, true);
    int M = 4;
    if (!C) { C = f4_keep<2>(s, low, d, hl, L, true); M = 3; }
    if (!C) { C = f4_keep<1>(s, low, d, hl, L, true); M = 2; }
    if (!C) { C = L; M = 1; }
    const int T = f4_exact_moves(s, d, hl);
    const int Me = f4_open_moves(s, d, hl, T);
    bad += (Me != M || C != L);
    up += Me > T;
  }
  *raised = up;
  return bad;
}

// ---- turn_block_free against the rule itself ------------------------------
// does die_filter remove a candidate at any node of the turn's sub-move tree
// (head rule ignored: a superset of the turn's nodes)?
static bool hc_binds_at(const Side& s, uint32_t low, int d) {
  const uint32_t C = die_candidates(s.O, s.P, d);
  return die_filter(s.O, s.S1o, block_info_low(s.O, low), C, d) != C;
}
static bool hc_binds(const Side& s, uint32_t low, int a, int b, int left) {
  if (left == 0) return false;
  if (hc_binds_at(s, low, a) || (b != a && hc_binds_at(s, low, b))) return true;
  for (int k = 0; k < (a == b ? 1 : 2); ++k) {
    const int x = k ? b : a, y = k ? a : b;
    uint32_t L = die_candidates(s.O, s.P, x);
    while (L) {
      const int p = __builtin_ctz(L);
      L &= L - 1u;
      Side c = s;
      apply_die(c, p, x);
      // two dice: one sub-move with the other die is left
      if (a == b ? hc_binds(c, low, a, a, left - 1) : hc_binds_at(c, low, y)) return true;
    }
  }
  return false;
}

// the most sub-moves of die d (up to n) from s by the plain walk: every
// list through die_filter, no shortcut
static int hc_depth_plain(const Side& s, uint32_t low, int d, int hl, int n) {
  if (n == 0) return 0;
  uint32_t L = die_filter(s.O, s.S1o, block_info_low(s.O, low), die_candidates(s.O, s.P, d), d);
  if (hl <= 0) L &= ~HEAD;
  int best = 0;
  while (L) {
    const int p = __builtin_ctz(L);
    L &= L - 1u;
    Side c = s;
    apply_die(c, p, d);
    const int v = 1 + hc_depth_plain(c, low, d, hl - (p == 23 ? 1 : 0), n - 1);
    best = v > best ? v : best;
  }
  return best;
}

// n random block-prone positions (an own 6-window with 0-4 holes, the
// opponent mostly past it so the rule applies), half doubles: a turn
// turn_block_free calls block-free must never have the rule remove a
// candidate.  Returns such turns; *freed = turns the hole count alone calls
// block-bound that the per-window test frees; *bound = turns where the rule
// really binds; *safe4 = block-bound doubles turns f4_safe_bound settles.
extern "C" int64_t hc_block_free_random(int64_t n, uint32_t seed, int64_t* freed, int64_t* bound,
                                        int64_t* safe4) {
  uint64_t x = 0x94D049BB133111EBull ^ seed;
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, fr = 0, bd = 0, fast = 0;
  for (int64_t done = 0; done < n; ++done) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const int i0 = (int)rnd(19);
    const uint32_t W = 0x3Fu << i0;
    const int holes = (int)rnd(5);
    uint32_t Hm = 0u;
    while (__builtin_popcount(Hm) < holes) Hm |= 1u << (i0 + (int)rnd(6));
    int left = 15;
    for (int p = i0; p < i0 + 6; ++p)
      if (!((Hm >> p) & 1u)) {
        const int c = 1 + (rnd(3) == 0 ? 1 : 0);
        for (int j = 0; j < c; ++j) nib_inc(s.own, p);
        left -= c;
      }
    while (left > 0) {
      const int p = (int)rnd(24);
      if ((Hm >> p) & 1u && rnd(2)) continue;  // keep most holes open
      nib_inc(s.own, p);
      --left;
    }
    uint32_t used = 0u;
    for (int p = 0; p < 24; ++p) used |= nib_get(s.own, p) ? (1u << p) : 0u;
    // opponent: mostly on points above the window (the rule applies),
    // sometimes anywhere; a few on the holes' feeder points
    const int lo_min = rnd(4) == 0 ? 0 : i0 + 1;
    for (int lo = 15; lo > 0;) {
      const int p = lo_min + (int)rnd((uint32_t)(24 - lo_min));
      if ((used >> p) & 1u) {
        if (lo_min > 0 && !(used & ~(MASK24 >> (24 - p)) & ~W)) { /* no free point */ }
        bool any = false;
        for (int q = lo_min; q < 24; ++q) any |= !((used >> q) & 1u);
        if (!any) break;
        continue;
      }
      nib_inc(s.opp, p);
      --lo;
    }
    s.ft_own = 0u;
    side_masks(s);
    const int a = 1 + (int)rnd(6), b = rnd(2) ? a : 1 + (int)rnd(6);
    const int dh = a > b ? a : b, dl = a > b ? b : a;
    const uint32_t low = block_lowmask(s.P);
    const bool bf = turn_block_free(s.O, s.S1o, s.P, low, dh, dl);
    // the hole count alone (the test before the per-window refinement)
    uint32_t U;
    if (dh == dl) {
      uint32_t S = s.O;
      U = s.O;
      for (int k = 0; k < 4; ++k) { S = land_step(S, s.P, dh); U |= S; }
    } else {
      const uint32_t A = s.O | land_step(s.O, s.P, dh) | land_step(s.O, s.P, dl);
      U = A | land_step(A, s.P, dh) | land_step(A, s.P, dl);
    }
    const bool coarse = (runs6(U) & low & windows_few_holes(s.O, dh == dl ? 4 : 2)) == 0u;
    const bool binds = hc_binds(s, low, dh, dl, dh == dl ? 4 : 2);
    bad += bf && binds;
    if (dh == dl) {
      // fewer sub-moves left (a node inside a turn): dbl_block_free(k) is
      // sound for each k, and the searches that stop at block-free nodes
      // (f4_depth / f4_reach) agree with the plain walk
      const int hl = 1 + (int)rnd(2);
      for (int k = 1; k <= 4; ++k) {
        bad += dbl_block_free(s.O, s.S1o, s.P, low, dh, k) && hc_binds(s, low, dh, dh, k);
        const int ref = hc_depth_plain(s, low, dh, hl, k);
        const int got = k == 1 ? f4_depth<1>(s, low, dh, hl, false)
                               : (k == 2 ? f4_depth<2>(s, low, dh, hl, false)
                                         : (k == 3 ? f4_depth<3>(s, low, dh, hl, false)
                                                   : f4_depth<4>(s, low, dh, hl, false)));
        const bool reach = k == 1 ? f4_reach<1>(s, low, dh, hl, false)
                                  : (k == 2 ? f4_reach<2>(s, low, dh, hl, false)
                                            : (k == 3 ? f4_reach<3>(s, low, dh, hl, false)
                                                      : f4_reach<4>(s, low, dh, hl, false)));
        bad += got != ref;
        bad += reach != (ref >= k);
      }
      // f4_safe_bound >= 4 (block-bound 'fast'): M = 4 and every first and
      // second sub-move keeps the rest of the turn playable
      if (!bf && f4_safe_bound(s, dh, hl, dbl_block_windows(s.O, s.S1o, s.P, low, dh, 4)) >= 4) {
        ++fast;
        bad += hc_depth_plain(s, low, dh, hl, 4) != 4;
        uint32_t L = legal1(s, low, dh, false);
        if (hl <= 0) L &= ~HEAD;
        while (L) {
          const int p = __builtin_ctz(L);
          L &= L - 1u;
          Side c = s;
          apply_die(c, p, dh);
          const int h2 = hl - (p == 23 ? 1 : 0);
          bad += hc_depth_plain(c, low, dh, h2, 3) != 3;
          uint32_t L2 = legal1(c, low, dh, false);
          if (h2 <= 0) L2 &= ~HEAD;
          while (L2) {
            const int q = __builtin_ctz(L2);
            L2 &= L2 - 1u;
            Side c2 = c;
            apply_die(c2, q, dh);
            bad += hc_depth_plain(c2, low, dh, h2 - (q == 23 ? 1 : 0), 2) != 2;
          }
        }
      }
    }
    bad += coarse && !bf;  // the refinement only ever frees turns
    fr += bf && !coarse;
    bd += binds;
  }
  *freed = fr;
  *bound = bd;
  *safe4 = fast;
  return bad;
}

// f4_sure_pair against f4_keep_pair on n random block-prone two-dice turns
// (hc_block_free_random's generator, two dice only): every sure first move
// keeps a move of the other die.  Returns violations; *sure = sure sources,
// *total = first-move sources checked.
extern "C" int64_t hc_sure_pair_random(int64_t n, uint32_t seed, int64_t* sure, int64_t* total) {
  uint64_t x = 0xBF58476D1CE4E5B9ull ^ seed;
  auto rnd = [&x](uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  };
  int64_t bad = 0, su = 0, tot = 0, done = 0;
  while (done < n) {
    Side s = side_start(0u);
    for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
    const int i0 = (int)rnd(19);
    uint32_t Hm = 0u;
    const int holes = (int)rnd(3);
    while (__builtin_popcount(Hm) < holes) Hm |= 1u << (i0 + (int)rnd(6));
    int left = 15;
    for (int p = i0; p < i0 + 6; ++p)
      if (!((Hm >> p) & 1u)) {
        const int c = 1 + (rnd(3) == 0 ? 1 : 0);
        for (int j = 0; j < c; ++j) nib_inc(s.own, p);
        left -= c;
      }
    while (left > 0) {
      const int p = (int)rnd(24);
      if ((Hm >> p) & 1u) continue;
      nib_inc(s.own, p);
      --left;
    }
    uint32_t used = 0u;
    for (int p = 0; p < 24; ++p) used |= nib_get(s.own, p) ? (1u << p) : 0u;
    const int lo_min = rnd(4) == 0 ? 0 : i0 + 1;
    bool any = false;
    for (int q = lo_min; q < 24; ++q) any |= !((used >> q) & 1u);
    if (!any) continue;
    for (int lo = 15; lo > 0;) {
      const int p = lo_min + (int)rnd((uint32_t)(24 - lo_min));
      if ((used >> p) & 1u) continue;
      nib_inc(s.opp, p);
      --lo;
    }
    side_masks(s);
    const int a = 1 + (int)rnd(6), b = 1 + (int)rnd(6);
    if (a == b) continue;
    const int dh = a > b ? a : b, dl = a > b ? b : a;
    const uint32_t low = block_lowmask(s.P);
    bool bound;
    const uint32_t hs = two_block_holes(s.O, s.S1o, s.P, low, dh, dl, bound);
    if (!bound) continue;
    ++done;
    for (int k = 0; k < 2; ++k) {
      const int u = k ? dl : dh, v = k ? dh : dl;
      const uint32_t L = legal1(s, low, u, false);
      const uint32_t sr = f4_sure_pair(s.O, s.P, v, L, hs);
      bad += (sr & ~f4_keep_pair(s, low, u, v, L, false)) != 0u;
      su += __builtin_popcount(sr);
      tot += __builtin_popcount(L);
    }
  }
  *sure = su;
  *total = tot;
  return bad;
}

// windows_few_holes (two carry-save adders) against the plain bit-sliced
// counter it replaced, over every 24-bit own mask; returns mismatches
static uint32_t wfh_ref(uint32_t O, int k) {
  const uint32_t h = ~O & MASK24;
  uint32_t s0 = 0u, s1 = 0u, s2 = 0u;
  for (int j = 0; j < 6; ++j) {
    const uint32_t x = h >> j;
    const uint32_t c0 = s0 & x;
    s0 ^= x;
    const uint32_t c1 = s1 & c0;
    s1 ^= c0;
    s2 |= c1;
  }
  return k >= 4 ? ~(s2 & (s1 | s0)) : ~s2 & ~(s1 & s0);
}
extern "C" int64_t hc_windows_few_holes_all() {
  int64_t bad = 0;
  for (uint32_t O = 0; O < (1u << 24); ++O)
    bad += (wfh_ref(O, 2) != windows_few_holes(O, 2)) + (wfh_ref(O, 4) != windows_few_holes(O, 4));
  return bad;
}

// ===========================================================================
// ply_bound_turn (gym-narde_amd/csrc/full4_wave.h) on 64 emulated lanes
// (ADVICE r04): the rollout's turn for a wave holding a block-bound doubles
// lane, compiled for the CPU with its two cross-lane operations emulated --
// every lane is a host thread, __ballot and __builtin_amdgcn_readlane meet
// at a 64-thread barrier (each lane publishes its value, all read, all leave)
// -- and held to env_turn_full (the host turn, itself held to the oracle and
// full4.npz) lane by lane: C_0 | M, the played sub-moves, reward / done and
// the post-turn state, on waves mixing block-bound doubles lanes (the
// f4_safe_bound fast path and the searched ones), block-bound two-dice lanes
// and free lanes.
#include <atomic>
#include <thread>
#include <vector>

namespace wave_emu {
// a sense-counting barrier (atomics, yielding spin: 64 threads on a few cores)
struct Wave {
  std::atomic<int> arrived{0};
  std::atomic<uint64_t> gen{0};
  uint32_t v[64];
  void sync() {
    const uint64_t g = gen.load(std::memory_order_acquire);
    if (arrived.fetch_add(1, std::memory_order_acq_rel) == 63) {
      arrived.store(0, std::memory_order_relaxed);
      gen.store(g + 1, std::memory_order_release);
    } else {
      while (gen.load(std::memory_order_acquire) == g) std::this_thread::yield();
    }
  }
};
Wave* g_wave = nullptr;
thread_local int t_lane = 0;
inline uint32_t readlane(uint32_t x, int l) {
  g_wave->v[t_lane] = x;
  g_wave->sync();
  const uint32_t r = g_wave->v[l];
  g_wave->sync();
  return r;
}
inline uint64_t ballot(bool b) {
  g_wave->v[t_lane] = b ? 1u : 0u;
  g_wave->sync();
  uint64_t r = 0;
  for (int l = 0; l < 64; ++l) r |= (uint64_t)(g_wave->v[l] & 1u) << l;
  g_wave->sync();
  return r;
}
}  // namespace wave_emu

#define __ballot(x) wave_emu::ballot(x)
#define __builtin_amdgcn_readlane(x, l) ((int)wave_emu::readlane((uint32_t)(x), (l)))
#include "../../gym-narde_amd/csrc/full4_wave.h"
#undef __ballot
#undef __builtin_amdgcn_readlane

namespace {
struct Rnd {
  uint64_t x;
  uint32_t operator()(uint32_t m) {
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    return (uint32_t)(((x * 0x2545F4914F6CDD1Dull) >> 32) % m);
  }
};

// a run-heavy position (hc_dbl_bound_w_random's generator): a run of 3-7
// own points from a random start, the rest of the 15 anywhere, the
// opponent's 15 mostly above the run
bool gen_position(Rnd& rnd, Side& s) {
  s = side_start(0u);
  for (int k = 0; k < 3; ++k) { s.own.w[k] = 0u; s.opp.w[k] = 0u; }
  const int r0 = (int)rnd(18), rl = 3 + (int)rnd(5);
  int left = 15;
  uint32_t used = 0u;
  for (int p = r0; p < r0 + rl && p < 24 && left > 0; ++p) {
    const int c = 1 + (int)rnd(left < 3 ? left : 3);
    for (int j = 0; j < c; ++j) nib_inc(s.own, p);
    used |= 1u << p;
    left -= c;
  }
  while (left > 0) {
    const int p = (int)rnd(24);
    nib_inc(s.own, p);
    used |= 1u << p;
    --left;
  }
  int lo = 15;
  for (int tries = 0; lo > 0 && tries < 1000; ++tries) {
    const int p = rnd(3) == 0 ? (int)rnd(24) : r0 + (int)rnd(24 - r0);
    if (p > 23 || ((used >> p) & 1u)) continue;
    nib_inc(s.opp, p);
    --lo;
  }
  if (lo > 0) return false;
  s.ft_own = rnd(3) == 0;
  side_masks(s);
  return true;
}

// a lane of the given kind: 0 block-bound doubles, 1 block-bound two dice,
// 2 anything (random dice)
void gen_lane(Rnd& rnd, int kind, Side& s, int& dh, int& dl) {
  for (;;) {
    if (!gen_position(rnd, s)) continue;
    int a = 1 + (int)rnd(6), b = 1 + (int)rnd(6);
    if (kind == 0) b = a;
    if (kind == 1 && a == b) continue;
    dh = a > b ? a : b;
    dl = a > b ? b : a;
    if (kind == 2) return;
    uint32_t fw;
    if (turn_block_set_sl(s.O, s.S1o, s.P, block_lowmask(s.P), dh, dl, fw) != 0u) return;
  }
}
}  // namespace

// `waves` waves of 64 lanes: returns the number of lanes whose result
// differs; counts[0..3] = block-bound doubles lanes, of them with the full
// search (not f4_safe_bound's fast path), block-bound two-dice lanes, lanes
extern "C" int64_t hc_ply_bound_turn_random(int64_t waves, uint32_t seed, int64_t* counts) {
  Rnd rnd{0x9E3779B97F4A7C15ull ^ ((uint64_t)seed << 17)};
  int64_t bad = 0;
  counts[0] = counts[1] = counts[2] = counts[3] = 0;
  for (int64_t wv = 0; wv < waves; ++wv) {
    Side s[64], got[64];
    int dh[64], dl[64];
    uint32_t w[64][4];
    TurnOut o[64];
    for (int l = 0; l < 64; ++l) {
      const uint32_t u = rnd(8);
      const int kind = l == 0 ? 0 : (u < 2 ? 0 : (u < 4 ? 1 : 2));
      gen_lane(rnd, kind, s[l], dh[l], dl[l]);
      for (int k = 0; k < 4; ++k) w[l][k] = (uint32_t)rnd(0xFFFFFFFFu) ^ ((uint32_t)rnd(65536) << 16);
    }
    wave_emu::Wave wave;
    wave_emu::g_wave = &wave;
    std::vector<std::thread> th;
    for (int l = 0; l < 64; ++l) {
      th.emplace_back([&, l] {
        wave_emu::t_lane = l;
        Side x = s[l];
        uint32_t fw;
        const uint32_t bs = turn_block_set_sl(x.O, x.S1o, x.P, block_lowmask(x.P), dh[l], dl[l], fw);
        ply_bound_turn(x, dh[l], dl[l], bs, fw, w[l], false, o[l], l);
        got[l] = x;
      });
    }
    for (auto& t : th) t.join();
    wave_emu::g_wave = nullptr;
    for (int l = 0; l < 64; ++l) {
      Side e = s[l];
      TurnOut oe;
      env_turn_full(e, dh[l], dl[l], false, 0ull, w[l], oe);
      uint4 a1, b1, a2, b2;
      side_to_record(got[l], a1, b1);
      side_to_record(e, a2, b2);
      const bool same = o[l].legal == oe.legal && o[l].played == oe.played && o[l].term == oe.term &&
                        o[l].reward == oe.reward && o[l].max_dice == oe.max_dice && a1.x == a2.x &&
                        a1.y == a2.y && a1.z == a2.z && a1.w == a2.w && b1.x == b2.x && b1.y == b2.y &&
                        b1.z == b2.z && got[l].O == e.O && got[l].P == e.P && got[l].S1o == e.S1o &&
                        got[l].S1p == e.S1p;
      bad += same ? 0 : 1;
      uint32_t fw;
      const uint32_t bs = turn_block_set_sl(s[l].O, s[l].S1o, s[l].P, block_lowmask(s[l].P), dh[l], dl[l], fw);
      const int hl = (s[l].ft_own && (dh[l] == 3 || dh[l] == 4 || dh[l] == 6)) ? 2 : 1;
      if (bs && dh[l] == dl[l]) {
        ++counts[0];
        counts[1] += f4_safe_bound(s[l], dh[l], hl, bs) < 4;
      }
      counts[2] += bs && dh[l] != dl[l];
      ++counts[3];
    }
  }
  return bad;
}

// ply_bound_turn on emulated waves whose block-bound doubles lanes come from
// random-legal self-play (round 5, the pair pass coop_pair_w): `envs` envs
// play `plies` plies with env_turn_full; every searching block-bound
// doubles turn met (f4_safe_bound < 4, a non-empty filtered root list) is
// kept, and the kept turns are replayed 64 to a wave through ply_bound_turn
// against env_turn_full, every field hc_ply_bound_turn_random compares.
// Returns the lanes that differ; counts[0] = turns kept, counts[1] = of
// them, turns whose sub-move 1 checks differ between one and two more
// sub-moves for the source the turn picks (the case that tells the pair
// pass's two result sets apart), counts[2] = waves run, counts[3] = kept
// turns coop_pair_w leaves to coop_depth_w (more than 8 root sources, or a
// list after some source longer than 8), counts[4] = kept turns whose
// sub-move 1 takes the pair pass's checked list (done there, M >= 3) -- so
// the caller can assert that both branches of the pass ran.
extern "C" int64_t hc_pair_pass_selfplay(int64_t envs, int64_t plies, int64_t* counts) {
  struct Kept {
    Side s;
    int d;
    uint32_t w[4];
  };
  std::vector<Kept> kept;
  std::vector<Side> S((size_t)envs);
  for (int64_t i = 0; i < envs; ++i) {
    uint32_t r[4];
    philox4x32_10(0, (uint32_t)i, 0u, 1u, 0u, 0u, r);
    S[i] = side_reset(r[0]);
    S[i].t = 0;
  }
  counts[0] = counts[1] = counts[2] = counts[3] = counts[4] = 0;
  for (int64_t p = 0; p < plies; ++p) {
    for (int64_t i = 0; i < envs; ++i) {
      Side& s = S[i];
      uint32_t R[4], r[4];
      ply_block(s.t, (uint32_t)i, 0u, 0u, R);
      ply_words_of(R, s.t, 0, r);
      int d0, d1;
      dice_from(r[0], 0, d0, d1);
      const int dh = d0 > d1 ? d0 : d1, dl = d0 > d1 ? d1 : d0;
      uint32_t w[4];
      turn_words(r, w);
      uint32_t fw;
      const uint32_t bs = turn_block_set_sl(s.O, s.S1o, s.P, block_lowmask(s.P), dh, dl, fw);
      if (bs && dh == dl) {
        const int hl = (s.ft_own && (dh == 3 || dh == 4 || dh == 6)) ? 2 : 1;
        const uint32_t Lh = die_candidates(s.O, s.P, dh);
        const uint32_t Lb = Lh & ~block_reject_w(s.O, s.S1o, fw, Lh, dh);
        if (f4_safe_bound(s, dh, hl, bs) < 4 && Lb) {
          Kept k;
          k.s = s;
          k.d = dh;
          for (int j = 0; j < 4; ++j) k.w[j] = w[j];
          kept.push_back(k);
          // coop_pair_w's branch for this owner: the pairs (<= 8 root sources,
          // <= 8 entries after each) or coop_depth_w's fallback
          bool wide = __builtin_popcount(Lb) > 8;
          for (uint32_t m = Lb; m && !wide; m &= m - 1u) {
            const int q = __builtin_ctz(m);
            Side a = s;
            apply_die(a, q, dh);
            uint32_t L1 = die_candidates_sl(a.O, a.P, dh);
            L1 &= ~block_reject_w(a.O, a.S1o, fw, L1, dh);
            if (hl - (q == 23 ? 1 : 0) <= 0) L1 &= ~HEAD;
            wide = __builtin_popcount(L1) > 8;
          }
          // the source env_turn_full's first pick takes, and its sub-move 1 sets
          Side e = s;
          TurnOut oe;
          env_turn_full(e, dh, dh, false, 0ull, w, oe);
          counts[3] += wide;
          counts[4] += !wide && oe.max_dice >= 3;
          if (oe.max_dice == 4) {
            const int p0 = (int)(oe.played & 0xFFu);
            Side a = s;
            apply_die(a, p0, dh);
            const int h1 = hl - (p0 == 23 ? 1 : 0);
            uint32_t L1 = die_candidates_sl(a.O, a.P, dh);
            L1 &= ~block_reject_w(a.O, a.S1o, fw, L1, dh);
            if (h1 <= 0) L1 &= ~HEAD;
            uint32_t c1 = 0u, c2 = 0u;
            for (uint32_t m = L1; m; m &= m - 1u) {
              const int q = __builtin_ctz(m);
              Side b = a;
              apply_die(b, q, dh);
              const int dd = f4_depth_w<2>(b, fw, dh, h1 - (q == 23 ? 1 : 0));
              c1 |= dd >= 1 ? 1u << q : 0u;
              c2 |= dd >= 2 ? 1u << q : 0u;
            }
            counts[1] += c1 != c2;
          }
        }
      }
      const uint32_t mb = s.black;
      TurnOut o;
      env_turn_full(s, d0, d1, false, 0ull, w, o);
      int4 st = make_int4(0, 0, 0, 0);
      int tm, tr;
      ply_close(s, st, o.term, o.reward, mb, r[3], 1000, true, tm, tr);
    }
  }
  counts[0] = (int64_t)kept.size();
  int64_t bad = 0;
  if (kept.empty()) return 0;  // (the caller asserts that turns were kept)
  for (size_t w0 = 0; w0 < kept.size(); w0 += 64) {
    Side s[64], got[64];
    int dh[64];
    uint32_t w[64][4];
    TurnOut o[64];
    for (int l = 0; l < 64; ++l) {
      const Kept& k = kept[(w0 + (size_t)l) % kept.size()];
      s[l] = k.s;
      dh[l] = k.d;
      for (int j = 0; j < 4; ++j) w[l][j] = k.w[j];
    }
    wave_emu::Wave wave;
    wave_emu::g_wave = &wave;
    std::vector<std::thread> th;
    for (int l = 0; l < 64; ++l) {
      th.emplace_back([&, l] {
        wave_emu::t_lane = l;
        Side x = s[l];
        uint32_t fw;
        const uint32_t bs = turn_block_set_sl(x.O, x.S1o, x.P, block_lowmask(x.P), dh[l], dh[l], fw);
        ply_bound_turn(x, dh[l], dh[l], bs, fw, w[l], false, o[l], l);
        got[l] = x;
      });
    }
    for (auto& t : th) t.join();
    wave_emu::g_wave = nullptr;
    ++counts[2];
    for (int l = 0; l < 64; ++l) {
      Side e = s[l];
      TurnOut oe;
      env_turn_full(e, dh[l], dh[l], false, 0ull, w[l], oe);
      uint4 a1, b1, a2, b2;
      side_to_record(got[l], a1, b1);
      side_to_record(e, a2, b2);
      const bool same = o[l].legal == oe.legal && o[l].played == oe.played && o[l].term == oe.term &&
                        o[l].reward == oe.reward && o[l].max_dice == oe.max_dice && a1.x == a2.x &&
                        a1.y == a2.y && a1.z == a2.z && a1.w == a2.w && b1.x == b2.x && b1.y == b2.y &&
                        b1.z == b2.z && got[l].O == e.O && got[l].P == e.P && got[l].S1o == e.S1o &&
                        got[l].S1p == e.S1p;
      bad += same ? 0 : 1;
    }
  }
  return bad;
}
