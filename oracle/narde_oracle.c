/*
 * narde_oracle.c -- CPU restatement of the reference gym-narde hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker the HIP path is
 * compared against; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (gym-narde_amd/) never links,
 * loads or falls back to it.
 *
 * It follows the reference's LOOP STRUCTURE (not the kernel's bitmask
 * formulation), so a match between the two is a real differential check.
 * Parity pinned: every function here is checked against golden vectors
 * captured from the imported reference (tools/capture_golden.py ->
 * tests/golden/<name>.npz) by tests/test_oracle_golden.py.
 *
 * Reference citations are /root/reference/<path>:<line>.
 *   rotate_board               gym_narde/envs/narde.py:16-17
 *   get_valid_moves            gym_narde/envs/narde.py:58-92
 *   _validate_head_moves       gym_narde/envs/narde.py:94-106
 *   _filter_head_moves         gym_narde/envs/narde.py:127-137
 *   _violates_block_rule       gym_narde/envs/narde.py:139-184
 *   execute_rotated_move       gym_narde/envs/narde.py:36-56 (+ _execute_move :108-125)
 *   NardeEnv.step              gym_narde/envs/narde_env.py:27-103
 *   NardeEnv._check_game_ended gym_narde/envs/narde_env.py:134-141
 *   NardeEnv.reset             gym_narde/envs/narde_env.py:105-120
 *
 * Move encoding: (from, to) with to = 24 for the reference's 'off'.
 * The self-play driver at the bottom (Philox dice + random legal policy +
 * auto-reset) is this build's own synthetic workload;
 * it is restated here independently of the kernel so trajectories can be
 * compared bit for bit.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_OFF 24
#define OR_MAXM 64

static uint32_t mulhi_n(uint32_t r, uint32_t n) { return (uint32_t)(((uint64_t)r * n) >> 32); }

typedef struct {
    int32_t board[24]; /* absolute: white > 0, black < 0 */
    int32_t off_w, off_b;
    int32_t ft_w, ft_b;
    int32_t player; /* +1 white, -1 black */
    int32_t elapsed; /* steps in episode (TimeLimit) */
} or_state;

/* narde.py:16-17  rotate_board(board) = concat(-board[12:], -board[:12]) */
void or_rotate_board(const int32_t *in, int32_t *out) {
    for (int i = 0; i < 12; ++i) out[i] = -in[i + 12];
    for (int i = 12; i < 24; ++i) out[i] = -in[i - 12];
}

/* narde.py:139-184 */
int or_violates_block_rule(const int32_t *board) {
    int i = 0;
    while (i < 24) {
        if (board[i] > 0) {
            int block_start = i, block_length = 1, j = i + 1;
            while (j < 24 && board[j] > 0) { block_length++; j++; }
            if (block_length >= 6) {
                int has_opponent_ahead = 0;
                for (int k = 0; k < block_start; ++k)
                    if (board[k] < 0) { has_opponent_ahead = 1; break; }
                if (!has_opponent_ahead) return 1;
            }
            i = j;
        } else {
            i++;
        }
    }
    return 0;
}

/* narde.py:58-92 (+ :94-106 and :127-137).  roll has n <= 4 dice.
 * grp (optional): for each returned entry, the index into the sorted roll of
 * the die whose loop iteration (narde.py:64) produced it. */
static int or_get_valid_moves_g(const int32_t *abs_board, int ft_w, int ft_b,
                                const int32_t *roll_in, int n, int player,
                                int32_t (*out)[2], int8_t *grp) {
    int32_t roll[4];
    for (int i = 0; i < n; ++i) roll[i] = roll_in[i];
    /* sorted(roll, reverse=True): insertion sort, descending */
    for (int i = 1; i < n; ++i)
        for (int j = i; j > 0 && roll[j] > roll[j - 1]; --j) {
            int32_t t = roll[j]; roll[j] = roll[j - 1]; roll[j - 1] = t;
        }
    int32_t board[24];
    if (player == 1) memcpy(board, abs_board, sizeof board);
    else or_rotate_board(abs_board, board);

    int32_t moves[OR_MAXM * 2][2];
    int8_t mg[OR_MAXM * 2];
    int nm = 0;
    for (int di = 0; di < n; ++di) {
        int die = roll[di];
        for (int pos = 0; pos < 24; ++pos) {
            if (board[pos] <= 0) continue;
            int np_ = pos - die;
            if (np_ >= 0 && np_ < 24) {
                if (board[np_] >= 0) { moves[nm][0] = pos; moves[nm][1] = np_; mg[nm] = (int8_t)di; nm++; }
            } else if (np_ < 0) {
                int32_t s = 0;
                for (int k = 6; k < 24; ++k) s += board[k] > 0 ? board[k] : 0;
                if (s == 0 && die >= pos + 1) { moves[nm][0] = pos; moves[nm][1] = OR_OFF; mg[nm] = (int8_t)di; nm++; }
            }
        }
    }
    /* block-rule filter (narde.py:78-89) */
    int32_t filt[OR_MAXM * 2][2];
    int8_t fg[OR_MAXM * 2];
    int nf = 0;
    for (int m = 0; m < nm; ++m) {
        int32_t bc[24];
        memcpy(bc, board, sizeof bc);
        bc[moves[m][0]] -= 1;
        if (moves[m][1] != OR_OFF) bc[moves[m][1]] += 1;
        if (!or_violates_block_rule(bc)) { filt[nf][0] = moves[m][0]; filt[nf][1] = moves[m][1]; fg[nf] = mg[m]; nf++; }
    }
    /* _validate_head_moves: sorted(roll) in [[3,3],[4,4],[6,6]] */
    int first_turn = player == 1 ? ft_w : ft_b;
    int max_head = 1;
    if (first_turn && n == 2 && roll[0] == roll[1] && (roll[0] == 3 || roll[0] == 4 || roll[0] == 6))
        max_head = 2;
    /* _filter_head_moves */
    int cnt = 0, head = 0;
    for (int m = 0; m < nf; ++m) {
        if (filt[m][0] == 23) {
            if (head < max_head) {
                if (grp) grp[cnt] = fg[m];
                out[cnt][0] = filt[m][0]; out[cnt][1] = filt[m][1]; cnt++; head++;
            }
        } else {
            if (grp) grp[cnt] = fg[m];
            out[cnt][0] = filt[m][0]; out[cnt][1] = filt[m][1]; cnt++;
        }
    }
    return cnt;
}

int or_get_valid_moves(const int32_t *abs_board, int ft_w, int ft_b,
                       const int32_t *roll_in, int n, int player,
                       int32_t (*out)[2]) {
    return or_get_valid_moves_g(abs_board, ft_w, ft_b, roll_in, n, player, out, NULL);
}

/* The build's compact form of a two-dice list,
 * computed from the list itself: bit `from` of word 0 for an entry of the
 * higher die's loop, of word 1 for the lower die's (grp from
 * or_get_valid_moves_g), | d_hi<<48 | d_lo<<52.  The decoding (entries in
 * die-major, ascending-source order, to = from - die or 'off') reproduces
 * the list exactly, so equal words are equal lists. */
static uint64_t or_compact2(const int32_t (*list)[2], const int8_t *grp, int cnt, const int32_t dice[2]) {
    uint32_t L[2] = {0u, 0u};
    for (int k = 0; k < cnt; ++k) L[grp[k]] |= 1u << list[k][0];
    uint32_t hi = dice[0] > dice[1] ? dice[0] : dice[1], lo = dice[0] > dice[1] ? dice[1] : dice[0];
    return (uint64_t)L[0] | ((uint64_t)L[1] << 24) | ((uint64_t)hi << 48) | ((uint64_t)lo << 52);
}

/* narde.py:108-125 */
static void or_execute_move(or_state *s, int from, int to) {
    if (to == OR_OFF) {
        if (s->board[from] > 0) { s->board[from] -= 1; s->off_w += 1; }
        else { s->board[from] += 1; s->off_b += 1; }
    } else {
        if (s->board[from] > 0) { s->board[from] -= 1; s->board[to] += 1; }
        else { s->board[from] += 1; s->board[to] -= 1; }
    }
}

/* narde.py:36-56 */
void or_execute_rotated_move(or_state *s, int from, int to, int player) {
    if (player != 1) {
        int rf = (from + 12) % 24;
        int rt = to == OR_OFF ? OR_OFF : (to + 12) % 24;
        or_execute_move(s, rf, rt);
    } else {
        or_execute_move(s, from, to);
    }
    if (player == 1) s->ft_w = 0; else s->ft_b = 0;
}

/* narde_env.py:134-141 */
static void or_check_game_ended(const or_state *s, int *done, int *reward) {
    if (s->player == 1 && s->off_w == 15) { *done = 1; *reward = s->off_b > 0 ? 1 : 2; return; }
    if (s->player == -1 && s->off_b == 15) { *done = 1; *reward = s->off_w > 0 ? 1 : 2; return; }
    *done = 0; *reward = 0;
}

/* narde.py:31-34 */
void or_perspective(const or_state *s, int player, int32_t *out) {
    if (player == 1) memcpy(out, s->board, 24 * sizeof(int32_t));
    else or_rotate_board(s->board, out);
}

/* narde_env.py:45-54: code -> move.  Python's // and % floor; a code
 * outside [0, 576) can never equal a listed move (from would be < 0 or
 * >= 24), so it decodes to an impossible move. */
static void or_decode(int code, int *from, int *to) {
    if (code < 0 || code >= 576) { *from = -1; *to = -1; return; }
    *from = code / 24;
    *to = code % 24;
    if (*to == 0 && *from >= 0 && *from <= 5) *to = OR_OFF;
}

static int or_in_list(int32_t (*l)[2], int n, int f, int t) {
    for (int i = 0; i < n; ++i) if (l[i][0] == f && l[i][1] == t) return 1;
    return 0;
}

static int or_encode(int f, int t) { return f * 24 + (t == OR_OFF ? 0 : t); }

typedef struct {
    int32_t obs[24];
    int32_t reward, terminated;
    int32_t count1, count2; /* count2 = -1 when no second list was made */
    int32_t list1[OR_MAXM][2];
    int32_t list2[OR_MAXM][2];
    int32_t roll2;
    int32_t code1, code2; /* actions actually used (policy mode) */
    uint64_t legal1;      /* or_compact2 of list1 */
} or_step_out;

/*
 * narde_env.py:27-103 with the dice given (the reference draws them with
 * np.random.randint at :29; parity is defined on injected dice).
 * policy != 0 selects the build's random-legal policy: code1 is drawn from
 * list1 with r1, and code2 from the env's own second list with r2.
 */
static void or_step_core(or_state *s, const int32_t dice[2], int code1, int code2,
                         int policy, uint32_t r1, uint32_t r2, or_step_out *o) {
    o->count2 = -1;
    o->roll2 = 0;
    int8_t g1[OR_MAXM];
    int n1 = or_get_valid_moves_g(s->board, s->ft_w, s->ft_b, dice, 2, s->player, o->list1, g1);
    o->count1 = n1;
    o->legal1 = or_compact2((const int32_t (*)[2])o->list1, g1, n1, dice);
    if (policy) {
        code1 = 0; code2 = 0;
        if (n1 >= 2) {
            uint32_t i1 = (uint32_t)(((uint64_t)r1 * (uint32_t)n1) >> 32);
            code1 = or_encode(o->list1[i1][0], o->list1[i1][1]);
        }
    }
    o->code1 = code1; o->code2 = code2;
    if (n1 == 0) {
        int done, rew;
        or_check_game_ended(s, &done, &rew);
        if (!done) s->player = -s->player;
        or_perspective(s, s->player, o->obs);
        o->reward = rew; o->terminated = done;
        return;
    } else if (n1 == 1) {
        or_execute_rotated_move(s, o->list1[0][0], o->list1[0][1], s->player);
    } else {
        int f1, t1, f2, t2;
        or_decode(code1, &f1, &t1);
        if (or_in_list(o->list1, n1, f1, t1)) {
            or_execute_rotated_move(s, f1, t1, s->player);
            int dist = t1 == OR_OFF ? f1 + 1 : abs(f1 - t1);
            int32_t temp[2] = {dice[0], dice[1]};
            int nt = 2;
            if (temp[0] == dist) { temp[0] = temp[1]; nt = 1; }
            else if (temp[1] == dist) { nt = 1; }
            else { temp[0] = temp[1]; nt = 1; } /* pop(0) */
            if (nt > 0) {
                o->roll2 = temp[0];
                int n2 = or_get_valid_moves(s->board, s->ft_w, s->ft_b, temp, 1, s->player, o->list2);
                o->count2 = n2;
                if (policy) {
                    if (n2 > 0) {
                        uint32_t i2 = (uint32_t)(((uint64_t)r2 * (uint32_t)n2) >> 32);
                        code2 = or_encode(o->list2[i2][0], o->list2[i2][1]);
                    } else {
                        code2 = 0;
                    }
                    o->code2 = code2;
                }
                or_decode(code2, &f2, &t2);
                if (or_in_list(o->list2, n2, f2, t2)) or_execute_rotated_move(s, f2, t2, s->player);
            }
        }
    }
    int done, rew;
    or_check_game_ended(s, &done, &rew);
    if (!done) s->player = -s->player;
    or_perspective(s, s->player, o->obs);
    o->reward = rew; o->terminated = done;
}

/* ---------------- batched entry points (ctypes) ---------------- */

static void load_state(or_state *s, const int8_t *board, const uint8_t *off,
                       const uint8_t *ft, int8_t player) {
    for (int k = 0; k < 24; ++k) s->board[k] = board[k];
    s->off_w = off[0]; s->off_b = off[1];
    s->ft_w = ft[0]; s->ft_b = ft[1];
    s->player = player;
    s->elapsed = 0;
}

static void store_state(const or_state *s, int8_t *board, uint8_t *off, uint8_t *ft, int8_t *player) {
    for (int k = 0; k < 24; ++k) board[k] = (int8_t)s->board[k];
    off[0] = (uint8_t)s->off_w; off[1] = (uint8_t)s->off_b;
    ft[0] = (uint8_t)s->ft_w; ft[1] = (uint8_t)s->ft_b;
    if (player) *player = (int8_t)s->player;
}

/* get_valid_moves over a batch. moves: [n][OR_MAXM][2] int8, -1 padded. */
void or_legal_batch(int64_t n, const int8_t *board, const uint8_t *off, const uint8_t *ft,
                    const int8_t *player, const uint8_t *roll, const uint8_t *nroll,
                    int8_t *moves, int16_t *count) {
    (void)off;
    for (int64_t i = 0; i < n; ++i) {
        int32_t b[24], r[4], out[OR_MAXM][2];
        for (int k = 0; k < 24; ++k) b[k] = board[i * 24 + k];
        for (int k = 0; k < nroll[i]; ++k) r[k] = roll[i * 4 + k];
        int c = or_get_valid_moves(b, ft[i * 2], ft[i * 2 + 1], r, nroll[i], player[i], out);
        count[i] = (int16_t)c;
        for (int k = 0; k < OR_MAXM; ++k) {
            moves[(i * OR_MAXM + k) * 2 + 0] = k < c ? (int8_t)out[k][0] : -1;
            moves[(i * OR_MAXM + k) * 2 + 1] = k < c ? (int8_t)out[k][1] : -1;
        }
    }
}

void or_block_batch(int64_t n, const int8_t *board, uint8_t *out) {
    for (int64_t i = 0; i < n; ++i) {
        int32_t b[24];
        for (int k = 0; k < 24; ++k) b[k] = board[i * 24 + k];
        out[i] = (uint8_t)or_violates_block_rule(b);
    }
}

void or_apply_batch(int64_t n, int8_t *board, uint8_t *off, uint8_t *ft,
                    const int8_t *player, const int8_t *move) {
    for (int64_t i = 0; i < n; ++i) {
        or_state s;
        load_state(&s, board + i * 24, off + i * 2, ft + i * 2, player[i]);
        or_execute_rotated_move(&s, move[i * 2], move[i * 2 + 1], player[i]);
        store_state(&s, board + i * 24, off + i * 2, ft + i * 2, NULL);
    }
}

/* NardeEnv.step over a batch with injected dice and given action codes.
 * State arrays are updated in place. */
void or_step_batch(int64_t n, int8_t *board, uint8_t *off, uint8_t *ft, int8_t *player,
                   const uint8_t *dice, const int16_t *action,
                   int8_t *obs, int8_t *reward, uint8_t *terminated,
                   int8_t *list1, int16_t *count1, int8_t *list2, int16_t *count2, uint8_t *roll2,
                   uint64_t *legal1) {
    for (int64_t i = 0; i < n; ++i) {
        or_state s;
        or_step_out o;
        load_state(&s, board + i * 24, off + i * 2, ft + i * 2, player[i]);
        int32_t d[2] = {dice[i * 2], dice[i * 2 + 1]};
        or_step_core(&s, d, action[i * 2], action[i * 2 + 1], 0, 0, 0, &o);
        store_state(&s, board + i * 24, off + i * 2, ft + i * 2, player + i);
        for (int k = 0; k < 24; ++k) obs[i * 24 + k] = (int8_t)o.obs[k];
        reward[i] = (int8_t)o.reward;
        terminated[i] = (uint8_t)o.terminated;
        if (list1) {
            for (int k = 0; k < OR_MAXM; ++k) {
                list1[(i * OR_MAXM + k) * 2] = k < o.count1 ? (int8_t)o.list1[k][0] : -1;
                list1[(i * OR_MAXM + k) * 2 + 1] = k < o.count1 ? (int8_t)o.list1[k][1] : -1;
                list2[(i * OR_MAXM + k) * 2] = k < o.count2 ? (int8_t)o.list2[k][0] : -1;
                list2[(i * OR_MAXM + k) * 2 + 1] = k < o.count2 ? (int8_t)o.list2[k][1] : -1;
            }
            count1[i] = (int16_t)o.count1;
            count2[i] = (int16_t)o.count2;
            roll2[i] = (uint8_t)o.roll2;
        }
        if (legal1) legal1[i] = o.legal1;
    }
}

/* ================= FULL4 rules mode (build extension) =================
 * Whole turns with 4-move doubles and the max-dice-used rule (SURVEY.md
 * section 8 row f-2; spec README.md:27-30).  The reference env never plays
 * them, so the composition rule is the build's; every
 * sub-move is the reference's own single-die primitive: or_get_valid_moves
 * with ONE die (narde.py:58-92 incl. the block filter :139-184) applied with
 * or_execute_rotated_move (narde.py:36-56).  Pinned to tests/golden/full4.npz
 * (tools/capture_full4.py: the same composition over the imported
 * reference's Narde objects).
 *   D = [a]*4 if a == b else [max, min];  H = 2 if first_turn and a == b in
 *   {3,4,6} else 1 (narde.py:94-106's condition) = head moves allowed;
 *   options = (v, p) for each distinct remaining die v descending, each entry
 *   of get_valid_moves([v]) ascending, except a head move beyond H;
 *   M = max sub-moves over all sequences; C_k = options whose child still
 *   reaches M; two different dice with M == 1: the higher die if it has an
 *   option; sub-move k plays entry mulhi(w[k], |C_k|) of C_k.
 */
typedef struct { int32_t v, from, to; } or_opt;

static int or_f4_options(const or_state *s, const int32_t *R, int nR, int h, int H, or_opt *opt) {
    int vals[4], nv = 0;
    for (int i = 0; i < nR; ++i) {
        int dup = 0;
        for (int j = 0; j < nv; ++j) dup |= vals[j] == R[i];
        if (!dup) vals[nv++] = R[i];
    }
    for (int i = 1; i < nv; ++i)
        for (int j = i; j > 0 && vals[j] > vals[j - 1]; --j) { int t = vals[j]; vals[j] = vals[j - 1]; vals[j - 1] = t; }
    int no = 0;
    for (int i = 0; i < nv; ++i) {
        int32_t die = vals[i], list[OR_MAXM][2];
        int c = or_get_valid_moves(s->board, s->ft_w, s->ft_b, &die, 1, s->player, list);
        for (int k = 0; k < c; ++k) {
            if (list[k][0] == 23 && h >= H) continue;
            opt[no].v = die; opt[no].from = list[k][0]; opt[no].to = list[k][1]; no++;
        }
    }
    return no;
}

static void or_f4_child(const or_state *s, const int32_t *R, int nR, int h, const or_opt *o,
                        or_state *c, int32_t *R2, int *nR2, int *h2) {
    *c = *s;
    or_execute_rotated_move(c, o->from, o->to, s->player);
    int removed = 0, n = 0;
    for (int i = 0; i < nR; ++i) {
        if (!removed && R[i] == o->v) { removed = 1; continue; }
        R2[n++] = R[i];
    }
    *nR2 = n;
    *h2 = h + (o->from == 23);
}

static int or_f4_depth(const or_state *s, const int32_t *R, int nR, int h, int H) {
    if (nR == 0) return 0;
    or_opt opt[64];
    int no = or_f4_options(s, R, nR, h, H, opt), best = 0;
    for (int i = 0; i < no && best < nR; ++i) {
        or_state c; int32_t R2[4]; int nR2, h2;
        or_f4_child(s, R, nR, h, &opt[i], &c, R2, &nR2, &h2);
        int d = 1 + or_f4_depth(&c, R2, nR2, h2, H);
        if (d > best) best = d;
    }
    return best;
}

/* One FULL4 turn of the mover, in place.  cm[k][0/1] = C_k source masks of
 * the higher/lower die (doubles: column 0); played[k] = (from, die), -1 pad. */
static int or_full4_turn(or_state *s, const int32_t dice[2], const uint32_t w[4],
                         uint32_t cm[4][2], int8_t played[4][2]) {
    int32_t a = dice[0], b = dice[1], hi = a > b ? a : b, lo = a > b ? b : a;
    int32_t R[4];
    int nR;
    if (a == b) { R[0] = R[1] = R[2] = R[3] = a; nR = 4; }
    else { R[0] = hi; R[1] = lo; nR = 2; }
    int ft = s->player == 1 ? s->ft_w : s->ft_b;
    int H = (ft && a == b && (a == 3 || a == 4 || a == 6)) ? 2 : 1, h = 0;
    int M = or_f4_depth(s, R, nR, h, H);
    for (int k = 0; k < 4; ++k) { cm[k][0] = cm[k][1] = 0; played[k][0] = played[k][1] = -1; }
    for (int k = 0; k < M; ++k) {
        or_opt opt[64], C[64];
        int no = or_f4_options(s, R, nR, h, H, opt), nc = 0;
        for (int i = 0; i < no; ++i) {
            or_state c; int32_t R2[4]; int nR2, h2;
            or_f4_child(s, R, nR, h, &opt[i], &c, R2, &nR2, &h2);
            if (or_f4_depth(&c, R2, nR2, h2, H) == M - k - 1) C[nc++] = opt[i];
        }
        if (k == 0 && M == 1 && a != b) {
            int any_hi = 0;
            for (int i = 0; i < nc; ++i) any_hi |= C[i].v == hi;
            if (any_hi) {
                int m = 0;
                for (int i = 0; i < nc; ++i) if (C[i].v == hi) C[m++] = C[i];
                nc = m;
            }
        }
        if (nc == 0) return M; /* unreachable: C_k is non-empty below M */
        for (int i = 0; i < nc; ++i) cm[k][C[i].v == hi ? 0 : 1] |= 1u << C[i].from;
        const or_opt *o = &C[mulhi_n(w[k], (uint32_t)nc)];
        played[k][0] = (int8_t)o->from; played[k][1] = (int8_t)o->v;
        or_state c; int32_t R2[4]; int nR2, h2;
        or_f4_child(s, R, nR, h, o, &c, R2, &nR2, &h2);
        *s = c; memcpy(R, R2, sizeof R2); nR = nR2; h = h2;
    }
    return M;
}

/* FULL4 turns over a batch with given dice and pick words; state updated in
 * place (no player flip: the caller sees the post-turn board). */
void or_full4_batch(int64_t n, int8_t *board, uint8_t *off, uint8_t *ft, const int8_t *player,
                    const uint8_t *dice, const uint32_t *words, int8_t *max_dice, uint32_t *cmask,
                    int8_t *played, int8_t *reward, uint8_t *done) {
    for (int64_t i = 0; i < n; ++i) {
        or_state s;
        load_state(&s, board + i * 24, off + i * 2, ft + i * 2, player[i]);
        int32_t d[2] = {dice[i * 2], dice[i * 2 + 1]};
        uint32_t cm[4][2];
        int8_t pl[4][2];
        max_dice[i] = (int8_t)or_full4_turn(&s, d, words + i * 4, cm, pl);
        memcpy(cmask + i * 8, cm, sizeof cm);
        memcpy(played + i * 8, pl, sizeof pl);
        int dn, rw;
        or_check_game_ended(&s, &dn, &rw);
        reward[i] = (int8_t)rw; done[i] = (uint8_t)dn;
        store_state(&s, board + i * 24, off + i * 2, ft + i * 2, NULL);
    }
}

/* 198-float Tesauro-style observation, README.md:42-102 (spec only; the
 * reference has no implementation -> parity unpinned).  Absolute points,
 * white block [0..97], black block [98..195], player one-hot [196..197]. */
void or_tesauro198(const int32_t *board, int off_w, int off_b, int player, float *out) {
    memset(out, 0, 198 * sizeof(float));
    for (int side = 0; side < 2; ++side) {
        float *o = out + side * 98;
        for (int p = 0; p < 24; ++p) {
            int v = board[p];
            int c = side == 0 ? (v > 0 ? v : 0) : (v < 0 ? -v : 0);
            if (c >= 1) o[p * 4 + 0] = 1.0f;
            if (c >= 2) o[p * 4 + 1] = 1.0f;
            if (c >= 3) { o[p * 4 + 2] = 1.0f; o[p * 4 + 3] = (float)(c - 3) / 2.0f; }
        }
        o[96] = 0.0f; /* bar: Narde has none */
        o[97] = (float)(side == 0 ? off_w : off_b) / 15.0f;
    }
    out[196] = player == 1 ? 1.0f : 0.0f;
    out[197] = player == 1 ? 0.0f : 1.0f;
}

void or_tesauro198_batch(int64_t n, const int8_t *board, const uint8_t *off, const int8_t *player, float *out) {
    for (int64_t i = 0; i < n; ++i) {
        int32_t b[24];
        for (int k = 0; k < 24; ++k) b[k] = board[i * 24 + k];
        or_tesauro198(b, off[i * 2], off[i * 2 + 1], player[i], out + i * 198);
    }
}

/* ---------------- Philox4x32-10 (Salmon et al., SC'11) ---------------- */

void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}


/* dice_mode 0: all 36 ordered pairs; 1: the 30 non-double ordered pairs. */
static void or_dice_from(uint32_t r, int dice_mode, int32_t d[2]) {
    if (dice_mode == 1) {
        uint32_t k = mulhi_n(r, 30);
        int a = (int)(k / 5) + 1, j = (int)(k % 5);
        d[0] = a; d[1] = j < a - 1 ? j + 1 : j + 2;
    } else {
        uint32_t k = mulhi_n(r, 36);
        d[0] = (int)(k / 6) + 1; d[1] = (int)(k % 6) + 1;
    }
}

/* Opening roll (narde_env.py:111-117): the reference redraws equal pairs;
 * drawing uniformly over the 30 unequal ordered pairs has the same law. */
static void or_reset_state(or_state *s, uint32_t r) {
    memset(s, 0, sizeof *s);
    s->board[23] = 15; s->board[11] = -15;
    s->ft_w = 1; s->ft_b = 1;
    int32_t d[2];
    or_dice_from(r, 1, d);
    s->player = d[0] > d[1] ? 1 : -1;
}

/*
 * Self-play driver restatement.  For env e (global id) and lockstep ply t:
 *   R = Philox4x32-10(ctr = {t >> 1, e, 0, 0}, key = {seed_lo, seed_hi})
 *   (one block per ply pair), (wa, wb) = (R0, R1) for even t, (R2, R3) for
 *   odd t, and the ply's words
 *   r0 = wa dice, r1 = wa * m mod 2^32 move1 pick (m = 36, or 30 for the
 *   non-double dice law), r2 = wb move2 pick, r3 = wb * 0x9E3779B9 opening
 *   roll of the episode that starts if this ply ends the current one.
 * Reset of env e with reset-epoch q: ctr = {q, e, 0, 1}, r0 = opening roll.
 */
static void or_ply_words(const uint32_t R[4], uint32_t t, int dice_mode, uint32_t r[4]) {
    uint32_t wa = (t & 1u) ? R[2] : R[0];
    uint32_t wb = (t & 1u) ? R[3] : R[1];
    r[0] = wa;
    r[1] = wa * (dice_mode == 1 ? 30u : 36u);
    r[2] = wb;
    r[3] = wb * 0x9E3779B9u;
}

static void or_ply_draw(uint32_t t, int64_t e, const uint32_t key[2], int first, int dice_mode,
                        uint32_t R[4], uint32_t r[4]) {
    if (first || (t & 1u) == 0u) {
        uint32_t ctr[4] = {t >> 1, (uint32_t)e, 0, 0};
        or_philox4x32_10(ctr, key, R);
    }
    or_ply_words(R, t, dice_mode, r);
}
void or_reset_batch(int64_t n, int64_t env0, uint64_t seed, uint32_t epoch,
                    int8_t *board, uint8_t *off, uint8_t *ft, int8_t *player, uint16_t *elapsed) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; ++i) {
        uint32_t ctr[4] = {epoch, (uint32_t)(env0 + i), 0, 1}, r[4];
        or_philox4x32_10(ctr, key, r);
        or_state s;
        or_reset_state(&s, r[0]);
        store_state(&s, board + i * 24, off + i * 2, ft + i * 2, player + i);
        elapsed[i] = 0;
    }
}

/*
 * Run `plies` lockstep plies t0..t0+plies-1 of random-legal self-play over n
 * envs.  Per-ply outputs (optional, NULL to skip) are [plies][n][...]:
 * obs int8[24] (next mover's perspective, after auto-reset), reward,
 * terminated, truncated, dice[2], action codes[2], count1, legal1 (list #1
 * in the build's compact form, or_compact2).
 * stats[n][3] accumulates {games, white points, black points}.
 */
void or_selfplay(int64_t n, int64_t env0, uint64_t seed, uint32_t t0, int plies,
                 int dice_mode, int max_steps,
                 int8_t *board, uint8_t *off, uint8_t *ft, int8_t *player, uint16_t *elapsed,
                 int32_t *stats,
                 int8_t *obs, int8_t *reward, uint8_t *terminated, uint8_t *truncated,
                 uint8_t *dice_out, int16_t *action_out, int16_t *count1_out, uint64_t *legal_out) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; ++i) {
        or_state s;
        load_state(&s, board + i * 24, off + i * 2, ft + i * 2, player[i]);
        s.elapsed = elapsed[i];
        uint32_t R[4];
        for (int p = 0; p < plies; ++p) {
            uint32_t r[4];
            or_ply_draw(t0 + (uint32_t)p, env0 + i, key, p == 0, dice_mode, R, r);
            int32_t d[2];
            or_dice_from(r[0], dice_mode, d);
            or_step_out o;
            int mover = s.player;
            or_step_core(&s, d, 0, 0, 1, r[1], r[2], &o);
            s.elapsed += 1;
            int term = o.terminated;
            int trunc = s.elapsed >= max_steps;
            int64_t ix = (int64_t)p * n + i;
            if (term) {
                stats[i * 3 + 0] += 1;
                stats[i * 3 + (mover == 1 ? 1 : 2)] += o.reward;
            } else if (trunc) {
                stats[i * 3 + 0] += 1;
            }
            if (term || trunc) {
                or_reset_state(&s, r[3]);
                or_perspective(&s, s.player, o.obs);
            }
            if (obs) for (int k = 0; k < 24; ++k) obs[ix * 24 + k] = (int8_t)o.obs[k];
            if (reward) reward[ix] = (int8_t)o.reward;
            if (terminated) terminated[ix] = (uint8_t)term;
            if (truncated) truncated[ix] = (uint8_t)trunc;
            if (dice_out) { dice_out[ix * 2] = (uint8_t)d[0]; dice_out[ix * 2 + 1] = (uint8_t)d[1]; }
            if (action_out) { action_out[ix * 2] = (int16_t)o.code1; action_out[ix * 2 + 1] = (int16_t)o.code2; }
            if (count1_out) count1_out[ix] = (int16_t)o.count1;
            if (legal_out) legal_out[ix] = o.legal1;
        }
        store_state(&s, board + i * 24, off + i * 2, ft + i * 2, player + i);
        elapsed[i] = (uint16_t)s.elapsed;
    }
}


/*
 * FULL4 self-play driver restatement: as or_selfplay
 * with a whole FULL4 turn per step.  Pick words w = {r1, r2, r1 * 0x85EBCA6B,
 * r2 * 0xC2B2AE35} (mod 2^32; the last two only matter on doubles).  Per-ply
 * outputs (optional): obs, reward, terminated, truncated, dice, legal u64
 * (C_0 masks | d_hi<<48 | d_lo<<52 | M<<56), played u64 (bytes 2k/2k+1 =
 * from/die of sub-move k, 0xFF = none).
 */
void or_selfplay_full(int64_t n, int64_t env0, uint64_t seed, uint32_t t0, int plies,
                      int dice_mode, int max_steps,
                      int8_t *board, uint8_t *off, uint8_t *ft, int8_t *player, uint16_t *elapsed,
                      int32_t *stats,
                      int8_t *obs, int8_t *reward, uint8_t *terminated, uint8_t *truncated,
                      uint8_t *dice_out, uint64_t *legal_out, uint64_t *played_out) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; ++i) {
        or_state s;
        load_state(&s, board + i * 24, off + i * 2, ft + i * 2, player[i]);
        s.elapsed = elapsed[i];
        uint32_t R[4];
        for (int p = 0; p < plies; ++p) {
            uint32_t r[4];
            or_ply_draw(t0 + (uint32_t)p, env0 + i, key, p == 0, dice_mode, R, r);
            int32_t d[2];
            or_dice_from(r[0], dice_mode, d);
            uint32_t w[4] = {r[1], r[2], r[1] * 0x85EBCA6Bu, r[2] * 0xC2B2AE35u};
            int mover = s.player;
            uint32_t cm[4][2];
            int8_t pl[4][2];
            int M = or_full4_turn(&s, d, w, cm, pl);
            int term, rew;
            or_check_game_ended(&s, &term, &rew);
            if (!term) s.player = -s.player;
            s.elapsed += 1;
            int trunc = max_steps > 0 && s.elapsed >= max_steps;
            if (term) {
                stats[i * 3 + 0] += 1;
                stats[i * 3 + (mover == 1 ? 1 : 2)] += rew;
            } else if (trunc) {
                stats[i * 3 + 0] += 1;
            }
            if (term || trunc) or_reset_state(&s, r[3]);
            int64_t ix = (int64_t)p * n + i;
            if (obs) {
                int32_t o[24];
                or_perspective(&s, s.player, o);
                for (int k = 0; k < 24; ++k) obs[ix * 24 + k] = (int8_t)o[k];
            }
            if (reward) reward[ix] = (int8_t)rew;
            if (terminated) terminated[ix] = (uint8_t)term;
            if (truncated) truncated[ix] = (uint8_t)trunc;
            if (dice_out) { dice_out[ix * 2] = (uint8_t)d[0]; dice_out[ix * 2 + 1] = (uint8_t)d[1]; }
            if (legal_out) {
                uint32_t hi = d[0] > d[1] ? d[0] : d[1], lo = d[0] > d[1] ? d[1] : d[0];
                legal_out[ix] = (uint64_t)cm[0][0] | ((uint64_t)cm[0][1] << 24) |
                                ((uint64_t)hi << 48) | ((uint64_t)lo << 52) | ((uint64_t)M << 56);
            }
            if (played_out) {
                uint64_t v = 0;
                for (int k = 0; k < 4; ++k)
                    v |= (uint64_t)(((uint32_t)(uint8_t)pl[k][1] << 8) | (uint8_t)pl[k][0]) << (16 * k);
                played_out[ix] = v;
            }
        }
        store_state(&s, board + i * 24, off + i * 2, ft + i * 2, player + i);
        elapsed[i] = (uint16_t)s.elapsed;
    }
}
