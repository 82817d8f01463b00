/*
 * narde.h -- C ABI of libnarde, the MI355X-native batched Narde environment.
 *
 * The reference (dmytroleonenko/gym-narde) is pure Python and has no FFI;
 * this ABI is the boundary UNDER a Python facade that reproduces its
 * gymnasium surface (gym-narde_amd/gym_narde/).  Each entry point names the
 * reference function it replaces (paths under the reference checkout):
 *
 *   narde_reset              NardeEnv.reset           gym_narde/envs/narde_env.py:105-120
 *   narde_legal_moves        Narde.get_valid_moves    gym_narde/envs/narde.py:58-92
 *   narde_step               NardeEnv.step            gym_narde/envs/narde_env.py:27-103
 *   narde_apply_moves        Narde.execute_rotated_move gym_narde/envs/narde.py:36-56
 *   narde_violates_block_rule Narde._violates_block_rule gym_narde/envs/narde.py:139-184
 *   narde_observe            NardeEnv._get_obs / get_perspective_board
 *                                                     gym_narde/envs/narde_env.py:24-25,
 *                                                     gym_narde/envs/narde.py:31-34
 *                            + 198-float Tesauro obs   README.md:42-102 (spec only)
 *   narde_get/set_state      direct `env.unwrapped.game` attribute access
 *                            (train_deepq_pytorch.py:867-931, evaluate_model.py:22-134)
 *   narde_selfplay           random-policy self-play loop (no reference equivalent;
 *                            the benchmark workload of BASELINE.json)
 *   narde_host_*             the same rules on small HOST batches (the scalar
 *                            gym facade): staged through pinned memory, synchronous.
 *
 * Conventions
 *   - Every pointer argument of a non-host entry point is a DEVICE pointer on
 *     the handle's device (e.g. a torch tensor's data_ptr()); NULL means
 *     "not requested" where documented.  Arrays are C-contiguous.
 *   - `stream` is a hipStream_t (NULL = the null stream).  Calls are stream-
 *     ordered and never synchronise unless documented (narde_host_*).
 *   - Board layout = the reference's: int8[24] absolute points, white > 0,
 *     black < 0 (point p = index p, white head 23, black head 11).
 *     off = {borne_off_white, borne_off_black}; first_turn = {white, black};
 *     player = current mover, +1 white / -1 black.
 *   - A move is (from, to) in the MOVER's perspective, to = 24 for 'off'.
 *   - Action codes are the reference's: from*24 + to, with to == 0 and
 *     from <= 5 meaning (from, 'off') (narde_env.py:238-254).
 *   - Return value: 0 on success, negative NARDE_E* on error;
 *     narde_last_error() gives a message (thread-local).
 */
#ifndef NARDE_H
#define NARDE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NARDE_OK 0
#define NARDE_EINVAL (-1)
#define NARDE_EHIP (-2)
#define NARDE_ENOMEM (-3)

#define NARDE_DICE_ALL36 0      /* dice uniform over the 36 ordered pairs      */
#define NARDE_DICE_NODOUBLES 1  /* uniform over the 30 non-double ordered pairs */

#define NARDE_MAX_MOVES 64      /* list capacity per env (4-die rolls give <= 60) */
#define NARDE_OFF 24

typedef struct narde_env narde_env; /* B envs resident in HBM on one device */

int narde_version(void);
const char *narde_last_error(void);

/* Allocate B = num_envs env records on `device`.  Global env ids are
 * env_id_offset .. env_id_offset+B-1 (device RNG is keyed by the global id,
 * so a sharded run reproduces a single-GPU run).  max_episode_steps is the
 * gymnasium TimeLimit (reference registers 1000: gym_narde/__init__.py:3-7);
 * 0 disables truncation.  Envs start in the reset state of epoch 0. */
int narde_create(int device, int64_t num_envs, int64_t env_id_offset, uint64_t seed,
                 int dice_mode, int max_episode_steps, narde_env **out);
int narde_destroy(narde_env *env);
int64_t narde_num_envs(const narde_env *env);
/* Per-env RNG ply counter t (kept in the env record, +1 per step, kept
 * across episodes): the device dice/policy draws of an env's next step are
 * Philox4x32-10(ctr = {t, global_env_id, 0, 0}, key = seed).  Because t lives
 * in device state, narde_step / narde_rollout launches can be captured in a
 * hipGraph and replayed.  get_ply reads env 0's counter and set_ply sets
 * every env's counter; both synchronise the whole device first
 * (hipDeviceSynchronize), so work queued on any stream is ordered before
 * them -- a device-wide barrier: they also wait for every other stream of
 * the process on that device, unrelated work (training, other handles)
 * included.  Neither belongs in a hot loop. */
int narde_get_ply(const narde_env *env, uint32_t *t);
int narde_set_ply(narde_env *env, uint32_t t);

/* NardeEnv.reset: start position + opening roll.  mask[B] (u8) selects envs,
 * NULL = all.  opening (optional) u8[B][pairs][2]: each env's opening draws
 * (white roll, black roll) in the order the reference draws them
 * (narde_env.py:111-117): the first pair of different dice decides, the
 * higher roll moves first; pairs with a die outside 1..6 are padding, and an
 * env whose row has no deciding pair (or opening = NULL) takes the device
 * draw, uniform over the 30 unequal ordered pairs.  Zeroes the per-env
 * statistics of reset envs. */
int narde_reset(narde_env *env, const uint8_t *mask, const uint8_t *opening, int pairs,
                void *stream);

/* Direct state access.  elapsed may be NULL (set: 0).  The device path does
 * NOT validate: a board value outside [-15, 15], more than 15 checkers (on
 * the board + off) of a colour, off > 15 or a player other than +1/-1 wraps
 * into neighbouring 4-bit fields of the record, so callers must pass legal
 * positions.  The narde_host_* entry points check every position and return
 * NARDE_EINVAL instead. */
int narde_set_state(narde_env *env, const int8_t *board, const uint8_t *off,
                    const uint8_t *first_turn, const int8_t *player, const uint16_t *elapsed,
                    void *stream);
int narde_get_state(narde_env *env, int8_t *board, uint8_t *off, uint8_t *first_turn,
                    int8_t *player, uint16_t *elapsed, void *stream);

/* Dice the next narde_step(dice = NULL) will use, in roll order: u8[B][2]. */
int narde_peek_dice(narde_env *env, uint8_t *dice, void *stream);

/* Narde.get_valid_moves(roll, current_player) for every env's mover.
 * dice: u8[B][4], 1..4 dice per env, unused slots 0; NULL = the next step's
 * device dice.  out_count: i16[B].  out_moves (optional): i8[B][64][2] (from,
 * to), -1 padded, exactly the reference's list (order + duplicates).
 * out_compact (optional, only for <= 2 dice): u64[B] = L_hi | L_lo<<24 |
 * d_hi<<48 | d_lo<<52 where L_* are the per-die 24-bit source masks. */
int narde_legal_moves(narde_env *env, const uint8_t *dice, int16_t *out_count,
                      int8_t *out_moves, uint64_t *out_compact, void *stream);

/* NardeEnv.step for all B envs.  actions i16[B][2] = (move1_code,
 * move2_code); NULL = in-kernel random legal policy.  dice u8[B][2] in roll
 * order; NULL = device RNG at each env's counter t.  A given die outside 1..6
 * makes that env's ply one with no legal move (list #1 empty: no checker
 * moves, the player changes, t and the TimeLimit count advance); the same
 * holds for the given dice of narde_step_full / narde_legal_full /
 * narde_legal_mask576_move2 (no sub-move / legal word 0 / empty mask).  Outputs (each optional, NULL = skip):
 * obs i32[B][24] (next mover's perspective), reward i32[B], terminated u8[B],
 * truncated u8[B], legal_compact u64[B] (list #1, format above),
 * actions_out i16[B][2] (codes actually used).  autoreset != 0: envs that
 * terminate or truncate are reset in the same call (obs is then the new
 * episode's first obs) and counted in the statistics.  Increments every
 * env's t. */
int narde_step(narde_env *env, const int16_t *actions, const uint8_t *dice, int32_t *obs,
               int32_t *reward, uint8_t *terminated, uint8_t *truncated,
               uint64_t *legal_compact, int16_t *actions_out, int autoreset, void *stream);

/* `plies` plies of random-legal self-play with auto-reset in ONE launch, the
 * env record kept in registers across plies.  Every ply's outputs are
 * streamed to rollout buffers laid out [plies][B][...] with the per-ply
 * formats of narde_step (each optional, NULL = skip).  Statistics accumulate
 * as in narde_step.  Equivalent to `plies` narde_step(actions = NULL,
 * dice = NULL, autoreset = 1) calls. */
int narde_rollout(narde_env *env, int plies, int32_t *obs, int32_t *reward, uint8_t *terminated,
                  uint8_t *truncated, uint64_t *legal_compact, int16_t *actions_out, void *stream);

/* narde_rollout with no per-ply outputs (statistics only). */
int narde_selfplay(narde_env *env, int plies, void *stream);

/* ---- FULL4 rules mode (build extension) -------------
 * One step = the mover's WHOLE turn: four sub-moves on doubles, the
 * max-dice-used rule, the higher die when only one of two dice can be used,
 * at most one checker off the head per turn (two on a first-turn 3-3, 4-4 or
 * 6-6).  Every sub-move is the reference's single-die primitive
 * (Narde.get_valid_moves([die]) narde.py:58-92, execute_rotated_move
 * narde.py:36-56); the reference env itself stops after two checker moves
 * (narde_env.py:45-93), so whole-turn parity is against the build's oracle,
 * which is pinned sub-move by sub-move to the reference (tests/golden/full4.npz).
 * A sub-move is (from, die), from in the mover's perspective; the landing
 * point is from - die, or 'off' when negative.
 *   legal_first u64[B] = C_hi | C_lo<<24 | d_hi<<48 | d_lo<<52 | M<<56: the
 *     sources playable as the FIRST sub-move with the higher / lower die
 *     (doubles: C_lo = 0, d_lo = d_hi) and M = max dice usable (0..4).
 *   played u64[B]: bytes 2k / 2k+1 = from / die of sub-move k, 0xFF unused.
 *   play i8[B][4][2] (from, die): applied while each sub-move keeps M
 *     reachable; the first one that does not ends the turn (illegal actions
 *     are ignored, as in narde_env.py:56-93).  NULL = in-kernel random policy
 *     (sub-move k uniform over its legal set). */
int narde_step_full(narde_env *env, const int8_t *play, const uint8_t *dice, int32_t *obs,
                    int32_t *reward, uint8_t *terminated, uint8_t *truncated,
                    uint64_t *legal_first, uint64_t *played, int autoreset, void *stream);
/* `plies` FULL4 random-policy turns per env in ONE launch (outputs [plies][B]). */
int narde_rollout_full(narde_env *env, int plies, int32_t *obs, int32_t *reward,
                       uint8_t *terminated, uint8_t *truncated, uint64_t *legal_first,
                       uint64_t *played, void *stream);
int narde_selfplay_full(narde_env *env, int plies, void *stream);
/* narde_rollout (full = 0; `last` = actions i16[plies][B][2]) or
 * narde_rollout_full (full = 1; `last` = played u64[plies][B]) with HIP
 * events recorded on `stream` just before the launch (ev_start) and just
 * after it (ev_stop), each optional (NULL): a timed launch is one call
 * instead of three (bench.py's timed region).  totals (optional): the
 * launch also writes the statistics of narde_get_stats after it, summed per
 * workgroup of 256 envs, as i64[NARDE_WG_ROWS(B)][3] {episodes, white
 * points, black points} (row r: envs 256 r .. 256 r + 255) -- the self-play
 * driver's per-run result with no second launch.  plies = 0 launches
 * nothing (and then totals must be NULL). */
#define NARDE_WG_ROWS(num_envs) (((num_envs) + 255) / 256)
int narde_rollout_timed(narde_env *env, int full, int plies, int32_t *obs, int32_t *reward,
                        uint8_t *terminated, uint8_t *truncated, uint64_t *legal, void *last,
                        void *ev_start, void *ev_stop, int64_t *totals, void *stream);
/* narde_rollout_timed pre-bound (round 6): _create checks the arguments,
 * chooses the kernel and packs its arguments once (plies > 0; the calling
 * thread's current device must be the env's); _launch then records ev_start,
 * launches and records ev_stop on `stream` -- the same launch as
 * narde_rollout_timed with the same arguments, one pointer per call (the
 * caller keeps the thread's current device and every buffer as at create);
 * _destroy frees the plan (host memory only). */
int narde_rollout_plan_create(narde_env *env, int full, int plies, int32_t *obs, int32_t *reward,
                              uint8_t *terminated, uint8_t *truncated, uint64_t *legal,
                              void *last, void *ev_start, void *ev_stop, int64_t *totals,
                              void *stream, void **plan);
int narde_rollout_plan_launch(void *plan);
int narde_rollout_plan_destroy(void *plan);
/* Timing events for narde_rollout_timed on `device`: a HIP event (returned
 * as void*) created with hipEventCreateWithFlags(flags); flags 0 = HIP's
 * default, 0x20000000 = hipEventDisableSystemFence (the event's record does
 * no system-scope cache write-back / invalidate: a timing-only marker, what
 * bench.py uses).  elapsed_ms = hipEventElapsedTime (both recorded and
 * complete). */
int narde_timing_event_create(int device, unsigned flags, void **event);
int narde_timing_event_destroy(void *event);
int narde_timing_event_elapsed_ms(void *start, void *stop, float *ms);
/* C_0 and M for dice u8[B][2] (NULL = the next step's device dice). */
int narde_legal_full(narde_env *env, const uint8_t *dice, uint64_t *legal_first, void *stream);

/* Per-env statistics i32[B][3] = {episodes finished, white points, black
 * points} since the last reset of that env. */
int narde_get_stats(narde_env *env, int32_t *stats, void *stream);

/* The same statistics summed over the handle's envs, as NARDE_TOTAL_ROWS
 * partial rows i64[NARDE_TOTAL_ROWS][3] (row b: the b-th contiguous range
 * of envs); the totals are the column sums.  One launch -- what a sharded
 * self-play run all-gathers per rank (the reference's returns, collected
 * by its training loops: train_deepq_pytorch.py:855-1081). */
#define NARDE_TOTAL_ROWS 64
int narde_get_totals(narde_env *env, int64_t *rows, void *stream);

/* execute_rotated_move(move, player) per env: moves i8[B][2] in the
 * perspective of player[B] (+1/-1; NULL = each env's current mover);
 * from < 0 skips the env.  Clears that player's first_turn flag.  A move the
 * record cannot hold -- the source has none of the player's checkers, or the
 * target holds opponent checkers (the reference, narde.py:108-125, would
 * conjure or cancel checkers) -- leaves that env unchanged; every listed move
 * is executable.  narde_host_apply_moves returns NARDE_EINVAL for one. */
int narde_apply_moves(narde_env *env, const int8_t *moves, const int8_t *player, void *stream);

/* obs i32[B][24] (current mover's perspective) and/or the 198-float
 * Tesauro observation f32[B][198] (absolute points; white block first). */
int narde_observe(narde_env *env, int32_t *obs, float *tesauro198, void *stream);

/* 576-bit mask of legal move1 action codes for the next step's dice:
 * u64[B][9], bit c set iff the reference would accept code c as move1. */
int narde_legal_mask576(narde_env *env, uint64_t *mask, void *stream);

/* Move-2 acceptance mask u64[B][9] given each env's move-1 code i16[B] and
 * dice u8[B][2] in roll order (NULL = the next step's device dice): bit c
 * set iff NardeEnv.step would play code c as move2 after move1
 * (narde_env.py:56-93); all zero when move1 would not be played.  With
 * narde_legal_mask576 it gives a policy the exact legal set of (move1,
 * move2) codes (train_deepq_pytorch.py:411-600 approximates it). */
int narde_legal_mask576_move2(narde_env *env, const int16_t *move1, const uint8_t *dice,
                              uint64_t *mask, void *stream);

/* The plays of each env's two-dice roll (the README's get_valid_actions,
 * README.md:156-165), for dice u8[B][2] in roll order (NULL = the next
 * step's device dice).  Replaces the per-env Python lists of
 * DQNAgent.act (train_deepq_pytorch.py:430-507, kind 0) and the (m1, m2)
 * set NardeEnv.step carries out (narde_env.py:45-93, kind 1; the facade's
 * Narde.get_valid_plays).  Outputs: legal u64[B] (optional) = list #1 in
 * the compact format above; table u32[B][2][24]: for each list-#1 entry
 * (k = 0 the higher die's list, k = 1 the lower's; source p) the word
 * second-move sources (24 bits) | rem << 24 | 1 << 27, 0 where (k, p) is no
 * entry -- kind 0: rem = the roll less the die act() matches to move 1
 * (exact distance in roll order; a bear-off from p: the first die >= p+1),
 * its list get_valid_moves([rem]) on the pre-move board; kind 1: move 1
 * applied, rem per the step's bookkeeping, list #2 on the post-move board
 * (a one-entry list #1: word 1 << 27, played alone); count i32[B]: kind 0
 * len(valid_move_combinations) (every entry, duplicates included, times
 * max(1, |its list|)), kind 1 the number of distinct plays.  A die outside
 * 1..6: list 0, count 0. */
int narde_play_set(narde_env *env, const uint8_t *dice, int kind, uint64_t *legal, uint32_t *table,
                   int32_t *count, void *stream);

/* DQNAgent.act's greedy candidate sets (train_deepq_pytorch.py:520-560) as
 * 576-bit masks u64[B][9], for dice u8[B][2] in roll order (NULL = the next
 * step's device dice).  move1 NULL: bit c set iff c is the code act() gives
 * some list-#1 entry (valid_first_moves' keys).  move1 int64 (element i at
 * move1[i * ld_move1]): the move-2 codes act() offers after move 1 --
 * valid_first_moves[move1]: the pre-move second list of the LAST list-#1
 * entry with that code, bit 0 alone if that list is empty, no bit if no
 * entry has that code. */
int narde_act_masks(narde_env *env, const uint8_t *dice, const int64_t *move1, int64_t ld_move1,
                    uint64_t *mask, void *stream);

/* The DQN driver's exploration (train_deepq_pytorch.py:514-515): for the
 * rows whose explore draw Philox4x32-10({*tag, row, 0, 5}, seed) r0 <
 * *epsilon * 2^32 (the policy kernels' shared decision), writes play
 * mulhi(r1, count) of act()'s combination list (kind 0 above: uniform over
 * (move1, move2) combinations) into out[row * ld_out + 0..1] (int64 codes);
 * other rows, and rows with no play, are left untouched.  dice as above. */
int narde_explore_plays(narde_env *env, const uint8_t *dice, const float *epsilon, uint64_t seed,
                        const int64_t *tag, int64_t *out, int64_t ld_out, void *stream);

/* Masked epsilon-greedy over the 576 codes (the policy of
 * train_deepq_pytorch.py:411-600, batched; stateless): q f32[n][ldq]
 * (ldq >= 576) Q-values, mask u64[n][9] legal codes (the two mask entry
 * points above).  out i64[n] = the legal code with the largest Q (lowest
 * code on ties, as torch.argmax), or with probability epsilon a legal code
 * uniformly at random, or 0 when none is legal.  Draws are Philox4x32-10
 * ({tag, row, 0, 5}, seed); the explore decision depends only on (seed, tag,
 * row), so both heads of one step called with the same tag explore together
 * (head 0 / 1 select independent picks). */
int narde_policy_masked_argmax576(int device, const float *q, int64_t ldq, const uint64_t *mask,
                                  int64_t n, float epsilon, uint64_t seed, uint32_t tag, int head,
                                  int64_t *out, void *stream);

/* The same with epsilon (f32) and tag (int64, low 32 bits used) read from
 * DEVICE memory at run time, so a captured hipGraph replays with the values
 * current at each replay (the DQN driver's decaying epsilon and step tag).
 * Optional addend: with add_tab != NULL the greedy value of code c is
 * q[i][c] + add_tab[add_row[i] * ld_add + c] -- the move-2 head's one-hot
 * column (W[:, 256 + move1], pre-transposed into rows) fused into the
 * argmax instead of materialising a second (n, 576) matrix. */
int narde_policy_masked_argmax576_dev(int device, const float *q, int64_t ldq, const uint64_t *mask,
                                      int64_t n, const float *epsilon, uint64_t seed,
                                      const int64_t *tag, int head, const float *add_tab,
                                      int64_t ld_add, const int64_t *add_row, int64_t *out,
                                      void *stream);

/* narde_policy_masked_argmax576_dev with the head computed inside, for the
 * legal codes only: q_c = f[row] . w[c][0:256] + bias[c] (+ addcol[c * ldw +
 * add_row[row]] when addcol is given: the move-2 head's one-hot column of
 * DecomposedDQN, train_deepq_pytorch.py:184-277), masked argmax (first
 * maximum in code order) or epsilon exploration (the same draws as
 * narde_policy_masked_argmax576_dev).  f f32[B][ldf] (feat = 256), w
 * f32[576][ldw], rows 16-B aligned.  The fp32 sums round differently from a
 * dense GEMM's; a greedy pick can differ only between codes whose Q-values
 * tie to rounding.  The codes go to out[row * ld_out] (i64) and, if out16 is
 * given, out16[row * ld_out16] (i16): straight into a column of the (B, 2)
 * action rows; add_row is read as add_row[row * ld_row]. */
int narde_head_policy576_dev(int device, const float *f, int64_t ldf, int64_t feat, const float *w,
                             int64_t ldw, const float *bias, const uint64_t *mask, int64_t n,
                             const float *epsilon, uint64_t seed, const int64_t *tag, int head,
                             const float *addcol, const int64_t *add_row, int64_t ld_row,
                             int64_t *out, int64_t ld_out, int16_t *out16, int64_t ld_out16,
                             void *stream);

/* One DQN transition for all B envs, fused (the batched trainer of
 * gym_narde/dqn.py, config 4; reward shaping as train_deepq_pytorch.py:
 * 885-912).  After a narde_step: s' = the Tesauro-198 observation of each
 * env's record; r' = reward (+ shaping if `shaping`: for the player the
 * trainer names after the step -- at a step that ended the game the winner
 * (15 off) or, truncated, the other player of the pre-step record -- +1 per
 * checker newly borne off since its off_seen tracker and +0.1 x its off
 * count; none when list #1 was empty; trackers f32[B][2] updated, zeroed on
 * done); done = terminated | truncated.
 *   legal u64[B]: the step's compact list #1 (NULL = every env could move);
 *   misc i32[B]: off_white | off_black << 4 | black_to_move << 10 of each
 *     env before the step on entry (the caller seeds it once from
 *     narde_get_state), after it on return.
 * Replay ring (capacity rows, capacity >= 2B): row j holds transition j's
 * observation s, and s' is row (j + B) % capacity.  This step's transitions
 * are rows (pos + i) % capacity -- their s must already be there -- and get
 * (actions[i], r', done) and priority *max_prio; s' goes to row
 * (pos + B + i) % capacity, whose priority becomes 0 until the next step
 * completes it; state[i] <- s'.  state f32[B][198] out, actions i64[B][2],
 * reward i32[B], terminated/truncated u8[B]; r_obs f32[capacity][198],
 * r_action i64[capacity][2], r_reward/r_done/r_prio f32[capacity]; max_prio
 * f32 and pos i64 are device scalars, 0 <= *pos < capacity (the caller
 * advances pos by B).  B * 198 < 2^31. */
int narde_dqn_transition(narde_env *env, float *state, const int64_t *actions,
                         const int32_t *reward, const uint8_t *terminated,
                         const uint8_t *truncated, const uint64_t *legal, int32_t *misc,
                         float *off_seen, int shaping, float *r_obs, int64_t *r_action,
                         float *r_reward, float *r_done, float *r_prio, const float *max_prio,
                         const int64_t *pos, int64_t capacity, void *stream);

/* ---- DQN learner (gym-narde_amd/csrc/dqn_learner.hip; config 4) ---------
 * The non-GEMM chains of train_deepq_pytorch.py's replay() (:602-750) and
 * PrioritizedReplayBuffer (:279-342) at batch scale, fp32, each one kernel.
 * Device scalars (counter i64, beta f64, max_prio / epsilon f32) are read
 * and updated in place, so the calls can be captured in a graph. */

/* Prioritized sample of `batch` rows from p f32[n] (priority^alpha) and its
 * inclusive prefix sum cdf f32[n]: u_j = Philox4x32-10({*counter, j, 0, 7},
 * seed) (24-bit uniform, written to u if non-NULL), idx_j = first k with
 * cdf[k] > u_j * cdf[n-1] (clamped to n-1), w_j = (n p[idx_j] /
 * cdf[n-1])^-beta / max_j; then beta = min(1, beta + beta_inc), counter += 1.
 * scratch: unused (may be NULL; kept for the ABI).  Two
 * launches: a 64-ary search, one wave per sample, then the normalisation. */
int narde_per_sample(int device, const float *p, const float *cdf, int64_t n, int64_t batch,
                     uint64_t seed, int64_t *counter, double *beta, double beta_inc, int64_t *idx,
                     float *w, float *u, uint32_t *scratch, void *stream);

/* narde_per_sample's inputs from the priorities prio f32[n] (round 6): p =
 * prio^alpha (powf) and cdf = its inclusive prefix sum, in chunks of 1,024
 * rows (chunk f32[chunks] scratch, chunks >= ceil(n / 1024): each chunk's
 * total, then each chunk's rows scanned on top of the totals before it) --
 * the same order on every run; replaces `prio ** alpha` + torch.cumsum
 * (train_deepq_pytorch.py:279-342's probabilities).  prio, p, cdf 16-byte
 * aligned.  Two launches. */
int narde_per_prefix(int device, const float *prio, int64_t n, double alpha, float *p, float *cdf,
                     float *chunk, int64_t chunks, void *stream);

/* Minibatch rows idx i64[batch] of the replay ring (narde_dqn_transition's
 * layout): s = obs[idx], ns = obs[(idx + next_stride) % capacity] (f32
 * [batch][state_size]), a i64[batch][2], r/d f32[batch]. */
int narde_gather_batch(int device, const int64_t *idx, int64_t batch, int state_size,
                       const float *obs, int64_t next_stride, int64_t capacity,
                       const int64_t *action, const float *reward, const float *done, float *s,
                       float *ns, int64_t *a, float *r, float *d, void *stream);

/* out[i] = max_c base[i][c] + tab[rows[i]][c] over the 576 codes (the target
 * move-2 head's max with its one-hot column added on the fly). */
int narde_rowmax_addend(int device, const float *base, int64_t ld, const float *tab,
                        int64_t ld_tab, const int64_t *rows, int64_t n, float *out, void *stream);

/* The online network's two heads (DecomposedDQN.move1_head / move2_head,
 * train_deepq_pytorch.py:184-222) at the stored codes only -- what the loss
 * of train_deepq_pytorch.py:653-720 reads (q.gather(1, action)):
 *   q1[i] = f[i] . w1[a1] + b1[a1],
 *   q2[i] = (f[i] . w2[a2][:256] + b2[a2]) + w2[a2][256 + a1]
 * with (a1, a2) = a[i][0..1] (i64; codes clamped to 0..575), f f32[n][ldf]
 * (256 features), w1 f32[576][ldw1 >= 256], w2 f32[576][ldw2 >= 832] (the
 * move-2 head's weight: 256 feature columns, then 576 one-hot columns);
 * f, w1, w2 16-byte aligned, leading dimensions multiples of 4. */
int narde_dqn_heads_forward(int device, const float *f, int64_t ldf, const float *w1,
                            int64_t ldw1, const float *b1, const float *w2, int64_t ldw2,
                            const float *b2, const int64_t *a, int64_t n, float *q1, float *q2,
                            void *stream);

/* The backward of narde_dqn_heads_forward for dloss/dq1 = g1, dloss/dq2 = g2
 * (f32[n]): gf f32[n][256] (dense, 16-byte aligned), and the heads' whole
 * gradients gw1 f32[576][256], gb1 f32[576], gw2 f32[576][832], gb2
 * f32[576] (every element written; zero for codes no row holds).  Each sum
 * runs in a fixed order: deterministic. */
int narde_dqn_heads_backward(int device, const float *g1, const float *g2, const float *f,
                             int64_t ldf, const float *w1, int64_t ldw1, const float *w2,
                             int64_t ldw2, const int64_t *a, int64_t n, float *gf, float *gw1,
                             float *gb1, float *gw2, float *gb2, void *stream);

/* The backward of h = relu(x W^T + b) up to the weight GEMM (the learner's
 * feature layers, train_deepq_pytorch.py:184-201): g = gh * (h > 0) and db =
 * the column sums of g, for gh, h, g f32[n][cols] (cols <= 4096).
 * scratch: f32[ceil(n / 64) * cols] of device memory.  Deterministic. */
int narde_relu_bias_grad(int device, const float *gh, const float *h, int64_t n, int64_t cols,
                         float *g, float *db, float *scratch, void *stream);

/* The decomposed DQN loss (train_deepq_pytorch.py:653-720) on batch rows:
 * t = r + (1 - d) * gamma * m (m1/m2 the target heads' maxima), td =
 * clamp(|t1 - q1| + |t2 - q2|, 0, 100), *loss = mean(w (q1 - t1)^2) +
 * mean(w (q2 - t2)^2) (also to *loss_copy if non-NULL), g1/g2 = dloss/dq1,
 * dloss/dq2. */
int narde_dqn_loss(int device, const float *q1, const float *q2, const float *m1, const float *m2,
                   const float *r, const float *d, const float *w, int64_t batch, float gamma,
                   float *td, float *loss, float *loss_copy, float *g1, float *g2, void *stream);

/* prio[idx_j] = td_j + eps; *max_prio = max(*max_prio, max_j); then, if
 * epsilon is non-NULL, *epsilon *= eps_decay when *epsilon > eps_min; if
 * cursor is non-NULL, *cursor = (*cursor + cursor_add) % cursor_mod (the
 * replay ring's write cursor); if tag is non-NULL, *tag += 1 (the driver's
 * step tag) -- device scalars a step's bookkeeping advances. */
int narde_prio_update(int device, const int64_t *idx, const float *td, int64_t batch, float eps,
                      float *prio, float *max_prio, float *epsilon, float eps_min,
                      float eps_decay, int64_t *cursor, int64_t cursor_add, int64_t cursor_mod,
                      int64_t *tag, void *stream);

/* torch.nn.utils.clip_grad_norm_(max_norm) + one torch.optim.Adam step
 * (train_deepq_pytorch.py's optimizer) over n_tensors <= 8 fp32 parameter
 * tensors (params/grads/m/v: arrays of n_tensors device pointers, sizes in
 * elements).  *step (device i64) is advanced first; scratch: >= 1026 floats
 * of device memory, its last word zero before the first call (left zero). */
int narde_adam_clip(int device, int n_tensors, float *const *params, const float *const *grads,
                    float *const *m, float *const *v, const int64_t *sizes, int64_t *step, float lr,
                    float beta1, float beta2, float eps, float max_norm, float *scratch,
                    void *stream);

/* Round 6's one-launch forms of the learner's chains (the calls above stay
 * for the torch-restatement tests):
 * narde_per_sample_gather = narde_per_sample's search + narde_gather_batch's
 * rows in one launch, w UNNORMALISED ((n p / total)^-beta); beta and the
 * counter are NOT stepped (narde_dqn_loss_prio does both). */
int narde_per_sample_gather(int device, const float *p, const float *cdf, int64_t n, int64_t batch,
                            uint64_t seed, const int64_t *counter, const double *beta, int64_t *idx,
                            float *w, int state_size, const float *obs, int64_t next_stride,
                            int64_t capacity, const int64_t *action, const float *reward,
                            const float *done, float *s, float *ns, int64_t *a, float *r, float *d,
                            void *stream);

/* The target heads' maxima: m1[i] = max_c nq1[i][c], am1[i] = its argmax
 * (torch.max(dim): NaN wins, ties to the lowest code; am1 may be NULL),
 * m2[i] = max_c base[i][c] + tab[am1[i]][c] (narde_rowmax_addend's sum). */
int narde_target_max2(int device, const float *nq1, int64_t ld1, const float *base, int64_t ld,
                      const float *tab, int64_t ld_tab, int64_t n, float *m1, int64_t *am1,
                      float *m2, void *stream);

/* One block: w[j] /= max_j w[j] (narde_per_sample's normalisation, in place),
 * then narde_dqn_loss, then narde_prio_update on the same td, then beta =
 * min(1, beta + beta_inc) and *counter += 1 (narde_per_sample's steps). */
int narde_dqn_loss_prio(int device, const float *q1, const float *q2, const float *m1,
                        const float *m2, const float *r, const float *d, float *w, int64_t batch,
                        float gamma, float *td, float *loss, float *loss_copy, float *g1, float *g2,
                        const int64_t *idx, float eps, float *prio, float *max_prio, float *epsilon,
                        float eps_min, float eps_decay, int64_t *cursor, int64_t cursor_add,
                        int64_t cursor_mod, int64_t *tag, int64_t *counter, double *beta,
                        double beta_inc, void *stream);

/* A/B switch of narde_adam_clip's form: bit 1 = float4 passes where sizes
 * and pointers allow (default), else round 5's scalar passes.  Returns the
 * previous flags. */
int narde_learner_variant(int flags);

/* Stateless: Narde._violates_block_rule on n perspective boards i8[n][24]. */
int narde_violates_block_rule(int device, const int8_t *boards, int64_t n, uint8_t *out,
                              void *stream);

/* ---- host-memory entry points (scalar facade; synchronous) ----------------
 * Same semantics as above on n <= 4096 envs given explicitly in HOST memory.
 * The handle's own B envs are untouched.  Return NARDE_EINVAL for an invalid
 * position (see narde_set_state). */
int narde_host_legal_moves(narde_env *env, int64_t n, const int8_t *board, const uint8_t *off,
                           const uint8_t *first_turn, const int8_t *player, const uint8_t *dice4,
                           int16_t *count, int8_t *moves);
int narde_host_step(narde_env *env, int64_t n, int8_t *board, uint8_t *off, uint8_t *first_turn,
                    int8_t *player, const uint8_t *dice2, const int16_t *actions, int32_t *obs,
                    int32_t *reward, uint8_t *terminated);
int narde_host_apply_moves(narde_env *env, int64_t n, int8_t *board, uint8_t *off,
                           uint8_t *first_turn, const int8_t *player, const int8_t *moves);
int narde_host_violates_block_rule(narde_env *env, int64_t n, const int8_t *boards, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif /* NARDE_H */
