#!/usr/bin/env python3
"""Capture FULL4 golden vectors by composing the reference's own primitives
(THIS container only; test infrastructure, not product code).

FULL4 is the build's rules mode for whole turns with 4-move doubles and the
max-dice-used rule (spec README.md:27-30, web
turn manager my_game/narde_game_manager.py:154-157,980-1011).  The reference
env never plays it (NardeEnv.step stops after 2 checker moves), so there is
no reference arithmetic for a whole turn.  What IS pinned is every single
checker move: each sub-move comes from the reference's
`Narde.get_valid_moves([die], player)` (gym_narde/envs/narde.py:58-92, one
die => its block filter :139-184 on the post-move board) and is applied with
`Narde.execute_rotated_move` (narde.py:36-56), on deep copies of the
reference's own Narde objects.  The composition rule is the build's
(DESIGN.md section 10):

  dice (a, b): D = [a]*4 if a == b else [max(a,b), min(a,b)]
  H = 2 if the mover's first_turn and a == b in {3, 4, 6} else 1
      (narde.py:94-106's condition), else 1: at most H sub-moves from 23
  options(node) = for each distinct remaining die v (descending), for each
      (p, q) of get_valid_moves([v]) (ascending p): (v, p) unless p == 23
      and H head moves were already made
  M = max number of sub-moves over all sequences (max dice used)
  C_k = options whose child still reaches M sub-moves in total; for two
      different dice with M == 1 only the higher die if it has an option
  policy: sub-move k takes entry mulhi(w_k, |C_k|) of C_k
  then NardeEnv._check_game_ended (narde_env.py:134-141) as in REF2.

Writes tests/golden/full4.npz: per case the pre-state, dice, pick words, M,
the C_k sets as per-die source masks, the sub-moves played (die, from) and
the post-turn state/reward/done.
"""
import argparse
import copy
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture_golden as CG  # noqa: E402


def mulhi(w, n):
    return (int(w) * int(n)) >> 32


class Full4:
    """The FULL4 turn composed from reference primitives (memoised)."""

    def __init__(self, narde_mod):
        self.Narde = narde_mod.Narde
        self.memo = {}

    @staticmethod
    def key(game, R, h):
        return (game.board.tobytes(), int(game.borne_off_white), int(game.borne_off_black),
                tuple(R), h)

    def options(self, game, R, player, h, H):
        out = []
        for v in sorted(set(R), reverse=True):
            for (f, t) in game.get_valid_moves([v], player):
                if f == 23 and h >= H:
                    continue
                out.append((v, f, t))
        return out

    def child(self, game, R, player, h, opt):
        v, f, t = opt
        g2 = copy.deepcopy(game)
        g2.execute_rotated_move((f, t), player)
        R2 = list(R)
        R2.remove(v)
        return g2, tuple(R2), h + (1 if f == 23 else 0)

    def depth(self, game, R, player, h, H):
        if not R:
            return 0
        k = self.key(game, R, h) + (player, H)
        if k in self.memo:
            return self.memo[k]
        best = 0
        for opt in self.options(game, R, player, h, H):
            g2, R2, h2 = self.child(game, R, player, h, opt)
            best = max(best, 1 + self.depth(g2, R2, player, h2, H))
            if best == len(R):
                break
        self.memo[k] = best
        return best

    def turn(self, game, dice, player, words):
        """Play one FULL4 turn in place; returns (M, cmasks[4][2], played[4][2])."""
        a, b = dice
        R = (a,) * 4 if a == b else (max(a, b), min(a, b))
        ft = game.first_turn_white if player == 1 else game.first_turn_black
        H = 2 if (ft and a == b and a in (3, 4, 6)) else 1
        h = 0
        M = self.depth(game, R, player, h, H)
        cm = np.zeros((4, 2), np.uint32)
        played = np.full((4, 2), -1, np.int8)
        for k in range(M):
            need = M - k - 1
            C = []
            for opt in self.options(game, R, player, h, H):
                g2, R2, h2 = self.child(game, R, player, h, opt)
                if self.depth(g2, R2, player, h2, H) == need:
                    C.append(opt)
            if k == 0 and M == 1 and a != b and any(o[0] == max(a, b) for o in C):
                C = [o for o in C if o[0] == max(a, b)]
            assert C, "C_k empty below M"
            for (v, f, _) in C:
                col = 0 if (v == max(a, b)) else 1
                cm[k, col] |= np.uint32(1 << f)
            opt = C[mulhi(words[k], len(C))]
            played[k] = (opt[1], opt[0])
            game.execute_rotated_move((opt[1], opt[2]), player)
            R2 = list(R)
            R2.remove(opt[0])
            R = tuple(R2)
            h += 1 if opt[1] == 23 else 0
        return M, cm, played


def end_check(game, player):
    """narde_env.py:134-141."""
    if player == 1 and game.borne_off_white == 15:
        return True, (1 if game.borne_off_black > 0 else 2)
    if player == -1 and game.borne_off_black == 15:
        return True, (1 if game.borne_off_white > 0 else 2)
    return False, 0


def full4_selfplay_states(narde_mod, f4, n, rng):
    """Reachable pre-turn states of FULL4 random self-play."""
    states = []
    game = narde_mod.Narde()
    player = rng.choice([1, -1])
    steps = 0
    while len(states) < n:
        states.append(CG.snapshot(game) + (player,))
        dice = (rng.randint(1, 6), rng.randint(1, 6))
        words = [rng.getrandbits(32) for _ in range(4)]
        f4.turn(game, dice, player, words)
        done, _ = end_check(game, player)
        steps += 1
        if done or steps >= 1000:
            game = narde_mod.Narde()
            player = rng.choice([1, -1])
            steps = 0
            f4.memo.clear()
        else:
            player = -player
        if len(f4.memo) > 200000:
            f4.memo.clear()
    return states


def capture(narde_mod, NardeEnv, scale, rng):
    f4 = Full4(narde_mod)
    states = []
    states += full4_selfplay_states(narde_mod, f4, int(9000 * scale), rng)
    states += CG.selfplay_states(NardeEnv, int(3000 * scale), 7)
    states += [CG.synthetic_state(rng) for _ in range(int(3000 * scale))]
    states += [CG.endgame_state(rng) for _ in range(int(1500 * scale))]
    rolls = []
    for s in states:
        r = rng.random()
        if r < 0.35:  # oversample doubles (the FULL4-specific path)
            d = rng.randint(1, 6)
            rolls.append((d, d))
        else:
            rolls.append((rng.randint(1, 6), rng.randint(1, 6)))
    # every ordered roll from the start position, both movers, first turn
    start = narde_mod.Narde()
    for pl in (1, -1):
        for a in range(1, 7):
            for b in range(1, 7):
                states.append(CG.snapshot(start) + (pl,))
                rolls.append((a, b))
    N = len(states)
    out = dict(
        board=np.zeros((N, 24), np.int8), off=np.zeros((N, 2), np.uint8),
        ft=np.zeros((N, 2), np.uint8), player=np.zeros(N, np.int8),
        dice=np.zeros((N, 2), np.uint8), words=np.zeros((N, 4), np.uint32),
        max_dice=np.zeros(N, np.int8), cmask=np.zeros((N, 4, 2), np.uint32),
        played=np.zeros((N, 4, 2), np.int8), board_after=np.zeros((N, 24), np.int8),
        off_after=np.zeros((N, 2), np.uint8), ft_after=np.zeros((N, 2), np.uint8),
        reward=np.zeros(N, np.int8), done=np.zeros(N, np.uint8))
    game = narde_mod.Narde()
    for i, (st, dice) in enumerate(zip(states, rolls)):
        board, offw, offb, ftw, ftb, player = st
        CG.set_game(game, board, offw, offb, ftw, ftb)
        words = [rng.getrandbits(32) for _ in range(4)]
        out["board"][i] = board
        out["off"][i] = (offw, offb)
        out["ft"][i] = (ftw, ftb)
        out["player"][i] = player
        out["dice"][i] = dice
        out["words"][i] = words
        M, cm, played = f4.turn(game, dice, player, words)
        done, rew = end_check(game, player)
        out["max_dice"][i] = M
        out["cmask"][i] = cm
        out["played"][i] = played
        b2, ow, ob, fw, fb = CG.snapshot(game)
        out["board_after"][i] = b2
        out["off_after"][i] = (ow, ob)
        out["ft_after"][i] = (fw, fb)
        out["reward"][i] = rew
        out["done"][i] = done
        if len(f4.memo) > 200000:
            f4.memo.clear()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    narde_mod, NardeEnv = CG.load_reference()
    rng = random.Random(20251015)
    d = capture(narde_mod, NardeEnv, args.scale, rng)
    p = os.path.join(args.out, "full4.npz")
    np.savez_compressed(p, **d)
    M = d["max_dice"]
    dbl = d["dice"][:, 0] == d["dice"][:, 1]
    print(f"wrote {p} ({os.path.getsize(p) / 1e6:.2f} MB): {len(M)} turns, "
          f"doubles {int(dbl.sum())}, M hist {np.bincount(M, minlength=5).tolist()}, "
          f"done {int(d['done'].sum())}")


if __name__ == "__main__":
    main()
