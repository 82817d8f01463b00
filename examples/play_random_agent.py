#!/usr/bin/env python3
"""Working counterpart of the reference's examples/play_random_agent.py
(configs[0]: one env, random agent).  The reference file is stale -- it
imports WHITE/BLACK/COLORS/TOKEN that narde.py does not define (:6), uses
the old gym and a 4-tuple step (:43) -- so this keeps its structure (one
RandomAgent per colour, play until done, report the winner) on the
gymnasium 5-tuple API of the drop-in package.  The agent samples the action
space as the reference's does (:20-21), so most actions are illegal and are
ignored by the env exactly as in the reference (narde_env.py:56-93); pass
--legal to sample uniformly over legal move codes instead.

  python examples/play_random_agent.py [--games N] [--seed S] [--legal] [--render]
"""
import argparse
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-narde_amd"))

import gym_narde  # noqa: E402

WHITE, BLACK = 1, -1
COLORS = {WHITE: "White", BLACK: "Black"}


class RandomAgent:
    def __init__(self, color, legal, rng):
        self.color, self.legal, self.rng = color, legal, rng
        self.name = f"AgentExample({COLORS[color]})"

    def choose_best_action(self, env):
        if not self.legal:
            return (self.rng.randrange(576), self.rng.randrange(576))
        # the dice step() will roll, peeked from numpy's global RNG
        st = np.random.get_state()
        dice = [np.random.randint(1, 7), np.random.randint(1, 7)]
        np.random.set_state(st)
        moves = env.unwrapped.game.get_valid_moves(dice, env.unwrapped.current_player)
        if not moves:
            return (0, 0)
        f, t = self.rng.choice(moves)
        return (f * 24 + (0 if t == "off" else t), 0)


def make_plays(games=1, seed=0, legal=False, render=False):
    env = gym_narde.make("gym_narde:narde-v0")
    rng = random.Random(seed)
    np.random.seed(seed)
    wins = {WHITE: 0, BLACK: 0}
    agents = {c: RandomAgent(c, legal, rng) for c in (WHITE, BLACK)}
    lengths = []
    for g in range(games):
        env.reset()
        t = time.time()
        for i in range(1, 100000):
            agent = agents[env.unwrapped.current_player]
            _, reward, terminated, truncated, _ = env.step(agent.choose_best_action(env))
            if render:
                env.unwrapped.render()
            if terminated or truncated:
                winner = env.unwrapped.current_player
                if terminated:
                    wins[winner] += 1
                lengths.append(i)
                tot = max(1, wins[WHITE] + wins[BLACK])
                print(f"Game={g + 1} | {'Winner=' + COLORS[winner] if terminated else 'truncated'} "
                      f"after {i:<4} plays (reward {reward}) || Wins: White={wins[WHITE]} "
                      f"({wins[WHITE] / tot * 100:.1f}%) Black={wins[BLACK]} "
                      f"({wins[BLACK] / tot * 100:.1f}%) | Duration={time.time() - t:.3f} sec")
                break
    env.close()
    return wins, lengths


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--legal", action="store_true")
    ap.add_argument("--render", action="store_true")
    a = ap.parse_args()
    make_plays(a.games, a.seed, a.legal, a.render)
