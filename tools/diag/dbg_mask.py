"""DIAGNOSTIC: envs where the driver's move-1 code (legal per k_mask576) is
ignored by the oracle's NardeEnv.step with the peeked dice."""
import os
import sys

sys.path.insert(0, "gym-narde_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
import numpy as np
import torch

import oracle as O
from gym_narde.dqn import BatchedDQNDriver, expand_mask
from gym_narde.vector import VecNardeEnv

env = VecNardeEnv(2048, device="cuda:0", seed=17)
drv = BatchedDQNDriver(env, capacity=1 << 16, train_batch=1024)
env.selfplay(40)
drv.state = drv._observe()
a = drv.act(drv.state).cpu().numpy().astype(np.int16)
st = {k: v.cpu().numpy() for k, v in env.get_state().items()}
dice = env.dice().cpu().numpy()
ref = O.step(st["board"], st["off"], st["first_turn"], st["player"], dice, a)
bad = np.nonzero(~((ref["count2"] >= 0) | (ref["count1"] < 2)))[0]
print("bad", len(bad), "t", env.ply)
m1 = expand_mask(env.legal_mask()).cpu().numpy()
lm = env.legal_moves()
for i in bad[:5]:
    print(i, "board", st["board"][i].tolist(), "off", st["off"][i].tolist(), "ft", st["first_turn"][i].tolist(),
          "player", int(st["player"][i]), "dice", dice[i].tolist(), "a", a[i].tolist(),
          "mask codes", np.nonzero(m1[i])[0][:20].tolist(), "count1", int(ref["count1"][i]))
