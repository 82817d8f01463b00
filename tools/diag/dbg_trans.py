import sys, os
sys.path.insert(0, "gym-narde_amd"); sys.path.insert(0, "tests")
import torch
import test_gpu_dqn as T
# re-run the test body but print the mismatches
from gym_narde.dqn import BatchedDQNDriver
from gym_narde.vector import VecNardeEnv
n = 4096
env = VecNardeEnv(n, device="cuda:0", seed=23)
env.selfplay(260)
drv = BatchedDQNDriver(env, capacity=3 * n, train_batch=1024, shaping=True)
drv.state = drv._observe()
g = torch.Generator(device="cuda:0").manual_seed(4)
off0 = torch.randint(0, 16, (n, 2), device="cuda:0", generator=g).float()
state0 = drv.state.clone()
rp = drv.replay
a = drv.act(drv.state)
_, reward, term, trunc, _ = env.step(a.to(torch.int16))
reward, term, trunc = reward.clone(), term.clone(), trunc.clone()
def run(fn):
    drv.state.copy_(state0); drv.off_seen.copy_(off0)
    for t in (rp.obs, rp.next_obs, rp.action, rp.reward, rp.done, rp.prio): t.zero_()
    rp.pos_t.fill_(0)
    fn()
    return rp.reward[:n].clone(), drv.off_seen.clone()
f, fo = run(lambda: drv._transition_fused(a, reward, term, trunc))
r, ro = run(lambda: drv._transition_torch(drv.state, a, reward, term, trunc))
bad = (f != r).nonzero().flatten()
print("mismatch", bad.numel(), "of", n)
nx = drv._observe()
for i in bad[:10].tolist():
    print(i, float(f[i]), float(r[i]), "rew", int(reward[i]), "off0", off0[i].tolist(), "obs off", float(nx[i,97]*15), float(nx[i,195]*15), "pl", float(nx[i,196]), "done", int(term[i]|trunc[i]))
