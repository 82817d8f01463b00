"""Profiling target for the config-4 DQN driver (rocprofv3 --kernel-trace):
B envs, graph-captured step, N replays.  argv: [B] [steps] [eager];
$NARDE_GATHERED=0 takes the dense online heads in the learner,
$NARDE_FUSED_FEATURES=0 autograd's feature-layer backward, $NARDE_ONE_LAUNCH=0
round 5's learner (no one-launch chains, scalar clip + Adam)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-narde_amd"))
import torch  # noqa: E402

from gym_narde.dqn import BatchedDQNDriver, use_tuned_gemms  # noqa: E402
from gym_narde.vector import VecNardeEnv  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
eager = len(sys.argv) > 3 and sys.argv[3] == "eager"
if os.environ.get("NARDE_TUNED_GEMMS", "1") == "1":
    use_tuned_gemms()
env = VecNardeEnv(B, device="cuda:0", seed=1)
drv = BatchedDQNDriver(env, train_batch=4096, capacity=max(1 << 20, 4 * B),
                       gathered_heads=os.environ.get("NARDE_GATHERED", "1") == "1",
                       fused_features=os.environ.get("NARDE_FUSED_FEATURES", "1") == "1",
                       one_launch_chains=os.environ.get("NARDE_ONE_LAUNCH", "1") == "1")
if os.environ.get("NARDE_ONE_LAUNCH", "1") != "1":  # round 5's learner forms throughout
    from gym_narde.dqn import learner_variant

    learner_variant(0)
if not eager:
    drv.capture_graph(warmup=2)
for _ in range(3):
    drv.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    drv.step()
torch.cuda.synchronize()
print(f"{'eager' if eager else 'graph'} B={B}: {(time.perf_counter() - t0) / N * 1e3:.4f} ms/step")
