"""f-3: the reference's evaluate_model.py loop, run
through the drop-in facade, replays the games the same loop played on the
imported reference (tests/golden/callers.npz from tools/capture_callers.py):
every agent roll, action, observation, reward, end and mover.  Exercises the
`env.unwrapped.game` shim (get_perspective_board, get_valid_moves),
`current_player`, the numpy global RNG draw pattern and TimeLimit through
gym_narde.make."""
import numpy as np
import pytest
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_evaluate_loop_replays_reference_games():
    import callers
    from gym_narde import make

    d = golden("callers.npz")
    games, np_seed, py_seed, mseed = (int(x) for x in d["meta"])
    model = callers.build_model(mseed)
    assert abs(callers.fingerprint(model) - float(d["fingerprint"])) < 1e-9  # same seeded weights
    rec = callers.play(lambda: make("gym_narde:narde-v0"), model, games, np_seed, py_seed)
    assert len(rec["action"]) == len(d["action"])
    for k in ("game", "ai_color", "dice", "action", "obs", "reward", "done", "player"):
        assert np.array_equal(rec[k], d[k]), k
    assert d["done"].sum() == games
