"""Transition codes from the kernels (craft_transition, craft_step_ex) drive the
language teacher exactly like the reference's state pairs do."""
import numpy as np
import pytest
import torch

from psketch_amd import CraftSim
from tests.test_oracle_golden import _language_codes_from_oracle

pytestmark = pytest.mark.gpu


def _sim_from_fixture(fx):
    pool, spec = fx["pool"], fx["spec"]
    B = len(spec)
    sim = CraftSim("craft_medium_12x12", n_envs=B, device=0, pool_capacity=len(pool))
    sim.load_pool(pool)
    sp = np.stack([spec[:, 0], spec[:, 1], spec[:, 2], spec[:, 3], np.zeros(B, np.int32)], 1)
    ag = np.stack([spec[:, 1], spec[:, 2], spec[:, 3], np.full(B, 40)], 1)
    sim.set_state(sp, ag)
    return sim


def test_transition_codes_and_descriptions(golden, gpu, oracle_mod):
    from psketch_amd.language import WORDS, PrimitiveLanguageTeacher
    fx = golden("language.npz")
    want_codes = _language_codes_from_oracle(oracle_mod, fx)
    actions = fx["actions"]
    T, B = actions.shape
    sim = _sim_from_fixture(fx)
    teacher = PrimitiveLanguageTeacher(np.random.RandomState(5))
    codes = torch.empty(B, dtype=torch.int8, device=gpu)
    for t in range(T):
        a = torch.as_tensor(actions[t].astype(np.int32), device=gpu)
        sim.transition(a, codes=codes)
        got = codes.cpu().numpy()
        assert np.array_equal(got, want_codes[t]), t
        words = teacher.describe_batch(a, codes)
        assert [WORDS.index(w) for w in words] == fx["desc_tick"][t].tolist(), t
    sim.check()


def test_step_ex_codes_match_transition_codes(golden, gpu):
    """The rollout tick reports the same codes for envs that step, -1 for the rest."""
    fx = golden("language.npz")
    actions = fx["actions"]
    B = actions.shape[1]
    a_sim, b_sim = _sim_from_fixture(fx), _sim_from_fixture(fx)
    ca = torch.empty(B, dtype=torch.int8, device=gpu)
    cb = torch.empty(B, dtype=torch.int8, device=gpu)
    done = torch.empty(B, dtype=torch.uint8, device=gpu)
    for t in range(10):
        act = torch.as_tensor(actions[t].astype(np.int32), device=gpu)
        a_sim.step(act, tick=t, autoreset=False, done=done, transition_code=ca)
        b_sim.transition(act, codes=cb)
        d = done.cpu().numpy().astype(bool)
        got, want = ca.cpu().numpy(), cb.cpu().numpy()
        assert (got[d] == -1).all()
        if t == 0:       # before any env froze, every stepping env matches the pure transition
            assert np.array_equal(got[~d], want[~d])
    a_sim.check()
    b_sim.check()
