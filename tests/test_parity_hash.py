"""The full-size parity hash, pinned on the CPU (no GPU).

`zo_run_hashes` (the bulk OpenMP oracle run the full-size GPU tests compare against) must
equal stepping `OracleEnv` one env at a time with the bench's discrete action stream and
hashing each step with `numpy_step_hash` (the host twin of the GPU `StepHasher`).
"""
import numpy as np
import pytest

from libzombsole_amd import _abi
from libzombsole_amd.actions import DISCRETE_TRIPLES, discrete_action_id
from oracle.oracle import OracleEnv, run_hashes
from parity_hash import numpy_step_hash

CASES = {
    "c3_multi_int64": (lambda n: _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"],
                                                       initial_zombies=10, max_episode_steps=14), 7),
    "c5_multi_int16": (lambda n: _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"],
                                                       initial_zombies=20, obs_dtype=_abi.DTYPE_I16,
                                                       max_episode_steps=1000), 7),
    "single_world_int32": (lambda n: _abi.single_env_config(n, "extermination", [], "bridge", 0,
                                                            initial_zombies=10, observation_scope="world",
                                                            observation_position_encoding="simple",
                                                            max_episode_steps=9), 6),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("twice", [0, 3])
def test_run_hashes_equal_stepwise_oracle(case, twice):
    mk, nd = CASES[case]
    n, steps, seed0 = 5, 30, 77
    bulk = run_hashes(mk(1), seed0, n, steps, nd, threads=2, reset_twice_mod=twice)
    assert bulk.shape == (n, steps + 1)
    for i in range(n):
        seed = seed0 + i
        o = OracleEnv(mk(1))
        o.seed(seed)
        obs = o.reset()
        if twice and i % twice == 1:
            obs = o.reset()
        row = [numpy_step_hash(obs)]
        need = False
        for t in range(1, steps + 1):
            if need:
                row.append(numpy_step_hash(o.reset(), reset=True))
                need = False
                continue
            acts = np.stack([DISCRETE_TRIPLES[discrete_action_id(seed, t, a, nd)] for a in range(o.A)])
            obs, r, d, tr, lb = o.step(acts)
            multi = o.builder.cfg.reward_mode == _abi.REWARD_MULTI
            row.append(numpy_step_hash(obs, r[:o.A] if multi else r[:1], lb if multi else None, d, tr))
            need = d or tr
        assert np.array_equal(np.array(row, dtype=np.uint64), bulk[i]), (case, i)
