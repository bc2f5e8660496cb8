"""Parity of the timed path at the sizes it is timed (BASELINE.json configs C2..C5).

`bench.py` replays the step as a hipGraph (`zs_step_graph`: on-device discrete policy +
reset work + tick + observations) over 4 096 .. 65 536 envs.  At those sizes the persistent
observation kernels walk many envs per wave (C3: 32 per wave, with the next env prefetched
into registers), `k_reset` grid-strides over the pending list / mask, and the graph replays
both pending-list parities.  Every env and every step is compared with the oracle
(`oracle/zs_oracle.c`, the restatement of `zombsole/core.py:72-78` World.step and its env
glue) through 64-bit per-env step hashes of obs, listed rewards, done/truncated and the
autoreset flag (`tests/parity_hash.py`; the hash itself is pinned on the CPU by
`tests/test_parity_hash.py`).  At the end, the full canonical state of envs at every
wave-stride residue is compared with an oracle replay.
"""
import numpy as np
import pytest

from libzombsole_amd import _abi
from libzombsole_amd.actions import DISCRETE_TRIPLES, discrete_action_id

pytestmark = pytest.mark.gpu


def c3(n, max_steps=1000):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1"], initial_zombies=10,
                                 minimum_zombies=0, max_episode_steps=max_steps)


def c4(n, max_steps=1000):
    return _abi.multi_env_config(n, "safehouse", [], "city128", ["0", "1", "2", "3"], initial_zombies=50,
                                 minimum_zombies=50, max_episode_steps=max_steps)


def c5(n, max_steps=1000):
    return _abi.multi_env_config(n, "extermination", [], "bridge64", ["0", "1", "2", "3"], initial_zombies=20,
                                 minimum_zombies=0, max_episode_steps=max_steps, obs_dtype=_abi.DTYPE_I16)


def spot_envs(n):
    """Envs at every wave-stride position the persistent kernels use (256 CUs x 1..4 workgroups x
    4 waves: strides 1024 .. 4096), plus both ends."""
    s = {0, 1, 63, 64, n - 1, n - 2}
    for stride in (1024, 2048, 4096):
        for base in (0, 5, stride - 1):
            for k in (1, 2, 7, 15):
                e = base + k * stride
                if e < n:
                    s.add(e)
    return sorted(e for e in s if 0 <= e < n)


def oracle_state(make_builder, seed, steps, nd, twice):
    from oracle.oracle import OracleEnv
    o = OracleEnv(make_builder(1))
    o.seed(seed)
    o.reset()
    if twice:
        o.reset()
    need = False
    for t in range(1, steps + 1):
        if need:
            o.reset()
            need = False
            continue
        acts = np.stack([DISCRETE_TRIPLES[discrete_action_id(seed, t, a, nd)] for a in range(o.A)])
        _, _, d, tr, _ = o.step(acts)
        need = d or tr
    return o.state()


def run_full(make_builder, n, steps, nd=7, seed0=0, graph=True, twice=0, min_resets=1, launch=None, after=None,
             graph_steps=1):
    import torch

    from libzombsole_amd.engine import Engine
    from oracle.oracle import run_hashes
    from parity_hash import StepHasher

    eng = Engine(make_builder(n).set_launch(launch))
    eng.seed([seed0 + i for i in range(n)])
    eng.reset()
    if twice:  # a masked reset of every twice-th env (zs_reset mask mode over the whole grid)
        mask = (torch.arange(n, device=eng.device) % twice == 1).to(torch.uint8)
        eng.reset(mask)
    hs = StepHasher(eng)
    got = np.zeros((n, steps + 1), dtype=np.uint64)
    got[:, 0] = hs.obs_hash().cpu().numpy().view(np.uint64)
    resets = 0
    for t in range(1, steps + 1):
        if graph_steps > 1:  # zs_step_graph_n: the outputs of every graph_steps-th step are seen
            if t % graph_steps:
                continue
            eng.step_graph(t - graph_steps + 1, nd, steps=graph_steps)
        elif graph:
            eng.step_graph(t, nd)
        else:
            eng.gen_actions(t, nd)
            eng.step()
        got[:, t] = hs.step_hash().cpu().numpy().view(np.uint64)
        resets += int(eng.was_reset.sum().item())
    exp = run_hashes(make_builder(1), seed0, n, steps, nd, threads=0, reset_twice_mod=twice)
    if graph_steps > 1:
        seen = [0] + list(range(graph_steps, steps + 1, graph_steps))
        got, exp = got[:, seen], exp[:, seen]
    bad = np.argwhere(got != exp)
    assert bad.size == 0, "%d of %d env-steps differ; first (env, step): %s" % (
        len(bad), got.size, bad[:12].tolist())
    assert resets >= min_resets, ("too few autoresets to cover the reset path", resets)
    kinds = [o[2] for o in eng.builder.map.obstacles]
    for e in spot_envs(n):
        exp_state = oracle_state(make_builder, seed0 + e, steps, nd, twice and e % twice == 1)
        assert eng.get_state(e).canonical(kinds) == exp_state, ("state", e)
    if after:
        after(eng)
    eng.close()
    return resets


def test_c3_65536_graph():
    """The headline (BASELINE metric, C3 at N=1): 65 536 envs, k_tick, the side-stream reset, k_obs_ring."""
    run_full(c3, 65536, 40)


def _expect_launch(step_kernel, obs_kernel):
    def check(eng):
        d = eng.describe()
        assert (d["step_kernel"], d["obs_kernel"]) == (step_kernel, obs_kernel), d
    return check


@pytest.mark.parametrize("n", [12288, 16384, 32768])
def test_c3_strong_scaling_shards(n):
    """The C3 shards of a strong-scaling run at N = 4 and 2 (16 384, 32 768 envs per GPU) and the ring's
    lower bound (12 288: 48 envs per CU): the step launch with the reset work inside it over up to two
    resident rounds, and k_obs_ring."""
    run_full(c3, n, 40, seed0=3 * n, after=_expect_launch("k_step", "k_obs_ring"))


def test_c5_16384_int16_fused_two_rounds():
    """C5 at 16 384 envs: the fused step launch over two resident rounds, int16 ring."""
    run_full(c5, 16384, 40, seed0=7, after=_expect_launch("k_step", "k_obs_ring"))


def test_c3_65536_truncation_waves():
    """TimeLimit 16: every env truncates at steps 16 and 33 -> 65 536-env autoreset waves (k_reset list
    mode grid-striding far past 2 048 pending envs), plus a masked reset of 21 846 envs before step 1."""
    r = run_full(lambda n: c3(n, max_steps=16), 65536, 40, twice=3, min_resets=2 * 65536)
    assert r >= 2 * 65536


def test_c2_4096_graph():
    run_full(c3, 4096, 60, seed0=4242)


def test_c2_4096_one_obs_workgroup_per_cu():
    """obs_wgs = 1: the persistent observation kernel (k_obs_patch, the int64 ring off) at 1 workgroup
    per CU walks several envs per wave at 4 096."""
    run_full(c3, 4096, 40, seed0=99, launch={"obs_wgs": 1, "obs_lds": 1, "obs_ring": -1})


def test_c2_4096_ring():
    """k_obs_ring (encoder / writer waves through an LDS ring; C3's default) at 4 096 envs: 16 envs per
    workgroup, every ring slot reused."""
    run_full(c3, 4096, 40, seed0=1234, launch={"obs_lds": 1, "obs_ring": 1})


def test_c5_65536_int16_ring():
    """k_obs_ring on C5's int16 blocks of 4 agents (10 584-B envs, two 16-B phases)."""
    run_full(c5, 65536, 12, min_resets=0, launch={"obs_ring": 1})


def test_c5_odd_int16_ring_pairs():
    """k_obs_ring's two-env units (C5's int16 envs end on 16-B boundaries in pairs) over an odd env
    count: one workgroup's last unit holds a single env."""
    run_full(c5, 4097, 24, seed0=555, min_resets=0, launch={"obs_ring": 1})


def test_c2_4096_ring_select_encoders():
    """k_obs_ring with its select-chain encoders instead of the padded-table ones (its fallback)."""
    run_full(c3, 4096, 40, seed0=4321, launch={"obs_lds": 1, "obs_ring": 1, "obs_ring_patch": -1})


def test_c2_4096_one_obs_workgroup_per_cu_cells():
    """The same walk through k_obs_pipe's per-cell stores."""
    run_full(c3, 4096, 40, seed0=7, launch={"obs_wgs": 1, "obs_lds": -1})


def test_c5_65536_int16_graph():
    """C5's engine side: 4 agents + 20 zombies, int16 observations (the gathered form); k_obs_ring
    with the padded-table encoders; episodes ending (extermination) and their autoresets at full size."""
    run_full(c5, 65536, 40, min_resets=1)


def test_c5_8192_int16_shard_graph():
    """C5's per-GPU shard at N=8 (8 192 envs, int16, rank 5's env range): the fused step launch."""
    run_full(c5, 8192, 48, seed0=5 * 8192, min_resets=1)


def test_c5_65536_int16_patch():
    """C5 through k_obs_patch (the padded-table encoder with per-wave flushes)."""
    run_full(c5, 65536, 32, seed0=77, min_resets=0, launch={"obs_ring": -1})


def test_c5_65536_int16_truncation_waves():
    """C5 with TimeLimit 12: 65 536-env autoreset waves at steps 12 and 25 (int16 reset observations)
    and a masked reset of every 4th env before step 1."""
    run_full(lambda n: c5(n, max_steps=12), 65536, 30, twice=4, min_resets=2 * 65536)


def test_c4_16384_graph():
    """C4: city128 safehouse, 4 agents + 50 zombies (minimum 50): k_obs_pbring (window-only encoders and
    writer waves), k_respawn after zombie deaths and safehouse / all-dead autoresets, at full size."""
    def respawned(eng):
        assert eng.describe()["obs_kernel"] == "k_obs_pbring"
        # every zombie death leaves a deficit under minimum 50 that the same step's respawn fills
        zd = sum(eng.get_state(e).zombie_deaths for e in range(0, 16384, 97))
        assert zd > 0, "no zombie died in the sampled envs: k_respawn untested"
        assert eng.describe()["respawn"] == "k_respawn"
    run_full(c4, 16384, 80, min_resets=1, after=respawned)


def test_c4_4096_gather():
    """C4's map through k_obs_gather (the big-map kernel without writer waves)."""
    def gather(eng):
        assert eng.describe()["obs_kernel"] == "k_obs_gather"
    run_full(c4, 4096, 40, min_resets=0, launch={"obs_ring": -1}, after=gather)


def test_c3_8192_shard_eager():
    """The N=8 shard size (8 192 envs per GPU) through per-kernel launches (zs_step), env range of rank 3."""
    run_full(c3, 8192, 40, seed0=3 * 8192, graph=False)


def test_c3_8192_shard_graph():
    """The N=8 headline's per-GPU run as bench.py times it: graph replay, the policy and the reset work
    inside the fused step launch (k_step), the lanes' parallel execution; env range of rank 6."""
    def fused(eng):
        desc = eng.describe()
        assert desc["step_kernel"] == "k_step" and desc["par_exec"] == 1, desc
    run_full(c3, 8192, 60, seed0=6 * 8192, after=fused)


def test_c3_8192_shard_multistep_graph():
    """Eight steps per graph launch (zs_step_graph_n) at the shard size, TimeLimit 15 so that autoresets
    fall inside a launch: the outputs of every eighth step and the final states against the oracle."""
    r = run_full(lambda n: c3(n, max_steps=15), 8192, 48, seed0=4 * 8192, graph_steps=8, min_resets=1)
    assert r >= 1


def test_c2_4096_multistep_graph_odd():
    """Three steps per graph launch: an odd count, so consecutive launches start on alternate pending-list
    parities (two graphs per buffer set)."""
    run_full(lambda n: c3(n, max_steps=10), 4096, 45, seed0=7 * 4096, graph_steps=3, min_resets=1)


def test_c3_8192_shard_serial_exec():
    """The same shard with the leader's serial execution (zs_launch.par_exec = -1)."""
    run_full(c3, 8192, 40, seed0=2 * 8192, launch={"par_exec": -1})


def _side_reset(eng):
    desc = eng.describe()
    assert desc["step_kernel"] == "k_tick" and desc["reset_side_stream"] == 1, desc


def test_c3_65536_multistep_graph_side_reset():
    """Five steps per graph launch at the headline size (zs_step_graph_n), the reset work on the side
    stream forked and joined inside every captured step; TimeLimit 14, so 65 536-env autoreset waves fall
    inside launches (their reset work at steps 15 and 30, the last steps of launches, whose outputs are
    seen).  Every fifth step's outputs and the final states against the oracle."""
    r = run_full(lambda n: c3(n, max_steps=14), 65536, 40, graph_steps=5, min_resets=2 * 65536, after=_side_reset)
    assert r >= 2 * 65536


def test_c5_65536_multistep_graph_side_reset():
    """Eight steps per graph launch at C5's size (int16, side-stream reset), TimeLimit 15 (autoresets at
    steps 16 and 32, the last steps of launches; the episodes' ends inside them)."""
    run_full(lambda n: c5(n, max_steps=15), 65536, 32, graph_steps=8, min_resets=2 * 65536, after=_side_reset)


def test_c4_16384_multistep_graph_respawn():
    """Eight steps per graph launch at C4 (side-stream reset, k_respawn after every tick), TimeLimit 15: the
    16 384-env autoreset waves at steps 16 and 32 are the last steps of launches."""
    def check(eng):
        _side_reset(eng)
        assert eng.describe()["respawn"] == "k_respawn"
    run_full(lambda n: c4(n, max_steps=15), 16384, 48, graph_steps=8, min_resets=2 * 16384, after=check)


