"""The per-call host path (zs_host_step / zs_host_reset / zs_host_observe, include/zombsole_mi355x.h) on a handle
of several envs: every section of every env's record equals what the batched calls give on a twin handle
(zs_reset / zs_step outputs, zs_get_state, zs_get_rng, zs_action_log, zs_death_log), with the envs' streams
moved in through the record path on some calls and left in place on others."""
import numpy as np
import pytest

from libzombsole_amd import _abi

pytestmark = pytest.mark.gpu

HOST_FLAGS, HOST_ERR, HOST_ALOG_N, HOST_DLOG_N, HOST_RNG = 0, 1, 2, 3, 4


def _cfg(n, surface):
    if surface == "multi":
        b = _abi.multi_env_config(n, "extermination", ["terminator"], "bridge", ["0", "1", "2"], initial_zombies=12,
                                  minimum_zombies=6, max_episode_steps=0, obs_dtype=_abi.DTYPE_I64, autoreset=False)
    else:
        b = _abi.single_env_config(n, "survival", ["hamster"], "boxed", 0, initial_zombies=3, minimum_zombies=2,
                                   observation_scope="world", observation_position_encoding="channels",
                                   max_episode_steps=0, obs_dtype=_abi.DTYPE_I32, autoreset=False)
    b.cfg.flags |= _abi.FLAG_DEATH_LOG
    return b


@pytest.mark.parametrize("surface", ["multi", "single"])
def test_host_records_equal_batched_calls(surface):
    import torch

    from libzombsole_amd.actions import DISCRETE_TRIPLES
    from libzombsole_amd.engine import Engine, decode_action_log, decode_death_log
    n = 5
    host, ref = Engine(_cfg(n, surface)), Engine(_cfg(n, surface))
    lay = host.host_layout()
    seeds = [70 + i for i in range(n)]
    ref.seed(seeds)
    # the host handle gets the same streams through the record path: seed a scratch handle, read its rings
    scratch = Engine(_cfg(n, surface))
    scratch.seed(seeds)
    rng = np.stack([scratch.get_rng(e) for e in range(n)]).astype(np.uint32)
    scratch.close()
    rec = host.host_record()
    host.host_reset(rng, rec)
    ref.reset()
    torch.cuda.synchronize()

    def compare(rec, step, where):
        obs = ref.obs.cpu().numpy()
        for e in range(n):
            r = rec[e]
            ob = r[lay["obs"]:].view(np.uint8)[:lay["obs_bytes"]].view(obs.dtype).reshape(obs.shape[1:])
            assert np.array_equal(ob, obs[e]), (where, e, "obs")
            st = ref.get_state(e).buf
            assert np.array_equal(r[lay["state"]:lay["state"] + len(st)], st), (where, e, "state")
            assert np.array_equal(r[HOST_RNG:HOST_RNG + 625].view(np.uint32), ref.get_rng(e)), (where, e, "rng")
            if step:
                rw = r[lay["rew"]:lay["rew"] + 2 * lay["R"]].view(np.float64)
                assert np.array_equal(rw, ref.rewards[e].cpu().numpy()), (where, e, "rewards")
                assert r[HOST_FLAGS] & 3 == int(ref.done[e]) | (int(ref.trunc[e]) << 1), (where, e, "flags")
                acts, _ = ref.action_log(e)
                assert decode_action_log(r[lay["alog"]:], int(r[HOST_ALOG_N]), ref.E)[0] == acts, (where, e, "alog")
                assert decode_death_log(r[lay["dlog"]:], int(r[HOST_DLOG_N]), ref.E) == ref.death_log(e), \
                    (where, e, "dlog")

    compare(rec, False, "reset")
    rec_prev = rec
    rs = np.random.default_rng(5)
    for t in range(1, 41):
        acts = np.zeros((n, ref.A, 3), dtype=np.int32)
        acts[:] = DISCRETE_TRIPLES[rs.integers(0, len(DISCRETE_TRIPLES), size=(n, ref.A))]
        ref.actions.copy_(torch.from_numpy(acts))
        ref.step()
        rec = host.host_record()
        # the streams: moved in through the record path every third call (the engine's own values), else left
        rng = np.stack([rec_prev[e][HOST_RNG:HOST_RNG + 625].view(np.uint32) for e in range(n)]) if t % 3 == 0 else None
        host.host_step(acts, rng, rec)
        torch.cuda.synchronize()
        compare(rec, True, "step %d" % t)
        rec_prev = rec
        if t == 20:  # zs_host_observe re-encodes the same state
            obs_rec = host.host_record()
            host.host_observe(obs_rec)
            for e in range(n):
                a = obs_rec[e][lay["obs"]:lay["obs"] + lay["obs_bytes"] // 4]
                b = rec[e][lay["obs"]:lay["obs"] + lay["obs_bytes"] // 4]
                assert np.array_equal(a, b), ("observe", e)
    host.close()
    ref.close()
