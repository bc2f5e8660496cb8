"""Per-env step hashes of the engine's outputs, computed on the GPU (test infrastructure).

Full-size parity (tests/test_fullsize_parity.py): the oracle cannot hand back 65 536 envs'
observations every step cheaply, so both sides reduce every env's step to one 64-bit hash
with the same definition (oracle/zs_oracle.c zo_run_hashes):

    h = sum_i obs[i] * W(i)                                        (mod 2^64)
      + stepped ? sum_a listed_a * bits(rew[a]) * W(R+a) + done * W(D) + trunc * W(T)
                : W(X)                                             (the env was autoreset)

W(i) are odd pseudo-random 64-bit weights, so a change of any single output word changes
the hash.  Here the sums run as int64 torch reductions on the device (two's-complement
wrap-around = arithmetic mod 2^64); `numpy_step_hash` is the same definition on host arrays
(pinned against the oracle in tests/test_parity_hash.py).
"""
import numpy as np

from oracle.oracle import HASH_D, HASH_R, hash_weights


def _i64(u):
    return np.asarray(u, dtype=np.uint64).view(np.int64)


class StepHasher(object):
    def __init__(self, eng, chunk=8192):
        torch = eng.torch
        self.eng, self.torch, self.chunk = eng, torch, chunk
        per = eng.obs[0].numel()
        dev = eng.device
        self.w_obs = torch.from_numpy(_i64(hash_weights(range(per)))).to(dev)
        nr = eng.rewards.shape[1]
        self.w_rew = torch.from_numpy(_i64(hash_weights([HASH_R + a for a in range(nr)]))).to(dev)
        wd, wt, wx = (int(v) for v in _i64(hash_weights([HASH_D, HASH_D + 1, HASH_D + 2])))
        self.wd, self.wt, self.wx = wd, wt, wx

    def obs_hash(self):
        """[N] int64: the observation part only (the reset column)."""
        t = self.torch
        eng = self.eng
        obs = eng.obs.view(eng.N, -1)
        out = t.empty(eng.N, dtype=t.int64, device=eng.device)
        for s in range(0, eng.N, self.chunk):
            out[s:s + self.chunk] = (obs[s:s + self.chunk].to(t.int64) * self.w_obs).sum(1)
        return out

    def step_hash(self):
        """[N] int64 hash of the last zs_step's outputs."""
        t = self.torch
        eng = self.eng
        h = self.obs_hash()
        reset = eng.was_reset.to(t.int64)
        stepped = 1 - reset
        bits = eng.rewards.view(t.int64)
        if eng.multi:
            bits = bits * eng.listed.to(t.int64)
        r = (bits * self.w_rew).sum(1)
        r = r + eng.done.to(t.int64) * self.wd + eng.trunc.to(t.int64) * self.wt
        return h + stepped * r + reset * self.wx


def numpy_step_hash(obs, rew=None, listed=None, done=False, trunc=False, reset=False):
    """The same definition for one env on host arrays (rew=None: the reset column)."""
    with np.errstate(over="ignore"):
        flat = np.asarray(obs).reshape(-1).astype(np.int64).view(np.uint64)
        h = np.uint64(np.sum(flat * hash_weights(range(flat.size)), dtype=np.uint64))
        if reset:
            return h + hash_weights([HASH_D + 2])[0]
        if rew is None:
            return h
        bits = np.asarray(rew, dtype=np.float64).view(np.uint64)
        if listed is not None:
            bits = bits * np.asarray(listed, dtype=np.uint64)
        h = h + np.sum(bits * hash_weights([HASH_R + a for a in range(bits.size)]), dtype=np.uint64)
        wd, wt = hash_weights([HASH_D, HASH_D + 1])
        return h + np.uint64(done) * wd + np.uint64(trunc) * wt
