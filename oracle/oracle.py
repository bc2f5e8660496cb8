"""ctypes binding of the C oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() import
this module.  The product path (libzombsole_amd) never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libzs_oracle.so")


def build(asan=False):
    target = "_build/libzs_oracle_asan.so" if asan else "_build/libzs_oracle.so"
    subprocess.check_call(["make", "-s", "-C", HERE, target])
    return os.path.join(HERE, target)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = load(LIB)
    return _lib


def load(path):
    L = C.CDLL(path)
    L.zo_create.restype = C.c_void_p
    L.zo_create.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    L.zo_destroy.argtypes = [C.c_void_p]
    L.zo_seed.argtypes = [C.c_void_p, C.c_uint64]
    L.zo_reset.argtypes = [C.c_void_p]
    L.zo_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.zo_obs.argtypes = [C.c_void_p, C.c_void_p]
    L.zo_state.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.zo_rng_draws.restype = C.c_uint64
    L.zo_rng_draws.argtypes = [C.c_void_p]
    L.zo_poke_life.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
    L.zo_poke_obstacle.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.zo_poke_dead.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.zo_poke_obstacle_gone.argtypes = [C.c_void_p, C.c_int]
    L.zo_run_batch.restype = C.c_int64
    L.zo_run_batch.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                               C.POINTER(C.c_uint64)]
    L.zo_hash_weight.restype = C.c_uint64
    L.zo_hash_weight.argtypes = [C.c_uint64]
    L.zo_run_hashes.restype = C.c_int64
    L.zo_run_hashes.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                C.c_void_p]
    L.zo_run_hashes_census.restype = C.c_int64
    L.zo_run_hashes_census.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                       C.c_void_p, C.c_int32, C.c_void_p]
    L.zo_set_census.argtypes = [C.c_void_p, C.c_int]
    L.zo_census.argtypes = [C.c_void_p, C.c_void_p]
    return L


def parse_state(buf):
    """Flat zo_state record -> the dict layout of tests/golden records."""
    it = iter(int(v) for v in buf)
    n = next(it)
    dyn = [[next(it) for _ in range(6)] for _ in range(n)]
    n = next(it)
    obst = [[next(it) for _ in range(3)] for _ in range(n)]
    n = next(it)
    dead = [next(it) for _ in range(n)]
    ctr = [next(it), next(it), next(it)]
    n = next(it)
    agents = [[next(it) for _ in range(4)] for _ in range(n)]
    n = next(it)
    players = [[next(it) for _ in range(4)] for _ in range(n)]
    return {"dyn": dyn, "obst": obst, "dead": dead, "ctr": ctr, "agents": agents, "players": players}


ZO_RAISED = 100


class OracleRaised(Exception):
    """The step stopped at an agent whose action is ZS_ACT_RAISE (World.get_actions re-raising)."""


class OracleEnv(object):
    """One reference env restated in C; `builder` is a libzombsole_amd._abi.ConfigBuilder."""

    def __init__(self, builder, path=None):
        self.L = load(path) if path else lib()
        self.builder = builder
        err = C.create_string_buffer(256)
        self.h = self.L.zo_create(C.cast(builder.ptr(), C.c_void_p), err, 256)
        if not self.h:
            raise ValueError(err.value.decode())
        self.A = builder.num_agents
        self.obs_shape = builder.obs_shape()
        from libzombsole_amd._abi import DTYPE_NP
        self.obs_dtype = DTYPE_NP[builder.cfg.obs_dtype]
        cap = 64 + 6 * (builder.num_agents + builder.num_bots + 4096) + 3 * len(builder.map.obstacles) \
            + builder.map.size[0] * builder.map.size[1] + 4 * (builder.num_agents + builder.num_bots)
        self._sbuf = np.zeros(cap, dtype=np.int32)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.zo_destroy(self.h)
            self.h = None

    def seed(self, s):
        self.L.zo_seed(self.h, s)

    def reset(self):
        rc = self.L.zo_reset(self.h)
        if rc:
            raise RuntimeError("zo_reset failed: %d" % rc)
        return self.obs()

    def step(self, actions):
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.int32).reshape(-1, 3))
        rew = np.zeros(max(self.A, 1), dtype=np.float64)
        done = np.zeros(1, np.uint8)
        trunc = np.zeros(1, np.uint8)
        listed = np.zeros(max(self.A, 1), np.uint8)
        rc = self.L.zo_step(self.h, a.ctypes.data, rew.ctypes.data, done.ctypes.data, trunc.ctypes.data,
                            listed.ctypes.data)
        if rc == ZO_RAISED:
            raise OracleRaised()
        if rc:
            raise RuntimeError("zo_step failed: %d" % rc)
        return self.obs(), rew, bool(done[0]), bool(trunc[0]), listed[:self.A].astype(bool)

    def obs(self):
        out = np.zeros(self.obs_shape, dtype=self.obs_dtype)
        self.L.zo_obs(self.h, out.ctypes.data)
        return out

    def state(self):
        n = self.L.zo_state(self.h, self._sbuf.ctypes.data, len(self._sbuf))
        if n < 0:
            raise RuntimeError("state buffer too small")
        return parse_state(self._sbuf[:n])

    def rng_draws(self):
        return int(self.L.zo_rng_draws(self.h))

    def poke_life(self, which, i, life):
        return self.L.zo_poke_life(self.h, which, i, life)

    def poke_obstacle(self, i, life):
        return self.L.zo_poke_obstacle(self.h, i, life)

    def poke_dead(self, x, y):
        return self.L.zo_poke_dead(self.h, x, y)

    def set_census(self, chunk_g):
        """Count the conflict cases of the engine's chunked execution with G = chunk_g (0 = off)."""
        self.L.zo_set_census(self.h, int(chunk_g))

    def census(self):
        out = np.zeros(len(CENSUS), dtype=np.int64)
        self.L.zo_census(self.h, out.ctypes.data)
        return dict(zip(CENSUS, (int(v) for v in out)))

    def poke_obstacle_gone(self, i):
        return self.L.zo_poke_obstacle_gone(self.h, i)


def run_batch(builder, seed0, n_envs, steps, n_discrete, threads=1):
    csum = C.c_uint64(0)
    n = lib().zo_run_batch(C.cast(builder.ptr(), C.c_void_p), seed0, n_envs, steps, n_discrete, threads,
                           C.byref(csum))
    return int(n), int(csum.value)


def hash_weights(idx):
    """zo_hash_weight(i) for every i of `idx` (uint64 array)."""
    L = lib()
    return np.array([L.zo_hash_weight(int(i)) for i in idx], dtype=np.uint64)


HASH_R, HASH_D = 1 << 20, 1 << 21  # weight offsets of rewards / done, truncated, autoreset (zs_oracle.c)


# conflict census of the engine's chunked execution (zs_oracle.h ZO_CF_*), in index order
CENSUS = ("enter_vacated", "same_dest", "target_moved", "target_later", "multi_hit", "hit_dead", "heal_clamp",
          "obst_int16", "lists", "lists_serial", "chunks", "max_in_chunk", "chunks_all6")
CENSUS_CASES = CENSUS[:8]


def run_hashes(builder, seed0, n_envs, steps, n_discrete, threads=0, reset_twice_mod=0, chunk_g=0):
    """Per env and step output hashes of the bench workload: uint64 [n_envs, steps + 1]
    (column 0 = the reset observation), see zo_run_hashes.  chunk_g > 0: also the conflict census of
    every env summed (a dict, CENSUS), returned as (hashes, census)."""
    out = np.zeros((n_envs, steps + 1), dtype=np.uint64)
    if chunk_g <= 0:
        lib().zo_run_hashes(C.cast(builder.ptr(), C.c_void_p), seed0, n_envs, steps, n_discrete, threads,
                            reset_twice_mod, out.ctypes.data)
        return out
    cen = np.zeros(len(CENSUS), dtype=np.int64)
    lib().zo_run_hashes_census(C.cast(builder.ptr(), C.c_void_p), seed0, n_envs, steps, n_discrete, threads,
                               reset_twice_mod, out.ctypes.data, int(chunk_g), cen.ctypes.data)
    return out, dict(zip(CENSUS, (int(v) for v in cen)))
