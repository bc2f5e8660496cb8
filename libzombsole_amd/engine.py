"""Runtime binding of the HIP engine (libzombsole_mi355x.so) through its C ABI.

`Engine` owns one `zs_handle` (N envs on one GPU) plus the torch device
tensors the engine writes its outputs into.  There is no CPU fallback: if
the shared library or a HIP device is missing, construction raises.
"""
import ctypes as C
import os

import numpy as np

from . import _abi

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libzombsole_mi355x.so")
SYMBOLS = ["zs_last_error", "zs_create", "zs_destroy", "zs_obs_shape", "zs_seed", "zs_reset", "zs_step", "zs_observe",
           "zs_gen_actions", "zs_step_graph", "zs_step_graph_n", "zs_state_size", "zs_get_state", "zs_set_state", "zs_get_rng", "zs_set_rng", "zs_overflow", "zs_profile", "zs_profile_read", "zs_describe",
           "zs_debug_stamps", "zs_debug_stamps_wg", "zs_debug_timeline", "zs_debug_lists", "zs_death_log", "zs_action_log",
           "zs_host_layout", "zs_host_step", "zs_host_reset", "zs_host_observe"]

_lib = None


class EngineUnavailable(RuntimeError):
    pass


def load_library(path=None):
    """Load the engine .so (no device call is made).  The product library unless `path` names
    another build of the same sources; use_library(path) makes such a build the process's engine
    (diagnostic tools: tools/stamps.py, A/B runs).  No environment variable selects the library."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise EngineUnavailable("HIP engine library not built: %s (run __graft_entry__.build())" % p)
    # torch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1; load it first so the engine
    # binds to that same runtime (same SONAME) instead of pulling a second HIP runtime from
    # /opt/rocm into the process, which cannot open the device once torch's runtime owns it.
    import torch  # noqa: F401
    L = C.CDLL(p)
    vp, i32, u64 = C.c_void_p, C.c_int32, C.c_uint64
    L.zs_last_error.restype = C.c_char_p
    L.zs_create.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.zs_destroy.argtypes = [vp]
    L.zs_obs_shape.argtypes = [vp, C.POINTER(i32)]
    L.zs_seed.argtypes = [vp, i32, i32, C.POINTER(u64), vp]
    L.zs_reset.argtypes = [vp, vp, vp, vp]
    L.zs_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.zs_observe.argtypes = [vp, vp, vp, vp]
    L.zs_gen_actions.argtypes = [vp, u64, i32, vp, vp]
    L.zs_step_graph.argtypes = [vp, u64, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.zs_step_graph_n.argtypes = [vp, u64, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.zs_state_size.argtypes = [vp, C.POINTER(i32)]
    L.zs_get_state.argtypes = [vp, i32, vp, vp]
    L.zs_set_state.argtypes = [vp, i32, vp, vp]
    L.zs_get_rng.argtypes = [vp, i32, vp, vp]
    L.zs_set_rng.argtypes = [vp, i32, vp, vp]
    L.zs_overflow.argtypes = [vp, C.POINTER(C.c_uint32), i32, vp]
    L.zs_profile.argtypes = [vp, i32]
    L.zs_profile_read.argtypes = [vp, C.POINTER(C.c_double)]
    L.zs_debug_stamps.argtypes = [vp, vp, vp, i32]
    L.zs_describe.argtypes = [vp, C.c_char_p, i32]
    L.zs_debug_lists.argtypes = [vp, C.POINTER(i32), vp]
    L.zs_death_log.argtypes = [vp, i32, C.POINTER(i32), i32, C.POINTER(i32), vp]
    L.zs_action_log.argtypes = [vp, i32, C.POINTER(i32), i32, C.POINTER(i32), vp]
    L.zs_debug_timeline.argtypes = [vp, vp, i32]
    L.zs_debug_stamps_wg.argtypes = [vp, vp, i32, i32]
    L.zs_host_layout.argtypes = [vp, C.POINTER(i32)]
    L.zs_host_step.argtypes = [vp, vp, vp, vp, vp]
    L.zs_host_reset.argtypes = [vp, vp, vp, vp]
    L.zs_host_observe.argtypes = [vp, vp, vp]
    for s in SYMBOLS:
        if s != "zs_last_error":
            getattr(L, s).restype = C.c_int
    if path is None:
        _lib = L
    return L


def use_library(path):
    """Tools only: make the build at `path` (e.g. a -DZS_STAMPS diagnostic build) the library every
    later Engine of this process binds."""
    global _lib
    _lib = load_library(path)
    return _lib


class EngineError(RuntimeError):
    pass


def _raise(L, rc, what):
    msg = (L.zs_last_error() or b"").decode(errors="replace")
    if rc == _abi.ZS_EINVAL:
        raise ValueError("%s: %s" % (what, msg))
    if rc == _abi.ZS_ENOSPACE:
        raise Exception(msg or "Not enough space to spawn")  # core.py:62-64 raises a bare Exception
    raise EngineError("%s failed (%d): %s" % (what, rc, msg))


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _np_ptr(a):
    """A host buffer argument: None, bytes (e.g. struct-packed) or a numpy array."""
    if a is None or isinstance(a, bytes):
        return a
    return C.c_void_p(a.ctypes.data)


def decode_action_log(words, n, E):
    """(actions, raised) from zs_action_log's words and count (n < 0: a debug raise, -1 - n entries)."""
    raised = n < 0
    k = min(-1 - n if raised else n, E)
    w = words[:2 * k].tolist()
    return [(w[2 * j] & 0xff, (w[2 * j] >> 8) & 0xff, w[2 * j + 1]) for j in range(k)], raised


def decode_death_log(words, n, E):
    """[(slot, serial, x, y, life)] from zs_death_log's words and count."""
    k = max(0, min(n, E))
    w = words[:5 * k].tolist()
    return [tuple(w[5 * j:5 * j + 5]) for j in range(k)]


class Engine(object):
    """N lock-step envs on one MI355X."""

    def __init__(self, builder, device=None):
        import torch
        if not torch.cuda.is_available():
            raise EngineUnavailable("no HIP device visible: the zombsole engine runs only on the GPU")
        self.torch = torch
        self.L = load_library()
        self.builder = builder
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        # Initialise torch's HIP runtime on this device first: the engine .so binds to the same
        # libamdhip64 torch loaded (one runtime per process), and a bare is_available() leaves
        # that runtime without a device context (hipSetDevice then reports no device).
        torch.zeros(1, device=self.device)
        self.h = C.c_void_p()
        rc = self.L.zs_create(C.cast(builder.ptr(), C.c_void_p), self.device.index, C.byref(self.h))
        if rc:
            _raise(self.L, rc, "zs_create")
        shp = (C.c_int32 * 4)()
        self.L.zs_obs_shape(self.h, shp)
        self.obs_shape = tuple(int(v) for v in shp)
        self.N = builder.cfg.num_envs
        self.A = builder.num_agents
        c = builder.cfg
        self.E = self.A + builder.num_bots + max(c.initial_zombies, c.minimum_zombies)  # entity slots (zs_create)
        self.multi = builder.cfg.reward_mode == _abi.REWARD_MULTI
        dt = {_abi.DTYPE_I32: torch.int32, _abi.DTYPE_I64: torch.int64, _abi.DTYPE_I16: torch.int16}
        self.obs_dtype = dt[builder.cfg.obs_dtype]
        kw = dict(device=self.device)
        self.out = self.outputs()
        self.obs, self.rewards, self.done, self.trunc = self.out.obs, self.out.rewards, self.out.done, self.out.trunc
        self.listed, self.was_reset = self.out.listed, self.out.was_reset
        self.actions = torch.zeros((self.N, self.A, 3), dtype=torch.int32, **kw)
        n = C.c_int32()
        self.L.zs_state_size(self.h, C.byref(n))
        self.state_words = int(n.value)

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.L.zs_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def seed(self, seeds, env0=0):
        arr = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).reshape(-1))
        rc = self.L.zs_seed(self.h, env0, len(arr), arr.ctypes.data_as(C.POINTER(C.c_uint64)), self._stream())
        if rc:
            _raise(self.L, rc, "zs_seed")

    def reset(self, mask=None):
        """Reset envs (all, or where the uint8 device tensor `mask` is nonzero)."""
        rc = self.L.zs_reset(self.h, _ptr(mask), _ptr(self.obs), self._stream())
        if rc:
            _raise(self.L, rc, "zs_reset")
        return self.obs

    def outputs(self, rows=None, obs=None, flat=None):
        """A set of step output buffers (StepOutputs) with `rows` >= N rows; the engine writes the
        first N.  Steps may alternate between sets (double-buffered outputs, vector.StepGather).  obs / flat,
        when given, are the storage to use (e.g. this rank's slice of a gather buffer)."""
        return StepOutputs(self, self.N if rows is None else max(int(rows), self.N), obs, flat)

    def step(self, actions=None, out=None):
        """One tick for all envs; `actions` int32 [N, A, 3] device tensor (default: self.actions);
        outputs into `out` (default: self.out)."""
        a = self.actions if actions is None else actions
        o = self.out if out is None else out
        rc = self.L.zs_step(self.h, _ptr(a), _ptr(o.obs), _ptr(o.rewards), _ptr(o.done),
                            _ptr(o.trunc), _ptr(o.listed), _ptr(o.was_reset), self._stream())
        if rc:
            _raise(self.L, rc, "zs_step")
        return o.obs[:self.N], o.rewards[:self.N], o.done[:self.N], o.trunc[:self.N]

    def step_graph(self, step0, n_discrete, out=None, steps=1, actions=None):
        """gen_actions(t, n_discrete) + step() as one replayed hipGraph (t = step0 on the first call,
        then advancing by one per step on the device).  steps > 1: that many steps per graph launch
        (zs_step_graph_n), the outputs holding the last one's.  n_discrete = 0: no policy, the graph
        replays step(actions) on the caller's action tensor (default self.actions), which the caller
        fills on the current stream before each call (see step_graphed)."""
        o = self.out if out is None else out
        a = self.actions if actions is None else actions
        if steps == 1:
            rc = self.L.zs_step_graph(self.h, int(step0), int(n_discrete), _ptr(a), _ptr(o.obs),
                                      _ptr(o.rewards), _ptr(o.done), _ptr(o.trunc), _ptr(o.listed),
                                      _ptr(o.was_reset), self._stream())
        else:
            rc = self.L.zs_step_graph_n(self.h, int(step0), int(n_discrete), int(steps), _ptr(a),
                                        _ptr(o.obs), _ptr(o.rewards), _ptr(o.done), _ptr(o.trunc), _ptr(o.listed),
                                        _ptr(o.was_reset), self._stream())
        if rc:
            _raise(self.L, rc, "zs_step_graph")
        return o.obs[:self.N], o.rewards[:self.N], o.done[:self.N], o.trunc[:self.N]

    def step_graphed(self, actions=None, out=None):
        """step(actions) as one replayed hipGraph launch (zs_step_graph with n_discrete = 0): the
        learner's per-step call (gym/multiagent_env.py:111-171) without the 3-5 host dispatches of an
        eager zs_step.  The graph is keyed on the action and output buffers, so a caller keeps them
        fixed (self.actions, an output set) and rewrites their contents each step."""
        return self.step_graph(0, 0, out=out, actions=actions)

    def observe(self, mask=None):
        """Re-encode observations from the current state (after pokes)."""
        rc = self.L.zs_observe(self.h, _ptr(mask), _ptr(self.obs), self._stream())
        if rc:
            _raise(self.L, rc, "zs_observe")
        return self.obs

    def gen_actions(self, step, n_discrete, out=None):
        o = self.actions if out is None else out
        rc = self.L.zs_gen_actions(self.h, int(step), int(n_discrete), _ptr(o), self._stream())
        if rc:
            _raise(self.L, rc, "zs_gen_actions")
        return o

    def profile(self, enable=True):
        """Bracket every k_tick / k_obs launch with HIP events on its stream."""
        self.L.zs_profile(self.h, 1 if enable else 0)

    def profile_read(self):
        """Per-kernel totals: tick_ms/tick_n, obs_ms/obs_n, reset_ms/reset_n, respawn_ms/respawn_n."""
        out = (C.c_double * 8)()
        rc = self.L.zs_profile_read(self.h, out)
        if rc:
            _raise(self.L, rc, "zs_profile_read")
        return {"tick_ms": out[0], "tick_n": int(out[1]), "obs_ms": out[2], "obs_n": int(out[3]),
                "reset_ms": out[4], "reset_n": int(out[5]), "respawn_ms": out[6], "respawn_n": int(out[7])}

    def describe(self):
        """The launch configuration the engine chose (zs_describe), as a dict."""
        import json
        buf = C.create_string_buffer(1024)
        rc = self.L.zs_describe(self.h, buf, len(buf))
        if rc:
            _raise(self.L, rc, "zs_describe")
        return json.loads(buf.value.decode())

    def debug_stamps(self, n=5):
        """Per-phase k_tick cycle sums / maxima (diagnostic -DZS_STAMPS build only)."""
        ssum = np.zeros(n, dtype=np.uint64)
        smax = np.zeros(n, dtype=np.uint64)
        rc = self.L.zs_debug_stamps(self.h, C.c_void_p(ssum.ctypes.data), C.c_void_p(smax.ctypes.data), n)
        if rc:
            _raise(self.L, rc, "zs_debug_stamps")
        return ssum, smax

    def debug_stamps_wg(self, n_wgs, n_phase):
        """Per-workgroup phase cycles of the step launches since the last stamps read, shape [n_wgs, n_phase]
        (diagnostic -DZS_STAMPS build only)."""
        out = np.zeros((n_wgs, n_phase), dtype=np.uint64)
        rc = self.L.zs_debug_stamps_wg(self.h, C.c_void_p(out.ctypes.data), n_wgs, n_phase)
        if rc:
            _raise(self.L, rc, "zs_debug_stamps_wg")
        return out

    def debug_timeline(self, n):
        """Start / end s_memrealtime (100 MHz) of the first n workgroups of the last fused step launch,
        shape [n, 2] (diagnostic -DZS_STAMPS build only)."""
        out = np.zeros((n, 2), dtype=np.uint64)
        rc = self.L.zs_debug_timeline(self.h, C.c_void_p(out.ctypes.data), n)
        if rc:
            _raise(self.L, rc, "zs_debug_timeline")
        return out

    def debug_lists(self):
        """(pending-reset count of list 0, of list 1, deferred-respawn count, parity drained next)."""
        out = (C.c_int32 * 4)()
        rc = self.L.zs_debug_lists(self.h, out, self._stream())
        if rc:
            _raise(self.L, rc, "zs_debug_lists")
        return tuple(int(v) for v in out)

    def death_log(self, env):
        """The things env's last step removed in clean_dead_things (core.py:121-138), in removal order:
        a list of (slot, serial, x, y, life).  Needs a config with FLAG_DEATH_LOG."""
        out = (C.c_int32 * (5 * max(1, self.E)))()
        n = C.c_int32(0)
        rc = self.L.zs_death_log(self.h, int(env), out, int(self.E), C.byref(n), self._stream())
        if rc:
            _raise(self.L, rc, "zs_death_log")
        return decode_death_log(np.frombuffer(out, dtype=np.int32), n.value, self.E)

    def action_log(self, env):
        """The actions env's last step executed, in execution order (core.py:76,103-119): a list of
        (slot, kind, target), kind 1 move (target: destination x | y << 16), 2 attack, 3 heal (target: an
        entity slot, or -1 - obstacle index).  Needs a config with FLAG_DEATH_LOG.  Returns (actions, raised):
        raised when a debug raise stopped the step, the actions then being the decided actions of the actors
        before the raising one, in dict order."""
        out = (C.c_int32 * (2 * max(1, self.E)))()
        n = C.c_int32(0)
        rc = self.L.zs_action_log(self.h, int(env), out, int(self.E), C.byref(n), self._stream())
        if rc:
            _raise(self.L, rc, "zs_action_log")
        return decode_action_log(np.frombuffer(out, dtype=np.int32), n.value, self.E)

    # -- the drop-ins' per-call path (zs_host_*): one copy in, one copy out, one synchronisation ----------
    def host_layout(self):
        """Word offsets of a zs_host_* record's sections (zs_host_layout)."""
        if getattr(self, "_hl", None) is None:
            out = (C.c_int32 * 8)()
            rc = self.L.zs_host_layout(self.h, out)
            if rc:
                _raise(self.L, rc, "zs_host_layout")
            self._hl = dict(zip(("words", "rew", "alog", "dlog", "state", "obs", "obs_bytes", "R"), [int(v) for v in out]))
        return self._hl

    def host_record(self):
        """A fresh record buffer for one zs_host_* call over all N envs (int32 [N][words])."""
        return np.empty((self.N, self.host_layout()["words"]), dtype=np.int32)

    def host_step(self, actions, rng, rec):
        """zs_host_step: actions int32 [N, A, 3] (host), rng [N][625] uint32 words (random.getstate() form;
        a numpy array or packed bytes) or None, rec from host_record() (filled)."""
        a = np.ascontiguousarray(actions, dtype=np.int32)
        rc = self.L.zs_host_step(self.h, C.c_void_p(a.ctypes.data), _np_ptr(rng), C.c_void_p(rec.ctypes.data),
                                 self._stream())
        if rc:
            _raise(self.L, rc, "zs_host_step")
        return rec

    def host_reset(self, rng, rec):
        """zs_host_reset: every env rebuilt (Game.__initialize_world__), record filled.  On ZS_ENOSPACE the
        record still holds the envs' streams (the caller moves them back before re-raising)."""
        rc = self.L.zs_host_reset(self.h, _np_ptr(rng), C.c_void_p(rec.ctypes.data), self._stream())
        if rc:
            _raise(self.L, rc, "zs_host_reset")
        return rec

    def host_observe(self, rec):
        rc = self.L.zs_host_observe(self.h, C.c_void_p(rec.ctypes.data), self._stream())
        if rc:
            _raise(self.L, rc, "zs_host_observe")
        return rec

    def get_state(self, env):
        buf = np.zeros(self.state_words, dtype=np.int32)
        rc = self.L.zs_get_state(self.h, int(env), C.c_void_p(buf.ctypes.data), self._stream())
        if rc:
            _raise(self.L, rc, "zs_get_state")
        return StateView(self, buf)

    def set_state(self, env, view):
        rc = self.L.zs_set_state(self.h, int(env), C.c_void_p(view.buf.ctypes.data), self._stream())
        if rc:
            _raise(self.L, rc, "zs_set_state")


    def overflow(self, clear=False):
        """Sticky range flags (_abi.OVF_INT16 | OVF_INT32) of every env since creation / the last clear."""
        f = C.c_uint32(0)
        rc = self.L.zs_overflow(self.h, C.byref(f), 1 if clear else 0, self._stream())
        if rc:
            _raise(self.L, rc, "zs_overflow")
        return int(f.value)

    def check_lossless(self):
        """Raise OverflowError when an obstacle life left what this engine's outputs hold exactly: below
        the int16 range with int16 observations, or saturated at -2**31 + 1."""
        f = self.overflow()
        if f & _abi.OVF_INT32:
            raise OverflowError("an obstacle life fell below -2147483647 and saturated (reference: unbounded int)")
        if (f & _abi.OVF_INT16) and self.obs_dtype == self.torch.int16:
            raise OverflowError("an obstacle life fell below -32768: int16 observations saturated it")

    def get_rng(self, env):
        """(mt[624] uint32, index) of env's MT19937 stream, CPython getstate() form."""
        buf = np.zeros(625, dtype=np.uint32)
        rc = self.L.zs_get_rng(self.h, int(env), C.c_void_p(buf.ctypes.data), self._stream())
        if rc:
            _raise(self.L, rc, "zs_get_rng")
        return buf

    def set_rng(self, env, state):
        buf = np.ascontiguousarray(np.asarray(state, dtype=np.uint32).reshape(625))
        rc = self.L.zs_set_rng(self.h, int(env), C.c_void_p(buf.ctypes.data), self._stream())
        if rc:
            _raise(self.L, rc, "zs_set_rng")

    def load_python_random(self, env, rnd=None):
        """Move a `random.Random` (default: the module-global one) state into env."""
        import random as _random
        st = (rnd or _random).getstate()
        self.set_rng(env, np.asarray(st[1], dtype=np.uint64).astype(np.uint32))

    def store_python_random(self, env, rnd=None):
        """Write env's stream back into a `random.Random` (default: the module-global one)."""
        import random as _random
        buf = self.get_rng(env)
        r = rnd or _random
        r.setstate((3, tuple(int(v) for v in buf), None))


class StepOutputs(object):
    """One set of zs_step output buffers, `rows` >= N rows (rows past N are padding the engine never
    writes: equal-sized shards for a collective).  Everything but the observations lives in one flat byte
    tensor (`flat`), so a per-step exchange moves it in one collective (obs + reward +
    done/trunc/alive): float64 rewards [rows][R], then done [rows], truncated [rows], listed [rows][A] (the
    agents alive before the step: the keys of the reference's per-agent dicts, gym/multiagent_env.py:156-169)
    and was_reset [rows] (the observation is a reset's)."""

    @staticmethod
    def row_bytes(eng):
        R = eng.A if eng.multi else 1
        return 8 * R + 3 + eng.A

    def __init__(self, eng, rows, obs=None, flat=None):
        torch = eng.torch
        kw = dict(device=eng.device)
        R = eng.A if eng.multi else 1
        A = eng.A
        self.rows = rows
        nb = rows * self.row_bytes(eng)
        if obs is not None:
            assert obs.shape == (rows,) + tuple(eng.obs_shape) and obs.dtype == eng.obs_dtype and obs.is_contiguous()
        if flat is not None:
            assert flat.dim() == 1 and flat.numel() >= nb and flat.dtype == torch.uint8
            assert flat.is_contiguous() and flat.storage_offset() % 8 == 0
        self.obs = obs if obs is not None else torch.zeros((rows,) + eng.obs_shape, dtype=eng.obs_dtype, **kw)
        self.flat = flat if flat is not None else torch.zeros(nb, dtype=torch.uint8, **kw)
        o = 8 * R * rows
        self.rewards = self.flat[:o].view(torch.float64).view(rows, R)
        self.done = self.flat[o:o + rows]
        self.trunc = self.flat[o + rows:o + 2 * rows]
        self.listed = self.flat[o + 2 * rows:o + (2 + A) * rows].view(rows, A)
        self.was_reset = self.flat[o + (2 + A) * rows:o + (3 + A) * rows]


class StateView(object):
    """Decoded zs_get_state record (layout: include/zombsole_mi355x.h)."""

    def __init__(self, eng, buf):
        self.buf = buf
        b = buf
        self.E, self.O, self.W, self.H = int(b[6]), int(b[7]), int(b[8]), int(b[9])
        self.A = eng.A
        self.P = eng.builder.num_bots
        o = _abi.STATE_HEADER
        self.ent = b[o:o + _abi.STATE_ENTITY_WORDS * self.E].reshape(self.E, _abi.STATE_ENTITY_WORDS)
        o += _abi.STATE_ENTITY_WORDS * self.E
        self.order = b[o:o + self.E]
        o += self.E
        self.obst_life = b[o:o + self.O]
        o += self.O
        self.obst_present = b[o:o + self.O]
        o += self.O
        self.prev_life = b[o:o + self.A]
        o += self.A
        self.listed = b[o:o + self.A]
        o += self.A
        dw = (self.W * self.H + 31) // 32
        self.dead_words = b[o:o + dw]

    t = property(lambda s: int(s.buf[0]))
    deaths = property(lambda s: int(s.buf[1]))
    zombie_deaths = property(lambda s: int(s.buf[2]))
    n_order = property(lambda s: int(s.buf[4]))

    def dead_cells(self):
        w = self.dead_words.astype(np.uint32)
        bits = np.unpackbits(w.view(np.uint8), bitorder="little")
        return [int(c) for c in np.nonzero(bits[:self.W * self.H])[0]]

    def canonical(self, obstacle_kinds):
        """The canonical state dict of tests/golden records."""
        dyn = []
        for s in self.order[:self.n_order]:
            r = self.ent[int(s)]
            dyn.append([int(r[0]), int(r[2]), int(r[3]), int(r[4]), int(r[5]), int(r[6])])
        obst = []
        for i in range(self.O):
            ml = 10 if obstacle_kinds[i] == _abi.THING_BOX else 200
            if int(self.obst_life[i]) != ml or not self.obst_present[i]:
                obst.append([i, int(self.obst_life[i]), int(self.obst_present[i])])
        agents = [[int(r[2]), int(r[3]), int(r[4]), int(r[5])] for r in self.ent[:self.A]]
        players = [[int(r[2]), int(r[3]), int(r[4]), int(r[5])] for r in self.ent[self.A:self.A + self.P]]
        return {"dyn": dyn, "obst": obst, "dead": self.dead_cells(), "ctr": [self.t, self.deaths, self.zombie_deaths],
                "agents": agents, "players": players}
