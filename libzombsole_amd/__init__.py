"""libzombsole_amd — MI355X-native batched zombsole step engine.

Drop-in surfaces (mirroring jvstinian/libzombsole):
  * ``libzombsole_amd.gym_env.ZombsoleGymEnv`` / ``ZombsoleGymEnvDiscreteAction``
  * ``libzombsole_amd.multiagent_env.MultiagentZombsoleEnv`` /
    ``MultiagentZombsoleEnvDiscreteAction``
  * ``libzombsole_amd.vector.BatchedZombsole`` — the batched device API.

Every step runs in the HIP engine (``libzombsole_mi355x.so``); there is no CPU
fallback.  Submodules are imported lazily so that the pure-host pieces (map
parsing, action encoding) import without torch or a GPU.
"""
__version__ = "0.1.0"

import os as _os

# hipGraph launches: the HIP runtime's replay of pre-captured AQL packets costs this engine's two-kernel
# step graphs ~4 us more per graph launch than its plain dispatch path (one MI355X, one step per graph
# launch: 8 192-env shard 134 -> 144 M env-steps/s with it off, C2 86 -> 94 M, the caller's policy at the
# shard 110 -> 117 M; C3 / C4 / C5 even; profiles/r05b_env_ab.log).  The runtime reads it when it
# initialises, so it applies when this package is imported before the process's first HIP call
# (bench.py, tests/conftest.py and __graft_entry__.py import it first); a value the caller set wins.
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
