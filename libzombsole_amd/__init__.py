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


def plain_graph_dispatch():
    """Opt-in HIP runtime setting for processes whose hot loop replays this engine's step graphs (bench.py,
    the tests, __graft_entry__): DEBUG_CLR_GRAPH_PACKET_CAPTURE=0, HIP's plain dispatch path for graph
    launches instead of its replay of pre-captured AQL packets, which costs this engine's two-kernel step
    graphs ~4 us more per graph launch (one MI355X, one step per graph launch: 8 192-env shard 134 -> 144 M
    env-steps/s with it off, C2 86 -> 94 M, the caller's policy at the shard 110 -> 117 M; C3 / C4 / C5 even;
    profiles/r05b_env_ab.log).  The runtime reads it when it initialises, so call this before the process's
    first HIP call; it changes how every hipGraph of the process is launched (torch.cuda graphs included),
    which is why importing the package does not set it.  A value the caller already set wins.  Also:
    ZS_PLAIN_GRAPH_DISPATCH=1 in the environment makes the import call it."""
    _os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")


if _os.environ.get("ZS_PLAIN_GRAPH_DISPATCH") == "1":
    plain_graph_dispatch()
