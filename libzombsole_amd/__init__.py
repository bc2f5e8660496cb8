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
