"""Debug: compare k_reset's world against the oracle for a few seeds (prints entity tables)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from libzombsole_amd import _abi
from libzombsole_amd.engine import Engine
from oracle.oracle import OracleEnv

def mk(n):
    return _abi.multi_env_config(n, "extermination", [], sys.argv[1] if len(sys.argv) > 1 else "boxed",
                                 ["0", "1"], initial_zombies=int(sys.argv[2]) if len(sys.argv) > 2 else 1)
seeds = [9, 10, 11, 12]
eng = Engine(mk(len(seeds)))
eng.seed(seeds)
eng.reset()
torch.cuda.synchronize()
kinds = [o[2] for o in eng.builder.map.obstacles]
for k, s in enumerate(seeds):
    o = OracleEnv(mk(1)); o.seed(s); o.reset()
    st = eng.get_state(k)
    print("seed", s, "engine", st.canonical(kinds)["dyn"])
    print("seed", s, "oracle", o.state()["dyn"])
    print("   ent raw", st.ent.tolist())
