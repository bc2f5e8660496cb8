#!/usr/bin/env python3
"""Golden transcripts of the reference's JSON-over-stdio server (this container only).

Runs the REAL `zombsole/interactive_json.py` GymEnvManager (imported read-only, with the no-op
shims of ./shims plus an in-memory `docopt` stub, all absent from this image and none touching
game arithmetic) on scripted request sessions and records every response line it prints.  Two
changes to the reference's behaviour, both outside the game: `render()` is replaced by a no-op
(the reference's render() raises NameError without a renderer, gym_env.py:207, which would end
every session at its first GameAction), and stdin is a scripted line list.  Nothing of the
reference is copied: only the transcripts are written, to tests/golden/stdio_*.json.gz.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_stdio_golden.py
"""
import contextlib
import gzip
import io
import json
import os
import random
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "shims"))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

sys.modules.setdefault("docopt", types.SimpleNamespace(docopt=lambda doc, argv=None: {}))

from stdio_sessions import SESSIONS  # noqa: E402

import zombsole.interactive_json as ij  # noqa: E402
from zombsole.gym_env import ZombsoleGymEnv  # noqa: E402
from zombsole.gym.multiagent_env import MultiagentZombsoleEnv  # noqa: E402

ZombsoleGymEnv.render = lambda self: None
MultiagentZombsoleEnv.render = lambda self: None


def run_session(sess):
    lines = list(sess["requests"])

    def fake_input(prompt=""):
        if not lines:
            raise EOFError("EOF when reading a line")
        return lines.pop(0)

    out = io.StringIO()
    random.seed(sess["seed"])
    err = None
    ij.input = fake_input  # the module's global lookup of input()
    try:
        with contextlib.redirect_stdout(out):
            ij.GymEnvManager(None, sess["multi"]).run()
    except Exception as ex:  # the reference's server ends on these (recorded, not hidden)
        err = type(ex).__name__
    finally:
        del ij.input
    return {"name": sess["name"], "multi": sess["multi"], "seed": sess["seed"], "requests": sess["requests"],
            "responses": out.getvalue().splitlines(), "exception": err}


def main():
    for sess in SESSIONS:
        rec = run_session(sess)
        path = os.path.join(HERE, "stdio_%s.json.gz" % sess["name"])
        with gzip.open(path, "wt", encoding="utf-8") as f:
            json.dump(rec, f, separators=(",", ":"))
        print("%-28s %3d responses  exception=%s  %7d bytes" % (sess["name"], len(rec["responses"]), rec["exception"],
                                                                 os.path.getsize(path)))


if __name__ == "__main__":
    main()
