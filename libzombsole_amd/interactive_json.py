"""JSON over stdio on top of the MI355X engine (the reference's ``zombsole-stdio-json``).

Restates the request/response protocol of ``zombsole/interactive_json.py`` (SURVEY.md §8(f)
rank 4) over this package's drop-in envs, so an external-language client that drives the
reference through this protocol can be pointed at this server unchanged.  One JSON object per
line in each direction:

requests (``GameRequest.decode_hook``, interactive_json.py:130-149)
    ``{"tag": "GameConfigUpdate", "parameters": {GameConfig fields}}``
    ``{"tag": "GameStatus"}``  ``{"tag": "StartGame"}``  ``{"tag": "Exit"}``
    ``{"tag": "GameAction", "parameters": <action for env.step>}``
responses (interactive_json.py:27-89)
    ``{"tag": "GameState", "parameters": {"status", "active", "config_required", "last_observation"}}``
    ``{"tag": "GameObservation", "parameters": {"observation", "reward", "done", "truncated", "info"}}``
    ``{"tag": "Error", "parameters": "<message>"}``

Behaviour kept from the reference, quirks included, because a client may depend on them:
the status strings ``"wating for game"`` / ``"exiting"`` and a null status while a game is in
progress (``_env_status`` falls off its end, interactive_json.py:237-243); a request without a
``"tag"`` decodes to a plain dict and ends the server with ``AttributeError``
(interactive_json.py:148-149, 264); ``StartGame`` or ``GameAction`` before any config ends it
with ``AttributeError`` on ``None``; errors raised inside ``env.step`` propagate.

One deliberate divergence: the reference calls ``gym_env.render()`` after every
step (interactive_json.py:332), which without a renderer raises ``NameError`` (gym_env.py:207
formats an undefined ``mode``), so its server dies on the first ``GameAction`` unless run with
``-r opencv``.  Rendering is out of scope here; this server calls ``render()`` only when a
render mode was asked for (and that raises ``NotImplementedError``).
"""
import argparse
import json
import sys
from abc import ABC, abstractmethod
from json import JSONEncoder
from typing import Dict, Union

__all__ = ["GameResponse", "GameStateEncoder", "GameStateResponse", "GameObservationResponse",
           "ErrorResponse", "GameConfig", "GameManagementInterface", "GameRequest",
           "GameConfigUpdateRequest", "GameStatusRequest", "ExitRequest", "StartGameRequest",
           "GameActionRequest", "GymEnvManager", "play_interactive_json"]


class GameResponse(ABC):
    """interactive_json.py:27-40."""

    def to_dict(self) -> Dict:
        return {"tag": self.get_tag(), "parameters": self.get_parameters()}

    @abstractmethod
    def get_tag(self) -> str:
        pass

    @abstractmethod
    def get_parameters(self) -> Dict:
        pass


class GameStateEncoder(JSONEncoder):
    """interactive_json.py:42-51: responses encode through their to_dict()."""

    def default(self, o):
        to_dict = getattr(o, "to_dict", None)
        if to_dict is not None:
            try:
                return to_dict()
            except TypeError:
                pass
        return super().default(o)


class GameStateResponse(GameResponse):
    """interactive_json.py:53-69."""

    def __init__(self, status, active: bool, config_required: bool, last_observation: Union[None, Dict] = None):
        self.status = status
        self.active = active
        self.config_required = config_required
        self.last_observation = last_observation

    def get_tag(self) -> str:
        return "GameState"

    def get_parameters(self) -> Dict:
        return {"status": self.status, "active": self.active, "config_required": self.config_required,
                "last_observation": self.last_observation}


class GameObservationResponse(GameResponse):
    """interactive_json.py:71-79."""

    def __init__(self, last_observation: Dict = None):
        self.last_observation = last_observation

    def get_tag(self) -> str:
        return "GameObservation"

    def get_parameters(self) -> Dict:
        return self.last_observation


class ErrorResponse(GameResponse):
    """interactive_json.py:81-89."""

    def __init__(self, message: str):
        self.message = message

    def get_tag(self) -> str:
        return "Error"

    def get_parameters(self):
        return self.message


class GameConfig(object):
    """interactive_json.py:91-107.  Unknown or missing keys raise TypeError from the
    constructor, which the request loop reports as an Error response."""

    def __init__(self, rules_name: str, map_name: str, players, agent_ids, initial_zombies=10, minimum_zombies=10,
                 observation_scope="world", observation_position_encoding="simple"):
        self.rules_name = rules_name
        self.map_name = map_name
        self.players = players
        self.agent_ids = agent_ids
        self.initial_zombies = initial_zombies
        self.minimum_zombies = minimum_zombies
        self.observation_scope = observation_scope
        self.observation_position_encoding = observation_position_encoding

    @classmethod
    def from_dict(cls, d):
        return cls(**d)


class GameManagementInterface(ABC):
    """interactive_json.py:109-128."""

    @abstractmethod
    def set_game_config(self, game_config: GameConfig):
        pass

    @abstractmethod
    def get_game_status(self):
        pass

    @abstractmethod
    def start_game(self):
        pass

    @abstractmethod
    def step_with_agent_action(self, action: Dict):
        pass

    @abstractmethod
    def exit(self):
        pass


_TAGS = ("GameConfigUpdate", "GameAction", "GameStatus", "StartGame", "Exit")


class GameRequest(ABC):
    """interactive_json.py:130-153."""

    @staticmethod
    def decode_hook(jsonobj):
        if "tag" not in jsonobj:  # nested objects (parameters) pass through unchanged
            return jsonobj
        tag = jsonobj["tag"]
        if tag in ("GameConfigUpdate", "GameAction") and "parameters" not in jsonobj:
            raise ValueError(f"A GameRequest with tag {tag} must have key \"parameters\"")
        if tag == "GameConfigUpdate":
            return GameConfigUpdateRequest.from_dict(jsonobj["parameters"])
        if tag == "GameStatus":
            return GameStatusRequest()
        if tag == "Exit":
            return ExitRequest()
        if tag == "StartGame":
            return StartGameRequest()
        if tag == "GameAction":
            return GameActionRequest(jsonobj["parameters"])
        raise ValueError("GameRequest \"tag\" must be \"GameConfigUpdate\", \"GameAction\", \"GameStatus\", "
                         "\"StartGame\", or \"Exit\"")

    @abstractmethod
    def update_game_manager(self, game_manager):
        pass


class GameConfigUpdateRequest(GameRequest):
    def __init__(self, game_config: GameConfig):
        self.game_config = game_config

    @classmethod
    def from_dict(cls, game_config_obj: Dict):
        return cls(GameConfig.from_dict(game_config_obj))

    def update_game_manager(self, game_manager: GameManagementInterface):
        game_manager.set_game_config(self.game_config)


class GameStatusRequest(GameRequest):
    def update_game_manager(self, game_manager: GameManagementInterface):
        game_manager.get_game_status()


class ExitRequest(object):
    def update_game_manager(self, game_manager: GameManagementInterface):
        game_manager.exit()


class StartGameRequest(object):
    def update_game_manager(self, game_manager: GameManagementInterface):
        game_manager.start_game()


class GameActionRequest(object):
    def __init__(self, action: Dict):
        self.action = action

    def update_game_manager(self, game_manager: GameManagementInterface):
        game_manager.step_with_agent_action(self.action)


def _default_single(*args, **kwargs):
    from .gym_env import ZombsoleGymEnv
    return ZombsoleGymEnv(*args, **kwargs)


def _default_multi(*args, **kwargs):
    from .gym.multiagent_env import MultiagentZombsoleEnv
    return MultiagentZombsoleEnv(*args, **kwargs)


class GymEnvManager(GameManagementInterface):
    """The stdio game manager (interactive_json.py:195-344) over the engine's drop-in envs.

    ``stdin``/``stdout`` default to the process streams; ``single_env``/``multi_env`` are the
    env constructors (the engine-backed drop-ins by default) and exist so the protocol layer
    can be exercised without a GPU."""

    def __init__(self, render_mode: str, use_multiagent_env: bool, stdin=None, stdout=None,
                 single_env=None, multi_env=None):
        self.game_config = None
        self.gym_env = None
        self.keep_going = True
        self.last_observation = None
        self.response_encoder = GameStateEncoder(indent=None)
        self.render_mode = render_mode
        self.use_multiagent_env = use_multiagent_env
        self._stdin = stdin
        self._stdout = stdout
        self._single_env = single_env or _default_single
        self._multi_env = multi_env or _default_multi

    def _initialize_gym(self):
        cfg = self.game_config
        if cfg is None:
            return
        if self.gym_env is not None:  # release the previous game's device state
            close = getattr(self.gym_env, "close", None)
            self.gym_env = None
            if close is not None:
                close()
        if self.use_multiagent_env:
            scope = cfg.observation_scope
            swidth = int(scope[len("surroundings:"):]) if scope.startswith("surroundings:") else 21
            self.gym_env = self._multi_env(cfg.rules_name, cfg.players, cfg.map_name, cfg.agent_ids,
                                           initial_zombies=cfg.initial_zombies,
                                           minimum_zombies=cfg.minimum_zombies,
                                           observation_surroundings_width=swidth,
                                           render_mode=self.render_mode, debug=False)
        else:
            self.gym_env = self._single_env(cfg.rules_name, cfg.players, cfg.map_name, cfg.agent_ids[0],
                                            initial_zombies=cfg.initial_zombies,
                                            minimum_zombies=cfg.minimum_zombies,
                                            observation_scope=cfg.observation_scope,
                                            observation_position_encoding=cfg.observation_position_encoding,
                                            render_mode=self.render_mode, debug=False)
        self.last_observation = None

    def _env_status(self):
        if not self.keep_going:
            return "exiting"
        if self.last_observation is None:
            return "wating for game"
        return None  # the reference's "game in progress" branch returns nothing

    def _get_game_state(self):
        return GameStateResponse(self._env_status(), self.keep_going, self.game_config is None,
                                 self.last_observation)

    def _respond(self, response):
        out = self._stdout if self._stdout is not None else sys.stdout
        out.write(self.response_encoder.encode(response.to_dict()) + "\n")
        out.flush()

    def _readline(self):
        if self._stdin is None:
            return input()
        line = self._stdin.readline()
        if not line:
            raise EOFError("EOF when reading a line")
        return line.rstrip("\n")

    def run(self):
        self._respond(self._get_game_state())
        while self.keep_going:
            message = self._readline()
            try:
                obj = json.loads(message, object_hook=GameRequest.decode_hook)
            except Exception as ex:
                self._respond(ErrorResponse(str(ex)))
            else:
                obj.update_game_manager(self)

    def set_game_config(self, game_config: GameConfig):
        self.game_config = game_config
        self._initialize_gym()
        self._respond(self._get_game_state())

    def get_game_status(self):
        self._respond(self._get_game_state())

    def _observation_json_ready(self, observation):
        if self.use_multiagent_env:
            return {agent_id: observation[agent_id].tolist() for agent_id in observation}
        return observation.tolist()

    def _initial_values(self):
        if self.use_multiagent_env:
            ids = self.gym_env.possible_agents
            return ({a: 0 for a in ids}, {a: False for a in ids}, {a: False for a in ids}, {})
        return 0, False, False, None

    def start_game(self):
        origobs, _ = self.gym_env.reset()
        reward, done, truncated, info = self._initial_values()
        self.last_observation = {"observation": self._observation_json_ready(origobs), "reward": reward,
                                 "done": done, "truncated": truncated, "info": info}
        self._respond(GameObservationResponse(self.last_observation))

    def step_with_agent_action(self, action: Dict):
        observation, reward, done, truncated, info = self.gym_env.step(action)
        self.last_observation = {"observation": self._observation_json_ready(observation), "reward": reward,
                                 "done": done, "truncated": truncated, "info": info}
        if self.render_mode is not None:
            self.gym_env.render()
        self._respond(GameObservationResponse(self.last_observation))

    def exit(self):
        self.keep_going = False
        self._respond(self._get_game_state())


def play_interactive_json(argv=None):
    """``zombsole-stdio-json [-r RENDERER] [--multi-agent]`` (interactive_json.py:346-359)."""
    p = argparse.ArgumentParser(prog="zombsole-stdio-json",
                                description="Play Zombsole interactively using JSON over stdio")
    p.add_argument("-r", dest="renderer", default="none", help="The renderer to use, either opencv or none")
    p.add_argument("-m", "--multi-agent", action="store_true", help="Play Multi-Agent Zombsole")
    args = p.parse_args(argv)
    if args.renderer not in ("opencv", "none"):
        print("When using interactive JSON mode, renderer_id must be one of \"opencv\" or \"none\".  Exiting...",
              file=sys.stderr)
        sys.exit(1)
    render_mode = "human" if args.renderer == "opencv" else None
    GymEnvManager(render_mode, args.multi_agent).run()


if __name__ == "__main__":
    play_interactive_json()
