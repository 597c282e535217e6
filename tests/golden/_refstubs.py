"""Offline stand-ins for the reference's three missing third-party imports.

Used ONLY by ``gen_golden.py`` (run in the build container, never on the GPU box)
to import the read-only reference at /root/reference and record golden vectors.
The stubs carry plumbing only (agent registry, name property, exception type);
every line of hot-path arithmetic that produces the golden vectors is the
reference's own code. Mirrors the stub list recorded in SURVEY.md §8(c).
"""
import sys
import types


def install():
    if "unified_planning" in sys.modules and getattr(sys.modules["unified_planning"], "_rmx_stub", False):
        return

    pz = types.ModuleType("pettingzoo")

    class ParallelEnv:  # noqa: D401 - stub
        def __init__(self, *a, **k):
            pass

    pz.ParallelEnv = ParallelEnv

    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Discrete:
        def __init__(self, n, *a, **k):
            self.n = n

    class MultiDiscrete:
        def __init__(self, nvec, *a, **k):
            self.nvec = nvec

    spaces.Discrete = Discrete
    spaces.MultiDiscrete = MultiDiscrete
    gym.spaces = spaces

    up = types.ModuleType("unified_planning")
    up._rmx_stub = True
    shortcuts = types.ModuleType("unified_planning.shortcuts")
    shortcuts.__all__ = []
    model = types.ModuleType("unified_planning.model")
    ma = types.ModuleType("unified_planning.model.multi_agent")
    exc = types.ModuleType("unified_planning.exceptions")

    class UPValueError(ValueError):
        pass

    class MultiAgentProblem:
        def __init__(self, *a, **k):
            self._agents = []

        @property
        def agents(self):
            return self._agents

        def add_agent(self, agent):
            if any(a.name == agent.name for a in self._agents):
                raise UPValueError(f"duplicate agent {agent.name}")
            self._agents.append(agent)

    class Agent:
        def __init__(self, name, ma_problem=None):
            self._name = name

        @property
        def name(self):
            return self._name

        @name.setter
        def name(self, v):
            self._name = v

    ma.MultiAgentProblem = MultiAgentProblem
    ma.Agent = Agent
    ma.__all__ = ["MultiAgentProblem", "Agent"]
    exc.UPValueError = UPValueError
    up.shortcuts = shortcuts
    up.model = model
    up.exceptions = exc
    model.multi_agent = ma

    for name, mod in {
        "pettingzoo": pz,
        "gymnasium": gym,
        "gymnasium.spaces": spaces,
        "unified_planning": up,
        "unified_planning.shortcuts": shortcuts,
        "unified_planning.model": model,
        "unified_planning.model.multi_agent": ma,
        "unified_planning.exceptions": exc,
    }.items():
        sys.modules[name] = mod
