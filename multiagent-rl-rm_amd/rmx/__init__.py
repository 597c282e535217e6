"""rmx — MI355X-native vectorised multi-agent grid-world + Reward-Machine step engine.

Drop-in replacement for the hot path of Alee08/multiagent-rl-rm:
``RMEnvironmentWrapper.step`` over ``MultiAgentFrozenLake`` / ``MultiAgentOfficeWorld`` with the
``RewardMachine`` transition/reward lookup, batched over thousands of (env, agent) instances as
hand-written HIP kernels for gfx950 behind the C ABI of ``include/rmx.h``.

* ``rmx.tables``  — host table compiler (maps, walls, RM indices, final state, shaping potentials)
* ``rmx.engine``  — ``VecRMEnv``: batched device engine over the C ABI (torch tensors as buffers)
* ``rmx.compat``  — reference-shaped dict API (``RMEnvironmentWrapper``-style reset/step)
* ``rmx.dist``    — one-process-per-GPU env sharding + RCCL all-reduce of episode statistics
"""
__version__ = "0.1.0"

from .tables import (  # noqa: F401
    FROZEN_LAKE, OFFICE_WORLD, RewardMachineSpec, CompiledTables, compile_tables, compile_scenario,
    baseline_scenario, parse_map_emoji, parse_office_world, find_disconnected_pairs,
)


def __getattr__(name):  # lazy: the engine needs torch + the HIP library, the table compiler does not
    if name in ("VecRMEnv",):
        from .engine import VecRMEnv
        return VecRMEnv
    raise AttributeError(name)
