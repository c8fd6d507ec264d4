"""gsamd — MI355X-native vectorized-rollout + GAE + PPO-update path for gymnasium-solver.

Host side of the drop-in: mirrors the reference's plugin surface (``build_agent``,
``BaseAgent`` hooks, ``losses_for_batch``, ``RolloutCollector``, ``MultiPassRandomSampler``)
and drives the C-ABI HIP library ``libgsamd.so`` (csrc/, declared in include/gsamd.h).
Submodules are imported lazily so that pure-host pieces (config, synthetic env) load
without the device library.
"""
__all__ = ["build_agent", "needs_host_env"]


def build_agent(config, *args, **kwargs):
    """Mirror of agents/__init__.py:1-8 for the device path (algo_id == "ppo")."""
    from .ppo_agent import build_agent as _build
    return _build(config, *args, **kwargs)


def needs_host_env(config) -> bool:
    """True when build_agent(config) needs env= (the env_id has no device dynamics)."""
    from .config import needs_host_env as _needs
    return _needs(config)
