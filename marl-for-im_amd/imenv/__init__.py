"""imenv — MI355X-native vectorised inventory-management environment.

Host side of the hot path: a HIP kernel library (csrc/: the step kernel body imenv_device.h,
ahead-of-time instantiations imenv_step_nt*.hip, the hipRTC specialiser imenv_jit.hip and the C ABI
imenv_capi.hip; declared in include/imenv.h) driven from Python. Public surface:

  build_spec(kind, config)      reference config dict -> HostSpec (spec.py)
  VectorInvEnv(kind, config, n) batched envs on one GPU (vector_env.py)
  InvManagement, MultiAgentInvManagement, InvManagementDiv,
  MultiAgentInvManagementDiv    drop-in single-env adaptors (envs.py)
  BaseStockRollout, dfo_func, base_stock_policy,
  optimize_inventory_policy     base-stock policy search on the GPU (policy.py,
                                base_restock_policy.py's interface)
  PlanRollout, replay_plans     the LP scripts' plan replay loop on the GPU (plan.py)

torch is imported lazily so that the spec builder works without a GPU stack.
"""
from .spec import HostSpec, SpecError, build_spec  # noqa: F401
from ._native import ImEnvNativeError  # noqa: F401


def __getattr__(name):
    if name == "VectorInvEnv":
        from .vector_env import VectorInvEnv
        return VectorInvEnv
    if name in ("InvManagement", "MultiAgentInvManagement", "InvManagementDiv", "MultiAgentInvManagementDiv"):
        from . import envs
        return getattr(envs, name)
    if name in ("BaseStockRollout", "dfo_func", "base_stock_policy", "optimize_inventory_policy",
                "evaluate_base_stock"):
        from . import policy
        return getattr(policy, name)
    if name in ("PlanRollout", "replay_plans"):
        from . import plan
        return getattr(plan, name)
    raise AttributeError(name)
