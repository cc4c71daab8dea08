"""marllb_amd — MI355X-native vectorised load-balancing RL environment (lbsim).

The hot path of the MARLLB reference (problem-03 LoadBalanceEnv.step/reset + problem-01 reservoir
feature collector) as hand-written gfx950 HIP kernels behind a C ABI (include/lbsim.h,
liblbsim.so), with the reference's Gym-style API on top.
"""
from .env import FEATURE_NAMES, LoadBalanceEnv, LoadBalanceEnvGym, VecLoadBalanceEnv, make_config
from .multi_agent import MultiAgentLoadBalanceEnv, VecMultiAgentLoadBalanceEnv
from .spaces import Box, MultiDiscrete

__all__ = ["FEATURE_NAMES", "LoadBalanceEnv", "LoadBalanceEnvGym", "VecLoadBalanceEnv",
           "MultiAgentLoadBalanceEnv", "VecMultiAgentLoadBalanceEnv", "make_config", "Box",
           "MultiDiscrete"]
__version__ = "0.1.0"
