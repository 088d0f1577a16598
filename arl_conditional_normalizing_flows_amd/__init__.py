"""MI355X-native (gfx950) conditional RealNVP hot path — drop-in for the
`conv_cINN_make_model` layer/model API of USArmyResearchLab/ARL_Conditional_Normalizing_Flows.

    from arl_conditional_normalizing_flows_amd.make_model import cFlow

The compute runs in libcnf_hip.so (hand-written HIP kernels, C ABI in include/cnf.h).
"""
from .config import FlowConfig, PRESETS  # noqa: F401

__all__ = ['FlowConfig', 'PRESETS', 'make_model']
