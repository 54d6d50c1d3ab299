"""sentinel_amd — MI355X-native batch flow-check engine for Sentinel's
statistics-and-check hot path (LeapArray windows, FlowRule controllers,
ParamFlowRule, cluster TokenService).

``sentinel_amd.abi``      ctypes mirror of include/sentinel_flow.h (no GPU needed)
``sentinel_amd.engine``   the HIP engine behind the C-ABI (libsentinel_flow.so)
``sentinel_amd.rules``    FlowRuleManager / ParamFlowRuleManager host mirrors
``sentinel_amd.trace``    seeded synthetic traces for the BASELINE configs
"""
__version__ = "0.1.0"
