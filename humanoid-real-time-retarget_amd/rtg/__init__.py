"""rtg -- MI355X-native runtime of the retargeting hot path (host side).

``rtg._lib`` binds librtg_hip.so (include/rtg.h); ``rtg.runtime`` holds the
device-side Topology / Solver handles; ``rtg.ops`` exposes batched device ops;
``rtg.assets`` / ``rtg.synth`` provide the zero poses and synthetic mocap.
"""
__version__ = "0.1.0"
