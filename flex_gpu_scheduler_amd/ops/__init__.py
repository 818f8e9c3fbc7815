"""GPU-side operations: HIP/CDNA4 probes (HBM bandwidth, XCD census, health).

The scheduler's own hot path is host code (C++); the GPU is exercised where
the scheduler's promises meet hardware — partition bandwidth, device health,
and (in parallel/) RCCL placement validation.
"""
from .hip_probe import Bandwidth, HipProbe, ProbeError, probe  # noqa: F401
