"""Distributed pieces: one process per GPU over torch.distributed (RCCL on
ROCm) — the RCCL/xGMI placement probe and sharded benchmark coordination."""
from .dist import DistContext, init_distributed  # noqa: F401
