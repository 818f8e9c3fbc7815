"""RCCL-over-xGMI placement probe.

The scheduler's promise for a gang placed on one 8x MI355X node is that every
ring hop of the job's all-reduce rides xGMI (7 links x ~153 GB/s per GPU,
full mesh). This probe measures that: one process per GPU (torch.distributed
backend "nccl" = RCCL on ROCm), all-reduce over a size sweep, reporting
algorithm and bus bandwidth (busBW = algBW * 2(n-1)/n, the nccl-tests
convention). Run it on the ranks a PodGroup was placed on to validate the
placement (SURVEY.md §2.4 "xGMI placement probe").
"""
from __future__ import annotations

import time
from dataclasses import dataclass


@dataclass
class AllReduceResult:
    bytes: int
    ms: float
    algbw_gbps: float
    busbw_gbps: float


def allreduce_sweep(sizes_bytes=(1 << 20, 16 << 20, 128 << 20), iters: int = 10, warmup: int = 3,
                    dtype: str = "bfloat16") -> list[AllReduceResult]:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialized")
    n = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dt = getattr(torch, dtype) if dev.type == "cuda" else torch.float32
    esize = torch.tensor([], dtype=dt).element_size()
    out = []
    for nbytes in sizes_bytes:
        x = torch.ones(max(1, nbytes // esize), dtype=dt, device=dev)
        for _ in range(warmup):
            dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / iters
        alg = x.numel() * esize / t / 1e9
        out.append(AllReduceResult(x.numel() * esize, t * 1e3, alg, alg * 2 * (n - 1) / n if n > 1 else alg))
    return out
