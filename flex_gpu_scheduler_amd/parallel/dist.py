"""torch.distributed bootstrap for one-process-per-GPU jobs.

Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as set by
`torch.distributed.run`; uses backend "nccl" (RCCL on ROCm) when GPUs are
visible and "gloo" otherwise (CPU tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class DistContext:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    backend: str = "none"
    cuda: bool = False

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    def barrier(self) -> None:
        if self.distributed:
            import torch.distributed as dist

            dist.barrier()

    def sync(self) -> None:
        if self.cuda:
            import torch

            torch.cuda.synchronize()

    def all_max(self, v: float) -> float:
        return self._reduce(v, "max")

    def all_sum(self, v: float) -> float:
        return self._reduce(v, "sum")

    def _reduce(self, v: float, op: str) -> float:
        if not self.distributed:
            return v
        import torch
        import torch.distributed as dist

        t = torch.tensor([float(v)], dtype=torch.float64, device="cuda" if self.cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return float(t.item())

    def gather(self, obj):
        if not self.distributed:
            return [obj]
        import torch.distributed as dist

        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def close(self) -> None:
        if self.distributed:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()


def init_distributed(want_cuda: bool = True) -> DistContext:
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    ctx = DistContext(rank=rank, local_rank=local, world_size=ws)
    cuda = False
    if want_cuda:
        try:
            import torch

            cuda = torch.cuda.is_available()
            if cuda:
                torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        except Exception:
            cuda = False
    ctx.cuda = cuda
    if ws > 1:
        import datetime

        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if cuda else "gloo"
        if cuda:
            # A collective that times out raises in the caller (instead of the
            # watchdog aborting the process), so a failed rank cannot hang the
            # job or kill the headline line of the others.
            os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        timeout = datetime.timedelta(seconds=float(os.environ.get("XSCHED_DIST_TIMEOUT_S", "300")))
        dist.init_process_group(backend=backend, rank=rank, world_size=ws, timeout=timeout)
        ctx.backend = backend
    return ctx
