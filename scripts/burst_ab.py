"""Headline burst waves (bench.py's timed loop: Shard.run per wave) in a
fresh process, with or without torch and the GPU initialised first, to see
whether the GPU runtime in the process costs the scheduler throughput.

    python scripts/burst_ab.py [--torch] [--nodes 64] [--waves 160]

Prints one JSON line: pods/s over the timed waves.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--waves", type=int, default=160)
    ap.add_argument("--warmup", type=int, default=16)
    a = ap.parse_args()
    if a.torch:
        import torch

        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    from flex_gpu_scheduler_amd.utils.benchrun import Shard
    from flex_gpu_scheduler_amd.utils.cpuaffinity import apply
    from flex_gpu_scheduler_amd.utils.workload import ClusterSpec

    apply("l3")
    shard = Shard(ClusterSpec(nodes=a.nodes), namespace="burst", seed=0)
    try:
        ws = [shard.wave(i) for i in range(a.warmup + a.waves)]
        prepared = [w.chunks_json() for w in ws]
        for i in range(a.warmup):
            shard.run(ws[i], prepared=prepared[i], collect_gangs=False)
        t0 = time.perf_counter()
        pods = 0
        for i in range(a.warmup, a.warmup + a.waves):
            pods += shard.run(ws[i], prepared=prepared[i], collect_gangs=False).pods
        dt = time.perf_counter() - t0
    finally:
        shard.close()
    print(json.dumps({"torch": a.torch, "waves": a.waves, "pods": pods, "seconds": round(dt, 4),
                      "pods_per_s": round(pods / dt, 1)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
