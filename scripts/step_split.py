"""Where a bench step's wall clock goes: mean create / to-bound / delete+drain
split (ms) over the same waves bench.py times, plus the scheduler's counters.
Usage: python scripts/step_split.py [--nodes 64] [--steps 40] [--warmup 5]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flex_gpu_scheduler_amd.utils.benchrun import Shard  # noqa: E402
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nodes", type=int, default=64)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--options", default="{}")
ap.add_argument("--cpus", default="l3")
a = ap.parse_args()
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply as pin_cpus, ranked_domains  # noqa: E402

pin_cpus(a.cpus, 0, order=ranked_domains() if a.cpus.startswith("l3") else None)
sh = Shard(ClusterSpec(nodes=a.nodes), namespace="split", seed=0, options=json.loads(a.options))
waves = [sh.wave(i) for i in range(a.warmup + a.steps)]
prep = [(w.groups_json(), w.pods_json()) for w in waves]
for i in range(a.warmup):
    sh.run(waves[i], prepared=prep[i])
split: dict[str, list[float]] = {}
t0 = time.perf_counter()
pods = 0
for i in range(a.warmup, a.warmup + a.steps):
    r = sh.run(waves[i], prepared=prep[i])
    pods += r.pods
    for k, v in r.split_ms.items():
        split.setdefault(k, []).append(v)
el = time.perf_counter() - t0
sh.close()
print(json.dumps({"pods_per_s": round(pods / el, 1), "pods_per_step": pods // a.steps,
                  "ms_per_step": round(el * 1e3 / a.steps, 3),
                  "split_ms_mean": {k: round(sum(v) / len(v), 3) for k, v in split.items()},
                  "split_ms_min": {k: round(min(v), 3) for k, v in split.items()}}))
