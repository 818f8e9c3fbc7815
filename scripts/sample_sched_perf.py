"""One scheduler_perf workload (tools/sched_perf.py) under the timestamped
sampler: OUTDIR/<name>.samples for tools/sample_report.py.

    python scripts/sample_sched_perf.py OUTDIR CapacityScheduling-Reclaim --nodes 5000 --pods 1000
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from flex_gpu_scheduler_amd._native import native  # noqa: E402
from flex_gpu_scheduler_amd.tools.sched_perf import WORKLOADS, run_spec  # noqa: E402
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("workload")
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--hz", type=int, default=2000)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    apply("l3")
    spec = WORKLOADS[a.workload](a.nodes, a.pods)
    native().sampler_start(a.hz, 8_000_000)
    r = run_spec(spec)
    native().sampler_dump(os.path.join(a.out, f"{a.workload}.samples"))
    print(json.dumps(r))
    return 0


if __name__ == "__main__":
    sys.exit(main())
