"""Scheduling-thread timeline of one benchmark wave, from the scheduler's
Chrome trace: when the first and last cycles ran relative to the wave's
first informer batch, how much of that span the scheduling thread was busy
(algorithm + assume/reserve/permit) and the largest idle gaps. Shows whether
a wave is bound by the scheduling thread or by what feeds it.

    python -m flex_gpu_scheduler_amd.tools.timeline [--nodes 64] [--warmup 4] [--cpus l3]
"""
from __future__ import annotations

import argparse
import collections
import json

from ..utils.benchrun import Shard
from ..utils.cpuaffinity import apply as pin_cpus
from ..utils.workload import ClusterSpec


def timeline(nodes: int = 64, warmup: int = 4) -> dict:
    sh = Shard(ClusterSpec(nodes=nodes), seed=0)
    try:
        ws = [sh.wave(i) for i in range(warmup + 1)]
        for i in range(warmup):
            sh.run(ws[i])
        sh.sched.set_trace(True)
        r = sh.run(ws[warmup])
        tr = json.loads(sh.sched.trace_json())
        ev = [e for e in (tr["traceEvents"] if isinstance(tr, dict) else tr) if e.get("ph") == "X"]
        by = collections.defaultdict(list)
        for e in ev:
            by[e["name"]].append(e)
        t0 = min(e["ts"] for e in ev)
        sched = sorted(by["schedule"], key=lambda e: e["ts"])
        first = sched[0]["ts"] - t0
        last_end = max(e["ts"] + e["dur"] for e in by["schedule"] + by["assume_reserve_permit"]) - t0
        ends = sorted((e["ts"], e["ts"] + e["dur"]) for e in by["schedule"] + by["assume_reserve_permit"])
        # Busy = union of the spans (trace timestamps are rounded to 1 us, so
        # adjacent spans can overlap by a tick and must not count twice).
        gaps = []
        cur = ends[0][1]
        busy = ends[0][1] - ends[0][0]
        for s, e in ends[1:]:
            if s > cur:
                gaps.append((s - cur, round((cur - t0) / 1e3, 3)))
            busy += max(0, e - max(s, cur))
            cur = max(cur, e)
        gaps.sort(reverse=True)
        span = last_end - first
        return {
            "pods": r.pods, "step_split_ms": {k: round(v, 3) for k, v in r.split_ms.items()},
            "first_cycle_ms": round(first / 1e3, 3), "last_cycle_end_ms": round(last_end / 1e3, 3),
            "sched_thread_busy_ms": round(busy / 1e3, 3), "sched_thread_span_ms": round(span / 1e3, 3),
            "busy_fraction": round(busy / max(1, span), 3),
            "idle_gaps_total_ms": round(sum(g for g, _ in gaps) / 1e3, 3),
            "largest_gaps_us_at_ms": gaps[:8],
            "informer_batches": [(round((e["ts"] - t0) / 1e3, 3), round(e["dur"] / 1e3, 3))
                                 for e in sorted(by["informer_batch"], key=lambda e: e["ts"])][:12],
        }
    finally:
        sh.close()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--cpus", default="l3")
    a = ap.parse_args()
    cpus = pin_cpus(a.cpus)
    out = timeline(a.nodes, a.warmup)
    out["cpus"] = len(cpus) if cpus else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
