"""Per-phase profile of the benchmark workload from the scheduler's own
Chrome trace (csrc/scheduler/trace.cc): queue wait, snapshot, filter,
schedule (whole algorithm), permit wait and bind, averaged per pod, plus the
wall-clock pods/s of the traced waves and the equivalence-cache hit rate.

    python -m flex_gpu_scheduler_amd.tools.phase_profile [--nodes 64] [--waves 6] [--options JSON]
"""
from __future__ import annotations

import argparse
import collections
import json
import time

from ..utils.benchrun import Shard
from ..utils.workload import ClusterSpec


def profile(nodes: int = 64, waves: int = 6, warmup: int = 2, options: dict | None = None) -> dict:
    sh = Shard(ClusterSpec(nodes=nodes), seed=0, options=options or {})
    try:
        ws = [sh.wave(i) for i in range(warmup + waves)]
        prep = [(w.groups_json(), w.pods_json()) for w in ws]
        for i in range(warmup):
            sh.run(ws[i], prepared=prep[i])
        sh.sched.set_trace(True)
        t0 = time.perf_counter()
        results = [sh.run(ws[i], prepared=prep[i]) for i in range(warmup, warmup + waves)]
        wall = time.perf_counter() - t0
        pods = sum(r.pods for r in results)
        split = {k: round(sum(r.split_ms[k] for r in results) / len(results), 3) for k in results[0].split_ms}
        tr = json.loads(sh.sched.trace_json())
        events = tr["traceEvents"] if isinstance(tr, dict) else tr
        agg: dict[str, list[float]] = collections.defaultdict(lambda: [0, 0.0])
        for e in events:
            if e.get("ph") == "X":
                agg[e["name"]][0] += 1
                agg[e["name"]][1] += float(e.get("dur", 0))
        st = sh.sched.stats()
        totals_ms = {k: round(d / 1e3 / waves, 3) for k, (c, d) in sorted(agg.items()) if k != "queue_wait"}
        return {
            "pods": pods, "wall_ms": round(wall * 1e3, 2), "pods_per_s": round(pods / wall, 1),
            "wall_us_per_pod": round(wall * 1e6 / max(1, pods), 2),
            "step_split_ms": split,
            "phases_us_per_pod": {k: round(d / max(1, c), 2) for k, (c, d) in sorted(agg.items())},
            "phase_totals_ms_per_wave": totals_ms,
            "eq_filter_hit_rate": round(st["eq_filter_hits"] / max(1, st["eq_filter_hits"] + st["eq_filter_misses"]), 3),
            "options": options or {},
        }
    finally:
        sh.close()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--waves", type=int, default=6)
    ap.add_argument("--options", default="{}")
    a = ap.parse_args()
    print(json.dumps(profile(a.nodes, a.waves, options=json.loads(a.options))))


if __name__ == "__main__":
    main()
