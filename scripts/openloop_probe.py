"""Open-loop admission at a ladder of offered rates on one bench shard (64
nodes, pinned to one L3 domain like bench.py): per rate the wall time, hold,
mean arrival lag of the driver, p99 PG-create -> last-Bind per gang type,
unbound gangs and the scheduler's unschedulable attempts. Shows where and how
the open-loop capacity ends.

Usage: python scripts/openloop_probe.py [--rates 20000,27000,35000] [--seconds 1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply as pin_cpus, ranked_domains  # noqa: E402
from flex_gpu_scheduler_amd.utils.benchrun import Shard  # noqa: E402
from flex_gpu_scheduler_amd.utils.openloop import run_open_loop  # noqa: E402
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rates", default="10000,20000,27000,35000,45000")
ap.add_argument("--seconds", type=float, default=1.0)
ap.add_argument("--nodes", type=int, default=64)
ap.add_argument("--occupancy", type=float, default=0.5)
ap.add_argument("--cpus", default="l3")
ap.add_argument("--options", default="{}")
ap.add_argument("--trace", default="", help="write the scheduler's Chrome trace here (with options trace=true)")
a = ap.parse_args()


def thread_sched() -> dict:
    """Per thread role: CPU time, run-queue wait (runnable, not running) and
    involuntary context switches, from /proc/self/task/*/{schedstat,status}."""
    out: dict = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            base = f"/proc/self/task/{tid}"
            comm = open(f"{base}/comm").read().strip().rstrip("0123456789")
            run_ns, wait_ns, _ = (int(x) for x in open(f"{base}/schedstat").read().split())
            inv = next(int(line.split()[1]) for line in open(f"{base}/status")
                       if line.startswith("nonvoluntary_ctxt_switches"))
        except (OSError, ValueError, StopIteration):
            continue
        r = out.setdefault(comm, [0, 0, 0])
        r[0] += run_ns
        r[1] += wait_ns
        r[2] += inv
    return out


def sched_delta(a0: dict, a1: dict) -> dict:
    return {k: {"cpu_ms": round((v[0] - a0.get(k, [0, 0, 0])[0]) / 1e6, 1),
                "runqueue_wait_ms": round((v[1] - a0.get(k, [0, 0, 0])[1]) / 1e6, 1),
                "involuntary_switches": v[2] - a0.get(k, [0, 0, 0])[2]} for k, v in a1.items()}


pin_cpus(a.cpus, 0, order=ranked_domains() if a.cpus.startswith("l3") else None)
sh = Shard(ClusterSpec(nodes=a.nodes), namespace="olp", seed=0, options=json.loads(a.options))
try:
    for rate in (float(x) for x in a.rates.split(",")):
        s0 = sh.sched.stats()
        ts0 = thread_sched()
        r = run_open_loop(sh, rate, a.seconds, seed=0, occupancy=a.occupancy, timeline=True)
        s1 = sh.sched.stats()
        threads = sched_delta(ts0, thread_sched())
        # Why attempts failed: FailedScheduling events of this rate, by message.
        events, _ = sh.store.list("events", "openloop")
        why: dict[str, int] = {}
        for e in events:
            if e.get("reason") == "FailedScheduling":
                m = e.get("message", "")[:200]
                why[m] = why.get(m, 0) + int(e.get("count", 1))
        # Every gang is deleted by now: the cache must be empty and its
        # accounting consistent (cache debugger), else something leaked.
        drained = sh.sched.wait_cache_empty(5.0)
        chk = sh.sched.check_cache()
        fails = sorted((int(e["metadata"]["resourceVersion"]), e.get("message", "")[:300])
                       for e in events if e.get("reason") == "FailedScheduling")
        sh.store.delete_all("events", "openloop")
        print(json.dumps({
            "offered_pods_per_s": rate, "wall_s": r["wall_s"], "hold_ms": r["hold_ms"],
            "mean_arrival_lag_us": r.get("mean_arrival_lag_us"), "mean_delete_lag_us": r.get("mean_delete_lag_us"),
            "max_in_flight_pods": r.get("max_in_flight_pods"), "max_held_pods": r.get("max_held_pods"),
            "p99_create_to_bound_ms": {k: v["create_to_bound_ms"]["p99"] for k, v in r["by_gang"].items()},
            "p50_create_to_bound_ms": {k: v["create_to_bound_ms"]["p50"] for k, v in r["by_gang"].items()},
            "unbound": sum(v["unbound"] for v in r["by_gang"].values()),
            "unschedulable_attempts": s1["unschedulable"] - s0["unschedulable"],
            "attempts": s1["attempts"] - s0["attempts"],
            "first_failures": [m for _, m in fails[:3]],
            "threads": threads,
            "timeline_5ms": r.get("timeline"),
            "cache_drained": drained, "cache_clean": chk.get("clean"),
            "accounting_mismatches": len(chk.get("accounting", [])),
            "failed_scheduling": dict(sorted(why.items(), key=lambda kv: -kv[1])[:8])}), flush=True)
finally:
    if a.trace:
        with open(a.trace, "w") as f:
            f.write(sh.sched.trace_json())
    sh.close()
