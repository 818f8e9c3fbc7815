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
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--bench-sequence", type=float, default=0.0,
                help="first run bench.py's capacity search up to this burst rate (pods/s), then the rates")
ap.add_argument("--trace", default="", help="write the scheduler's Chrome trace here (with options trace=true)")
ap.add_argument("--sample-run", type=int, default=-1,
                help="wall-clock sample every thread during the rate of this index; dump to --sample")
ap.add_argument("--sample", default="/tmp/olp.samples")
ap.add_argument("--sample-hz", type=int, default=2000)
ap.add_argument("--trace-run", default="",
                help="comma-separated rate indexes to trace (4M-event ring each), written to <--trace>.<k>")
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


def cgroup_cpu() -> dict:
    """cgroup v2 cpu.stat counters (CFS quota throttling of this container)."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f)}
    except (OSError, ValueError):
        return {}


def cgroup_mem() -> dict:
    """cgroup v2 memory.events counters plus memory.current (bytes)."""
    out = {}
    try:
        with open("/sys/fs/cgroup/memory.events") as f:
            out = {k: int(v) for k, v in (line.split() for line in f)}
        with open("/sys/fs/cgroup/memory.current") as f:
            out["current"] = int(f.read())
    except (OSError, ValueError):
        pass
    return out


def sched_delta(a0: dict, a1: dict) -> dict:
    return {k: {"cpu_ms": round((v[0] - a0.get(k, [0, 0, 0])[0]) / 1e6, 1),
                "runqueue_wait_ms": round((v[1] - a0.get(k, [0, 0, 0])[1]) / 1e6, 1),
                "involuntary_switches": v[2] - a0.get(k, [0, 0, 0])[2]} for k, v in a1.items()}


pin_cpus(a.cpus, 0, order=ranked_domains() if a.cpus.startswith("l3") else None)
sh = Shard(ClusterSpec(nodes=a.nodes), namespace="olp", seed=0, options=json.loads(a.options))
try:
    if a.bench_sequence > 0:
        from flex_gpu_scheduler_amd.utils.openloop import open_loop_capacity

        log: list = []
        cap = open_loop_capacity(sh, a.bench_sequence, seed=0, log=log)
        print(json.dumps({"capacity_pods_per_s": cap, "search": log}), flush=True)
        if a.rates == "capacity":
            a.rates = f"{0.5 * cap},{0.9 * cap}"
    for k, rate in enumerate(float(x) for x in a.rates.split(",")):
        traced = str(k) in a.trace_run.split(",")
        if k == a.sample_run:
            from flex_gpu_scheduler_amd._native import native as _nat

            _nat().sampler_start(a.sample_hz)
        if traced:
            sh.sched.set_trace(True, 4 << 20)
        s0 = sh.sched.stats()
        ts0 = thread_sched()
        cg0 = cgroup_cpu()
        cm0 = cgroup_mem()
        r = run_open_loop(sh, rate, a.seconds, seed=a.seed, occupancy=a.occupancy, timeline=True)
        if k == a.sample_run:
            _nat().sampler_dump(a.sample)
        if traced:
            sh.sched.set_trace(False)
            with open(f"{a.trace}.{k}", "w") as f:
                f.write(sh.sched.trace_json())
        s1 = sh.sched.stats()
        threads = sched_delta(ts0, thread_sched())
        cg1 = cgroup_cpu()
        cgroup = {k: cg1[k] - cg0.get(k, 0) for k in ("nr_throttled", "throttled_usec", "usage_usec") if k in cg1}
        cm1 = cgroup_mem()
        cgroup["memory_events"] = {k: cm1[k] - cm0.get(k, 0) for k in cm1 if k != "current"}
        cgroup["memory_current_mib"] = cm1.get("current", 0) >> 20
        with open("/proc/self/status") as f:
            cgroup["rss_mib"] = next((int(x.split()[1]) >> 10 for x in f if x.startswith("VmRSS")), None)
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
            "parked_gangs": r.get("parked_gangs"), "denied_gangs": r["denials"]["total"],
            "p99_enqueue_to_allow_ms": {k: v["enqueue_to_allow_ms"]["p99"] for k, v in r["by_gang"].items()},
            "unschedulable_attempts": s1["unschedulable"] - s0["unschedulable"],
            "attempts": s1["attempts"] - s0["attempts"],
            "first_failures": [m for _, m in fails[:3]],
            "threads": threads, "cgroup_cpu": cgroup,
            "timeline_5ms": r.get("timeline"),
            "cache_drained": drained, "cache_clean": chk.get("clean"),
            "accounting_mismatches": len(chk.get("accounting", [])),
            "failed_scheduling": dict(sorted(why.items(), key=lambda kv: -kv[1])[:8])}), flush=True)
finally:
    if a.trace and not a.trace_run:
        with open(a.trace, "w") as f:
            f.write(sh.sched.trace_json())
    sh.close()
