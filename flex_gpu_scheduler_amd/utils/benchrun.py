"""Benchmark runner: one scheduler shard over a synthetic 8x MI355X cluster.

A "step" is one wave (utils/workload.py): create the PodGroups and pods of the
wave in the store, wait until every pod is bound, then delete the wave and
wait until the scheduler's cache has dropped it. Everything — API writes,
informer ingestion, scheduling and binding cycles, PodGroup status PATCHes,
deletions — happens inside the step.
"""
from __future__ import annotations

import json
import time
from dataclasses import dataclass, field

from ..config import load_config
from ..scheduler import Store, new_scheduler
from .workload import ClusterSpec, Wave, flagship_config, make_wave, percentile


class WaveTimeout(RuntimeError):
    pass


@dataclass
class StepResult:
    pods: int
    seconds: float
    gangs: list[dict] = field(default_factory=list)
    # wall-clock split of the step (ms): API writes, until every pod is bound,
    # deletion + cache drain
    split_ms: dict = field(default_factory=dict)


class Shard:
    def __init__(self, spec: ClusterSpec, *, namespace: str = "bench", seed: int = 0, config: dict | None = None,
                 options: dict | None = None):
        self.spec = spec
        self.ns = namespace
        self.seed = seed
        self.store = Store()
        self.store.create_many("nodes", json.dumps(spec.node_objects()))
        self.store.create_many("noderesourcetopologies", json.dumps(spec.nrt_objects()))
        opts = {"seed": seed + 1, **(options or {})}
        self.sched = new_scheduler(self.store, load_config(config or flagship_config()), **opts)
        self.sched.start()
        self._bound = 0

    def wave(self, step: int) -> Wave:
        return make_wave(self.spec, step, namespace=self.ns, seed=self.seed)

    def run(self, wave: Wave, timeout_s: float = 120.0, *,
            prepared: tuple[str, str] | list[tuple[str, str]] | None = None,
            check_cache: dict | None = None, collect_gangs: bool = True) -> StepResult:
        """One wave: create, wait until bound, delete, wait until the cache
        drained. `prepared` is the wave's JSON, either (PodGroups, pods) or
        Wave.chunks_json() (PodGroups written chunk by chunk just before their
        pods). With `check_cache` (a dict, filled in), the cache debugger
        runs once the wave is bound and no binding is in flight, before the
        deletion (untimed callers only). With `collect_gangs` False the gang
        records stay in the scheduler (a caller collects many waves' worth
        at once with sched.gang_records)."""
        chunks = prepared if isinstance(prepared, list) else [prepared or (wave.groups_json(), wave.pods_json())]
        n = len(wave.pods)
        target = self._bound + n
        t0 = time.perf_counter()
        for groups_js, pods_js in chunks:
            if groups_js != "[]":
                self.store.create_many("podgroups", groups_js)
            if pods_js != "[]":
                self.store.create_many("pods", pods_js)
        t_created = time.perf_counter()
        deadline = t0 + timeout_s
        sched = self.sched
        # Waits natively (no Python per poll, no stats lock): wait_bound polls
        # the scheduler's bound counter every 20 us with the GIL released.
        if not sched.wait_bound(target, max(0.0, deadline - time.perf_counter())):
            b = sched.stats()["bound"]
            raise WaveTimeout(f"wave not bound after {timeout_s}s: {b - self._bound}/{n} "
                              f"queue={sched.queue_counts()} stats={sched.stats()}")
        self._bound = target
        t_bound = time.perf_counter()
        if check_cache is not None:
            while sched.stats()["inflight_bindings"] > 0 and time.perf_counter() < deadline:
                time.sleep(0.0002)
            check_cache.update(sched.check_cache())
        gangs = sched.gang_records(True) if collect_gangs else []
        self.store.delete_all("pods", self.ns)
        self.store.delete_all("podgroups", self.ns)
        if not sched.wait_cache_empty(max(0.0, deadline - time.perf_counter())):
            raise WaveTimeout("wave deletion not observed by the scheduler cache")
        t_end = time.perf_counter()
        return StepResult(n, t_end - t0, gangs, {"create": (t_created - t0) * 1e3, "to_bound": (t_bound - t_created) * 1e3,
                                                 "delete_drain": (t_end - t_bound) * 1e3})

    def close(self) -> None:
        self.sched.stop()


def gang_type(g: dict) -> str:
    """"1" / "2" / "4" / "8" for whole-GPU gangs, "cpx4" for CPX quarter
    gangs (workload.make_wave names them "s<step>-<k>-q")."""
    return "cpx4" if g.get("pod_group", "").endswith("-q") else str(g["size"])


def gang_split_summary(gangs: list[dict]) -> dict:
    """Per gang type: how many gangs landed on more than one node (`split`),
    and how many of those could have been hosted by one node when their first
    rank was placed (`avoidable`: the record's `hostable` is 1). Gangs of one
    rank cannot split and are left out."""
    out: dict[str, dict] = {}
    for g in gangs:
        if g.get("size", 0) <= 1 or "nodes" not in g:
            continue
        row = out.setdefault(gang_type(g), {"n": 0, "split": 0, "avoidable": 0, "hostable": 0})
        row["n"] += 1
        split = g["nodes"] > 1
        row["split"] += split
        row["hostable"] += g.get("hostable", -1) == 1
        row["avoidable"] += split and g.get("hostable", -1) == 1
    for row in out.values():
        row["split_fraction"] = round(row["split"] / max(1, row["n"]), 6)
        row["avoidable_fraction"] = round(row["avoidable"] / max(1, row["n"]), 6)
    return dict(sorted(out.items(), key=lambda kv: (kv[0].startswith("cpx"), int(kv[0].lstrip("cpx")))))


def gang_latency_summary(gangs: list[dict], sizes: dict[str, int] | None = None, *, by_type: bool = False) -> dict:
    """p50/p99 first-member-enqueue -> last-member-bound (ms) per group size.

    With `by_type`, CPX quarter-GPU gangs (workload.make_wave names them
    "s<step>-<k>-q") are keyed "cpx4" apart from whole-GPU gangs of 4."""
    by: dict[str, list[float]] = {}
    for g in gangs:
        key = str(g["size"])
        if by_type and g.get("pod_group", "").endswith("-q"):
            key = "cpx4"
        by.setdefault(key, []).append((g["bound_us"] - g["first_enqueue_us"]) / 1000.0)
    out = {}
    for key in sorted(by, key=lambda k: (k.startswith("cpx"), int(k.lstrip("cpx")))):
        xs = by[key]
        out[key] = {"n": len(xs), "p50_ms": round(percentile(xs, 50), 3), "p99_ms": round(percentile(xs, 99), 3)}
    return out
