"""Open-loop gang admission latency (bench.py `config.gang_admit_open_loop`).

The headline step is a burst: a whole wave of gangs created at once, so the
p99 gang-admit latency it reports is mostly the time a gang queues behind the
rest of the burst (and the CPX quarter gangs, appended after the whole-GPU
gangs in a wave, always queue longest: the "size-4 anomaly" of the burst
numbers). This mode measures admission instead: gangs arrive one by one as a
Poisson process at a fixed fraction of the shard's measured throughput, gang
types interleaved at random (whole-GPU gangs of 1/2/4/8 ranks and CPX quarter
gangs of 4 x 0.25 MI355X), and each gang is deleted a hold time after it is
bound so the cluster stays at a steady occupancy. The native driver
(csrc/scheduler/openloop.cc) paces arrivals and records, per gang:

  enqueue_to_allow   first member enters the queue -> last member allowed at
                     Permit (scheduler-internal; the reference's
                     scheduler_permit_wait_duration_seconds family,
                     vendor/.../scheduler/metrics/metrics.go:158-166)
  create_to_bound    PodGroup + pods written -> last member bound (end to end)

both as p50/p99 per gang type.
"""
from __future__ import annotations

import json
import random

from ..models.mi355x import GPU, GPU_XCD
from ..models.objects import make_container, make_pod, make_pod_group
from .workload import ClusterSpec, percentile

GANG_TYPES = ("1", "2", "4", "8", "cpx4")  # whole-GPU ranks, or a CPX quarter-GPU gang of 4


def gang_objects(kind: str, name: str, ns: str, rng: random.Random) -> dict:
    req = {"cpu": f"{rng.choice([500, 1000, 2000, 4000])}m", "memory": f"{rng.choice([2, 4, 8, 16])}Gi"}
    if kind == "cpx4":
        size, limits, cname = 4, {GPU_XCD: "2"}, "shard"
    else:
        size, limits, cname = int(kind), {GPU: "1"}, "trainer"
    pods = [make_pod(f"{name}-r{r}", ns, containers=[make_container(cname, requests=req, limits=limits)],
                     pod_group=name) for r in range(size)]
    return {"podgroup": make_pod_group(name, ns, size), "pods": pods}


def plan(spec: ClusterSpec, rate_pods_per_s: float, duration_s: float, seed: int = 0, ns: str = "openloop",
         occupancy: float = 0.5, tag: str = "") -> tuple[list[dict], list[str], list[int], int]:
    """Gangs, their types, Poisson arrival offsets (us) and the hold time (us)
    that keeps ~`occupancy` of the SPX GPUs busy at this arrival rate. `tag`
    goes into every gang name, so consecutive runs on one shard do not reuse
    PodGroup names (Coscheduling remembers a denied group by name for
    deniedPGExpirationTimeSeconds)."""
    rng = random.Random(seed)
    mean_pods = sum(4 if t == "cpx4" else int(t) for t in GANG_TYPES) / len(GANG_TYPES)
    gang_rate = rate_pods_per_s / mean_pods
    n = max(1, int(gang_rate * duration_s))
    kinds = [rng.choice(GANG_TYPES) for _ in range(n)]
    t, offsets = 0.0, []
    for _ in range(n):
        t += rng.expovariate(gang_rate)
        offsets.append(int(t * 1e6))
    gangs = [gang_objects(k, f"ol{tag}{i}-{k}", ns, rng) for i, k in enumerate(kinds)]
    # Whole-GPU GPU-seconds arriving per second on the SPX side.
    whole = [int(k) for k in GANG_TYPES if k != "cpx4"]
    spx_gpu_rate = gang_rate * (len(whole) / len(GANG_TYPES)) * (sum(whole) / len(whole))
    hold_us = int(1e6 * occupancy * max(1, spec.spx_gpus) / max(spx_gpu_rate, 1e-9))
    return gangs, kinds, offsets, max(100, hold_us)  # occupancy 0: deleted as soon as bound


def _pct(xs: list[float]) -> dict:
    if not xs:
        return {"p50": None, "p99": None, "p999": None, "max": None}
    return {"p50": round(percentile(xs, 50), 3), "p99": round(percentile(xs, 99), 3),
            "p999": round(percentile(xs, 99.9), 3), "max": round(max(xs), 3)}


def _ms(v: float | None):
    return None if v is None else (round(v, 3) if v != float("inf") else "inf")


def summarize(kinds: list[str], gangs: list[dict], wall_us: int, late_us: int) -> dict:
    out: dict = {}
    for k in GANG_TYPES:
        rows = [g for kk, g in zip(kinds, gangs) if kk == k]
        ok = [g for g in rows if g["bound_us"]]
        if not rows:
            continue
        e2a = [(g["admit_us"] - g["first_enqueue_us"]) / 1e3 for g in ok]
        c2b = [(g["bound_us"] - g["create_us"]) / 1e3 for g in ok]
        multi = [g for g in ok if g.get("nodes", 0) and int(k.lstrip("cpx")) > 1]
        out[k] = {"n": len(rows), "unbound": len(rows) - len(ok),
                  "enqueue_to_allow_ms": _pct(e2a), "create_to_bound_ms": _pct(c2b),
                  # Bound gangs on more than one node, and those of them one
                  # node could have hosted when their first rank was placed.
                  "split": sum(1 for g in multi if g["nodes"] > 1),
                  "avoidable_split": sum(1 for g in multi if g["nodes"] > 1 and g.get("hostable") == 1),
                  "multi_rank_bound": len(multi)}
    # Over every gang, an unbound one counting as infinitely late (the
    # capacity criterion of open_loop_capacity).
    c2b_all = sorted((g["bound_us"] - g["create_us"]) / 1e3 if g["bound_us"] else float("inf") for g in gangs)
    n = len(gangs)
    multi = sum(v["multi_rank_bound"] for v in out.values())
    return {"by_gang": out, "gangs": n, "wall_s": round(wall_us / 1e6, 3),
            "gang_split_fraction": round(sum(v["split"] for v in out.values()) / max(1, multi), 6),
            "gang_avoidable_split_fraction": round(sum(v["avoidable_split"] for v in out.values()) / max(1, multi), 6),
            "all_gangs": {"n": n, "unbound": sum(1 for g in gangs if not g["bound_us"]),
                          "p99_create_to_bound_ms": _ms(percentile(c2b_all, 99) if c2b_all else None),
                          "p999_create_to_bound_ms": _ms(percentile(c2b_all, 99.9) if c2b_all else None),
                          "max_create_to_bound_ms": _ms(c2b_all[-1] if c2b_all else None)},
            "mean_arrival_lag_us": round(late_us / max(1, n), 1)}


def open_loop_capacity(shard, max_pods_per_s: float, duration_s: float = 1.0, seed: int = 0,
                       start_pods_per_s: float = 2000.0, occupancy: float = 0.5,
                       p99_budget_ms: float = 25.0, log: list | None = None, reset=None,
                       fine_step: float = 1.07, resume_at: float = 0.0, outcome: dict | None = None) -> float:
    """Sustained open-loop capacity (pods/s), an SLO capacity: the highest
    arrival rate of a rising ladder at which the p99 PG-create -> last-Bind
    over every gang of the run is within `p99_budget_ms` (a gang still
    unbound at the end counts as infinitely late). The ladder climbs x1.3 from
    `start_pods_per_s` while the next step stays a full x1.3 step under
    `max_pods_per_s` (the burst capacity), then in steps of `fine_step` (x1.07,
    the resolution two bisection steps of x1.3 gave) up to the burst rate
    itself. Gangs arrive one at a time and are held at `occupancy` of the SPX
    GPUs, as in the measured loads.

    The search ends at the first failed rate: the capacity is the rate below
    it. An overloaded trial leaves thousands of parked gangs and a lagging
    informer behind, and trials after one, even on a fresh shard in the same
    process, failed at rates that pass on their own (docs/ARCHITECTURE.md,
    "the open-loop edge is metastable"): climbing in fine steps, the first
    failure is at most one step past the edge, and no trial follows it.

    One trial per rate; two, with different arrival seeds, that must both
    pass, for rates within two x1.3 steps of the burst rate. No retries.
    `reset` is accepted for callers of the bisection version and not used.
    `resume_at` (a rung of the ladder) starts there instead, with no halving
    below it: 0.0 when it fails. `outcome["failed_at"]` receives the rate
    that ended the search (None when the burst rate itself passed).
    Every trial is appended to `log` with its parked gangs, its Coscheduling
    denials and their causes (Scheduler::note_gang_denied), p99.9 and max.
    Near capacity the hold time (a few ms) is comparable to the admission
    pipeline and GPUs held by gangs in flight push the SPX pool to full: a
    gang that finds it full parks until GPUs are released (Coscheduling
    transientShortage=Park) rather than being denied for the TTL as the
    reference's PostFilter does (which made a rate fail on < 1% of its
    gangs waiting 3 s)."""
    del reset
    top = max_pods_per_s / 1.3 ** 2  # rates within two x1.3 steps of the burst rate get a second trial

    def served(rate: float) -> bool:
        trials = 2 if rate >= top else 1
        ok = True
        for t in range(trials):
            r = run_open_loop(shard, rate, duration_s, seed=seed + 7 * t, occupancy=occupancy)
            p99 = r["all_gangs"]["p99_create_to_bound_ms"]
            ok_t = p99 is not None and p99 != "inf" and p99 <= p99_budget_ms
            if log is not None:
                log.append({"offered_pods_per_s": round(rate, 1), "served": ok_t, "trial": t + 1, "trials": trials,
                            "gangs": r["gangs"],
                            "unbound_gangs": r["all_gangs"]["unbound"], "p99_create_to_bound_ms": p99,
                            "p999_create_to_bound_ms": r["all_gangs"]["p999_create_to_bound_ms"],
                            "max_create_to_bound_ms": r["all_gangs"]["max_create_to_bound_ms"],
                            "wall_s": r["wall_s"], "denied_gangs": r["denials"]["total"],
                            "denied_gang_fraction": r["denied_gang_fraction"], "parked_gangs": r["parked_gangs"],
                            "denial_causes": r["denials"]["causes"],
                            "gang_split_fraction": r.get("gang_split_fraction"),
                            "gang_avoidable_split_fraction": r.get("gang_avoidable_split_fraction")})
            ok = ok and ok_t
            if not ok:
                break
        return ok

    if outcome is not None:
        outcome["failed_at"] = None

    def failed(rate: float, best: float) -> float:
        if outcome is not None:
            outcome["failed_at"] = rate
        return best

    if resume_at > 0:
        if not served(resume_at):
            return failed(resume_at, 0.0)
        rate = resume_at
    else:
        rate = min(start_pods_per_s, max(max_pods_per_s, 1.0))
        # A small cluster or a loaded host may not serve even the start rate:
        # halve down to it first (a few probes at most), then climb.
        floor = rate / 64
        while rate > floor and not served(rate):
            rate /= 2
        if rate <= floor:
            return failed(rate * 2, 0.0)
    best = rate
    coarse_top = max_pods_per_s / 1.3
    while True:
        nxt = rate * 1.3 if rate * 1.3 <= coarse_top else rate * fine_step
        if nxt > max_pods_per_s:
            # The last rung is the burst rate itself (otherwise the ladder,
            # not the scheduler, would cap the result just under it).
            if rate >= max_pods_per_s:
                return best
            nxt = max_pods_per_s
        if not served(nxt):
            return failed(nxt, best)
        best = rate = nxt


def denial_summary(total: int, recs: list[dict], keep: int = 3) -> dict:
    """Coscheduling group denials of one run: how many, by cause, and the
    first few records with the cache/store GPU census at that moment."""
    causes: dict[str, int] = {}
    for d in recs:
        causes[d["cause"]] = causes.get(d["cause"], 0) + 1
    return {"total": int(total), "causes": causes, "first": recs[:keep]}


_runs = 0  # run_open_loop calls in this process: the gang-name tag


def run_open_loop(shard, rate_pods_per_s: float, duration_s: float = 1.0, seed: int = 0,
                  occupancy: float = 0.5, timeline: bool = False) -> dict:
    """One load level on `shard` (utils/benchrun.py Shard, idle). With
    `timeline`, also [pods in flight, pods held] at the end of every 5 ms."""
    from .._native import native

    global _runs
    _runs += 1
    gangs, kinds, offsets, hold_us = plan(shard.spec, rate_pods_per_s, duration_s, seed, occupancy=occupancy,
                                          tag=f"{_runs}r")
    shard.sched.gang_denials(True)
    shard.sched.gang_parks(True)
    res = native().run_open_loop(shard.store, shard.sched, json.dumps(gangs), offsets, hold_us, 10_000_000)
    shard.sched.wait_idle(10_000)
    out = summarize(kinds, res["gangs"], res["wall_us"], res["late_us"])
    out["denials"] = denial_summary(*shard.sched.gang_denials(True))
    # Parked groups (Coscheduling transientShortage=Park): waited for GPUs to
    # be released instead of being denied for deniedPGExpirationTimeSeconds.
    out["parked_gangs"] = int(shard.sched.gang_parks(True))
    out["denied_gang_fraction"] = round(out["denials"]["total"] / max(1, len(res["gangs"])), 5)
    n = max(1, len(res["gangs"]))
    out.update({"mean_delete_lag_us": round(res.get("delete_late_us", 0) / n, 1),
                "max_in_flight_pods": res.get("max_in_flight_pods"), "max_held_pods": res.get("max_held_pods")})
    if timeline:
        out["timeline"] = [list(x) for x in res.get("timeline", [])]
    out.update({"offered_pods_per_s": round(rate_pods_per_s, 1), "hold_ms": round(hold_us / 1e3, 3)})
    return out


def capacity_report(shard, burst: float, seed: int = 0, reset=None) -> dict:
    """The bench's open-loop block on `shard`: the capacity search, then the
    50% and 90% loads of the capacity found (on a fresh shard when `reset`
    is given, so they do not follow the search's overloaded trials)."""
    search: list[dict] = []
    cap = open_loop_capacity(shard, burst, seed=seed, log=search, reset=reset) if burst > 0 else 0.0
    out = {"capacity": cap, "search": search}
    if cap > 0 and reset is not None:
        shard = reset()
    for f in (0.5, 0.9):
        if cap > 0:
            out[f"load_{int(f * 100)}"] = run_open_loop(shard, f * cap, duration_s=1.0, seed=seed + 1)
    return out


def capacity_in_child(nodes: int, seed: int, options: dict, burst: float, cpus: list[int] | None = None,
                      warm_waves: int = 16, hbm_gib: int = 288, timeout_s: float = 600.0,
                      colocation: str = "Preferred", deny_check: bool = False) -> dict:
    """capacity_report in a child Python process that never loads the GPU
    runtime, on a fresh shard of the same cluster (spec, seed, options),
    warmed with `warm_waves` burst waves and pinned to `cpus`.

    The scheduler runs without the GPU runtime in deployment (it is a
    control-plane process; the GPU probes run in the node agent). In the
    bench's rank process, torch and HIP are loaded, and near the capacity
    cliff an overloaded trial then leaves the process markedly slower for the
    next ones (profiles/r5ar_openloop_torch_loaded.txt vs
    r5aq_openloop_no_torch.txt), so the in-process search measured that
    interaction rather than the scheduler."""
    import subprocess
    import sys

    base = [sys.executable, "-m", "flex_gpu_scheduler_amd.utils.openloop", "--nodes", str(nodes),
            "--seed", str(seed), "--options", json.dumps(options), "--burst", repr(float(burst)),
            "--warm-waves", str(warm_waves), "--hbm-gib", str(hbm_gib), "--colocation", colocation]
    if cpus:
        base += ["--cpus", ",".join(map(str, cpus))]

    def child(extra: list[str]) -> dict:
        r = subprocess.run(base + extra, capture_output=True, text=True, timeout=timeout_s, check=False)
        if r.returncode != 0:
            raise RuntimeError(f"open-loop child exited {r.returncode}: {r.stderr[-2000:]}")
        return json.loads(r.stdout.strip().splitlines()[-1])

    # The search ends with an overloaded trial; the 50% / 90% loads then run
    # in a second fresh process, so they never follow it (a fresh shard in
    # the overloaded process still served the 90% load at 11 ms p99 where a
    # fresh process serves it at 1 ms: profiles/r6/README.md, r6ah).
    rep = child(["--search-only"])
    # A shared host's other tenants can fail one rung (two full benches on one
    # box: 90.2k then 60.6k, r6ap). The rung that failed is tried once more in
    # a fresh process; if it passes there, the ladder goes on from it in that
    # process until a rung fails again. One retry per search.
    failed_at = rep.get("failed_at")
    if failed_at and failed_at <= burst:
        again = child(["--search-only", "--resume-at", repr(float(failed_at))])
        for row in again["search"]:
            row["retry_in_fresh_process"] = True
        rep["search"] += again["search"]
        rep["retried_rate"] = round(failed_at, 1)
        if again["capacity"] > rep["capacity"]:
            rep["capacity"] = again["capacity"]
    if rep["capacity"] > 0:
        loads = child(["--loads-at", repr(float(rep["capacity"]))] + (["--deny-check"] if deny_check else []))
        rep.update({k: v for k, v in loads.items() if k.startswith(("load_", "deny_mode_"))})
    return rep


def _child_main(argv: list[str] | None = None) -> int:
    import argparse
    import os

    ap = argparse.ArgumentParser(description="open-loop capacity report on a fresh shard (bench.py child)")
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--options", default="{}")
    ap.add_argument("--burst", type=float, required=True)
    ap.add_argument("--warm-waves", type=int, default=16)
    ap.add_argument("--hbm-gib", type=int, default=288)
    ap.add_argument("--cpus", default="")
    ap.add_argument("--colocation", default="Preferred")
    ap.add_argument("--deny-check", action="store_true", help="also run the 90%% load in Deny mode")
    ap.add_argument("--no-reset", action="store_true", help="keep one shard through the whole search")
    ap.add_argument("--search-only", action="store_true", help="the capacity search alone (no 50%%/90%% loads)")
    ap.add_argument("--loads-at", type=float, default=0.0,
                    help="no search: the 50%% and 90%% loads of this capacity on a fresh shard")
    ap.add_argument("--resume-at", type=float, default=0.0, help="with --search-only: start the ladder at this rung")
    a = ap.parse_args(argv)
    if a.cpus:
        os.sched_setaffinity(0, [int(c) for c in a.cpus.split(",")])  # before the shard's threads start
    from .benchrun import Shard
    from .workload import flagship_config

    shards: list = []

    def fresh():
        """A new shard of the same cluster, warmed with burst waves (the
        previous one is closed)."""
        while shards:
            shards.pop().close()
        sh = Shard(ClusterSpec(nodes=a.nodes, hbm_gib=a.hbm_gib), namespace="bench-ol", seed=a.seed,
                   options=json.loads(a.options), config=flagship_config(gang_colocation=a.colocation))
        shards.append(sh)
        for i in range(a.warm_waves):
            w = sh.wave(i)
            sh.run(w, prepared=w.chunks_json(), collect_gangs=False)
        return sh

    try:
        if a.loads_at > 0:
            sh = fresh()
            rep = {"capacity": a.loads_at, "search": []}
            for f in (0.5, 0.9):
                rep[f"load_{int(f * 100)}"] = run_open_loop(sh, f * a.loads_at, duration_s=1.0, seed=a.seed + 1)
        elif a.search_only:
            search: list[dict] = []
            outcome: dict = {}
            cap = (open_loop_capacity(fresh(), a.burst, seed=a.seed, log=search, resume_at=a.resume_at,
                                      outcome=outcome) if a.burst > 0 else 0.0)
            rep = {"capacity": cap, "search": search, "failed_at": outcome.get("failed_at")}
        else:
            rep = capacity_report(fresh(), a.burst, seed=a.seed, reset=None if a.no_reset else fresh)
    finally:
        while shards:
            shards.pop().close()
    if a.deny_check and rep["capacity"] > 0:
        # The same 90% load with the reference's semantics
        # (transientShortage: Deny) on a fresh shard: the like-for-like
        # comparison for the Park-mode numbers.
        deny = Shard(ClusterSpec(nodes=a.nodes, hbm_gib=a.hbm_gib), namespace="bench-ol-deny", seed=a.seed,
                     options=json.loads(a.options),
                     config=flagship_config(gang_colocation=a.colocation, transient_shortage="Deny"))
        try:
            for i in range(a.warm_waves):
                w = deny.wave(i)
                deny.run(w, prepared=w.chunks_json(), collect_gangs=False)
            rep["deny_mode_load_90"] = run_open_loop(deny, 0.9 * rep["capacity"], duration_s=1.0, seed=a.seed + 1)
        finally:
            deny.close()
    print(json.dumps(rep))
    return 0


if __name__ == "__main__":
    raise SystemExit(_child_main())
