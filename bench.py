#!/usr/bin/env python
"""Headline benchmark: scheduling throughput (pods/s) and p99 PodGroup
gang-admit latency for 1/2/4/8-GPU groups on synthetic 8x MI355X nodes.

Metric and config come from BASELINE.json (the reference publishes no
numbers, so vs_baseline is null). One process per GPU; each rank runs one
scheduler shard (its own store + scheduler over `--nodes` 8x MI355X nodes),
so per-GPU work is fixed as N grows (weak scaling) and `value` is the sum of
pods/s over ranks divided by the slowest rank's time.

GPU use: every rank probes its own MI355X concurrently with the HIP probes
(device props, checksum health test, MFMA tile check and the per-partition
HBM bandwidth table the node agent publishes; untimed) -> `config.gpu_probes`,
one row per GPU, and sizes the synthetic nodes' HBM from it. After the timed
steps (untimed) the ranks validate placement end to end
(parallel/placement.py): the live node from discovery, PodGroups of 1/2/4/8
ranks scheduled, each rank resolved through the device plugin's Allocate, and
an RCCL all-reduce on exactly the allocated GPUs next to deliberately bad
placements, each row judged against an xGMI bus-bandwidth model ->
`config.rccl_placement`. That is the last collective: then ranks > 0 exit and
rank 0 alone runs the untimed extras (open-loop admission latency, a
1,024-node run, steady-state service mode, the BASELINE scenarios), so no rank
waits inside an RCCL collective while they run.

Every headline number is also a scalar key of `config`, ahead of every
dict-valued key, led by `headline` (one string with all of them):
p99_gang_admit_ms_<type> (burst), open_loop_p99_create_to_bound_ms_<type> (at
90% of the open-loop capacity), open_loop_capacity_pods_per_s,
nodes1024_pods_per_s, service_mode_pods_per_s (+ generator_limited),
denied_gang_fraction, parked_gang_fraction (over the served open-loop runs;
*_all_trials adds the failed overload rung), gang_split_fraction_<type> (gangs
placed on more than one node) and gang_avoidable_split_fraction (split although
one node could host the gang), and on >= 2 GPUs placement_verdict_<k> and
placed_busbw_GBps_<k>.

    python bench.py --gpus N --steps K --warmup W

Launch: under torch.distributed.run (WORLD_SIZE set) each process is one
rank. A bare `python bench.py --gpus N` with N > 1 starts its N ranks itself
(one child process per GPU, before anything touches the GPU) and exits with
their status; WORLD_SIZE != --gpus is refused, and `n_gpus` is always the
real world size.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "pods/sec sched throughput + p99 PodGroup gang-admit latency, 1/2/4/8-GPU groups"


def progress(msg: str) -> None:
    """One progress line on stderr per phase (long untimed extras keep a
    watcher that expects output every few minutes informed)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """Start ranks 0..n-1 of this script as child processes (the parent never
    initialises the GPU: it only counts devices) and wait for them. If one
    rank fails the others are stopped, so a broken rank cannot leave its peers
    blocked in a collective."""
    import signal
    import subprocess

    from flex_gpu_scheduler_amd.gpu.discovery import visible_gpu_count

    # Counted from amdgpu sysfs / KFD: the parent never loads HIP, so nothing
    # GPU-side is initialised before the ranks start.
    try:
        have = visible_gpu_count()
    except Exception:  # noqa: BLE001
        have = 0
    if have and have < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) are visible", file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def run_nodes(nodes: int, waves: int, seed: int, options: dict, colocation: str = "Preferred") -> dict:
    """Untimed run of the headline workload on one `nodes`-node shard: two
    warm-up waves, then `waves` timed waves (pods/s over those)."""
    from flex_gpu_scheduler_amd.utils.benchrun import Shard, gang_latency_summary, gang_split_summary
    from flex_gpu_scheduler_amd.utils.workload import ClusterSpec, flagship_config

    shard = Shard(ClusterSpec(nodes=nodes), namespace=f"bench-n{nodes}", seed=seed + 104729, options=options,
                  config=flagship_config(gang_colocation=colocation))
    try:
        ws = [shard.wave(i) for i in range(waves + 2)]
        prepared = [w.chunks_json() for w in ws]
        for i in range(2):
            shard.run(ws[i], prepared=prepared[i])
        shard.sched.gang_records(True)
        t0 = time.perf_counter()
        pods = 0
        split: dict[str, float] = {}
        for i in range(2, waves + 2):
            r = shard.run(ws[i], prepared=prepared[i], collect_gangs=False)
            pods += r.pods
            for k, v in r.split_ms.items():
                split[k] = split.get(k, 0.0) + v
        dt = time.perf_counter() - t0
        recs = shard.sched.gang_records(True)
        lat = gang_latency_summary(recs, by_type=True)
        # Where a wave's time goes: API writes (scheduling overlaps them),
        # until the last pod is bound, deletion + cache drain.
        return {"nodes": nodes, "waves": waves, "pods": pods, "seconds": round(dt, 3),
                "pods_per_s": round(pods / dt, 1) if dt > 0 else 0.0,
                "split_ms_per_wave": {k: round(v / max(1, waves), 2) for k, v in split.items()},
                "p99_gang_admit_ms": {k: v["p99_ms"] for k, v in lat.items()},
                "gang_split": gang_split_summary(recs)}
    finally:
        shard.close()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=64, help="8x MI355X nodes per scheduler shard")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-gpu-probe", action="store_true")
    ap.add_argument("--trace", default="", help="write a Chrome trace of rank 0's timed steps")
    ap.add_argument("--sched-options", default="{}",
                    help='JSON scheduler options for A/B runs, e.g. \'{"equivalenceCache": false}\'')
    ap.add_argument("--no-scenarios", action="store_true",
                    help="skip the per-BASELINE-config scenarios (untimed, reported under config.scenarios)")
    ap.add_argument("--cpus", default=os.environ.get("XSCHED_CPUS", "l3"),
                    help="shard CPU placement: none | l3 | l3xK | explicit list (utils/cpuaffinity.py)")
    ap.add_argument("--no-open-loop", action="store_true",
                    help="skip the untimed open-loop (Poisson arrivals) gang admission latency run")
    ap.add_argument("--open-loop-in-process", action="store_true",
                    help="run the open-loop search on this rank's shard instead of a GPU-free child (A/B)")
    ap.add_argument("--waves-per-step", type=int, default=16,
                    help="waves per timed step (one wave fills the shard's GPUs once)")
    ap.add_argument("--no-service-mode", action="store_true",
                    help="skip the untimed service-mode run (API server in another process, HTTP)")
    ap.add_argument("--no-placement", action="store_true",
                    help="skip the end-to-end placement validation (discovery -> scheduler -> Allocate -> RCCL)")
    ap.add_argument("--gang-colocation", default="Preferred", choices=("Preferred", "Required", "None"),
                    help="NRT gangColocation of the flagship profile (xGMI gang co-location)")
    ap.add_argument("--nodes1024-waves", type=int, default=6,
                    help="timed waves of the untimed 1,024-node run (0 skips it)")
    args = ap.parse_args()

    world = os.environ.get("WORLD_SIZE")
    if world is None and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    if world is not None and int(world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; one rank per GPU is required", file=sys.stderr)
        return 2

    from flex_gpu_scheduler_amd.parallel.dist import init_distributed
    from flex_gpu_scheduler_amd.utils.benchrun import Shard, gang_latency_summary, gang_split_summary
    from flex_gpu_scheduler_amd.utils.workload import ClusterSpec

    ctx = init_distributed(want_cuda=True)
    extras: dict = {}
    hbm_gib = 288
    if ctx.cuda and not args.no_gpu_probe:
        from flex_gpu_scheduler_amd.ops.hip_probe import probe

        pr = probe()
        props = pr.props(ctx.local_rank)
        health = pr.health(ctx.local_rank)
        if not health["healthy"]:
            raise SystemExit(f"GPU {ctx.local_rank} failed the checksum health test: {health}")
        mfma = pr.mfma_check(ctx.local_rank)
        if not mfma["healthy"]:
            raise SystemExit(f"GPU {ctx.local_rank} failed the MFMA tile check: {mfma}")
        hbm_gib = max(1, int(props["totalGlobalMem"]) // (1 << 30))
        extras["gpu"] = {"name": props.get("gcnArchName"), "computeUnits": props.get("computeUnits"),
                         "hbm_gib": hbm_gib}
        # The node agent's per-GPU table, measured on every rank's own GPU at
        # once (untimed); a failure is reported, not fatal.
        row = {"rank": ctx.rank, "local_rank": ctx.local_rank, "healthy": True, "mfma_ok": True,
               "pci_bus_id": props.get("pciBusID")}
        try:
            row["hbm"] = pr.partition_table(ctx.local_rank)
        except Exception as e:  # noqa: BLE001
            row["hbm"] = {"error": f"{type(e).__name__}: {e}"}
        probe_row = row
    else:
        probe_row = None
    probe_rows = ctx.gather(probe_row)
    if ctx.rank == 0 and any(probe_rows):
        extras["gpu_probes"] = [r for r in probe_rows if r]

    from flex_gpu_scheduler_amd.utils.cpuaffinity import apply as pin_cpus, ranked_domains

    # One L3 domain per shard (8 cores / 16 CPUs on the MI355X hosts): the
    # shard's threads hand work to each other ~10^5 times/s and floating over
    # 256 CPUs costs 2x throughput (profiles/r1g_affinity_ab.txt). Rank 0's
    # idle ranking is shared so the ranks of one node take disjoint domains.
    order = None
    if args.cpus.startswith("l3"):
        order = ctx.gather(ranked_domains())[0] if ctx.distributed else ranked_domains()
    cpus = pin_cpus(args.cpus, ctx.local_rank, order=order)  # before the shard's threads start
    if cpus:
        extras["cpus"] = {"mode": args.cpus, "n": len(cpus), "first": cpus[0]}
    spec = ClusterSpec(nodes=args.nodes, hbm_gib=hbm_gib)
    from flex_gpu_scheduler_amd.utils.workload import flagship_config

    shard = Shard(spec, namespace=f"bench-r{ctx.rank}", seed=args.seed + 7919 * ctx.rank,
                  options=json.loads(args.sched_options), config=flagship_config(gang_colocation=args.gang_colocation))
    # Pre-render every wave's JSON (data preparation, outside the timed region).
    wps = max(1, args.waves_per_step)
    n_waves = (args.warmup + args.steps) * wps
    waves = [shard.wave(i) for i in range(n_waves + 1)]  # +1: the untimed check wave
    # Each chunk's PodGroups are written just before its pods (as job
    # submitters do), unless XSCHED_BENCH_INTERLEAVE=0 (all PodGroups first;
    # A/B runs).
    interleave = os.environ.get("XSCHED_BENCH_INTERLEAVE", "1") != "0"
    prepared = [w.chunks_json() if interleave else (w.groups_json(), w.pods_json()) for w in waves]

    progress(f"rank {ctx.rank}: warm-up ({args.warmup * wps} waves)")
    for i in range(args.warmup * wps):
        shard.run(waves[i], prepared=prepared[i])
    progress(f"rank {ctx.rank}: timed steps")

    if args.trace and ctx.rank == 0:
        shard.sched.set_trace(True)
    shard.sched.gang_records(True)  # drop the warm-up waves' records
    ctx.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    pods = 0
    for i in range(args.warmup * wps, n_waves):
        # Gang latency records stay in the scheduler until the timed steps end
        # (converting them to Python per wave is bookkeeping, not scheduling).
        r = shard.run(waves[i], prepared=prepared[i], collect_gangs=False)
        pods += r.pods
    t_rank = time.perf_counter() - t0
    ctx.sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    gangs: list[dict] = shard.sched.gang_records(True)
    if args.trace and ctx.rank == 0:
        with open(args.trace, "w") as f:
            f.write(shard.sched.trace_json())

    # Untimed: one more wave, and once it is bound the cache debugger
    # compares the cache with the listers and re-derives every node's
    # accounting (resources, GPU ledger, gang counts) from its pods.
    check: dict = {}
    shard.run(waves[-1], prepared=prepared[-1], check_cache=check)
    extras["cache_check"] = {"clean": bool(check.get("clean")), "assumed": check.get("assumed"),
                             "accounting_mismatches": len(check.get("accounting", []))}
    t_max = ctx.all_max(elapsed)
    pods_total = ctx.all_sum(float(pods))
    all_gangs = [g for part in ctx.gather(gangs) for g in part]
    per_rank = ctx.gather(round(pods / t_rank, 1) if t_rank > 0 else 0.0)
    del waves, prepared
    stats = shard.sched.stats()
    if not args.no_placement and (ctx.distributed or ctx.cuda):
        # Untimed: gangs placed on the live node, resolved by the device
        # plugin, all-reduced on exactly those GPUs (parallel/placement.py).
        # A failure there is reported, not fatal to the headline line. The
        # last collective of the run: every rank takes part.
        from flex_gpu_scheduler_amd.parallel.placement import validate_placement

        try:
            tables = {r["local_rank"]: r["hbm"] for r in probe_rows if r and "error" not in r.get("hbm", {})}
            extras["rccl_placement"] = validate_placement(ctx, bandwidth_tables=tables)
        except Exception as e:  # noqa: BLE001
            extras["rccl_placement"] = {"error": f"{type(e).__name__}: {e}"}
    ctx.barrier()
    if ctx.rank != 0:
        # Ranks > 0 are done: rank 0's untimed extras below run without them.
        shard.close()
        ctx.close()
        return 0
    def repin() -> list[int] | None:
        # Rank 0's untimed extras run after the other ranks have exited: each
        # phase takes the L3 domain that is least busy now (other tenants of
        # the host may have moved onto the one ranked at the start).
        if not args.cpus.startswith("l3"):
            return None
        return pin_cpus(args.cpus, 0, order=ranked_domains())

    progress(f"timed region done: {pods / t_rank if t_rank > 0 else 0:.0f} pods/s on rank 0")
    if not args.no_open_loop:
        progress("open-loop capacity search")
        # Untimed: Poisson gang arrivals at 50% / 90% of this shard's measured
        # open-loop capacity, gang types interleaved, held then deleted
        # (utils/openloop.py) — admission latency rather than burst queueing.
        # In a child process that never loads the GPU runtime (the scheduler's
        # deployment shape), on a fresh shard of the same cluster pinned to
        # this shard's CPUs (this one is idle meanwhile): with torch and HIP in
        # the process, an overloaded trial near the cliff leaves it slower for
        # the next trials (utils/openloop.py capacity_in_child).
        from flex_gpu_scheduler_amd.utils.openloop import capacity_in_child, capacity_report

        burst = pods / t_rank if t_rank > 0 else 0.0
        if args.open_loop_in_process:
            rep = capacity_report(shard, burst, seed=args.seed)
        else:
            rep = capacity_in_child(args.nodes, args.seed + 7919 * ctx.rank, json.loads(args.sched_options), burst,
                                    cpus=repin() or cpus, hbm_gib=hbm_gib, colocation=args.gang_colocation,
                                    deny_check=True)
        cap = rep["capacity"]
        extras["gang_admit_open_loop"] = {
            "burst_capacity_pods_per_s": round(burst, 1),
            "capacity_pods_per_s": round(cap, 1),
            "capacity_rule": "highest rate of a rising ladder (x1.3 steps, then x1.07 steps from one x1.3 step "
                             "under the burst rate up to it) whose p99 PG-create->last-Bind over all gangs "
                             "(unbound = infinite) is <= 25 ms; the search stops at the first failed rate, which "
                             "is tried once more in a fresh process (the ladder goes on there if it passes); one "
                             "trial per rate, two (both must pass) within two x1.3 steps of the burst rate",
            "transient_shortage": "Park (gangs short of GPUs wait for a release; the reference denies them "
                                  "for deniedPGExpirationTimeSeconds)",
            "process": "this rank's" if args.open_loop_in_process else (
                "children without the GPU runtime: the search on one fresh shard, the 50%/90% loads on "
                "another in a second process"),
            "capacity_search": rep["search"],
            "retried_rate": rep.get("retried_rate"),
            **{k: rep[k] for k in ("load_50", "load_90", "deny_mode_load_90") if k in rep}}
        search = rep["search"]
        ol = extras["gang_admit_open_loop"]
        extras["open_loop_capacity_pods_per_s"] = round(cap, 1)
        l90 = ol.get("load_90") or {}
        for k, v in (l90.get("by_gang") or {}).items():
            extras[f"open_loop_p99_create_to_bound_ms_{k}"] = v["create_to_bound_ms"]["p99"]
        if l90:
            extras["open_loop_p999_create_to_bound_ms"] = l90["all_gangs"]["p999_create_to_bound_ms"]
            extras["open_loop_max_create_to_bound_ms"] = l90["all_gangs"]["max_create_to_bound_ms"]
        # Over the served open-loop runs (search rungs that passed and the two
        # loads); the rung that failed is an overload by construction, so its
        # parked gangs are reported apart (all_trials) instead of diluting the
        # fraction a user sees below capacity.
        extras.update(gang_fractions(search, [ol.get(f"load_{x}") for x in (50, 90) if ol.get(f"load_{x}")]))
        dn = ol.get("deny_mode_load_90")
        if dn:
            # The reference's semantics at the same load (Coscheduling
            # transientShortage: Deny), for a like-for-like comparison.
            extras["deny_mode_open_loop_p99_create_to_bound_ms"] = dn["all_gangs"]["p99_create_to_bound_ms"]
            extras["deny_mode_denied_gang_fraction"] = dn["denied_gang_fraction"]
        loads = [ol.get(f"load_{x}") for x in (50, 90) if ol.get(f"load_{x}")]
        if loads:
            extras["open_loop_gang_split_fraction"] = max(r.get("gang_split_fraction", 0.0) for r in loads)
            extras["open_loop_gang_avoidable_split_fraction"] = max(r.get("gang_avoidable_split_fraction", 0.0)
                                                                    for r in loads)
    shard.close()

    if args.nodes1024_waves > 0:
        progress("1,024-node run")
        # Untimed: the same workload on one 1,024-node shard (12k pods/wave).
        repin()
        try:
            extras["nodes1024"] = run_nodes(1024, args.nodes1024_waves, args.seed, json.loads(args.sched_options),
                                            args.gang_colocation)
            extras["nodes1024_pods_per_s"] = extras["nodes1024"]["pods_per_s"]
            sp = extras["nodes1024"]["gang_split"]
            n_multi = sum(v["n"] for v in sp.values())
            extras["nodes1024_gang_split_fraction"] = round(sum(v["split"] for v in sp.values()) / max(1, n_multi), 6)
            extras["nodes1024_gang_avoidable_split_fraction"] = round(
                sum(v["avoidable"] for v in sp.values()) / max(1, n_multi), 6)
        except Exception as e:  # noqa: BLE001
            extras["nodes1024"] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_service_mode:
        progress("service mode")
        # Untimed: the deployable shape — scheduler and API server in separate
        # processes over loopback HTTP (tools/remote_bench.py): steady state
        # (pods created over HTTP by other processes while it schedules), and
        # drains of pre-created plain pods / 8-rank gangs for comparison. The
        # steady rows climb the offered rate (pipelined creates) until the
        # scheduler, not the generator, is the limit: a row whose backlog grows
        # (generator_limited false) measures the scheduler's ceiling.
        try:
            from flex_gpu_scheduler_amd.tools.remote_bench import run as remote_run, run_steady

            rows = []
            for depth in (1, 16, 64):
                row = run_steady(128, 2.0, 8, depth=depth)
                rows.append(row)
                if not row["generator_limited"] and row["offered_creates_per_s"] >= 1.3 * row["pods_per_s"]:
                    break
            plain = remote_run(64, 4000, False, 16, 8)
            gang = remote_run(64, 512, True, 16, 8)
            limited = [r for r in rows if not r["generator_limited"]]
            best = max(limited or rows, key=lambda r: r["pods_per_s"])
            extras["service_mode"] = {
                "apiserver": "native HTTP/1.1 (csrc/apiserver), separate process, loopback",
                "steady": best,
                "steady_rows": rows,
                "drain_plain": {k: plain[k] for k in ("pods", "pods_per_s", "pods_per_s_after_sync", "sync_s",
                                                      "bound")},
                "drain_gang8": {k: gang[k] for k in ("pods", "pods_per_s", "pods_per_s_after_sync", "sync_s",
                                                     "bound")}}
            extras["service_mode_pods_per_s"] = best["pods_per_s"]
            extras["service_mode_offered_creates_per_s"] = best["offered_creates_per_s"]
            extras["service_mode_generator_limited"] = best["generator_limited"]
        except Exception as e:  # noqa: BLE001
            extras["service_mode"] = {"error": f"{type(e).__name__}: {e}"}

    value = pods_total / t_max if t_max > 0 else 0.0
    if not args.no_scenarios:
        # The five BASELINE.json configurations, each with its placement check
        # (outside the timed region; utils/scenarios.py).
        from flex_gpu_scheduler_amd.utils.scenarios import run_all

        progress("BASELINE scenarios")
        extras["scenarios"] = run_all()
    if ctx.rank == 0:
        lat = gang_latency_summary(all_gangs)
        by_type = gang_latency_summary(all_gangs, by_type=True)
        split = gang_split_summary(all_gangs)
        head = headline_scalars(value, by_type, split, extras, ctx.world_size)
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "pods/s",
            "n_gpus": ctx.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max * 1000.0 / max(1, args.steps), 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic pod specs / random resource requests (BASELINE.json configs)",
            "config": {
                # Scalars first (a reader that keeps only the first scalar keys
                # gets every headline number): the contract keys, a one-line
                # summary of every headline number, then each as its own key.
                "model": "FlexGPU(MI355X SPX/CPX/HBM) + Coscheduling + NRT xGMI gang placement",
                "global_batch": int(round(pods_total / max(1, args.steps))),
                "parallelism": f"{ctx.world_size} rank(s) x 1 scheduler shard, one rank per GPU "
                               f"({ctx.backend if ctx.distributed else 'single process'})",
                **head,
                "seq_len": None,
                "waves_per_step": wps,
                "timed_region_s": round(t_max, 3),
                "nodes_per_shard": args.nodes,
                "gpus_per_shard": args.nodes * 8,
                "gang_colocation": args.gang_colocation,
                "value_kind": "sum over independent per-rank scheduler shards (one shard per GPU)",
                "attempts": stats["attempts"],
                "unschedulable_attempts": stats["unschedulable"],
                "eq_cache_filter_hit_rate": round(stats["eq_filter_hits"] / max(1, stats["eq_filter_hits"] +
                                                                                 stats["eq_filter_misses"]), 3),
                **{k: v for k, v in extras.items() if not isinstance(v, (dict, list)) and k not in head},
                "per_rank": {"pods_per_s": per_rank,
                             "spread": round((max(per_rank) - min(per_rank)) / max(1e-9, sum(per_rank) / len(per_rank)), 3)},
                "p99_gang_admit_ms": {k: v["p99_ms"] for k, v in lat.items()},
                "gang_admit": lat,
                "gang_admit_by_type": by_type,
                "gang_split": split,
                **{k: v for k, v in extras.items() if isinstance(v, (dict, list))},
            },
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    return 0


def gang_fractions(search: list[dict], loads: list[dict]) -> dict:
    """Denied and parked gang fractions of the open loop: over the served runs
    (search rungs that passed, and the 50%/90% loads), and over every run
    including the failed rung (`*_all_trials`)."""
    def frac(rs: list[dict], key: str) -> float:
        n_g = sum(r["gangs"] for r in rs)
        if key == "denied":
            n = sum(r.get("denied_gangs", (r.get("denials") or {}).get("total", 0)) for r in rs)
        else:
            n = sum(r.get("parked_gangs", 0) for r in rs)
        return round(n / max(1, n_g), 6)

    served = [*(r for r in search if r.get("served")), *loads]
    every = [*search, *loads]
    return {"denied_gang_fraction": frac(served, "denied"), "parked_gang_fraction": frac(served, "parked"),
            "denied_gang_fraction_all_trials": frac(every, "denied"),
            "parked_gang_fraction_all_trials": frac(every, "parked")}


def headline_scalars(value: float, by_type: dict, split: dict, extras: dict, world: int) -> dict:
    """Every headline number as a scalar, in priority order, led by one
    summary string holding all of them (round-5 verdict item 2)."""
    types = ("1", "2", "4", "8", "cpx4")
    out: dict = {}
    for k in types:
        if k in by_type:
            out[f"p99_gang_admit_ms_{k}"] = by_type[k]["p99_ms"]
    for k in types:
        key = f"open_loop_p99_create_to_bound_ms_{k}"
        if key in extras:
            out[key] = extras[key]
    for key in ("open_loop_capacity_pods_per_s", "nodes1024_pods_per_s", "service_mode_pods_per_s",
                "service_mode_generator_limited", "denied_gang_fraction", "parked_gang_fraction"):
        if key in extras:
            out[key] = extras[key]
    for k in types[1:]:
        if k in split:
            out[f"gang_split_fraction_{k}"] = split[k]["split_fraction"]
    if split:
        n = sum(v["n"] for v in split.values())
        out["gang_avoidable_split_fraction"] = round(sum(v["avoidable"] for v in split.values()) / max(1, n), 6)
    for key in ("open_loop_gang_split_fraction", "open_loop_gang_avoidable_split_fraction",
                "nodes1024_gang_split_fraction", "nodes1024_gang_avoidable_split_fraction"):
        if key in extras:
            out[key] = extras[key]
    # Multi-GPU placement (n/a on one GPU): verdict and placed busBW per gang
    # size, the cross-socket ratio, and whether TLP saw every GPU.
    summ = (extras.get("rccl_placement") or {}).get("summary") or {}
    rows = {str(r.get("gang")): r for r in (extras.get("rccl_placement") or {}).get("gangs", [])}
    for k in ("2", "4", "8"):
        s = summ.get(k) or {}
        placed = s.get("placed") or {}
        out[f"placement_verdict_{k}"] = s.get("verdict", "n/a") if world > 1 else "n/a"
        out[f"placed_busbw_GBps_{k}"] = (max(placed.values()) if placed and all(
            isinstance(v, (int, float)) for v in placed.values()) else "n/a") if world > 1 else "n/a"
    ratios = [r.get("cross_socket_over_placed") for r in rows.values() if r.get("cross_socket_over_placed")]
    out["cross_socket_over_placed"] = round(min(ratios), 3) if ratios and world > 1 else "n/a"
    tlp = ((extras.get("scenarios") or {}).get("trimaran_tlp") or {})
    if "gpus_sampled" in tlp:
        out["tlp_gpus_sampled"] = tlp["gpus_sampled"]
        out["tlp_replicated_from_gpu0"] = tlp.get("replicated_from_gpu0")
    summary = [f"burst={value / 1e3:.1f}k"]
    summary.append("p99_ms[" + "/".join(k for k in types if f"p99_gang_admit_ms_{k}" in out) + "]=" +
                   "/".join(str(out[f"p99_gang_admit_ms_{k}"]) for k in types if f"p99_gang_admit_ms_{k}" in out))
    if "open_loop_capacity_pods_per_s" in out:
        summary.append(f"open_loop={out['open_loop_capacity_pods_per_s'] / 1e3:.1f}k")
        summary.append("ol_p99_ms=" + "/".join(str(out.get(f"open_loop_p99_create_to_bound_ms_{k}")) for k in types))
    for key, name in (("nodes1024_pods_per_s", "n1024"), ("service_mode_pods_per_s", "service")):
        if key in out:
            summary.append(f"{name}={out[key] / 1e3:.1f}k")
    if "service_mode_generator_limited" in out:
        summary.append(f"service_generator_limited={out['service_mode_generator_limited']}")
    for key, name in (("denied_gang_fraction", "denied"), ("parked_gang_fraction", "parked")):
        if key in out:
            summary.append(f"{name}={out[key]}")
    summary.append("split[2/4/8/cpx4]=" + "/".join(str(out.get(f"gang_split_fraction_{k}", "-")) for k in types[1:]))
    for key, name in (("gang_avoidable_split_fraction", "avoidable_split"),
                      ("open_loop_gang_split_fraction", "ol_split"), ("nodes1024_gang_split_fraction", "n1024_split"),
                      ("nodes1024_gang_avoidable_split_fraction", "n1024_avoidable_split")):
        if key in out:
            summary.append(f"{name}={out[key]}")
    summary.append("placement[2/4/8]=" + "/".join(str(out[f"placement_verdict_{k}"]) for k in ("2", "4", "8")))
    return {"headline": " ".join(summary), **out}


if __name__ == "__main__":
    sys.exit(main())
