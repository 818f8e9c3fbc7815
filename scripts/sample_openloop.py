"""One open-loop trial (utils/openloop.py, as the bench's capacity search runs
it) under the timestamped sampler, to see which thread limits the sustained
rate near the capacity cliff.

    python scripts/sample_openloop.py OUTDIR --rate 106000 [--nodes 64]
    python scripts/sample_openloop.py OUTDIR --sequence 102371,118500,106400

With --sequence, no sampling: the trials run back to back on one shard, as
the capacity search runs them, and each one's p99 is printed.

Writes OUTDIR/openloop.samples (symbolize against the extension .so) and
OUTDIR/openloop_trial.json (the trial's summary without per-gang rows).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from flex_gpu_scheduler_amd._native import native  # noqa: E402
from flex_gpu_scheduler_amd.utils.benchrun import Shard  # noqa: E402
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply  # noqa: E402
from flex_gpu_scheduler_amd.utils.openloop import run_open_loop  # noqa: E402
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--rate", type=float, default=106_000.0)
    ap.add_argument("--hz", type=int, default=4000)
    ap.add_argument("--sequence", default="")
    ap.add_argument("--seed", type=int, default=7, help="Shard seed (bench.py uses 0 for rank 0)")
    ap.add_argument("--waves", type=int, default=4, help="burst waves before the open-loop trials")
    ap.add_argument("--sample-last", action="store_true", help="with --sequence: sample the last trial")
    ap.add_argument("--trim", action="store_true", help="malloc_trim(0) after every trial (heap-state A/B)")
    ap.add_argument("--prerender", action="store_true",
                    help="render every warm wave's JSON up front and drop it afterwards, as bench.py does")
    ap.add_argument("--torch", action="store_true", help="initialise torch and the GPU first, as bench.py does")
    ap.add_argument("--options", default="{}", help="scheduler options JSON, e.g. '{\"events\": false}'")
    ap.add_argument("--fresh-sched-after", type=int, default=-2,
                    help="with --sequence: a new scheduler on the same store after trial N (0-based)")
    ap.add_argument("--fresh-after", type=int, default=-2,
                    help="with --sequence: replace the shard by a fresh one (same process) after trial N (0-based)")
    ap.add_argument("--torch-after-pin", action="store_true", help="initialise them after the CPU pinning")
    ap.add_argument("--colocation", default="Preferred", help="NRT gangColocation of the flagship profile")
    ap.add_argument("--settle", type=float, default=0.0,
                    help="with --fresh-after: seconds to wait (after malloc_trim) once the old shard is dropped")
    ap.add_argument("--pin", default="l3", help="shard CPU placement (utils/cpuaffinity.py): l3 | l3x2 | none")
    ap.add_argument("--detail", action="store_true",
                    help="with --sequence: per-type p99, generator lags and the 5-ms timeline of every trial")
    a = ap.parse_args()

    def init_torch():
        import torch

        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")

    if a.torch:
        init_torch()
    os.makedirs(a.out, exist_ok=True)
    apply(a.pin)
    if a.torch_after_pin:
        init_torch()
    from flex_gpu_scheduler_amd.utils.workload import flagship_config

    shard = Shard(ClusterSpec(nodes=a.nodes), namespace="sample", seed=a.seed, options=json.loads(a.options),
                  config=flagship_config(gang_colocation=a.colocation))
    try:
        # Warm the shard as the bench does before its search: burst waves,
        # then one open-loop trial well below the cliff.
        if a.prerender:
            ws = [shard.wave(i) for i in range(a.waves)]
            prepared = [w.chunks_json() for w in ws]
            for w, pj in zip(ws, prepared):
                shard.run(w, prepared=pj, collect_gangs=False)
            del ws, prepared
            if a.trim:
                import ctypes
                ctypes.CDLL("libc.so.6").malloc_trim(0)
        else:
            for i in range(a.waves):
                w = shard.wave(i)
                shard.run(w, prepared=w.chunks_json(), collect_gangs=False)
        if a.sequence:
            rows = []
            rates = [float(x) for x in a.sequence.split(",")]

            def gate_waits() -> dict:
                out = {}
                for line in shard.sched.metrics_text().splitlines():
                    if line.startswith("xsched_coscheduling_gate_waits_total{"):
                        k, v = line.rsplit(" ", 1)
                        out[k[k.index("{") + 1:k.rindex("}")].replace('"', "")] = float(v)
                return out
            for i, rate in enumerate(rates):
                if i == a.fresh_sched_after + 1:
                    # Scheduler state vs store state: the store (and its
                    # watchers' history) stays, the scheduler is new.
                    from flex_gpu_scheduler_amd import load_config, new_scheduler
                    from flex_gpu_scheduler_amd.utils.workload import flagship_config

                    shard.sched.stop()
                    shard.sched = new_scheduler(shard.store, load_config(flagship_config()), seed=shard.seed + 1)
                    shard.sched.start()
                    print(json.dumps({"fresh_scheduler_before_trial": i}), flush=True)
                if i == a.fresh_after + 1:
                    # Shard state vs process state: a new store and scheduler
                    # in the same process (same heap), warmed as the first.
                    shard.close()
                    shard = None
                    if a.settle > 0:
                        import ctypes
                        import gc
                        import time

                        gc.collect()
                        time.sleep(a.settle)
                        ctypes.CDLL("libc.so.6").malloc_trim(0)
                    shard = Shard(ClusterSpec(nodes=a.nodes), namespace="sample2", seed=a.seed,
                                  config=flagship_config(gang_colocation=a.colocation))
                    for j in range(4):
                        w = shard.wave(j)
                        shard.run(w, prepared=w.chunks_json(), collect_gangs=False)
                    print(json.dumps({"fresh_shard_before_trial": i}), flush=True)
                last = i == len(rates) - 1
                if last and a.sample_last:
                    native().sampler_start(a.hz, 4_000_000)
                gw0 = gate_waits() if a.detail else {}
                r = run_open_loop(shard, rate, 1.0, seed=0, timeline=a.detail)
                gw1 = gate_waits() if a.detail else {}
                if last and a.sample_last:
                    native().sampler_dump(os.path.join(a.out, "openloop.samples"))
                if a.trim:
                    import ctypes
                    ctypes.CDLL("libc.so.6").malloc_trim(0)
                rows.append({"offered_pods_per_s": rate, "wall_s": r["wall_s"], "parked_gangs": r["parked_gangs"],
                             **{k: r["all_gangs"][k] for k in ("p99_create_to_bound_ms", "max_create_to_bound_ms")},
                             "queue_after": shard.sched.queue_counts(),
                             "store_pods": len(shard.store.list("pods", "")[0]) if hasattr(shard, "store") else None})
                if a.detail:
                    rows[-1].update({
                        "by_type_p99_ms": {k: v["create_to_bound_ms"]["p99"] for k, v in r["by_gang"].items()},
                        "by_type_e2a_p99_ms": {k: v["enqueue_to_allow_ms"]["p99"] for k, v in r["by_gang"].items()},
                        "mean_arrival_lag_us": r.get("mean_arrival_lag_us"),
                        "mean_delete_lag_us": r.get("mean_delete_lag_us"),
                        "max_in_flight_pods": r.get("max_in_flight_pods"), "max_held_pods": r.get("max_held_pods"),
                        "hold_ms": r.get("hold_ms"), "denials": r.get("denials", {}).get("total"),
                        "gate_waits": {k: int(v - gw0.get(k, 0)) for k, v in gw1.items() if v - gw0.get(k, 0)},
                        # per 5 ms: pods in flight, pods held, attempts, unschedulable, parks
                        "timeline": r.get("timeline", [])})
                print(json.dumps({k: v for k, v in rows[-1].items() if k != "timeline"}), flush=True)
            with open(os.path.join(a.out, "openloop_sequence.jsonl"), "w") as f:
                f.writelines(json.dumps(x) + "\n" for x in rows)
            return 0
        run_open_loop(shard, a.rate / 2, 1.0, seed=0)
        native().sampler_start(a.hz, 4_000_000)
        r = run_open_loop(shard, a.rate, 1.0, seed=0, timeline=True)
        native().sampler_dump(os.path.join(a.out, "openloop.samples"))
    finally:
        shard.close()
    keep = {k: v for k, v in r.items() if k not in ("by_gang",)}
    with open(os.path.join(a.out, "openloop_trial.json"), "w") as f:
        json.dump(keep, f)
    print(json.dumps({k: keep[k] for k in ("offered_pods_per_s", "all_gangs", "wall_s", "parked_gangs",
                                             "max_in_flight_pods", "max_held_pods", "hold_ms")}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
