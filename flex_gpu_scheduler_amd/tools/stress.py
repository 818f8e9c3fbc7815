"""Write the inputs of the native stress driver (csrc/tools/stress_main.cc):
nodes, NRTs, the resolved flagship scheduler config and four waves."""
from __future__ import annotations

import argparse
import json
from pathlib import Path

from ..config import load_config
from ..utils.workload import ClusterSpec, flagship_config, make_wave


def write_inputs(out: str | Path, nodes: int = 64, seed: int = 0, options: dict | None = None) -> Path:
    d = Path(out)
    d.mkdir(parents=True, exist_ok=True)
    spec = ClusterSpec(nodes=nodes)
    (d / "nodes.json").write_text(json.dumps(spec.node_objects()))
    (d / "nrts.json").write_text(json.dumps(spec.nrt_objects()))
    cfg = load_config(flagship_config()).to_native(**(options or {}))
    (d / "config.json").write_text(json.dumps(cfg))
    for i in range(4):
        w = make_wave(spec, i, namespace="bench", seed=seed)
        (d / f"wave_{i}.json").write_text(json.dumps({"namespace": "bench", "podgroups": w.pod_groups, "pods": w.pods}))
    return d


def write_workload(out: str | Path, name: str, nodes: int, pods: int, options: dict | None = None) -> Path:
    """A tools/sched_perf.py workload as stress-driver input: the measured
    pods form every wave; init pods (init.json) are created and bound before
    each wave, untimed."""
    from .sched_perf import WORKLOADS

    w = WORKLOADS[name](nodes, pods)
    d = Path(out)
    d.mkdir(parents=True, exist_ok=True)
    (d / "nodes.json").write_text(json.dumps(w["nodes"]))
    (d / "nrts.json").write_text("[]")
    cfg = load_config(w["config"]).to_native(**{**w["options"], **(options or {})})
    (d / "config.json").write_text(json.dumps(cfg))
    extra = {k: v for k, v in (w.get("extra_objects") or {}).items() if k != "podgroups"}
    if extra:
        (d / "extra.json").write_text(json.dumps(extra))
    elif (d / "extra.json").exists():
        (d / "extra.json").unlink()
    if w["init_pods"]:
        (d / "init.json").write_text(json.dumps(w["init_pods"]))
    elif (d / "init.json").exists():
        (d / "init.json").unlink()
    ns = w["pods"][0]["metadata"].get("namespace", "default")
    for i in range(4):
        wave = {"namespace": ns, "podgroups": w["extra_objects"].get("podgroups", []), "pods": w["pods"]}
        if w.get("expect_bound") is not None:
            wave["expect_bound"] = w["expect_bound"]
        (d / f"wave_{i}.json").write_text(json.dumps(wave))
    return d


def write_openloop(out: str | Path, nodes: int, rate: float, seconds: float, occupancy: float = 0.5,
                   seed: int = 0, options: dict | None = None) -> Path:
    """Inputs of the stress driver's open-loop mode: the bench cluster and one
    planned run of utils/openloop.py (Poisson gang arrivals at `rate` pods/s)."""
    from ..utils.openloop import plan

    d = write_inputs(out, nodes, seed=seed, options=options)
    gangs, _, offsets, hold_us = plan(ClusterSpec(nodes=nodes), rate, seconds, seed, occupancy=occupancy)
    (d / "openloop.json").write_text(json.dumps({"gangs": gangs, "offsets_us": offsets, "hold_us": hold_us}))
    return d


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--pods", type=int, default=1000, help="pods per wave (--workload only)")
    ap.add_argument("--workload", default="", help="a tools/sched_perf.py workload instead of the bench waves")
    ap.add_argument("--parallelism", type=int, default=16)
    ap.add_argument("--openloop", type=float, default=0.0,
                    help="open-loop mode: Poisson gang arrivals at this many pods/s (utils/openloop.py)")
    ap.add_argument("--seconds", type=float, default=1.0, help="open-loop arrival window")
    ap.add_argument("--occupancy", type=float, default=0.5, help="open-loop hold, as SPX GPU occupancy")
    a = ap.parse_args()
    if a.openloop > 0:
        write_openloop(a.out, a.nodes, a.openloop, a.seconds, a.occupancy, options={"parallelism": a.parallelism})
        return
    if (Path(a.out) / "openloop.json").exists():
        (Path(a.out) / "openloop.json").unlink()
    if a.workload:
        write_workload(a.out, a.workload, a.nodes, a.pods, options={"parallelism": a.parallelism})
    else:
        write_inputs(a.out, a.nodes, options={"parallelism": a.parallelism})


if __name__ == "__main__":
    main()
