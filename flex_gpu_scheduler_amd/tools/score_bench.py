"""Score-path micro-benchmark, the reference's BenchmarkTargetLoadPackingPlugin
(pkg/trimaran/targetloadpacking/targetloadpacking_test.go:267-360): one pod
scored by TargetLoadPacking over 100 / 1,000 / 5,000 nodes of 64 CPUs and
346Gi, every node reporting 0% CPU (Latest), Score node-parallel then
NormalizeScore, per pass. The reference ships the harness without results;
this prints ours. `--mi355x` adds the MI355X scorers (FlexGPU, NRT
XGMIGangAffinity) on 8xMI355X nodes for the same node counts.

    python -m flex_gpu_scheduler_amd.tools.score_bench [--iterations 200] [--mi355x]
"""
from __future__ import annotations

import argparse
import json

from .. import Store, load_config, new_scheduler
from ..models import GPU, make_node, make_pod, mi355x_node, mi355x_nrt


def _cfg(mi355x: bool) -> dict:
    score = ([{"name": "FlexGPU", "weight": 1}, {"name": "NodeResourceTopologyMatch", "weight": 2}] if mi355x
             else [{"name": "TargetLoadPacking", "weight": 1}])
    plugins = {"score": {"enabled": score, "disabled": [{"name": "*"}]}}
    if mi355x:
        plugins["preScore"] = {"enabled": [{"name": "NodeResourceTopologyMatch"}], "disabled": [{"name": "*"}]}
    pc = [{"name": "NodeResourceTopologyMatch", "args": {"scoringStrategy": {"type": "XGMIGangAffinity"}}}] \
        if mi355x else [{"name": "TargetLoadPacking", "args": {"watcherAddress": "http://unused:2020"}}]
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": plugins, "pluginConfig": pc}]}


def run(nodes: int, iterations: int, mi355x: bool = False) -> dict:
    store = Store()
    if mi355x:
        store.create_many("nodes", json.dumps([mi355x_node(f"node-{i}") for i in range(nodes)]))
        store.create_many("noderesourcetopologies", json.dumps([mi355x_nrt(f"node-{i}") for i in range(nodes)]))
    else:
        store.create_many("nodes", json.dumps([make_node(f"node-{i}", {"cpu": "64000m", "memory": "346Gi",
                                                                         "pods": "110"}) for i in range(nodes)]))
        store.create("loadwatchermetrics", {
            "metadata": {"name": "load-watcher"}, "timestamp": 0, "window": {"duration": "15m", "start": 0, "end": 0},
            "source": "bench", "data": {"NodeMetricsMap": {
                f"node-{i}": {"metrics": [{"type": "CPU", "operator": "Latest", "value": 0}]} for i in range(nodes)}}})
    s = new_scheduler(store, load_config(_cfg(mi355x)))
    try:
        s.sync_informers(200)
        pod = make_pod("p", labels={"foo": ""}, limits={GPU: "1"}) if mi355x else make_pod("p", labels={"foo": ""})
        s.score_benchmark(pod, 5)  # warm
        r = s.score_benchmark(pod, iterations)
        return {"nodes": r["nodes"], "us_per_pass": round(r["us_per_pass"], 2),
                "ns_per_node": round(1000 * r["us_per_pass"] / max(1, r["nodes"]), 1),
                "scorers": "FlexGPU+NRT(XGMI)" if mi355x else "TargetLoadPacking"}
    finally:
        s.stop()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=200)
    ap.add_argument("--mi355x", action="store_true")
    a = ap.parse_args()
    out = [run(n, a.iterations, False) for n in (100, 1000, 5000)]
    if a.mi355x:
        out += [run(n, a.iterations, True) for n in (100, 1000, 5000)]
    print(json.dumps({"benchmark": "score pass (PreScore + parallel Score + NormalizeScore)", "results": out}))


if __name__ == "__main__":
    main()
