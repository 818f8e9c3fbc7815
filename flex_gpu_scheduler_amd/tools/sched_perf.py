"""scheduler_perf-style throughput matrix.

Upstream kube-scheduler measures its plugins with a matrix of workloads
(test/integration/scheduler_perf: SchedulingBasic, SchedulingPodAntiAffinity,
SchedulingPodAffinity, the Preferred* variants, TopologySpreading,
SchedulingNodeAffinity, PreemptionBasic, Unschedulable, ...) on 500 and
5,000 fake nodes. The reference suite inherits that harness through its
vendored scheduler but publishes no results. This tool runs the
same shapes against our scheduler — in-process store, default plugin set
unless the workload needs another profile — plus the MI355X workloads
(FlexGPU whole/XCD/HBM mix, Coscheduling gangs), and reports pods/s of the
measured phase (create the measured pods -> all bound).

    python -m flex_gpu_scheduler_amd.tools.sched_perf [--nodes 500] [--pods 1000] [--only NAME ...]
"""
from __future__ import annotations

import argparse
import json
import sys
import time

from ..config import load_config
from ..models import GPU, GPU_MEMORY, GPU_XCD, make_node, make_pod, make_pod_group, mi355x_node
from ..scheduler import Store, new_scheduler
from ..utils.workload import flagship_config

ZONE = "topology.kubernetes.io/zone"


def _nodes_plain(n: int) -> list[dict]:
    return [make_node(f"node-{i}", {"cpu": "32", "memory": "128Gi", "pods": "110"},
                      labels={ZONE: f"zone-{i % 3}", "disktype": "ssd" if i % 2 else "hdd"}) for i in range(n)]


def _wait_bound(sched, target: int, timeout: float) -> bool:
    return sched.wait_bound(target, timeout)  # native wait, GIL released


def _spec(name: str, nodes: list[dict], init_pods: list[dict], pods: list[dict], *, config=None, options=None,
          extra_objects: dict | None = None, expect_bound: int | None = None) -> dict:
    """A workload: everything needed to run it here or in the native stress
    driver (tools/stress.py --workload)."""
    return {"name": name, "nodes": nodes, "init_pods": init_pods, "pods": pods, "config": config,
            "options": options or {}, "extra_objects": extra_objects or {}, "expect_bound": expect_bound}


def run_spec(w: dict, timeout: float = 120.0) -> dict:
    return _run(w["name"], w["nodes"], w["init_pods"], w["pods"], config=w["config"], options=w["options"],
                extra_objects=w["extra_objects"], expect_bound=w.get("expect_bound"), timeout=timeout)


def _run(name: str, nodes: list[dict], init_pods: list[dict], pods: list[dict], *, config=None, options=None,
         extra_objects: dict | None = None, expect_bound: int | None = None, timeout: float = 120.0) -> dict:
    store = Store()
    store.create_many("nodes", json.dumps(nodes))
    for kind, objs in (extra_objects or {}).items():
        store.create_many(kind, json.dumps(objs))
    sched = new_scheduler(store, load_config(config), **(options or {}))
    sched.start()
    try:
        if init_pods:
            store.create_many("pods", json.dumps(init_pods))
            if not _wait_bound(sched, len(init_pods), timeout):
                return {"workload": name, "error": f"init pods not bound: {sched.stats()}"}
        base = sched.stats()["bound"]
        want = expect_bound if expect_bound is not None else len(pods)
        payload = json.dumps(pods)  # data preparation, outside the measured phase
        t0 = time.perf_counter()
        store.create_many("pods", payload)
        ok = _wait_bound(sched, base + want, timeout)
        dt = time.perf_counter() - t0
        st = sched.stats()
        out = {"workload": name, "nodes": len(nodes), "init_pods": len(init_pods), "pods": len(pods),
               "bound": st["bound"] - base, "seconds": round(dt, 4),
               "pods_per_s": round((st["bound"] - base) / dt, 1) if dt > 0 else None,
               "attempts": st["attempts"], "unschedulable_attempts": st["unschedulable"]}
        if not ok:
            out["error"] = f"timeout: {st['bound'] - base}/{want} bound"
        return out
    finally:
        sched.stop()


def scheduling_basic(n_nodes: int, n_pods: int) -> dict:
    init = [make_pod(f"init-{i}", requests={"cpu": "100m", "memory": "100Mi"}) for i in range(n_nodes)]
    pods = [make_pod(f"p-{i}", requests={"cpu": "100m", "memory": "100Mi"}) for i in range(n_pods)]
    return _spec("SchedulingBasic", _nodes_plain(n_nodes), init, pods)


def pod_anti_affinity(n_nodes: int, n_pods: int) -> dict:
    n = min(n_pods, n_nodes)  # one per node by construction
    aff = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"color": "green"}}, "topologyKey": "kubernetes.io/hostname"}]}}
    pods = [make_pod(f"aa-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"color": "green"}, affinity=aff)
            for i in range(n)]
    return _spec("SchedulingPodAntiAffinity", _nodes_plain(n_nodes), [], pods)


def topology_spreading(n_nodes: int, n_pods: int) -> dict:
    def pod(i):
        p = make_pod(f"ts-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"app": "spread"})
        p["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": ZONE,
                                                   "whenUnsatisfiable": "DoNotSchedule",
                                                   "labelSelector": {"matchLabels": {"app": "spread"}}}]
        return p
    return _spec("TopologySpreading", _nodes_plain(n_nodes), [], [pod(i) for i in range(n_pods)])


def pod_affinity(n_nodes: int, n_pods: int) -> dict:
    # Required affinity (zone) to a group of seed pods that all live in zone-0.
    init = [make_pod(f"seed-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"color": "blue"},
                     node_selector={ZONE: "zone-0"}) for i in range(max(1, n_nodes // 30))]
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"color": "blue"}}, "topologyKey": ZONE}]}}
    pods = [make_pod(f"pa-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"color": "blue"}, affinity=aff)
            for i in range(n_pods)]
    return _spec("SchedulingPodAffinity", _nodes_plain(n_nodes), init, pods)


def preferred_pod_affinity(n_nodes: int, n_pods: int) -> dict:
    aff = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 1, "podAffinityTerm": {"labelSelector": {"matchLabels": {"color": "red"}},
                                          "topologyKey": "kubernetes.io/hostname"}}]}}
    pods = [make_pod(f"ppa-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"color": "red"}, affinity=aff)
            for i in range(n_pods)]
    return _spec("SchedulingPreferredPodAffinity", _nodes_plain(n_nodes), [], pods)


def preferred_pod_anti_affinity(n_nodes: int, n_pods: int) -> dict:
    aff = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 1, "podAffinityTerm": {"labelSelector": {"matchLabels": {"color": "yellow"}},
                                          "topologyKey": "kubernetes.io/hostname"}}]}}
    pods = [make_pod(f"ppaa-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"color": "yellow"},
                     affinity=aff) for i in range(n_pods)]
    return _spec("SchedulingPreferredPodAntiAffinity", _nodes_plain(n_nodes), [], pods)


def preferred_topology_spreading(n_nodes: int, n_pods: int) -> dict:
    def pod(i):
        p = make_pod(f"pts-{i}", requests={"cpu": "100m", "memory": "100Mi"}, labels={"app": "soft"})
        p["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": ZONE,
                                                   "whenUnsatisfiable": "ScheduleAnyway",
                                                   "labelSelector": {"matchLabels": {"app": "soft"}}}]
        return p
    return _spec("PreferredTopologySpreading", _nodes_plain(n_nodes), [], [pod(i) for i in range(n_pods)])


def unschedulable(n_nodes: int, n_pods: int) -> dict:
    # 200 pods that fit nowhere sit in the unschedulable queue while the
    # measured pods schedule (upstream "Unschedulable" shape).
    stuck = [make_pod(f"huge-{i}", requests={"cpu": "9000", "memory": "1Gi"}) for i in range(200)]
    pods = [make_pod(f"u-{i}", requests={"cpu": "100m", "memory": "100Mi"}) for i in range(n_pods)]
    return _spec("Unschedulable", _nodes_plain(n_nodes), [], stuck + pods, expect_bound=n_pods)


def node_affinity(n_nodes: int, n_pods: int) -> dict:
    aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": "disktype", "operator": "In", "values": ["ssd"]}]}]}}}
    pods = [make_pod(f"na-{i}", requests={"cpu": "100m", "memory": "100Mi"}, affinity=aff) for i in range(n_pods)]
    return _spec("SchedulingNodeAffinity", _nodes_plain(n_nodes), [], pods)


def preemption_basic(n_nodes: int, n_pods: int) -> dict:
    # Fill every node with 4 low-priority pods of 8 CPUs, then ask for
    # high-priority 8-CPU pods that each need one victim (upstream shape).
    n = min(n_pods, n_nodes)
    init = [make_pod(f"low-{i}", requests={"cpu": "8", "memory": "1Gi"}, priority=1) for i in range(4 * n_nodes)]
    pods = [make_pod(f"high-{i}", requests={"cpu": "8", "memory": "1Gi"}, priority=1000) for i in range(n)]
    return _spec("PreemptionBasic", _nodes_plain(n_nodes), init, pods,
                options={"podInitialBackoffSeconds": 0.01, "podMaxBackoffSeconds": 0.1})


def mi355x_flexgpu_mix(n_nodes: int, n_pods: int) -> dict:
    nodes = [mi355x_node(f"mi355x-{i}", mode="cpx" if i % 4 == 3 else "spx") for i in range(n_nodes)]
    pods = []
    for i in range(n_pods):
        k = i % 4
        lim = {GPU: "1"} if k == 0 else {GPU_XCD: "2"} if k == 1 else {GPU_MEMORY: "24"} if k == 2 else {}
        pods.append(make_pod(f"g-{i}", requests={"cpu": "1", "memory": "4Gi"}, limits=lim or None))
    return _spec("MI355X-FlexGPUMix", nodes, [], pods, config=flagship_config())


def mi355x_gangs(n_nodes: int, n_pods: int) -> dict:
    nodes = [mi355x_node(f"mi355x-{i}") for i in range(n_nodes)]
    size = 8
    groups = max(1, n_pods // size)
    pgs = [make_pod_group(f"gang-{g}", "default", size) for g in range(groups)]
    pods = [make_pod(f"r-{g}-{r}", pod_group=f"gang-{g}", requests={"cpu": "8", "memory": "64Gi"}, limits={GPU: "1"})
            for g in range(groups) for r in range(size)]
    return _spec("MI355X-Gang8", nodes, [], pods, config=flagship_config(), extra_objects={"podgroups": pgs})


def _capacity_config() -> dict:
    """Default plugins plus CapacityScheduling (its PostFilter replaces
    DefaultPreemption), as manifests/capacityscheduling/scheduler-config.yaml."""
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": {
                "preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
                "postFilter": {"enabled": [{"name": "CapacityScheduling"}], "disabled": [{"name": "*"}]},
                "reserve": {"enabled": [{"name": "CapacityScheduling"}]}}}]}


def _quotas(n_nodes: int, share: float = 0.5) -> list[dict]:
    """Two namespaces, each guaranteed `share` of the cluster's CPU and
    memory and allowed to borrow up to all of it."""
    from ..models import make_elastic_quota

    cpu, mem = 32 * n_nodes, 128 * n_nodes
    mn = {"cpu": str(int(cpu * share)), "memory": f"{int(mem * share)}Gi"}
    mx = {"cpu": str(cpu), "memory": f"{mem}Gi"}
    return [make_elastic_quota(f"quota-{ns}", ns, min=mn, max=mx) for ns in ("team-a", "team-b")]


def capacity_admission(n_nodes: int, n_pods: int) -> dict:
    """SchedulingBasic with every pod under an ElasticQuota (2 namespaces
    sharing the cluster): the per-cycle quota snapshot, nominated-pod sums
    and Reserve accounting on the admission path."""
    init = [make_pod(f"init-{i}", ("team-a", "team-b")[i % 2], requests={"cpu": "100m", "memory": "100Mi"})
            for i in range(n_nodes)]
    pods = [make_pod(f"p-{i}", ("team-a", "team-b")[i % 2], requests={"cpu": "100m", "memory": "100Mi"})
            for i in range(n_pods)]
    return _spec("CapacityScheduling-Admission", _nodes_plain(n_nodes), init, pods, config=_capacity_config(),
                 extra_objects={"elasticquotas": _quotas(n_nodes)})


def capacity_reclaim(n_nodes: int, n_pods: int) -> dict:
    """PreemptionBasic across quotas: team-a borrowed the whole cluster (4
    pods of 8 CPUs per node, beyond its 50% min); team-b's pods, within its
    min, each reclaim one borrowed pod (capacity_scheduling.go:465-644)."""
    n = min(n_pods, n_nodes)
    init = [make_pod(f"borrow-{i}", "team-a", requests={"cpu": "8", "memory": "1Gi"}, priority=1)
            for i in range(4 * n_nodes)]
    pods = [make_pod(f"reclaim-{i}", "team-b", requests={"cpu": "8", "memory": "1Gi"}, priority=1)
            for i in range(n)]
    return _spec("CapacityScheduling-Reclaim", _nodes_plain(n_nodes), init, pods, config=_capacity_config(),
                 extra_objects={"elasticquotas": _quotas(n_nodes)},
                 options={"podInitialBackoffSeconds": 0.01, "podMaxBackoffSeconds": 0.1})


WORKLOADS = {
    "SchedulingBasic": scheduling_basic,
    "SchedulingPodAntiAffinity": pod_anti_affinity,
    "TopologySpreading": topology_spreading,
    "SchedulingPodAffinity": pod_affinity,
    "SchedulingPreferredPodAffinity": preferred_pod_affinity,
    "SchedulingPreferredPodAntiAffinity": preferred_pod_anti_affinity,
    "PreferredTopologySpreading": preferred_topology_spreading,
    "Unschedulable": unschedulable,
    "SchedulingNodeAffinity": node_affinity,
    "PreemptionBasic": preemption_basic,
    "MI355X-FlexGPUMix": mi355x_flexgpu_mix,
    "MI355X-Gang8": mi355x_gangs,
    "CapacityScheduling-Admission": capacity_admission,
    "CapacityScheduling-Reclaim": capacity_reclaim,
}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nodes", type=int, default=500)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--cpus", default="none", help="utils/cpuaffinity.py mode (l3 on the GPU box)")
    a = ap.parse_args()
    if a.cpus != "none":
        from ..utils.cpuaffinity import apply
        apply(a.cpus)
    for name, fn in WORKLOADS.items():
        if a.only and name not in a.only:
            continue
        try:
            r = run_spec(fn(a.nodes, a.pods))
        except Exception as e:  # noqa: BLE001 - one workload failing must not hide the others
            r = {"workload": name, "error": f"{type(e).__name__}: {e}"}
        print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
