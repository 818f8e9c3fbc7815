"""Synthetic MI355X cluster + gang workload generator (the benchmark's data).

BASELINE.json names the metric "pods/sec sched throughput + p99 PodGroup
gang-admit latency, 1/2/4/8-GPU groups" over synthetic pod specs with random
resource requests. A wave mixes, per the BASELINE configs:
  * PodGroups of 1, 2, 4 and 8 ranks, one whole MI355X per rank
    (distributed-training gangs, Coscheduling + FlexGPU + xGMI placement);
  * "4 pods x 0.25 amd.com/gpu" CPX fractional gangs (amd.com/gpu-xcd: 2);
  * shared-HBM slice pods (amd.com/gpu-memory) for inference-style packing;
with random CPU/memory requests. Waves are sized to a target fraction of
cluster GPU capacity so every wave is schedulable.
"""
from __future__ import annotations

import json
import random
from dataclasses import dataclass, field

from ..models.mi355x import GPU, GPU_MEMORY, GPU_XCD, default_gpus, mi355x_node, mi355x_nrt
from ..models.objects import POD_GROUP_LABEL, make_container, make_pod, make_pod_group

GROUP_SIZES = (1, 2, 4, 8)


@dataclass
class ClusterSpec:
    nodes: int = 64
    cpx_fraction: float = 0.25  # share of nodes whose GPUs run in CPX mode
    hbm_gib: int = 288
    cpu: str = "256"
    memory: str = "3Ti"

    def node_objects(self, prefix: str = "mi355x") -> list[dict]:
        out = []
        n_cpx = int(round(self.nodes * self.cpx_fraction))
        for i in range(self.nodes):
            mode = "cpx" if i < n_cpx else "spx"
            gpus = default_gpus(8, mode)
            for g in gpus:
                g.hbm_gib = self.hbm_gib
            out.append(mi355x_node(f"{prefix}-{i:04d}", gpus=gpus, cpu=self.cpu, memory=self.memory))
        return out

    def nrt_objects(self, prefix: str = "mi355x") -> list[dict]:
        return [mi355x_nrt(f"{prefix}-{i:04d}") for i in range(self.nodes)]

    @property
    def spx_gpus(self) -> int:
        return (self.nodes - int(round(self.nodes * self.cpx_fraction))) * 8

    @property
    def cpx_xcds(self) -> int:
        return int(round(self.nodes * self.cpx_fraction)) * 8 * 8


@dataclass
class Wave:
    pod_groups: list[dict] = field(default_factory=list)
    pods: list[dict] = field(default_factory=list)
    group_sizes: dict[str, int] = field(default_factory=dict)

    def pods_json(self) -> str:
        return json.dumps(self.pods)

    def groups_json(self) -> str:
        return json.dumps(self.pod_groups)

    def chunks_json(self, chunk: int = 64) -> list[tuple[str, str]]:
        """The wave as the API server would receive it from many job
        submitters: (PodGroups, pods) per chunk of >= `chunk` pods ending on a
        gang boundary, each chunk's PodGroups written just before its pods.
        The scheduler starts on the first gangs instead of after every
        PodGroup of the wave."""
        by_name = {pg["metadata"]["name"]: pg for pg in self.pod_groups}
        out: list[tuple[str, str]] = []
        groups: list[dict] = []
        pods: list[dict] = []
        seen: set[str] = set()
        for i, p in enumerate(self.pods):
            g = (p["metadata"].get("labels") or {}).get(POD_GROUP_LABEL, "")
            if g and g not in seen:
                seen.add(g)
                if g in by_name:
                    groups.append(by_name[g])
            pods.append(p)
            nxt = self.pods[i + 1] if i + 1 < len(self.pods) else None
            ng = (nxt["metadata"].get("labels") or {}).get(POD_GROUP_LABEL, "") if nxt else None
            if nxt is None or (len(pods) >= chunk and (not g or ng != g)):
                out.append((json.dumps(groups), json.dumps(pods)))
                groups, pods = [], []
        leftover = [pg for name, pg in by_name.items() if name not in seen]
        if leftover:  # groups without pods in this wave
            out.insert(0, (json.dumps(leftover), "[]"))
        return out


def _rand_cpu_mem(rng: random.Random) -> dict:
    return {"cpu": f"{rng.choice([500, 1000, 2000, 4000])}m", "memory": f"{rng.choice([2, 4, 8, 16])}Gi"}


def make_wave(spec: ClusterSpec, step: int, *, namespace: str = "bench", fill: float = 0.85, seed: int = 0,
              scheduler_name: str | None = None) -> Wave:
    """One wave of gangs filling ~`fill` of the SPX GPUs and CPX XCDs.

    Whole-GPU gangs (1/2/4/8 ranks) and CPX quarter gangs (4 x 0.25 GPU) are
    interleaved evenly in creation order, and named with one running index
    so the queue (PodGroup creation time, then ns/name) keeps that order: a
    burst no longer queues every CPX gang behind all whole-GPU gangs."""
    rng = random.Random(seed * 1_000_003 + step)
    w = Wave()
    gpu_budget = int(spec.spx_gpus * fill)
    # Whole-GPU gang sizes: cycle through sizes so each wave has all four.
    whole: list[int] = []
    gi = 0
    while gpu_budget > 0:
        size = GROUP_SIZES[gi % len(GROUP_SIZES)] if gi < 4 else rng.choice(GROUP_SIZES)
        gi += 1
        if size > gpu_budget:
            size = 1
        whole.append(size)
        gpu_budget -= size
    # CPX fractional gangs: 4 pods x 0.25 GPU (2 XCDs each) = one CPX GPU.
    n_cpx = max(0, int(spec.cpx_xcds * fill * 0.75) // 8)
    kinds: list[int] = []  # gang size, 0 = CPX quarter gang
    total = len(whole) + n_cpx
    wi = ci = 0
    for k in range(total):
        # Bresenham-style merge: CPX gangs at their share of the positions.
        if ci < n_cpx and (wi >= len(whole) or (ci + 1) * total <= (k + 1) * n_cpx):
            kinds.append(0)
            ci += 1
        else:
            kinds.append(whole[wi])
            wi += 1
    for k, size in enumerate(kinds):
        if size:
            name = f"s{step}-{k:04d}-x{size}"
            limits, cname, n = {GPU: "1"}, "trainer", size
        else:
            name = f"s{step}-{k:04d}-q"
            limits, cname, n = {GPU_XCD: "2"}, "shard", 4
        w.pod_groups.append(make_pod_group(name, namespace, n))
        w.group_sizes[f"{namespace}/{name}"] = n
        req = _rand_cpu_mem(rng)
        for r in range(n):
            c = make_container(cname, requests=req, limits=limits)
            w.pods.append(make_pod(f"{name}-r{r}", namespace, containers=[c], pod_group=name,
                                   scheduler_name=scheduler_name))
    # Shared-HBM inference pods packed into the remaining CPX partitions.
    for m in range(int(spec.cpx_xcds * fill * 0.25 / 2)):
        c = make_container("infer", requests=_rand_cpu_mem(rng), limits={GPU_MEMORY: str(rng.choice([8, 12, 16]))})
        w.pods.append(make_pod(f"s{step}-m{m}", namespace, containers=[c], scheduler_name=scheduler_name))
    return w


def flagship_config(permit_wait_s: int = 10, denied_s: int = 3, transient_shortage: str = "Park",
                    gang_colocation: str = "Preferred") -> dict:
    """KubeSchedulerConfiguration of the benchmark: Coscheduling gangs +
    FlexGPU MI355X packing (FlexGPU binds) + NRT xGMI gang placement.
    `transient_shortage`: "Park" (gangs short of free GPUs wait for a
    release) or "Deny" (the reference: denied for `denied_s`).
    `gang_colocation`: "Preferred" (a gang goes to a node that hosts all of
    its ranks whenever one exists), "Required" (it waits, parked, until one
    does) or "None" (score only)."""
    return {
        "apiVersion": "kubescheduler.config.k8s.io/v1beta3",
        "kind": "KubeSchedulerConfiguration",
        "profiles": [{
            "schedulerName": "default-scheduler",
            "plugins": {
                "queueSort": {"enabled": [{"name": "Coscheduling"}], "disabled": [{"name": "*"}]},
                "preFilter": {"enabled": [{"name": "Coscheduling"}, {"name": "NodeResourceTopologyMatch"}]},
                "filter": {"enabled": [{"name": "FlexGPU"}, {"name": "NodeResourceTopologyMatch"}]},
                "postFilter": {"enabled": [{"name": "Coscheduling"}]},
                "preScore": {"enabled": [{"name": "NodeResourceTopologyMatch"}]},
                "score": {"enabled": [{"name": "FlexGPU", "weight": 1},
                                      {"name": "NodeResourceTopologyMatch", "weight": 2}]},
                "reserve": {"enabled": [{"name": "Coscheduling"}, {"name": "FlexGPU"}]},
                "permit": {"enabled": [{"name": "Coscheduling"}]},
                "bind": {"enabled": [{"name": "FlexGPU"}], "disabled": [{"name": "DefaultBinder"}]},
                "postBind": {"enabled": [{"name": "Coscheduling"}]},
            },
            "pluginConfig": [
                {"name": "Coscheduling",
                 "args": {"permitWaitingTimeSeconds": permit_wait_s, "deniedPGExpirationTimeSeconds": denied_s,
                          "transientShortage": transient_shortage}},
                {"name": "NodeResourceTopologyMatch", "args": {"scoringStrategy": {"type": "XGMIGangAffinity"},
                                                               "gangColocation": gang_colocation}},
            ],
        }],
    }


def percentile(xs: list[float], q: float) -> float:
    if not xs:
        return float("nan")
    s = sorted(xs)
    k = max(0, min(len(s) - 1, int(round(q / 100.0 * (len(s) - 1)))))
    return s[k]
