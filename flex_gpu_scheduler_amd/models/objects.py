"""Builders for the Kubernetes objects the scheduler consumes.

Plays the role of the reference's test/util factories (test/util/utils.go:
MakePG, MakePod, MakeNodesAndPods) and of the typed API structs in
apis/scheduling/v1alpha1/types.go:30-193: every builder returns a plain
JSON-compatible dict in the exact wire shape the API server (or our store)
accepts.
"""
from __future__ import annotations

from typing import Any, Iterable, Mapping

POD_GROUP_LABEL = "pod-group.scheduling.sigs.k8s.io"
SCHEDULING_GROUP = "scheduling.sigs.k8s.io/v1alpha1"
TOPOLOGY_GROUP = "topology.node.k8s.io/v1alpha1"


def _rl(d: Mapping[str, Any] | None) -> dict:
    return {str(k): (v if isinstance(v, str) else str(v)) for k, v in (d or {}).items()}


def make_container(name: str = "c", requests: Mapping | None = None, limits: Mapping | None = None,
                   image: str = "busybox", ports: Iterable[dict] | None = None) -> dict:
    c: dict = {"name": name, "image": image, "resources": {}}
    if requests:
        c["resources"]["requests"] = _rl(requests)
    if limits:
        c["resources"]["limits"] = _rl(limits)
    if ports:
        c["ports"] = list(ports)
    return c


def make_pod(name: str, namespace: str = "default", *, requests: Mapping | None = None, limits: Mapping | None = None,
             containers: list[dict] | None = None, init_containers: list[dict] | None = None,
             pod_group: str | None = None, priority: int | None = None, priority_class: str | None = None,
             scheduler_name: str | None = None, node_name: str | None = None, labels: Mapping | None = None,
             annotations: Mapping | None = None, tolerations: list[dict] | None = None,
             node_selector: Mapping | None = None, affinity: dict | None = None, phase: str | None = None,
             overhead: Mapping | None = None, preemption_policy: str | None = None,
             uid: str | None = None) -> dict:
    md: dict = {"name": name, "namespace": namespace}
    lab = dict(labels or {})
    if pod_group:
        lab[POD_GROUP_LABEL] = pod_group
    if lab:
        md["labels"] = lab
    if annotations:
        md["annotations"] = dict(annotations)
    if uid:
        md["uid"] = uid
    spec: dict = {"containers": containers if containers is not None else [make_container(requests=requests, limits=limits)]}
    if init_containers:
        spec["initContainers"] = init_containers
    if priority is not None:
        spec["priority"] = int(priority)
    if priority_class:
        spec["priorityClassName"] = priority_class
    if scheduler_name:
        spec["schedulerName"] = scheduler_name
    if node_name:
        spec["nodeName"] = node_name
    if tolerations:
        spec["tolerations"] = tolerations
    if node_selector:
        spec["nodeSelector"] = dict(node_selector)
    if affinity:
        spec["affinity"] = affinity
    if overhead:
        spec["overhead"] = _rl(overhead)
    if preemption_policy:
        spec["preemptionPolicy"] = preemption_policy
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec}
    if phase:
        pod["status"] = {"phase": phase}
    return pod


def make_node(name: str, allocatable: Mapping | None = None, *, capacity: Mapping | None = None,
              labels: Mapping | None = None, annotations: Mapping | None = None, taints: list[dict] | None = None,
              unschedulable: bool = False) -> dict:
    alloc = _rl(allocatable or {"cpu": "32", "memory": "256Gi", "pods": "110"})
    md: dict = {"name": name, "labels": {"kubernetes.io/hostname": name, **dict(labels or {})}}
    if annotations:
        md["annotations"] = dict(annotations)
    spec: dict = {}
    if taints:
        spec["taints"] = taints
    if unschedulable:
        spec["unschedulable"] = True
    return {"apiVersion": "v1", "kind": "Node", "metadata": md, "spec": spec,
            "status": {"allocatable": alloc, "capacity": _rl(capacity) if capacity else dict(alloc)}}


def make_pod_group(name: str, namespace: str = "default", min_member: int = 1, *,
                   min_resources: Mapping | None = None, schedule_timeout_seconds: int | None = None) -> dict:
    spec: dict = {"minMember": int(min_member)}
    if min_resources:
        spec["minResources"] = _rl(min_resources)
    if schedule_timeout_seconds is not None:
        spec["scheduleTimeoutSeconds"] = int(schedule_timeout_seconds)
    return {"apiVersion": SCHEDULING_GROUP, "kind": "PodGroup", "metadata": {"name": name, "namespace": namespace},
            "spec": spec, "status": {}}


def make_elastic_quota(name: str, namespace: str, *, min: Mapping | None = None, max: Mapping | None = None) -> dict:
    spec: dict = {}
    if min is not None:
        spec["min"] = _rl(min)
    if max is not None:
        spec["max"] = _rl(max)
    return {"apiVersion": SCHEDULING_GROUP, "kind": "ElasticQuota", "metadata": {"name": name, "namespace": namespace},
            "spec": spec}


def make_nrt(node: str, zones: list[dict], policies: Iterable[str] = ("SingleNUMANodeContainerLevel",)) -> dict:
    return {"apiVersion": TOPOLOGY_GROUP, "kind": "NodeResourceTopology", "metadata": {"name": node},
            "topologyPolicies": list(policies), "zones": zones}


def nrt_zone(numa_id: int, resources: Mapping[str, Any], *, costs: Mapping[str, int] | None = None,
             available: Mapping[str, Any] | None = None) -> dict:
    res = []
    for k, v in resources.items():
        av = (available or {}).get(k, v)
        res.append({"name": k, "capacity": str(v), "allocatable": str(v), "available": str(av)})
    z: dict = {"name": f"node-{numa_id}", "type": "Node", "resources": res}
    if costs:
        z["costs"] = [{"name": k, "value": int(v)} for k, v in costs.items()]
    return z


def make_pdb(name: str, namespace: str, match_labels: Mapping[str, str], disruptions_allowed: int = 0) -> dict:
    return {"apiVersion": "policy/v1", "kind": "PodDisruptionBudget", "metadata": {"name": name, "namespace": namespace},
            "spec": {"selector": {"matchLabels": dict(match_labels)}},
            "status": {"disruptionsAllowed": int(disruptions_allowed)}}


def make_priority_class(name: str, value: int, *, annotations: Mapping | None = None,
                        preemption_policy: str | None = None, global_default: bool = False) -> dict:
    md: dict = {"name": name}
    if annotations:
        md["annotations"] = dict(annotations)
    pc: dict = {"apiVersion": "scheduling.k8s.io/v1", "kind": "PriorityClass", "metadata": md, "value": int(value),
                "globalDefault": global_default}
    if preemption_policy:
        pc["preemptionPolicy"] = preemption_policy
    return pc
