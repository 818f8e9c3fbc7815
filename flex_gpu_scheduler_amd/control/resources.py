"""REST resource table: store kind <-> Kubernetes API path.

The native ObjectStore keys objects by plural kind ("pods", "podgroups", ...).
The HTTP API server and the REST client map those kinds onto the Kubernetes
URL layout so the wire format matches kube-apiserver for every kind the
reference touches (core pods/nodes/events/PV/PVC, storage.k8s.io StorageClass
and CSINode, scheduling.k8s.io PriorityClass,
policy PDB, coordination Lease, the scheduling.sigs.k8s.io CRDs from
apis/scheduling/v1alpha1/types.go:30-193, topology.node.k8s.io NRT) plus the
load-watcher document (vendor/github.com/paypal/load-watcher/pkg/watcher/
watcher.go:63-101), published under our own group.
"""
from __future__ import annotations

from dataclasses import dataclass
from urllib.parse import quote


@dataclass(frozen=True)
class Resource:
    kind_plural: str      # store kind
    group: str            # "" for core
    version: str
    kind: str             # object Kind
    namespaced: bool
    short_names: tuple[str, ...] = ()

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @property
    def prefix(self) -> str:
        return f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"

    def collection_path(self, ns: str = "") -> str:
        if self.namespaced and ns:
            return f"{self.prefix}/namespaces/{quote(ns)}/{self.kind_plural}"
        return f"{self.prefix}/{self.kind_plural}"

    def object_path(self, ns: str, name: str, sub: str = "") -> str:
        base = self.collection_path(ns if self.namespaced else "") + "/" + quote(name)
        return base + ("/" + sub if sub else "")


SCHEDULING_GROUP = "scheduling.sigs.k8s.io"
XSCHED_GROUP = "xsched.amd.com"

RESOURCES: dict[str, Resource] = {r.kind_plural: r for r in [
    Resource("pods", "", "v1", "Pod", True, ("po",)),
    Resource("nodes", "", "v1", "Node", False, ("no",)),
    Resource("namespaces", "", "v1", "Namespace", False, ("ns",)),
    Resource("events", "", "v1", "Event", True, ("ev",)),
    Resource("persistentvolumes", "", "v1", "PersistentVolume", False, ("pv",)),
    Resource("persistentvolumeclaims", "", "v1", "PersistentVolumeClaim", True, ("pvc",)),
    Resource("storageclasses", "storage.k8s.io", "v1", "StorageClass", False, ("sc",)),
    Resource("csinodes", "storage.k8s.io", "v1", "CSINode", False),
    Resource("priorityclasses", "scheduling.k8s.io", "v1", "PriorityClass", False, ("pc",)),
    Resource("poddisruptionbudgets", "policy", "v1", "PodDisruptionBudget", True, ("pdb",)),
    Resource("leases", "coordination.k8s.io", "v1", "Lease", True),
    Resource("podgroups", SCHEDULING_GROUP, "v1alpha1", "PodGroup", True, ("pg", "pgs")),
    Resource("elasticquotas", SCHEDULING_GROUP, "v1alpha1", "ElasticQuota", True, ("eq", "eqs")),
    Resource("noderesourcetopologies", "topology.node.k8s.io", "v1alpha1", "NodeResourceTopology", False,
             ("node-res-topo",)),
    Resource("loadwatchermetrics", XSCHED_GROUP, "v1alpha1", "WatcherMetrics", False),
]}

# (group, version, plural) -> Resource, for routing.
BY_PATH: dict[tuple[str, str, str], Resource] = {(r.group, r.version, r.kind_plural): r for r in RESOURCES.values()}


def resource(kind: str) -> Resource:
    """Look up by plural kind, Kind or short name (case-insensitive)."""
    k = kind.lower()
    if k in RESOURCES:
        return RESOURCES[k]
    for r in RESOURCES.values():
        if k == r.kind.lower() or k in r.short_names or k + "s" == r.kind_plural:
            return r
    raise KeyError(f"unknown resource kind {kind!r}")


def parse_path(path: str) -> tuple[Resource, str, str, str] | None:
    """Split an API path into (resource, namespace, name, subresource).

    Returns None when the path names no known collection.
    """
    parts = [p for p in path.split("/") if p]
    if not parts:
        return None
    if parts[0] == "api" and len(parts) >= 2:
        group, version, rest = "", parts[1], parts[2:]
    elif parts[0] == "apis" and len(parts) >= 3:
        group, version, rest = parts[1], parts[2], parts[3:]
    else:
        return None
    ns = ""
    if len(rest) >= 2 and rest[0] == "namespaces" and (len(rest) > 2):
        ns, rest = rest[1], rest[2:]
    if not rest:
        return None
    r = BY_PATH.get((group, version, rest[0]))
    if r is None:
        # /api/v1/namespaces and /api/v1/namespaces/<name> themselves
        return None
    name = rest[1] if len(rest) > 1 else ""
    sub = rest[2] if len(rest) > 2 else ""
    return r, ns, name, sub


def with_type_meta(kind: str, obj: dict) -> dict:
    r = RESOURCES[kind]
    if "apiVersion" not in obj or "kind" not in obj:
        obj = dict(obj)
        obj.setdefault("apiVersion", r.api_version)
        obj.setdefault("kind", r.kind)
    return obj
