"""CustomResourceDefinitions for the scheduling API, generated from one
schema description (reference: apis/scheduling/v1alpha1/types.go:30-193 for
PodGroup/ElasticQuota, the noderesourcetopology-api v1alpha1 types for NRT).

Wire compatibility is what matters — group, version, kinds, plural/short
names, scope and field schema match the reference's CRDs (which have no
status subresource, so status is written through the main resource, as our
scheduler and controllers do). WatcherMetrics is our addition: the
load-watcher document stored as a cluster-scoped object.

    python -m flex_gpu_scheduler_amd.deploy.crds deploy/crds
"""
from __future__ import annotations

import os
import sys

import yaml

QUANTITY = {"anyOf": [{"type": "integer"}, {"type": "string"}],
            "pattern": (r"^(\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))"
                        r"(([KMGTPE]i)|[numkMGTPE]|([eE](\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))))?$"),
            "x-kubernetes-int-or-string": True}
RESOURCE_LIST = {"type": "object", "additionalProperties": QUANTITY}


def _obj(props: dict, required: list[str] | None = None, desc: str | None = None) -> dict:
    o: dict = {"type": "object", "properties": props}
    if required:
        o["required"] = required
    if desc:
        o["description"] = desc
    return o


def _crd(group: str, kind: str, plural: str, scope: str, short: list[str], spec_schema: dict,
         status_schema: dict | None = None, extra_root: dict | None = None, version: str = "v1alpha1",
         printer: list[dict] | None = None) -> dict:
    props = {"apiVersion": {"type": "string"}, "kind": {"type": "string"}, "metadata": {"type": "object"}}
    if spec_schema is not None:
        props["spec"] = spec_schema
    if status_schema is not None:
        props["status"] = status_schema
    props.update(extra_root or {})
    ver: dict = {"name": version, "served": True, "storage": True,
                 "schema": {"openAPIV3Schema": {"type": "object", "properties": props}}}
    if printer:
        ver["additionalPrinterColumns"] = printer
    names: dict = {"kind": kind, "listKind": kind + "List", "plural": plural, "singular": kind.lower()}
    if short:
        names["shortNames"] = short
    return {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
            "metadata": {"name": f"{plural}.{group}",
                         "annotations": {"api-approved.kubernetes.io":
                                         "https://github.com/kubernetes-sigs/scheduler-plugins/pull/50"}
                         if group.endswith(".k8s.io") or group == "scheduling.sigs.k8s.io" else {}},
            "spec": {"group": group, "names": names, "scope": scope, "versions": [ver]}}


def podgroup_crd() -> dict:
    spec = _obj({
        "minMember": {"type": "integer", "format": "int32", "minimum": 1,
                      "description": "Minimum number of members that must run together (gang size)."},
        "minResources": dict(RESOURCE_LIST, description="Minimum total resources the cluster must have for "
                                                        "the group to be admitted."),
        "scheduleTimeoutSeconds": {"type": "integer", "format": "int32",
                                   "description": "How long members may wait at Permit."},
    })
    status = _obj({
        "phase": {"type": "string", "enum": ["Pending", "PreScheduling", "Scheduling", "Scheduled", "Running",
                                             "Finished", "Failed", "Unknown"]},
        "occupiedBy": {"type": "string"},
        "scheduled": {"type": "integer", "format": "int32"},
        "running": {"type": "integer", "format": "int32"},
        "succeeded": {"type": "integer", "format": "int32"},
        "failed": {"type": "integer", "format": "int32"},
        "scheduleStartTime": {"type": "string", "format": "date-time"},
    })
    printer = [{"name": "Phase", "type": "string", "jsonPath": ".status.phase"},
               {"name": "MinMember", "type": "integer", "jsonPath": ".spec.minMember"},
               {"name": "Scheduled", "type": "integer", "jsonPath": ".status.scheduled"},
               {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}]
    return _crd("scheduling.sigs.k8s.io", "PodGroup", "podgroups", "Namespaced", ["pg", "pgs"], spec, status,
                printer=printer)


def elasticquota_crd() -> dict:
    spec = _obj({"min": RESOURCE_LIST, "max": RESOURCE_LIST})
    status = _obj({"used": RESOURCE_LIST})
    return _crd("scheduling.sigs.k8s.io", "ElasticQuota", "elasticquotas", "Namespaced", ["eq", "eqs"], spec, status)


def nrt_crd() -> dict:
    named_int = _obj({"name": {"type": "string"}, "value": {"type": "integer", "format": "int64"}},
                     ["name", "value"])
    named_str = _obj({"name": {"type": "string"}, "value": {"type": "string"}}, ["name", "value"])
    resource_info = _obj({"name": {"type": "string"}, "capacity": QUANTITY, "allocatable": QUANTITY,
                          "available": QUANTITY}, ["name", "capacity", "allocatable", "available"])
    zone = _obj({"name": {"type": "string"}, "type": {"type": "string"}, "parent": {"type": "string"},
                 "costs": {"type": "array", "items": named_int},
                 "attributes": {"type": "array", "items": named_str},
                 "resources": {"type": "array", "items": resource_info}}, ["name", "type"])
    extra = {"topologyPolicies": {"type": "array", "items": {"type": "string"}},
             "zones": {"type": "array", "items": zone}}
    return _crd("topology.node.k8s.io", "NodeResourceTopology", "noderesourcetopologies", "Cluster",
                ["node-res-topo"], None, None, extra_root=extra)


def watchermetrics_crd() -> dict:
    metric = _obj({"name": {"type": "string"}, "type": {"type": "string"}, "operator": {"type": "string"},
                   "rollup": {"type": "string"}, "value": {"type": "number"}})
    extra = {"timestamp": {"type": "integer", "format": "int64"},
             "window": _obj({"duration": {"type": "string"}, "start": {"type": "integer", "format": "int64"},
                             "end": {"type": "integer", "format": "int64"}}),
             "source": {"type": "string"},
             "data": _obj({"NodeMetricsMap": {"type": "object", "additionalProperties": _obj(
                 {"metrics": {"type": "array", "items": metric},
                  "tags": {"type": "object"}, "metadata": {"type": "object",
                                                           "x-kubernetes-preserve-unknown-fields": True}})}})}
    return _crd("xsched.amd.com", "WatcherMetrics", "loadwatchermetrics", "Cluster", ["lwm"], None, None,
                extra_root=extra)


ALL = {"scheduling.sigs.k8s.io_podgroups.yaml": podgroup_crd,
       "scheduling.sigs.k8s.io_elasticquotas.yaml": elasticquota_crd,
       "topology.node.k8s.io_noderesourcetopologies.yaml": nrt_crd,
       "xsched.amd.com_loadwatchermetrics.yaml": watchermetrics_crd}


def write_all(out_dir: str) -> list[str]:
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for fn, make in ALL.items():
        p = os.path.join(out_dir, fn)
        with open(p, "w") as f:
            f.write("# Generated by flex_gpu_scheduler_amd.deploy.crds; do not edit.\n---\n")
            yaml.safe_dump(make(), f, sort_keys=False, width=120)
        paths.append(p)
    return paths


if __name__ == "__main__":
    print("\n".join(write_all(sys.argv[1] if len(sys.argv) > 1 else "deploy/crds")))
