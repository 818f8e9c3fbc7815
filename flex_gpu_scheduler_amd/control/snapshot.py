"""Checkpoint / restore of the API store as JSON.

The reference keeps no scheduler checkpoint — all state is soft and rebuilt
from LIST/WATCH; its durable state lives in etcd. Our API
server's store is in-memory, so it can dump every object to a JSON file and
load it back (server restart, benchmark replay). Objects keep uid and
creationTimestamp; resourceVersions restart.
"""
from __future__ import annotations

import json
import os
import tempfile

from .resources import RESOURCES

# Restore order: namespaces and cluster objects first, pods last.
ORDER = ("namespaces", "priorityclasses", "storageclasses", "nodes", "csinodes", "noderesourcetopologies",
         "persistentvolumes", "persistentvolumeclaims", "podgroups", "elasticquotas",
         "poddisruptionbudgets", "leases", "loadwatchermetrics", "events", "pods")


def snapshot(store) -> dict:
    out = {"apiVersion": "xsched.amd.com/v1alpha1", "kind": "StoreSnapshot", "resourceVersion":
           store.resource_version, "objects": {}}
    for kind in RESOURCES:
        items, _ = store.list_json(kind, "")
        objs = json.loads(items)
        if objs:
            out["objects"][kind] = objs
    return out


def restore(store, snap: dict) -> int:
    n = 0
    objs = snap.get("objects") or {}
    for kind in list(ORDER) + [k for k in objs if k not in ORDER]:
        items = objs.get(kind) or []
        for o in items:
            o.get("metadata", {}).pop("resourceVersion", None)
        if items:
            n += store.create_many(kind, items)
    return n


def snapshot_to_file(store, path: str) -> None:
    data = json.dumps(snapshot(store), separators=(",", ":"))
    d = os.path.dirname(os.path.abspath(path))
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".snap-")
    with os.fdopen(fd, "w") as f:
        f.write(data)
    os.replace(tmp, path)
