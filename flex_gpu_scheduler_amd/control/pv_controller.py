"""PersistentVolume controller: the half of volume binding that is not the
scheduler's.

The scheduler's VolumeBinding plugin (csrc/plugins/volume.cc) picks a PV for
each WaitForFirstConsumer claim and writes `spec.claimRef` on it, or marks a
claim for provisioning with `volume.kubernetes.io/selected-node`, and then
waits until the claim is fully bound. In a cluster, kube-controller-manager's
PV controller (pkg/controller/volume/persistentvolume/pv_controller.go
syncClaim / syncVolume) and an external provisioner finish that work. This
controller does the same for clusters served by this framework's API server
(and for the integration tests, the envtest analog):

  * a PV whose claimRef names a claim gets bound to it: the claim's
    `spec.volumeName`, the `pv.kubernetes.io/bind-completed` annotation and
    phase Bound on both (syncVolume / bind);
  * an unbound claim of Immediate binding mode is matched to the smallest
    fitting Available PV of its class (FindMatchingVolume with no node) or
    provisioned at once;
  * a claim with `selected-node` is provisioned on that node: a PV named
    `pvc-<claim uid>` of the requested size, with a CSI source named after the
    class's provisioner and node affinity to the node's zone (or to the node
    itself), is created pre-bound and then bound;
  * new PVs without a phase become Available.

Provisioning is done for every StorageClass provisioner except
`kubernetes.io/no-provisioner`, unless `provisioners` restricts it.
"""
from __future__ import annotations

import logging
import time

from .client import Client, is_already_exists, is_not_found
from .controllers import _Controller
from .informer import InformerFactory, meta_key, split_key

log = logging.getLogger(__name__)

ANN_SELECTED_NODE = "volume.kubernetes.io/selected-node"
ANN_BIND_COMPLETED = "pv.kubernetes.io/bind-completed"
ANN_BOUND_BY_CONTROLLER = "pv.kubernetes.io/bound-by-controller"
ANN_PROVISIONED_BY = "pv.kubernetes.io/provisioned-by"
ANN_STORAGE_CLASS_BETA = "volume.beta.kubernetes.io/storage-class"
NO_PROVISIONER = "kubernetes.io/no-provisioner"
ZONE_LABEL = "topology.kubernetes.io/zone"


def _quantity_bytes(q) -> int:
    from .._native import native

    if q is None:
        return 0
    try:
        return int(native().parse_quantity(str(q))[1])
    except Exception:  # noqa: BLE001
        return 0


def claim_class(pvc: dict) -> str:
    ann = (pvc.get("metadata") or {}).get("annotations") or {}
    if ANN_STORAGE_CLASS_BETA in ann:
        return ann[ANN_STORAGE_CLASS_BETA]
    return (pvc.get("spec") or {}).get("storageClassName") or ""


def volume_class(pv: dict) -> str:
    cls = (pv.get("spec") or {}).get("storageClassName")
    if cls is not None:
        return cls
    return ((pv.get("metadata") or {}).get("annotations") or {}).get(ANN_STORAGE_CLASS_BETA, "")


def _bound_to(pv: dict, pvc: dict) -> bool:
    ref = (pv.get("spec") or {}).get("claimRef") or {}
    md = pvc.get("metadata") or {}
    if not ref or ref.get("name") != md.get("name") or ref.get("namespace", "default") != md.get("namespace",
                                                                                                "default"):
        return False
    return not ref.get("uid") or ref.get("uid") == md.get("uid")


class PersistentVolumeController(_Controller):
    name = "PersistentVolume"

    def __init__(self, client: Client, workers: int = 1, factory: InformerFactory | None = None,
                 provisioners: set[str] | None = None):
        super().__init__(client, workers, factory)
        self.provisioners = provisioners  # None: every provisioner but no-provisioner
        self.pvc_informer = self.factory.informer("persistentvolumeclaims")
        self.pv_informer = self.factory.informer("persistentvolumes")
        self.sc_informer = self.factory.informer("storageclasses")
        self.node_informer = self.factory.informer("nodes")
        self.pvc_informer.add_event_handler(self._claim_event, lambda o, n: self._claim_event(n))
        self.pv_informer.add_event_handler(self._volume_event, lambda o, n: self._volume_event(n))
        self.provisioned = 0
        self.bound = 0

    # ------------------------------------------------------------- events
    def _claim_event(self, pvc: dict) -> None:
        self.queue.add("claim/" + meta_key(pvc))

    def _volume_event(self, pv: dict) -> None:
        self.queue.add("volume/" + pv["metadata"]["name"])
        ref = (pv.get("spec") or {}).get("claimRef")
        if ref:
            self.queue.add(f"claim/{ref.get('namespace', 'default')}/{ref.get('name')}")

    # --------------------------------------------------------------- sync
    def sync(self, key: str) -> None:
        what, rest = key.split("/", 1)
        if what == "volume":
            self._sync_volume(rest)
        else:
            ns, name = split_key(rest)
            self._sync_claim(ns, name)

    def _sync_volume(self, name: str) -> None:
        pv = self.client.get("persistentvolumes", "", name)
        if pv is None or (pv.get("status") or {}).get("phase"):
            return
        phase = "Bound" if (pv.get("spec") or {}).get("claimRef") else "Available"
        self.client.patch("persistentvolumes", "", name, {"status": {"phase": phase}})

    def _sync_claim(self, ns: str, name: str) -> None:
        pvc = self.client.get("persistentvolumeclaims", ns, name)
        if pvc is None or (pvc.get("metadata") or {}).get("deletionTimestamp"):
            return
        spec = pvc.get("spec") or {}
        ann = (pvc.get("metadata") or {}).get("annotations") or {}
        if spec.get("volumeName"):
            pv = self.client.get("persistentvolumes", "", spec["volumeName"])
            if pv is None:
                if (pvc.get("status") or {}).get("phase") == "Bound":
                    self.client.patch("persistentvolumeclaims", ns, name, {"status": {"phase": "Lost"}})
                return
            ref = (pv.get("spec") or {}).get("claimRef")
            if ref and not _bound_to(pv, pvc):
                return  # the volume belongs to another claim: leave it pending
            self._bind(pv, pvc)
            return
        # A PV pre-bound to this claim (the scheduler's PreBind, or a user).
        for pv in self.pv_informer.list(None):
            if _bound_to(pv, pvc):
                self._bind(self.client.get("persistentvolumes", "", pv["metadata"]["name"]) or pv, pvc)
                return
        cls_name = claim_class(pvc)
        sc = self.sc_informer.get("", cls_name) if cls_name else None
        if cls_name and sc is None:
            # The class may be newer than this informer's view (upstream syncs
            # its caches before the first claim; our informers start together):
            # treating a WaitForFirstConsumer claim as Immediate would bind it
            # behind the scheduler's back.
            sc = self.client.get("storageclasses", "", cls_name)
        wffc = bool(sc and sc.get("volumeBindingMode") == "WaitForFirstConsumer")
        selected = ann.get(ANN_SELECTED_NODE)
        if wffc and not selected:
            return  # the scheduler chooses the node (and maybe the volume)
        if not wffc:
            pv = self._find_matching(pvc, cls_name)
            if pv is not None:
                self._bind(pv, pvc)
                return
        if sc is not None and self._provisions(sc.get("provisioner") or ""):
            self._provision(pvc, sc, selected)

    # ----------------------------------------------------------- matching
    def _find_matching(self, pvc: dict, cls_name: str) -> dict | None:
        """FindMatchingVolume with no node (the PV controller path)."""
        want = _quantity_bytes(((pvc.get("spec") or {}).get("resources") or {}).get("requests", {}).get("storage"))
        modes = set((pvc.get("spec") or {}).get("accessModes") or [])
        vmode = (pvc.get("spec") or {}).get("volumeMode") or "Filesystem"
        def free(pv: dict) -> bool:
            return not (pv.get("spec") or {}).get("claimRef") and \
                (pv.get("status") or {}).get("phase") in (None, "", "Available")

        fits = []
        for pv in self.pv_informer.list(None):
            spec = pv.get("spec") or {}
            if not free(pv):
                continue
            if volume_class(pv) != cls_name or (spec.get("volumeMode") or "Filesystem") != vmode:
                continue
            size = _quantity_bytes((spec.get("capacity") or {}).get("storage"))
            if size < want or not modes <= set(spec.get("accessModes") or []):
                continue
            fits.append((size, pv["metadata"]["name"]))
        # The informer can lag this controller's own claimRef patches (the
        # upstream controller keeps an assumed-volume store for the same
        # reason): confirm the volume is still free on the API object.
        for _, name in sorted(fits):
            pv = self.client.get("persistentvolumes", "", name)
            if pv is not None and free(pv):
                return pv
        return None

    def _provisions(self, provisioner: str) -> bool:
        if not provisioner or provisioner == NO_PROVISIONER:
            return False
        return self.provisioners is None or provisioner in self.provisioners

    # ----------------------------------------------------------- binding
    def _bind(self, pv: dict, pvc: dict) -> None:
        md = pvc["metadata"]
        ns, name = md.get("namespace", "default"), md["name"]
        pv_name = pv["metadata"]["name"]
        ref = (pv.get("spec") or {}).get("claimRef") or {}
        if not ref.get("uid"):
            # Conditional on the version _find_matching saw (a merge patch
            # carrying metadata.resourceVersion is a precondition): with
            # several workers two claims can pick the same free volume; the
            # loser gets a 409, its sync fails and the claim is requeued to
            # look again (upstream's assume cache plays this role).
            patch = {"spec": {"claimRef": {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": ns,
                                           "name": name, "uid": md.get("uid", "")}}}
            rv = (pv.get("metadata") or {}).get("resourceVersion")
            if rv:
                patch["metadata"] = {"resourceVersion": rv}
            pv = self.client.patch("persistentvolumes", "", pv_name, patch)
        if (pv.get("status") or {}).get("phase") != "Bound":
            self.client.patch("persistentvolumes", "", pv_name, {"status": {"phase": "Bound"}})
        ann = md.get("annotations") or {}
        if (pvc.get("spec") or {}).get("volumeName") == pv_name and ann.get(ANN_BIND_COMPLETED) and \
                (pvc.get("status") or {}).get("phase") == "Bound":
            return
        new_ann = {ANN_BIND_COMPLETED: "yes"}
        if not (pvc.get("spec") or {}).get("volumeName"):
            new_ann[ANN_BOUND_BY_CONTROLLER] = "yes"
        spec = pv.get("spec") or {}
        self.client.patch("persistentvolumeclaims", ns, name, {
            "metadata": {"annotations": new_ann},
            "spec": {"volumeName": pv_name},
            "status": {"phase": "Bound", "accessModes": spec.get("accessModes") or [],
                       "capacity": spec.get("capacity") or {}}})
        self.bound += 1

    def _provision(self, pvc: dict, sc: dict, node_name: str | None) -> None:
        md = pvc["metadata"]
        spec = pvc.get("spec") or {}
        pv_name = f"pvc-{md.get('uid') or md['name']}"
        affinity = None
        if node_name:
            node = self.node_informer.get("", node_name) or {}
            zone = ((node.get("metadata") or {}).get("labels") or {}).get(ZONE_LABEL)
            term = ({"matchExpressions": [{"key": ZONE_LABEL, "operator": "In", "values": [zone]}]} if zone else
                    {"matchFields": [{"key": "metadata.name", "operator": "In", "values": [node_name]}]})
            affinity = {"required": {"nodeSelectorTerms": [term]}}
        elif sc.get("allowedTopologies"):
            exprs = [{"key": e["key"], "operator": "In", "values": list(e.get("values") or [])}
                     for e in (sc["allowedTopologies"][0].get("matchLabelExpressions") or [])]
            affinity = {"required": {"nodeSelectorTerms": [{"matchExpressions": exprs}]}}
        pv = {
            "apiVersion": "v1", "kind": "PersistentVolume",
            "metadata": {"name": pv_name, "annotations": {ANN_PROVISIONED_BY: sc["provisioner"]}},
            "spec": {
                "capacity": {"storage": ((spec.get("resources") or {}).get("requests") or {}).get("storage", "1Gi")},
                "accessModes": spec.get("accessModes") or ["ReadWriteOnce"],
                "volumeMode": spec.get("volumeMode") or "Filesystem",
                "storageClassName": sc["metadata"]["name"],
                "persistentVolumeReclaimPolicy": sc.get("reclaimPolicy") or "Delete",
                "csi": {"driver": sc["provisioner"], "volumeHandle": pv_name},
                "claimRef": {"kind": "PersistentVolumeClaim", "apiVersion": "v1",
                             "namespace": md.get("namespace", "default"), "name": md["name"],
                             "uid": md.get("uid", "")},
            },
            "status": {"phase": "Bound"},
        }
        if affinity:
            pv["spec"]["nodeAffinity"] = affinity
        try:
            created = self.client.create("persistentvolumes", pv)
        except Exception as e:  # noqa: BLE001
            if not is_already_exists(e):
                raise
            created = self.client.get("persistentvolumes", "", pv_name)
        self.provisioned += 1
        log.info("provisioned %s for claim %s/%s on %s", pv_name, md.get("namespace"), md["name"], node_name or "-")
        self._bind(created, self.client.get("persistentvolumeclaims", md.get("namespace", "default"), md["name"]) or pvc)


def wait_bound(client: Client, ns: str, name: str, timeout: float = 10.0) -> dict:
    """Test helper: the claim once fully bound."""
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        c = client.get("persistentvolumeclaims", ns, name)
        if c and (c.get("spec") or {}).get("volumeName") and \
                ((c.get("metadata") or {}).get("annotations") or {}).get(ANN_BIND_COMPLETED):
            return c
        time.sleep(0.01)
    raise TimeoutError(f"claim {ns}/{name} not bound")


__all__ = ["PersistentVolumeController", "wait_bound", "is_not_found"]
