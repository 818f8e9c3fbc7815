"""The volume plugin family (csrc/plugins/volume.cc) and the PV controller
(control/pv_controller.py): the plugins kube-scheduler 1.23 enables by default
in every profile of the reference (vendor/k8s.io/kubernetes/pkg/scheduler/
apis/config/v1beta2/default_plugins.go:41-62,94-103)."""
import time

import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.control import LocalClient
from flex_gpu_scheduler_amd.control.pv_controller import ANN_SELECTED_NODE, PersistentVolumeController, wait_bound
from flex_gpu_scheduler_amd.models import make_node, make_pod, make_pod_group
from helpers import coscheduling_config, placements, wait_bound as wait_pods_bound

V1B2 = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration"}
ZONE = "topology.kubernetes.io/zone"


def node(name, zone=None, **alloc):
    labels = {"kubernetes.io/hostname": name}
    if zone:
        labels[ZONE] = zone
    return make_node(name, {"cpu": "16", "memory": "64Gi", "pods": "110", **alloc}, labels=labels)


def sc(name, mode="WaitForFirstConsumer", provisioner="kubernetes.io/no-provisioner", topologies=None):
    o = {"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": name},
         "provisioner": provisioner, "volumeBindingMode": mode}
    if topologies:
        o["allowedTopologies"] = [{"matchLabelExpressions": [{"key": k, "values": v} for k, v in topologies.items()]}]
    return o


def pv(name, size="10Gi", cls="local", node_name=None, zone=None, claim=None, csi=None, labels=None, phase="Available"):
    o = {"apiVersion": "v1", "kind": "PersistentVolume", "metadata": {"name": name, "labels": dict(labels or {})},
         "spec": {"capacity": {"storage": size}, "accessModes": ["ReadWriteOnce"], "storageClassName": cls},
         "status": {"phase": phase}}
    if node_name:
        o["spec"]["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
            {"key": "kubernetes.io/hostname", "operator": "In", "values": [node_name]}]}]}}
    if zone:
        o["metadata"]["labels"][ZONE] = zone
    if claim:
        o["spec"]["claimRef"] = {"namespace": "default", "name": claim}
    if csi:
        o["spec"]["csi"] = {"driver": csi, "volumeHandle": name}
    return o


def pvc(name, size="5Gi", cls="local", volume=None, bound=False):
    o = {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": "default"},
         "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": size}},
                  "storageClassName": cls}}
    if volume:
        o["spec"]["volumeName"] = volume
    if bound:
        o["metadata"]["annotations"] = {"pv.kubernetes.io/bind-completed": "yes"}
        o["status"] = {"phase": "Bound"}
    return o


def with_claims(p, *claims):
    p["spec"]["volumes"] = [{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}} for i, c in enumerate(claims)]
    return p


def condition(store, name):
    for c in (store.get("pods", "default", name).get("status") or {}).get("conditions") or []:
        if c.get("type") == "PodScheduled":
            return c
    return {}


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while not pred():
        assert time.time() - t0 < timeout, "timed out"
        time.sleep(0.005)


@pytest.fixture
def pvctl(store):
    c = PersistentVolumeController(LocalClient(store)).run()
    yield c
    c.stop()


def test_default_profiles_run_the_volume_family():
    for api in ("v1beta2", "v1beta3"):
        c = load_config({"apiVersion": f"kubescheduler.config.k8s.io/{api}", "kind": "KubeSchedulerConfiguration"})
        p = c.profiles[0].plugins
        for name in ("VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits",
                     "VolumeBinding", "VolumeZone"):
            assert name in p["filter"], (api, name)
        assert "VolumeBinding" in p["preFilter"] and "VolumeBinding" in p["reserve"] and "VolumeBinding" in p["preBind"]
        assert "VolumeRestrictions" in p["preFilter"]


def test_zonal_pv_steers_placement(store):
    for n, z in (("n0", "a"), ("n1", "b"), ("n2", "c")):
        store.create("nodes", node(n, z))
    store.create("persistentvolumes", pv("data", zone="b", claim="data", cls="", phase="Bound"))
    c = pvc("data", cls="", volume="data", bound=True)
    store.create("persistentvolumeclaims", c)
    s = new_scheduler(store, load_config(V1B2), start=True)
    try:
        store.create("pods", with_claims(make_pod("p", requests={"cpu": "1"}), "data"))
        wait_pods_bound(s, 1)
        assert placements(store) == {"p": "n1"}
        out = s.explain(with_claims(make_pod("q", requests={"cpu": "1"}), "data"))
        assert out["filtered"]["n0"]["plugin"] == "VolumeZone"
        assert out["filtered"]["n0"]["reason"] == "node(s) had no available volume zone"
    finally:
        s.stop()


def test_wait_for_first_consumer_static_binding(store, pvctl):
    """Only n1 has a local PV big enough: the pod goes there, PreBind writes
    the claimRef and waits, the PV controller completes the binding."""
    for n in ("n0", "n1"):
        store.create("nodes", node(n))
    store.create("storageclasses", sc("local"))
    store.create("persistentvolumes", pv("small-n0", size="1Gi", node_name="n0"))
    store.create("persistentvolumes", pv("big-n1", size="20Gi", node_name="n1"))
    store.create("persistentvolumes", pv("mid-n1", size="8Gi", node_name="n1"))
    store.create("persistentvolumeclaims", pvc("c", size="5Gi"))
    s = new_scheduler(store, load_config(V1B2), start=True)
    try:
        store.create("pods", with_claims(make_pod("p", requests={"cpu": "1"}), "c"))
        wait_pods_bound(s, 1)
        assert placements(store) == {"p": "n1"}
        claim = wait_bound(LocalClient(store), "default", "c")
        assert claim["spec"]["volumeName"] == "mid-n1"  # smallest fit
        vol = store.get("persistentvolumes", "", "mid-n1")
        assert vol["spec"]["claimRef"]["name"] == "c" and vol["status"]["phase"] == "Bound"
        assert vol["metadata"]["annotations"]["pv.kubernetes.io/bound-by-controller"] == "yes"
    finally:
        s.stop()


def test_dynamic_provisioning_on_the_selected_node(store, pvctl):
    store.create("nodes", node("n0", "a"))
    store.create("nodes", node("n1", "b"))
    store.create("storageclasses", sc("fast", provisioner="nvme.csi.amd.com", topologies={ZONE: ["b"]}))
    store.create("persistentvolumeclaims", pvc("scratch", size="100Gi", cls="fast"))
    s = new_scheduler(store, load_config(V1B2), start=True)
    try:
        store.create("pods", with_claims(make_pod("p", requests={"cpu": "1"}), "scratch"))
        wait_pods_bound(s, 1)
        assert placements(store) == {"p": "n1"}  # allowedTopologies
        claim = wait_bound(LocalClient(store), "default", "scratch")
        assert claim["metadata"]["annotations"][ANN_SELECTED_NODE] == "n1"
        vol = store.get("persistentvolumes", "", claim["spec"]["volumeName"])
        assert vol["spec"]["csi"]["driver"] == "nvme.csi.amd.com" and pvctl.provisioned == 1
    finally:
        s.stop()


def test_gang_with_per_rank_claims_gets_distinct_volumes(store, pvctl):
    """Four ranks, four WaitForFirstConsumer claims and exactly four local PVs
    on one node: the assume cache keeps two ranks from picking the same PV
    before PreBind lands."""
    store.create("nodes", node("n0"))
    store.create("nodes", node("n1"))
    store.create("storageclasses", sc("local"))
    for i in range(4):
        store.create("persistentvolumes", pv(f"nvme{i}", node_name="n1"))
        store.create("persistentvolumeclaims", pvc(f"ckpt-{i}"))
    s = new_scheduler(store, load_config(coscheduling_config()), start=True)
    try:
        store.create("podgroups", make_pod_group("train", min_member=4))
        for i in range(4):
            store.create("pods", with_claims(make_pod(f"r{i}", pod_group="train", requests={"cpu": "1"}), f"ckpt-{i}"))
        wait_pods_bound(s, 4)
        assert set(placements(store).values()) == {"n1"}
        vols = {wait_bound(LocalClient(store), "default", f"ckpt-{i}")["spec"]["volumeName"] for i in range(4)}
        assert vols == {f"nvme{i}" for i in range(4)}
    finally:
        s.stop()


def test_pv_controller_with_stale_informers(store):
    """The controller's informers can lag the API: a StorageClass it has not
    seen yet must not turn a WaitForFirstConsumer claim into an Immediate one,
    and a PV it still sees as free must not be bound to a second claim."""
    store.create("storageclasses", sc("local"))
    store.create("storageclasses", sc("imm", mode="Immediate"))
    store.create("persistentvolumes", pv("only", cls="imm"))
    for name, cls in (("wffc", "local"), ("a", "imm"), ("b", "imm")):
        store.create("persistentvolumeclaims", pvc(name, cls=cls))
    c = PersistentVolumeController(LocalClient(store))  # informers never started: always stale
    stale_pv = store.get("persistentvolumes", "", "only")
    c.pv_informer.list = lambda _sel=None: [stale_pv]
    for name in ("wffc", "a", "b"):
        c.sync(f"claim/default/{name}")
    get = lambda n: store.get("persistentvolumeclaims", "default", n)  # noqa: E731
    assert not get("wffc")["spec"].get("volumeName")  # left for the scheduler
    assert get("a")["spec"].get("volumeName") == "only"
    assert not get("b")["spec"].get("volumeName")  # "only" is taken on the API object
    assert store.get("persistentvolumes", "", "only")["spec"]["claimRef"]["name"] == "a"


def test_claim_errors_are_unresolvable(store):
    store.create("nodes", node("n0"))
    store.create("storageclasses", sc("imm", mode="Immediate"))
    store.create("persistentvolumeclaims", pvc("pending", cls="imm"))
    s = new_scheduler(store, load_config(V1B2), start=True)
    try:
        store.create("pods", with_claims(make_pod("missing"), "nope"))
        store.create("pods", with_claims(make_pod("immediate"), "pending"))
        wait_for(lambda: condition(store, "missing").get("reason") == "Unschedulable")
        wait_for(lambda: condition(store, "immediate").get("reason") == "Unschedulable")
        assert 'persistentvolumeclaim "nope" not found' in condition(store, "missing")["message"]
        assert "pod has unbound immediate PersistentVolumeClaims" in condition(store, "immediate")["message"]
    finally:
        s.stop()


def test_no_matching_volume_and_no_provisioner(store):
    store.create("nodes", node("n0"))
    store.create("storageclasses", sc("local"))
    store.create("persistentvolumes", pv("tiny", size="1Gi", node_name="n0"))
    store.create("persistentvolumeclaims", pvc("c", size="5Gi"))
    s = new_scheduler(store, load_config(V1B2))
    s.sync_informers(50)
    out = s.explain(with_claims(make_pod("p"), "c"))
    assert out["filtered"]["n0"]["plugin"] == "VolumeBinding"
    assert out["filtered"]["n0"]["code"] == "UnschedulableAndUnresolvable"
    assert "didn't find available persistent volumes to bind" in out["filtered"]["n0"]["reason"]
    s.stop()


def test_bound_pv_node_affinity_conflict(store):
    store.create("nodes", node("n0"))
    store.create("nodes", node("n1"))
    store.create("persistentvolumes", pv("v", node_name="n0", claim="c", cls="", phase="Bound"))
    store.create("persistentvolumeclaims", pvc("c", cls="", volume="v", bound=True))
    s = new_scheduler(store, load_config(V1B2))
    s.sync_informers(50)
    out = s.explain(with_claims(make_pod("p"), "c"))
    assert out["feasible"] == ["n0"]
    assert out["filtered"]["n1"]["reason"] == "node(s) had volume node affinity conflict"
    s.stop()


def test_csi_attach_limit(store):
    store.create("nodes", node("n0"))
    store.create("csinodes", {"apiVersion": "storage.k8s.io/v1", "kind": "CSINode", "metadata": {"name": "n0"},
                              "spec": {"drivers": [{"name": "nvme.csi.amd.com", "nodeID": "n0",
                                                    "allocatable": {"count": 1}}]}})
    for i in range(2):
        store.create("persistentvolumes", pv(f"v{i}", cls="", claim=f"c{i}", csi="nvme.csi.amd.com", phase="Bound"))
        store.create("persistentvolumeclaims", pvc(f"c{i}", cls="", volume=f"v{i}", bound=True))
    store.create("pods", with_claims(make_pod("first", node_name="n0"), "c0"))
    s = new_scheduler(store, load_config(V1B2))
    s.sync_informers(50)
    out = s.explain(with_claims(make_pod("second"), "c1"))
    assert out["filtered"]["n0"]["plugin"] == "NodeVolumeLimits"
    assert out["filtered"]["n0"]["reason"] == "node(s) exceed max volume count"
    # The same volume again does not count twice.
    assert s.explain(with_claims(make_pod("again"), "c0"))["feasible"] == ["n0"]
    s.stop()


def test_intree_limits_and_disk_conflicts(store):
    store.create("nodes", node("n0", **{"attachable-volumes-aws-ebs": "1"}))
    ebs = lambda vid: [{"name": "d", "awsElasticBlockStore": {"volumeID": vid}}]  # noqa: E731
    gce = lambda pd, ro=False: [{"name": "g", "gcePersistentDisk": {"pdName": pd, "readOnly": ro}}]  # noqa: E731
    a = make_pod("a", node_name="n0")
    a["spec"]["volumes"] = ebs("vol-1") + gce("pd-1", ro=True)
    store.create("pods", a)
    s = new_scheduler(store, load_config(V1B2))
    s.sync_informers(50)

    def verdict(vols):
        p = make_pod("x")
        p["spec"]["volumes"] = vols
        out = s.explain(p)
        return out["filtered"].get("n0", {}).get("plugin", "ok"), out["filtered"].get("n0", {}).get("reason", "")

    assert verdict(ebs("vol-2")) == ("EBSLimits", "node(s) exceed max volume count")
    # EBS: any second use of the same volume conflicts.
    assert verdict(ebs("vol-1")) == ("VolumeRestrictions", "node(s) had no available disk")
    assert verdict(gce("pd-1", ro=True)) == ("ok", "")          # read-only sharing is fine
    assert verdict(gce("pd-1", ro=False)) == ("VolumeRestrictions", "node(s) had no available disk")
    s.stop()


def test_pods_without_volumes_skip_the_volume_filters(store):
    """Plugin::skip_filter: the default profile's volume plugins are not even
    called for a pod with no volumes (explain reports no volume plugin)."""
    store.create("nodes", node("n0"))
    s = new_scheduler(store, load_config(V1B2))
    s.sync_informers(50)
    out = s.explain(make_pod("p", requests={"cpu": "100"}))  # fails NodeResourcesFit only
    assert out["filtered"]["n0"]["plugin"] == "NodeResourcesFit"
    s.stop()


def test_prebind_waits_do_not_starve_other_bindings(store):
    """More pods whose claims never bind than there are binder workers: each
    VolumeBinding PreBind waits (no PV controller runs), the pool adds a worker
    per blocked wait, and an unrelated pod still binds at once (upstream
    blocks one goroutine per pod, vendor/k8s.io/kubernetes/pkg/scheduler/
    framework/plugins/volumebinding/binder.go BindPodVolumes)."""
    store.create("nodes", node("n0"))
    store.create("storageclasses", sc("fast", provisioner="nvme.csi.amd.com"))
    cfg = {**V1B2, "profiles": [{"schedulerName": "default-scheduler", "pluginConfig": [
        {"name": "VolumeBinding", "args": {"bindTimeoutSeconds": 3}}]}]}
    s = new_scheduler(store, load_config(cfg), start=True, bindWorkers=4)
    try:
        for i in range(10):
            store.create("persistentvolumeclaims", pvc(f"scratch-{i}", size="1Gi", cls="fast"))
            store.create("pods", with_claims(make_pod(f"vol-{i}", requests={"cpu": "100m"}), f"scratch-{i}"))
        wait_for(lambda: s.stats()["inflight_bindings"] >= 10, timeout=5)
        assert s.stats()["bind_threads"] >= 4 + 10 - 1
        t0 = time.time()
        store.create("pods", make_pod("plain", requests={"cpu": "100m"}))
        wait_for(lambda: placements(store).get("plain") == "n0", timeout=2)
        assert time.time() - t0 < 1.0
    finally:
        s.stop()


def test_pv_controller_claimref_patch_is_conditional(store):
    """Two claims that both saw one free volume: the second claimRef patch
    carries the version it matched against, fails with 409 (its sync is
    retried), and the volume stays bound to the first claim."""
    from flex_gpu_scheduler_amd.control.client import ApiException

    client = LocalClient(store)
    ctl = PersistentVolumeController(client)
    store.create("storageclasses", sc("imm", mode="Immediate"))
    store.create("persistentvolumes", pv("only", cls="imm"))
    a = store.create("persistentvolumeclaims", pvc("a", cls="imm"))
    b = store.create("persistentvolumeclaims", pvc("b", cls="imm"))
    stale = client.get("persistentvolumes", "", "only")
    ctl._bind(stale, a)
    with pytest.raises(ApiException) as ei:
        ctl._bind(stale, b)
    assert ei.value.code == 409
    vol = client.get("persistentvolumes", "", "only")
    assert vol["spec"]["claimRef"]["name"] == "a"
