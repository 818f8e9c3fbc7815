"""Volume binding end to end over HTTP (the envtest analog of
test/integration): the API server over the native store, the remote-mode
scheduler (its own mirror, informers and native REST writes) and the PV
controller as separate clients. A gang whose ranks mount WaitForFirstConsumer
claims gets its PVs bound at PreBind, and a zonal PV steers placement."""
import time

import pytest

from flex_gpu_scheduler_amd import load_config
from flex_gpu_scheduler_amd.control import ApiServer, RestClient
from flex_gpu_scheduler_amd.control.pv_controller import PersistentVolumeController, wait_bound
from flex_gpu_scheduler_amd.control.remote import RemoteScheduler
from flex_gpu_scheduler_amd.models import GPU, make_pod, make_pod_group, mi355x_node
from helpers import FLEXGPU_PLUGINS, coscheduling_config
from test_volumes import ZONE, pv, pvc, sc, with_claims


def _wait(fn, timeout=20.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if fn():
            return True
        time.sleep(0.02)
    return bool(fn())


@pytest.fixture
def cluster(store):
    srv = ApiServer(store).start()
    client = RestClient(srv.url)
    client.url = srv.url
    ctl = PersistentVolumeController(RestClient(srv.url)).run()
    yield client
    ctl.stop()
    srv.stop()


def _node(name, zone):
    n = mi355x_node(name)
    n["metadata"]["labels"].update({ZONE: zone, "kubernetes.io/hostname": name})
    return n


def _scheduler(client):
    return RemoteScheduler(RestClient(client.url), load_config(coscheduling_config(FLEXGPU_PLUGINS))).start()


def test_gang_with_wait_for_first_consumer_claims_binds_over_http(cluster):
    client = cluster
    client.create("nodes", _node("gpu-a", "a"))
    client.create("nodes", _node("gpu-b", "b"))
    client.create("storageclasses", sc("local-nvme"))
    # Local NVMe PVs only on gpu-b: the gang must land there.
    for i in range(4):
        client.create("persistentvolumes", pv(f"nvme-b{i}", size="100Gi", cls="local-nvme", node_name="gpu-b"))
    rs = _scheduler(client)
    try:
        assert rs.native_io
        client.create("podgroups", make_pod_group("train", min_member=4))
        for i in range(4):
            client.create("persistentvolumeclaims", pvc(f"ckpt-{i}", size="50Gi", cls="local-nvme"))
            client.create("pods", with_claims(make_pod(f"rank-{i}", pod_group="train", limits={GPU: "1"},
                                                       requests={GPU: "1"}), f"ckpt-{i}"))
        assert _wait(lambda: all(p["spec"].get("nodeName") for p in client.list("pods", "default")[0]))
        pods = {p["metadata"]["name"]: p for p in client.list("pods", "default")[0]}
        assert {p["spec"]["nodeName"] for p in pods.values()} == {"gpu-b"}
        vols = set()
        for i in range(4):
            claim = wait_bound(client, "default", f"ckpt-{i}")
            vols.add(claim["spec"]["volumeName"])
            vol = client.get("persistentvolumes", "", claim["spec"]["volumeName"])
            assert vol["spec"]["claimRef"]["name"] == f"ckpt-{i}" and vol["status"]["phase"] == "Bound"
        assert vols == {f"nvme-b{i}" for i in range(4)}
        assert _wait(lambda: client.get("podgroups", "default", "train")["status"].get("phase") == "Scheduled")
    finally:
        rs.stop()


def test_zonal_pv_steers_placement_over_http(cluster):
    client = cluster
    for name, zone in (("gpu-a", "a"), ("gpu-b", "b"), ("gpu-c", "c")):
        client.create("nodes", _node(name, zone))
    client.create("persistentvolumes", pv("dataset", size="1Ti", cls="", zone="c", claim="dataset", phase="Bound"))
    client.create("persistentvolumeclaims", pvc("dataset", size="1Ti", cls="", volume="dataset"))
    rs = _scheduler(client)
    try:
        wait_bound(client, "default", "dataset")  # the PV controller completes the pre-binding
        client.create("pods", with_claims(make_pod("reader", limits={GPU: "1"}, requests={GPU: "1"}), "dataset"))
        assert _wait(lambda: client.get("pods", "default", "reader")["spec"].get("nodeName"))
        assert client.get("pods", "default", "reader")["spec"]["nodeName"] == "gpu-c"
    finally:
        rs.stop()


def test_dynamic_provisioning_over_http(cluster):
    client = cluster
    client.create("nodes", _node("gpu-a", "a"))
    client.create("nodes", _node("gpu-b", "b"))
    client.create("storageclasses", sc("scratch", provisioner="nvme.csi.amd.com", topologies={ZONE: ["a"]}))
    client.create("persistentvolumeclaims", pvc("tmp", size="200Gi", cls="scratch"))
    rs = _scheduler(client)
    try:
        client.create("pods", with_claims(make_pod("job", limits={GPU: "2"}, requests={GPU: "2"}), "tmp"))
        assert _wait(lambda: client.get("pods", "default", "job")["spec"].get("nodeName"))
        assert client.get("pods", "default", "job")["spec"]["nodeName"] == "gpu-a"
        claim = wait_bound(client, "default", "tmp")
        vol = client.get("persistentvolumes", "", claim["spec"]["volumeName"])
        assert vol["spec"]["nodeAffinity"]["required"]["nodeSelectorTerms"][0]["matchExpressions"][0]["values"] == ["a"]
    finally:
        rs.stop()
