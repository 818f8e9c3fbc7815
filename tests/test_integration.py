"""Multi-process-shaped integration: API server + remote-mode scheduler +
controllers talking over HTTP (the reference's envtest tier,
test/integration/coscheduling_test.go:127-372, with fake MI355X nodes as plain
API objects and no kubelet)."""
import time

import pytest

from flex_gpu_scheduler_amd import load_config
from flex_gpu_scheduler_amd.control import ApiServer, ControllerManager, RestClient
from flex_gpu_scheduler_amd.control.remote import RemoteScheduler
from flex_gpu_scheduler_amd.models import GPU, INDEX_ANNOTATION, make_pod, make_pod_group, mi355x_node

from helpers import FLEXGPU_PLUGINS, coscheduling_config


def wait_for(fn, timeout=10.0):
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
    yield srv, client
    srv.stop()


def test_remote_scheduler_places_gang_over_http(store, cluster):
    srv, client = cluster
    for n in ("n0", "n1"):
        client.create("nodes", mi355x_node(n))
    cfg = load_config(coscheduling_config(FLEXGPU_PLUGINS))
    rs = RemoteScheduler(RestClient(srv.url), cfg).start()
    mgr = ControllerManager(RestClient(srv.url)).run()
    try:
        client.create("podgroups", make_pod_group("g", min_member=4))
        for i in range(4):
            client.create("pods", make_pod(f"w{i}", pod_group="g", limits={GPU: "1"}, requests={GPU: "1"}))
        assert wait_for(lambda: all(p["spec"].get("nodeName") for p in client.list("pods", "default")[0]))
        pods = client.list("pods", "default")[0]
        assert len({p["spec"]["nodeName"] for p in pods}) >= 1
        # FlexGPU's Bind carried the GPU index annotation through v1.Binding.
        idx = [(p["spec"]["nodeName"], p["metadata"]["annotations"][INDEX_ANNOTATION]) for p in pods]
        assert len(set(idx)) == 4
        # Coscheduling PostBind patched the group through the remote API.
        assert wait_for(lambda: client.get("podgroups", "default", "g")["status"].get("phase") == "Scheduled")
        assert client.get("podgroups", "default", "g")["status"]["scheduled"] == 4
        # The controller takes it to Running once the pods run.
        for p in pods:
            client.patch("pods", "default", p["metadata"]["name"], {"status": {"phase": "Running"}})
        assert wait_for(lambda: client.get("podgroups", "default", "g")["status"].get("phase") == "Running")
    finally:
        mgr.stop()
        rs.stop()


def test_remote_scheduler_gang_waits_for_min_member(store, cluster):
    srv, client = cluster
    client.create("nodes", mi355x_node("n0"))
    rs = RemoteScheduler(RestClient(srv.url), load_config(coscheduling_config(FLEXGPU_PLUGINS, permit_wait=2))).start()
    try:
        client.create("podgroups", make_pod_group("g", min_member=3))
        for i in range(2):
            client.create("pods", make_pod(f"w{i}", pod_group="g", limits={GPU: "1"}, requests={GPU: "1"}))
        time.sleep(1.0)
        assert not any(p["spec"].get("nodeName") for p in client.list("pods", "default")[0])
        client.create("pods", make_pod("w2", pod_group="g", limits={GPU: "1"}, requests={GPU: "1"}))
        assert wait_for(lambda: all(p["spec"].get("nodeName") for p in client.list("pods", "default")[0]), 20)
    finally:
        rs.stop()
