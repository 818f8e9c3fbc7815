"""Node agent, sysfs discovery and telemetry — replayed against a capture of
a real 8x MI355X box (tests/fixtures/mi355x_box, taken with
`python -m flex_gpu_scheduler_amd.tools.capture_hw` through gpurun)."""
import json
import os
import time
import urllib.request

import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.control import ApiServer, LocalClient, RestClient
from flex_gpu_scheduler_amd.control.httpserve import ServiceHTTP
from flex_gpu_scheduler_amd.control.node_agent import UNHEALTHY_TAINT, NodeAgent
from flex_gpu_scheduler_amd.gpu import HostSampler, LoadWatcherService, NodeTelemetry, WatcherFetcher, discover_host
from flex_gpu_scheduler_amd.gpu.discovery import fake_host, parse_cpulist
from flex_gpu_scheduler_amd.gpu.telemetry import Sample, merge_documents
from flex_gpu_scheduler_amd.models import GPU, TOPOLOGY_ANNOTATION, make_pod

BOX = os.path.join(os.path.dirname(__file__), "fixtures", "mi355x_box", "root")


def test_discovery_on_real_capture():
    h = discover_host(BOX)
    assert len(h.gpus) == 8
    assert [g.bdf for g in h.gpus] == sorted(g.bdf for g in h.gpus)
    assert {g.compute_partition for g in h.gpus} == {"SPX"} and {g.memory_partition for g in h.gpus} == {"NPS1"}
    assert all(g.hbm_gib == 288 for g in h.gpus)
    assert [g.numa for g in h.gpus] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert h.cpus == 256 and h.numa_nodes == [0, 1] and len(h.numa_cpus[1]) == 128
    # The container could open one GPU: its KFD node carries the compute and
    # xGMI details (7 XGMI links, 256 CUs, 8 XCCs, one hive).
    (vis,) = [g for g in h.gpus if g.kfd_node is not None]
    assert vis.bdf == "0000:8b:00.0" and vis.cus == 256 and vis.num_xcc == 8 and len(vis.xgmi_links) == 7
    assert all(lk.bandwidth_mbps == 76000 for lk in vis.xgmi_links)
    assert h.xgmi_hive is not None
    assert parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


def test_agent_publishes_node_and_nrt(store):
    c = LocalClient(store)
    agent = NodeAgent(c, "mi355x-0", host_fn=lambda: discover_host(BOX), publish_metrics=False)
    agent.sync()
    node = store.get("nodes", "", "mi355x-0")
    alloc = node["status"]["allocatable"]
    assert alloc[GPU] == "8" and alloc["amd.com/gpu-xcd"] == "64" and alloc["amd.com/gpu-memory"] == "2304"
    assert node["metadata"]["labels"]["amd.com/gpu.compute-partition"] == "spx"
    assert node["metadata"]["labels"]["amd.com/gpu.memory-partition"] == "NPS1"
    topo = json.loads(node["metadata"]["annotations"][TOPOLOGY_ANNOTATION])
    assert [g["numa"] for g in topo["gpus"]] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert topo["gpus"][4]["xgmiLinks"] == 7
    nrt = store.get("noderesourcetopologies", "", "mi355x-0")
    zone_gpus = [next(r["available"] for r in z["resources"] if r["name"] == GPU) for z in nrt["zones"]]
    assert zone_gpus == ["4", "4"]
    # A scheduler sees the node and places a 4-GPU pod on it.
    s = new_scheduler(store, load_config(None))
    s.sync_informers(50)
    out = s.explain(make_pod("p", requests={GPU: "4"}, limits={GPU: "4"}))
    assert out["selected"] == "mi355x-0"
    s.stop()


def test_agent_preserves_cordon_and_withholds_unhealthy(store):
    c = LocalClient(store)
    agent = NodeAgent(c, "n", host_fn=lambda: fake_host(8), publish_metrics=False)
    agent.sync()
    store.patch("nodes", "", "n", {"spec": {"unschedulable": True, "taints": [{"key": "admin", "effect": "NoSchedule"}]}})
    agent.health_fn = lambda dev: dev != 3
    agent.sync()
    node = store.get("nodes", "", "n")
    assert node["spec"]["unschedulable"] is True
    assert node["spec"]["taints"] == [{"key": "admin", "effect": "NoSchedule"}]
    assert node["status"]["allocatable"][GPU] == "7" and node["status"]["capacity"][GPU] == "8"
    assert json.loads(node["metadata"]["annotations"][TOPOLOGY_ANNOTATION])["unhealthy"] == [3]
    agent.health_fn = lambda dev: False
    agent.sync()
    node = store.get("nodes", "", "n")
    assert UNHEALTHY_TAINT in node["spec"]["taints"] and node["status"]["allocatable"][GPU] == "0"
    agent.health_fn = None
    agent.sync()
    assert UNHEALTHY_TAINT not in store.get("nodes", "", "n")["spec"]["taints"]


def test_agent_heartbeat_over_http(store):
    with ApiServer(store) as srv:
        agent = NodeAgent(RestClient(srv.url), "n", host_fn=lambda: fake_host(4), heartbeat=0.05,
                          publish_metrics=False).start()
        try:
            first = store.get("nodes", "", "n")["metadata"]["resourceVersion"]
            deadline = time.time() + 5
            while time.time() < deadline and store.get("nodes", "", "n")["metadata"]["resourceVersion"] == first:
                time.sleep(0.02)
            node = store.get("nodes", "", "n")
            assert node["metadata"]["resourceVersion"] != first
            assert node["status"]["conditions"][0]["type"] == "Ready"
        finally:
            agent.stop()


def test_sampler_reads_gpu_sysfs():
    s = HostSampler(BOX)
    smp = s.sample()
    assert smp.cpu is None  # needs two /proc/stat reads
    assert 0 <= smp.memory <= 100
    busy = [b for b, _ in s.gpu_samples()]
    assert len(busy) == 8 and 100 in busy  # one GPU of the box was busy at capture time
    assert smp.gpu == pytest.approx(sum(busy) / 8)


class _Seq:
    def __init__(self, values):
        self.values = list(values)

    def sample(self):
        cpu, gpu = self.values.pop(0)
        return Sample(time.time(), cpu, 50.0, gpu, 10.0)


def test_telemetry_windows_and_wire_format():
    t = NodeTelemetry("n", _Seq([(10, 90), (30, 70)]))
    t.sample()
    t.sample()
    doc = t.watcher_metrics()
    assert doc["window"]["duration"] == "15m" and doc["window"]["end"] - doc["window"]["start"] == 900
    ms = {(m["type"], m["operator"]): m["value"] for m in doc["data"]["NodeMetricsMap"]["n"]["metrics"]}
    assert ms[("CPU", "AVG")] == 20 and ms[("CPU", "STD")] == 10 and ms[("CPU", "Latest")] == 30
    assert ms[("GPU", "AVG")] == 80 and ms[("Memory", "AVG")] == 50 and ms[("GPUMemory", "Latest")] == 10


def test_node_metrics_feed_trimaran(store):
    """Per-node documents from agents drive TargetLoadPacking (GPU mode)."""
    from flex_gpu_scheduler_amd.models import make_node
    c = LocalClient(store)
    for n in ("busy", "idle"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110", GPU: "8"}))
    for n, gpu in (("busy", [95, 95]), ("idle", [20, 30])):
        agent = NodeAgent(c, n, host_fn=lambda: fake_host(8), sampler=_Seq([(10, g) for g in gpu]))
        agent.telemetry = NodeTelemetry(n, agent._sampler)
        agent.sample_and_publish()
        agent.sample_and_publish()
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "score": {"enabled": [{"name": "TargetLoadPacking"}], "disabled": [{"name": "*"}]}},
               "pluginConfig": [{"name": "TargetLoadPacking", "args": {"resourceType": "GPU"}}]}]}
    s = new_scheduler(store, load_config(cfg))
    s.sync_informers(50)
    out = s.explain(make_pod("p", limits={GPU: "1"}, requests={GPU: "1"}))
    # idle: 25% + 12.5% = 37.5% -> 96; busy: 107.5% -> 0
    assert out["scores"]["idle"]["TargetLoadPacking*1"] == 96 and out["scores"]["busy"]["TargetLoadPacking*1"] == 0
    s.stop()


def test_load_watcher_service_and_fetcher(store):
    c = LocalClient(store)
    for n, v in (("a", 10), ("b", 20)):
        t = NodeTelemetry(n, _Seq([(v, v)]))
        t.sample()
        from flex_gpu_scheduler_amd.gpu.telemetry import publish
        publish(c, t.watcher_metrics())
    http = ServiceHTTP().start()
    LoadWatcherService(c, http)
    try:
        doc = json.loads(urllib.request.urlopen(http.url + "/watcher").read())
        assert sorted(doc["data"]["NodeMetricsMap"]) == ["a", "b"]
        one = json.loads(urllib.request.urlopen(http.url + "/watcher?host=b").read())
        assert list(one["data"]["NodeMetricsMap"]) == ["b"]
        # A scheduler-side fetcher mirrors the service document into another store.
        from flex_gpu_scheduler_amd import Store
        other = Store()
        f = WatcherFetcher(http.url, LocalClient(other))
        assert f.fetch_once()
        got = other.get("loadwatchermetrics", "", "load-watcher")
        assert sorted(got["data"]["NodeMetricsMap"]) == ["a", "b"]
        assert f.fetch_once()  # second fetch replaces the document
    finally:
        http.stop()
    assert merge_documents([]) is None


def test_partition_bandwidth_table_is_published(store):
    """measure_bandwidth runs the (injected) partition probe once per healthy
    GPU and build_node publishes the table as amd.com/gpu-hbm-bandwidth."""
    import json as _json

    from flex_gpu_scheduler_amd.control import LocalClient
    from flex_gpu_scheduler_amd.control.node_agent import BANDWIDTH_ANNOTATION, NodeAgent
    from flex_gpu_scheduler_amd.gpu.discovery import fake_host

    calls = []

    def bw(dev):
        calls.append(dev)
        return {"bytes": 1 << 30, "partitions": {"CPX": {"xcds": 1, "read_GBps": 1000.0 + dev},
                                                  "SPX": {"xcds": 8, "read_GBps": 5000.0 + dev}}}

    agent = NodeAgent(LocalClient(store), "n0", host_fn=lambda: fake_host(4), bandwidth_fn=bw,
                      health_fn=lambda dev: dev != 2, publish_metrics=False)
    agent.sync()
    agent.sync()  # measured once per GPU
    assert sorted(calls) == [0, 1, 3]
    ann = _json.loads(store.get("nodes", "", "n0")["metadata"]["annotations"][BANDWIDTH_ANNOTATION])
    assert sorted(ann) == ["0", "1", "3"] and ann["3"]["partitions"]["SPX"]["read_GBps"] == 5003.0


def test_failed_bandwidth_probe_is_not_retried_every_heartbeat(store):
    from flex_gpu_scheduler_amd.control import LocalClient
    from flex_gpu_scheduler_amd.control.node_agent import NodeAgent
    from flex_gpu_scheduler_amd.gpu.discovery import fake_host

    calls = []

    def bw(dev):
        calls.append(dev)
        if dev == 1:
            raise RuntimeError("probe failed")
        return {"bytes": 1 << 30, "partitions": {}}

    agent = NodeAgent(LocalClient(store), "n0", host_fn=lambda: fake_host(2), bandwidth_fn=bw, publish_metrics=False)
    agent.sync()
    agent.sync()
    agent.sync()
    assert sorted(calls) == [0, 1]  # GPU 1 failed once and waits for its retry time
    agent.bandwidth_retry_s = 0.0
    agent._bandwidth_retry_at.clear()
    agent.sync()
    assert calls.count(1) == 2
