"""The reference's Trimaran plugin-level Score tables and the load-aware and
QoS integration flows, case for case.

Unit tables (the plugin's Score against a watcher that serves the case's
WatcherMetrics over HTTP, as the reference's httptest server does):
* pkg/trimaran/loadvariationriskbalancing/loadvariationriskbalancing_test.go:124  TestScore (6 cases)
* pkg/trimaran/targetloadpacking/targetloadpacking_test.go:106                 TestTargetLoadPackingScoring (4)

Integration flows (HTTP ApiServer + remote-mode scheduler, the envtest analog
of tests/test_envtest_parity.py):
* test/integration/targetloadpacking_test.go         TestTargetLoadPackingPlugin
* test/integration/loadVariationRiskBalancing_test.go TestLoadVariationRiskBalancingPlugin
* test/integration/qos_test.go                       TestQOSPlugin
* test/integration/elasticquota_controller_test.go   TestElasticController (3 cases)

The watcher documents are the reference's Go values as json.Marshal writes
them (an empty WatcherMetrics marshals NodeMetricsMap as null: the "404"
cases). The metrics reach the native plugins the way `watcherAddress` does in
a deployment: gpu/telemetry.WatcherFetcher GETs <address>/watcher and
publishes the document as a loadwatchermetrics object.
"""
import http.server
import json
import threading
import time

import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.control import ApiServer, ElasticQuotaController, RestClient
from flex_gpu_scheduler_amd.control.client import LocalClient
from flex_gpu_scheduler_amd.control.remote import RemoteScheduler
from flex_gpu_scheduler_amd.gpu.telemetry import WatcherFetcher
from flex_gpu_scheduler_amd.models import make_elastic_quota, make_node, make_pod
from flex_gpu_scheduler_amd.models.objects import make_container

MEGA = 1024 * 1024


def go_metric(type_, op, value):
    """watcher.Metric as json.Marshal writes it (rollup omitted when empty)."""
    return {"name": "", "type": type_, "operator": op, "value": value}


def watcher_doc(node_metrics: dict | None) -> dict:
    """watcher.WatcherMetrics{Window: {}, Data: {NodeMetricsMap: ...}}."""
    nmm = None if node_metrics is None else {
        n: {"metrics": ms, "tags": {}, "metadata": {}} for n, ms in node_metrics.items()}
    return {"timestamp": 0, "window": {"duration": "", "start": 0, "end": 0}, "source": "",
            "data": {"NodeMetricsMap": nmm}}


class WatcherServer:
    """httptest.NewServer serving one WatcherMetrics document."""

    def __init__(self, doc: dict):
        body = json.dumps(doc).encode()

        class H(http.server.BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):  # noqa: D401
                pass

        self.srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        self.t = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.t.start()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


def score_config(plugin: str, args: dict) -> dict:
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler", "plugins": {
                "score": {"enabled": [{"name": plugin}], "disabled": [{"name": "*"}]}},
                "pluginConfig": [{"name": plugin, "args": args}]}]}


def plugin_scores(store, plugin, args, nodes, doc, pod) -> dict:
    """The case's nodes, the watcher serving `doc`, one Score per node."""
    for n in nodes:
        store.create("nodes", n)
    srv = WatcherServer(doc)
    s = new_scheduler(store, load_config(score_config(plugin, {**args, "watcherAddress": srv.url})))
    try:
        assert WatcherFetcher(srv.url, LocalClient(store)).fetch_once()
        s.sync_informers(50)
        return s.plugin_call(plugin, "score", {"pod": pod})["raw"]
    finally:
        s.stop()
        srv.close()


NODE_RESOURCES = {"cpu": "1000m", "memory": "1Gi"}


def ref_node(name="node-1"):
    """st.MakeNode().Name(name).Capacity(nodeResources): capacity and allocatable."""
    return make_node(name, NODE_RESOURCES, capacity=NODE_RESOURCES)


def lvrb_pod(cpu_m: int, mem: int):
    """getPodWithContainersAndOverhead(0, 0, 0, []int64{cpu}, []int64{mem})
    (loadvariationriskbalancing_test.go:398)."""
    c = make_container("test-container-0", requests={"cpu": f"{cpu_m}m", "memory": str(mem)},
                       limits={"cpu": f"{cpu_m}m", "memory": str(mem)})
    init = make_container("test-init", requests={"cpu": "0m", "memory": "0"})
    return make_pod("p", containers=[c], init_containers=[init], overhead={"cpu": "0m"})


LVRB_SCORE = [
    ("new node", make_pod("p", containers=[]), {"node-1": [go_metric("CPU", "AVG", 50)]}, 75),
    ("hot node", make_pod("p", containers=[]), {"node-1": [go_metric("CPU", "AVG", 100)]}, 50),
    ("average and stDev metrics", lvrb_pod(200, 256 * MEGA),
     {"node-1": [go_metric("CPU", "AVG", 30), go_metric("CPU", "STD", 16)]}, 67),
    ("CPU and Memory metrics", lvrb_pod(100, 512 * MEGA),
     {"node-1": [go_metric("CPU", "AVG", 40), go_metric("CPU", "STD", 16), go_metric("Memory", "AVG", 50),
                 go_metric("Memory", "STD", 10)]}, 45),
    ("pick worst case: CPU or Memory", lvrb_pod(100, 512 * MEGA),
     {"node-1": [go_metric("CPU", "AVG", 80), go_metric("CPU", "STD", 20), go_metric("Memory", "AVG", 25),
                 go_metric("Memory", "STD", 15)]}, 45),
    ("404 resp from watcher", make_pod("p", containers=[]), None, 0),
]


@pytest.mark.parametrize("name,pod,metrics,expected", LVRB_SCORE, ids=[c[0] for c in LVRB_SCORE])
def test_lvrb_score(store, name, pod, metrics, expected):
    raw = plugin_scores(store, "LoadVariationRiskBalancing", {"safeVarianceMargin": 1, "safeVarianceSensitivity": 1},
                        [ref_node()], watcher_doc(metrics), pod)
    assert raw == {"node-1": expected}


def tlp_pod(overhead_m: int, *requests_m: int):
    """getPodWithContainersAndOverhead (targetloadpacking_test.go:415):
    requests == limits per container, CPU overhead."""
    conts = [make_container(f"test-container-{i}", requests={"cpu": f"{r}m"}, limits={"cpu": f"{r}m"})
             for i, r in enumerate(requests_m)]
    return make_pod("p", containers=conts, overhead={"cpu": f"{overhead_m}m"})


TLP_SCORE = [
    ("new node", make_pod("p", containers=[]), {"node-1": [go_metric("CPU", "Latest", 0)]}, 40),
    ("hot node", make_pod("p", containers=[]), {"node-1": [go_metric("CPU", "Latest", 40 + 10)]}, 33),
    ("excess utilization returns min score", tlp_pod(0, 1000), {"node-1": [go_metric("CPU", "Latest", 30)]}, 0),
    ("404 resp from watcher", make_pod("p", containers=[]), None, 0),
]


@pytest.mark.parametrize("name,pod,metrics,expected", TLP_SCORE, ids=[c[0] for c in TLP_SCORE])
def test_tlp_scoring(store, name, pod, metrics, expected):
    # TargetLoadPackingArgs{TargetUtilization: 40, DefaultRequestsMultiplier: 1.5, WatcherAddress}
    # (no DefaultRequests: a container without CPU requests predicts 0).
    raw = plugin_scores(store, "TargetLoadPacking",
                        {"targetUtilization": 40, "defaultRequestsMultiplier": "1.5", "defaultRequests": {"cpu": "0"}},
                        [ref_node()], watcher_doc(metrics), pod)
    assert raw == {"node-1": expected}


# ------------------------------------------------------------ integration --
@pytest.fixture
def http_cluster(store):
    srv = ApiServer(store).start()
    yield RestClient(srv.url)
    srv.stop()


def _wait(fn, timeout=10.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if fn():
            return True
        time.sleep(0.02)
    return bool(fn())


def _node_of(client, ns, name):
    p = client.get("pods", ns, name)
    return (p or {}).get("spec", {}).get("nodeName", "")


INTEGRATION_METRICS = {"node-1": [go_metric("CPU", "Latest", 10)], "node-2": [go_metric("CPU", "Latest", 60)],
                       "node-3": [go_metric("CPU", "Latest", 0)]}


def _load_aware_flow(client, plugin, args, expected):
    """Three nodes of 2 CPUs / 256 bytes / 32 pods with CPU at 10% / 60% / 0%;
    pods of 300m then 100m CPU (50 bytes memory); both land on `expected`."""
    srv = WatcherServer(watcher_doc(INTEGRATION_METRICS))
    fetch = WatcherFetcher(srv.url, client)
    assert fetch.fetch_once()
    rs = None
    try:
        for n in ("node-1", "node-2", "node-3"):
            res = {"pods": "32", "cpu": "2", "memory": "256"}
            client.create("nodes", make_node(n, res, capacity=res, labels={"node": n}))
        rs = RemoteScheduler(client, load_config(score_config(plugin, {**args, "watcherAddress": srv.url}))).start()
        for name, cpu in (("pod-1", 300), ("pod-2", 100)):
            client.create("pods", make_pod(name, "integration", requests={"cpu": f"{cpu}m", "memory": "50"}))
            assert _wait(lambda: _node_of(client, "integration", name)), name
            assert _node_of(client, "integration", name) == expected, name
    finally:
        if rs:
            rs.stop()
        srv.close()


def test_integration_target_load_packing(http_cluster):
    # TargetLoadPackingArgs{WatcherAddress, TargetUtilization: 40, DefaultRequestsMultiplier: 1.5}
    _load_aware_flow(http_cluster, "TargetLoadPacking",
                     {"targetUtilization": 40, "defaultRequestsMultiplier": "1.5", "defaultRequests": {"cpu": "0"}},
                     "node-1")


def test_integration_load_variation_risk_balancing(http_cluster):
    # LoadVariationRiskBalancingArgs{WatcherAddress, SafeVarianceMargin: 1}
    _load_aware_flow(http_cluster, "LoadVariationRiskBalancing", {"safeVarianceMargin": 1}, "node-3")


def test_integration_qos_queue_sort(store):
    """Three pods created BestEffort, Burstable, Guaranteed on a scheduler
    that is not running: NextPod pops them in the reverse (QoS) order."""
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "queueSort": {"enabled": [{"name": "QOSSort"}], "disabled": [{"name": "*"}]}}}]}
    res = {"pods": "32", "cpu": "500m", "memory": "500"}
    store.create("nodes", make_node("fake-node", res, capacity=res, labels={"node": "fake-node"}))
    names = ["bestefforts", "burstable", "guaranteed"]
    reqs = [None, ({"memory": "100"}, {"memory": "200"}), ({"memory": "100"}, {"memory": "100"})]
    # As in the reference, the scheduler's informers are synced before the
    # pods are created one by one (each reaches the queue as a watch event).
    s = new_scheduler(store, load_config(cfg))
    try:
        s.sync_informers(50)
        for name, rl in zip(names, reqs):
            c = make_container("pause") if rl is None else make_container("pause", requests=rl[0], limits=rl[1])
            store.create("pods", make_pod(name, "integration", containers=[c]))
            s.sync_informers(50)
        assert _wait(lambda: s.sync_informers(20) >= 0 and s.queue_counts()["active"] == 3)
        popped = [s.next_pod(1000) for _ in names]
        assert popped == [f"integration/{n}" for n in reversed(names)]
    finally:
        s.stop()


# ElasticQuota controller: cases of elasticquota_controller_test.go. Each
# case: quotas (min, max), existing pods (created, scheduled by the default
# profile; Running ones get their status), the `used` expected then, the
# status updates of the incoming pods and the `used` expected after them.
def _rl(cpu=None, mem=None):
    out = {}
    if cpu is not None:
        out["cpu"] = str(cpu)
    if mem is not None:
        out["memory"] = str(mem)
    return out


EQ_CASES = [
    ("The status of the pod changes from pending to running",
     [("ns1", "t1-eq1", _rl(100, 1000), _rl(100, 1000)), ("ns2", "t1-eq2", _rl(100, 1000), _rl(100, 1000))],
     [("ns1", "t1-p1", 10, 20, None), ("ns1", "t1-p2", 10, 10, None), ("ns1", "t1-p3", 10, 10, None),
      ("ns2", "t1-p4", 10, 10, None)],
     {("ns1", "t1-eq1"): _rl(0, 0), ("ns2", "t1-eq2"): _rl(0, 0)},
     [("ns1", "t1-p1", "Running"), ("ns1", "t1-p2", "Running"), ("ns1", "t1-p3", "Running"),
      ("ns2", "t1-p4", "Running")],
     {("ns1", "t1-eq1"): _rl(30, 40), ("ns2", "t1-eq2"): _rl(10, 10)}),
    ("The status of the pod changes from running to others",
     [("ns1", "t2-eq1", _rl(100, 1000), _rl(100, 1000)), ("ns2", "t2-eq2", _rl(100, 1000), _rl(100, 1000))],
     [("ns1", "t2-p1", 10, 20, "Running"), ("ns1", "t2-p2", 10, 10, "Running"), ("ns1", "t2-p3", 10, 10, "Running"),
      ("ns2", "t2-p4", 10, 10, "Running")],
     {("ns1", "t2-eq1"): _rl(30, 40), ("ns2", "t2-eq2"): _rl(10, 10)},
     [("ns1", "t2-p1", "Succeeded"), ("ns1", "t2-p3", "Failed")],
     {("ns1", "t2-eq1"): _rl(10, 10), ("ns2", "t2-eq2"): _rl(10, 10)}),
    ("Different resource between max and min",
     [("ns1", "t3-eq1", _rl(mem=1000), _rl(cpu=100))],
     [("ns1", "t3-p1", 10, 20, None)],
     {("ns1", "t3-eq1"): _rl(0, 0)},
     [("ns1", "t3-p1", "Running")],
     {("ns1", "t3-eq1"): _rl(10, 20)}),
]


def _used_equals(got: dict, want: dict) -> bool:
    """quota.Equals: the same keys with equal quantities."""
    from flex_gpu_scheduler_amd._native import native

    n = native()
    got = got or {}
    return set(got) == set(want) and all(n.quantity_cmp(str(got[k]), str(v)) == 0 for k, v in want.items())


def test_integration_elastic_quota_controller(http_cluster):
    client = http_cluster
    res = {"pods": "300", "cpu": "300", "memory": "3000"}
    client.create("nodes", make_node("fake-node", res, capacity=res, labels={"node": "fake-node"}))
    ctrl = ElasticQuotaController(client).run()
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler"}]}
    rs = RemoteScheduler(client, load_config(cfg)).start()
    try:
        for name, eqs, existing, used, incoming, want in EQ_CASES:
            for ns, eqn, mn, mx in eqs:
                client.create("elasticquotas", make_elastic_quota(eqn, ns, min=mn, max=mx))
            for ns, pn, cpu, mem, phase in existing:
                client.create("pods", make_pod(pn, ns, containers=[make_container(
                    "c", requests=_rl(cpu, mem), limits=_rl(cpu, mem))]))
            assert _wait(lambda: all(_node_of(client, ns, pn) for ns, pn, *_ in existing)), name
            for ns, pn, _c, _m, phase in existing:
                if phase:
                    client.patch("pods", ns, pn, {"status": {"phase": phase}})

            def used_is(expect):
                for (ns, eqn), u in expect.items():
                    eq = client.get("elasticquotas", ns, eqn)
                    if not _used_equals((eq.get("status") or {}).get("used"), u):
                        return False
                return True

            assert _wait(lambda: used_is(used)), (name, "used before", [client.get("elasticquotas", ns, e)
                                                                       for ns, e, *_ in eqs])
            for ns, pn, phase in incoming:
                client.patch("pods", ns, pn, {"status": {"phase": phase}})
            assert _wait(lambda: used_is(want)), (name, "used after", [client.get("elasticquotas", ns, e)
                                                                      for ns, e, *_ in eqs])
            for ns, pn, *_ in existing:
                client.delete("pods", ns, pn)
            for ns, eqn, *_ in eqs:
                client.delete("elasticquotas", ns, eqn)
    finally:
        rs.stop()
        ctrl.stop()
