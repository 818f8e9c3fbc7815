"""load-watcher library mode (vendor/github.com/paypal/load-watcher/pkg/watcher/
watcher.go:104-203, internal/metricsprovider/{k8s,prometheus,signalfx}.go):
providers against fake HTTP backends, the 15/10/5-minute fallback, and the
end-to-end path Prometheus -> Watcher -> store -> native TargetLoadPacking.

The reference tests providers the same way (collector_test.go:78-128 serves a
hand-built WatcherMetrics from httptest); the Prometheus / SignalFx payloads
below follow the shapes those providers decode (model.Vector; the
timeserieswindow + metrictimeseries sample payloads in signalfx.go)."""
import pytest

from flex_gpu_scheduler_amd import load_config, new_scheduler
from flex_gpu_scheduler_amd.control.client import LocalClient
from flex_gpu_scheduler_amd.control.httpserve import ServiceHTTP
from flex_gpu_scheduler_amd.gpu.providers import (FIFTEEN, FIVE, TEN, KubernetesMetricsServerProvider,
                                                  PrometheusProvider, SignalFxProvider, Watcher, new_provider, window)
from flex_gpu_scheduler_amd.models import GPU, make_node, make_pod


def _vector(series):
    return {"status": "success", "data": {"resultType": "vector", "result": [
        {"metric": labels, "value": [1700000000.0, str(v)]} for labels, v in series]}}


@pytest.fixture
def prom():
    http = ServiceHTTP()
    seen = []

    def query(q, body):
        promql = q["query"]
        seen.append(promql)
        if promql.startswith("avg_over_time(instance:node_cpu:ratio"):
            return 200, "application/json", _vector([({"instance": "a"}, 0.25), ({"instance": "b"}, 0.5)])
        if promql.startswith("stddev_over_time(instance:node_cpu:ratio"):
            return 200, "application/json", _vector([({"instance": "a"}, 0.05)])
        if promql.startswith("avg_over_time(instance:node_memory"):
            return 200, "application/json", _vector([({"instance": "a"}, 0.1)])
        if promql.startswith("stddev_over_time(instance:node_memory"):
            return 200, "application/json", _vector([])
        if "gpu_gfx_activity" in promql and "avg_over_time" in promql:
            return 200, "application/json", _vector([({"hostname": "a"}, 80.0), ({"hostname": "b"}, 5.0)])
        if "gpu_used_vram" in promql:
            return 200, "application/json", _vector([({"hostname": "a"}, 40.0)])
        return 200, "application/json", _vector([])

    http.add_route("GET", "/api/v1/query", query)
    http.start()
    yield http, seen
    http.stop()


def test_prometheus_queries_and_values(prom):
    http, seen = prom
    p = PrometheusProvider(http.url)
    out = p.fetch_all_hosts_metrics(window(FIFTEEN))
    assert "avg_over_time(instance:node_cpu:ratio[15m])" in seen
    assert "stddev_over_time(instance:node_memory_utilisation:ratio[15m])" in seen
    a = {(m["type"], m["operator"]): m["value"] for m in out["a"]}
    assert a[("CPU", "AVG")] == pytest.approx(25.0)
    assert a[("CPU", "STD")] == pytest.approx(5.0)
    assert a[("Memory", "AVG")] == pytest.approx(10.0)
    assert a[("GPU", "AVG")] == pytest.approx(80.0)       # percent already, not x100
    assert a[("GPUMemory", "AVG")] == pytest.approx(40.0)
    assert {(m["type"], m["operator"]) for m in out["b"]} >= {("CPU", "AVG"), ("GPU", "AVG")}
    assert all(m["rollup"] == "15m" for m in out["a"])


def test_prometheus_host_query_shape():
    assert PrometheusProvider.build_query("n1", "instance:node_cpu:ratio", "avg_over_time", "5m") == \
        'avg_over_time(instance:node_cpu:ratio{instance="n1"}[5m])'


def test_prometheus_unreachable_raises():
    p = PrometheusProvider("http://127.0.0.1:9", gpu=False)
    with pytest.raises(Exception):
        p.fetch_all_hosts_metrics(window(FIVE))
    assert not p.health()


def test_signalfx_joins_metadata_and_averages():
    http = ServiceHTTP()
    calls = []

    def tsw(q, body):
        calls.append(("tsw", q))
        return 200, "application/json", {"data": {"id1": [[1, 10.0], [2, 30.0]], "id2": [[1, 50.0]], "orphan": [[1, 1]]}}

    def meta(q, body):
        calls.append(("meta", q))
        return 200, "application/json", {"count": 2, "results": [
            {"id": "id1", "dimensions": {"host": "node-a.dev.example.com"}},
            {"id": "id2", "dimensions": {"host": "node-b"}}]}

    http.add_route("GET", "/v1/timeserieswindow", tsw)
    http.add_route("GET", "/v2/metrictimeseries", meta)
    http.start()
    try:
        p = SignalFxProvider(http.url, token="t", cluster="c1")
        w = window(FIFTEEN, now=1000)
        out = p.fetch_all_hosts_metrics(w)
    finally:
        http.stop()
    assert out["node-a"][0] == {"name": 'sf_metric:"cpu.utilization"', "type": "CPU", "operator": "AVG", "rollup": "",
                                "value": 20.0}
    assert out["node-b"][0]["value"] == 50.0
    assert {m["type"] for m in out["node-a"]} == {"CPU", "Memory"}
    q = calls[0][1]
    assert q["query"] == 'host:* AND cluster:c1 AND sf_metric:"cpu.utilization"'
    assert q["startMs"] == str(100 * 1000) and q["endMs"] == str(1000 * 1000) and q["resolution"] == "60000"
    with pytest.raises(ValueError):
        SignalFxProvider(http.url, token="")


class _MetricsServerClient(LocalClient):
    """A LocalClient that also answers metrics.k8s.io like a RestClient."""

    def __init__(self, store, node_metrics):
        super().__init__(store)
        self.node_metrics = node_metrics

    def request(self, method, path, body=None, **kw):
        assert (method, path) == ("GET", "/apis/metrics.k8s.io/v1beta1/nodes")
        return {"kind": "NodeMetricsList", "items": self.node_metrics}


def test_metrics_server_latest_percentages(store):
    store.create("nodes", make_node("a", {"cpu": "64", "memory": "256Gi", "pods": "110"}))
    nm = [{"metadata": {"name": "a"}, "usage": {"cpu": "16", "memory": "64Gi"}},
          {"metadata": {"name": "ghost"}, "usage": {"cpu": "1", "memory": "1Gi"}}]
    p = new_provider({"type": "KubernetesMetricsServer"}, _MetricsServerClient(store, nm))
    assert isinstance(p, KubernetesMetricsServerProvider) and p.health()
    out = p.fetch_all_hosts_metrics(window(FIFTEEN))
    assert set(out) == {"a"}  # unknown hosts are skipped (k8s.go)
    assert {(m["type"], m["operator"], m["value"]) for m in out["a"]} == {("CPU", "Latest", 25.0),
                                                                          ("Memory", "Latest", 25.0)}


class _Flaky:
    name = "Fake"

    def __init__(self, fail_for=()):
        self.fail_for = set(fail_for)

    def fetch_all_hosts_metrics(self, win):
        if win["duration"] in self.fail_for:
            raise RuntimeError("down")
        return {"n": [{"type": "CPU", "operator": "AVG", "value": {"15m": 15, "10m": 10, "5m": 5}[win["duration"]]}]}

    def health(self):
        return True


def test_watcher_window_fallback():
    w = Watcher(_Flaky(fail_for={FIFTEEN}))
    w.fetch_all()
    assert w.latest(FIFTEEN)["window"]["duration"] == TEN   # 15m missing -> 10m
    assert w.latest(FIVE)["window"]["duration"] == FIVE
    w2 = Watcher(_Flaky(fail_for={FIFTEEN, TEN, FIVE}))
    w2.fetch_all()
    assert w2.latest(FIFTEEN) is None and w2.errors == 3
    w3 = Watcher(_Flaky())
    for _ in range(7):
        w3.fetch_all()
    assert len(w3._cache[FIFTEEN]) == Watcher.CACHE_SIZE  # bounded cache (sizePerWindow 5)


def test_watcher_serves_watcher_endpoint():
    import json
    import urllib.request

    http = ServiceHTTP()
    w = Watcher(_Flaky()).serve(http)
    http.start()
    try:
        w.fetch_all()
        doc = json.loads(urllib.request.urlopen(http.url + "/watcher").read())
        assert doc["data"]["NodeMetricsMap"]["n"]["metrics"][0]["value"] == 15
        assert urllib.request.urlopen(http.url + "/watcher/health").status == 200
    finally:
        http.stop()


def test_prometheus_to_native_tlp_end_to_end(store, prom):
    http, _ = prom
    for n in ("a", "b"):
        store.create("nodes", make_node(n, {"cpu": "64", "memory": "256Gi", "pods": "110", GPU: "8"}))
    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "score": {"enabled": [{"name": "TargetLoadPacking"}], "disabled": [{"name": "*"}]}},
               "pluginConfig": [{"name": "TargetLoadPacking", "args": {
                   "resourceType": "GPU", "metricProvider": {"type": "Prometheus", "address": http.url}}}]}]}
    from flex_gpu_scheduler_amd.cli import _library_watchers

    conf = load_config(cfg)
    ws = _library_watchers(conf, LocalClient(store), LocalClient(store))
    assert len(ws) == 1
    ws[0].fetch_all()
    s = new_scheduler(store, conf)
    try:
        s.sync_informers(20)
        sc = s.explain(make_pod("p", limits={GPU: "1"}))["scores"]
        # a: 80% busy + 1/8 GPU = 92.5% -> round(40*(100-92.5)/60) = 5; b: 5% + 12.5% = 17.5% -> round(60*17.5/40+40) = 66
        assert sc["a"]["TargetLoadPacking*1"] == 5 and sc["b"]["TargetLoadPacking*1"] == 66
    finally:
        s.stop()


def test_metrics_server_watcher_skipped_without_metrics_api(store):
    from flex_gpu_scheduler_amd.cli import _library_watchers

    cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration",
           "profiles": [{"schedulerName": "default-scheduler", "plugins": {
               "score": {"enabled": [{"name": "TargetLoadPacking"}]}}}]}
    # LocalClient has no metrics.k8s.io: node agents stay the metrics source.
    assert _library_watchers(load_config(cfg), LocalClient(store), LocalClient(store)) == []
