"""load-watcher library mode: metric providers + the windowed Watcher.

The reference's Trimaran plugins, when no `watcherAddress` is given, run the
vendored paypal/load-watcher in-process (vendor/github.com/paypal/load-watcher/
pkg/watcher/watcher.go:104-203) over one of three providers chosen by
`metricProvider.type` (apis/config/types.go MetricProviderType; defaults.go:66
picks KubernetesMetricsServer):

  * KubernetesMetricsServer (internal/metricsprovider/k8s.go): per node,
    Latest CPU % = usage.cpu / capacity.cpu and Memory % = usage.memory /
    capacity.memory from metrics.k8s.io/v1beta1 NodeMetrics;
  * Prometheus (prometheus.go): `avg_over_time` and `stddev_over_time` of
    `instance:node_cpu:ratio` / `instance:node_memory_utilisation:ratio` over
    the window, keyed by the `instance` label, value x100;
  * SignalFx (signalfx.go): `/v1/timeserieswindow` for cpu.utilization /
    memory.utilization at 1-minute resolution joined with `/v2/metrictimeseries`
    metadata (tsid -> host dimension, FQDN cut at the first dot), averaged, AVG.

MI355X additions, opt-in per provider: Prometheus also asks for GPU busy % and
HBM used % as exported by the AMD GPU metrics exporter (`gpu_gfx_activity`,
`gpu_used_vram` / `gpu_total_vram`, keyed by `hostname`) and emits them as
the "GPU" / "GPUMemory" metric types the node agent uses, so
TargetLoadPacking with `resourceType: GPU` works off a Prometheus stack too.

`Watcher` keeps the 15/10/5-minute windows (fetched once at start, then every
minute, 5 documents cached per window) and `latest()` applies the same
15 -> 10 -> 5 minute fallback as GetLatestWatcherMetrics. `publish_to()`
writes the latest document into the API store as
`loadwatchermetrics/<name>`, where the native plugins read it, exactly like
the node agents' own documents (gpu/telemetry.py).
"""
from __future__ import annotations

import json
import logging
import ssl
import threading
import time
import urllib.parse
import urllib.request
from collections import deque
from typing import Callable, Protocol

log = logging.getLogger(__name__)

FIFTEEN, TEN, FIVE = "15m", "10m", "5m"
WINDOW_SECONDS = {FIFTEEN: 900, TEN: 600, FIVE: 300}

K8S_CLIENT_NAME = "KubernetesMetricsServer"
PROM_CLIENT_NAME = "Prometheus"
SIGNALFX_CLIENT_NAME = "SignalFx"

PROM_CPU = "instance:node_cpu:ratio"
PROM_MEM = "instance:node_memory_utilisation:ratio"
PROM_HOST_KEY = "instance"
DEFAULT_PROM_ADDRESS = "http://prometheus-k8s:9090"
# AMD GPU metrics exporter series (percent / bytes), labelled by hostname.
PROM_GPU_BUSY = "gpu_gfx_activity"
PROM_GPU_VRAM_USED = "gpu_used_vram"
PROM_GPU_VRAM_TOTAL = "gpu_total_vram"
PROM_GPU_HOST_KEY = "hostname"

DEFAULT_SIGNALFX_ADDRESS = "https://api.signalfx.com"
SFX_CPU = 'sf_metric:"cpu.utilization"'
SFX_MEM = 'sf_metric:"memory.utilization"'


def window(duration: str, now: float | None = None) -> dict:
    end = int(now if now is not None else time.time())
    return {"duration": duration, "start": end - WINDOW_SECONDS[duration], "end": end}


class MetricsProvider(Protocol):
    name: str

    def fetch_all_hosts_metrics(self, win: dict) -> dict[str, list[dict]]: ...

    def health(self) -> bool: ...


def _http_json(url: str, headers: dict | None = None, timeout: float = 10.0, insecure: bool = False):
    req = urllib.request.Request(url, headers=headers or {})
    ctx = None
    if url.startswith("https") and insecure:
        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    with urllib.request.urlopen(req, timeout=timeout, context=ctx) as r:
        return json.loads(r.read())


def _head_ok(url: str, timeout: float = 5.0) -> bool:
    try:
        req = urllib.request.Request(url, method="HEAD")
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status == 200
    except Exception:  # noqa: BLE001
        return False


# ------------------------------------------------------- metrics-server ----
def _milli(q) -> float:
    """Quantity -> milli-units, exact k8s parsing (native Quantity)."""
    from .._native import native

    return float(native().parse_quantity(str(q))[0])


class KubernetesMetricsServerProvider:
    """Latest CPU/memory utilisation from metrics.k8s.io NodeMetrics.

    `list_node_metrics()` returns NodeMetrics objects (`usage.cpu`,
    `usage.memory`); by default it GETs /apis/metrics.k8s.io/v1beta1/nodes
    through a RestClient. `list_nodes()` returns Node objects."""

    name = K8S_CLIENT_NAME

    def __init__(self, client, list_node_metrics: Callable[[], list[dict]] | None = None):
        self.client = client
        self._list_nm = list_node_metrics or self._rest_node_metrics

    def _rest_node_metrics(self) -> list[dict]:
        out = self.client.request("GET", "/apis/metrics.k8s.io/v1beta1/nodes")
        return list((out or {}).get("items") or [])

    def fetch_all_hosts_metrics(self, win: dict) -> dict[str, list[dict]]:
        nodes, _ = self.client.list("nodes")
        cap = {}
        for n in nodes:
            c = ((n.get("status") or {}).get("capacity")) or {}
            cap[n["metadata"]["name"]] = (_milli(c.get("cpu", "0")), _milli(c.get("memory", "0")) / 1000.0)
        out: dict[str, list[dict]] = {}
        for nm in self._list_nm():
            host = nm["metadata"]["name"]
            if host not in cap:
                log.error("unable to find host %s in node list caching cpu capacity", host)
                continue
            usage = nm.get("usage") or {}
            cpu_cap, mem_cap = cap[host]
            ms = []
            if cpu_cap > 0:
                ms.append({"name": "", "type": "CPU", "operator": "Latest", "rollup": "",
                           "value": 100.0 * _milli(usage.get("cpu", "0")) / cpu_cap})
            if mem_cap > 0:
                ms.append({"name": "", "type": "Memory", "operator": "Latest", "rollup": "",
                           "value": 100.0 * (_milli(usage.get("memory", "0")) / 1000.0) / mem_cap})
            out[host] = ms
        return out

    def health(self) -> bool:
        try:
            self._list_nm()
            return True
        except Exception:  # noqa: BLE001
            return False


# ------------------------------------------------------------ Prometheus ----
class PrometheusProvider:
    name = PROM_CLIENT_NAME

    def __init__(self, address: str = "", token: str = "", insecure_skip_verify: bool = True, gpu: bool = True):
        self.address = (address or DEFAULT_PROM_ADDRESS).rstrip("/")
        self.token = token
        self.insecure = insecure_skip_verify
        self.gpu = gpu

    def _query(self, promql: str) -> list[dict]:
        url = f"{self.address}/api/v1/query?" + urllib.parse.urlencode({"query": promql, "time": f"{time.time():.3f}"})
        headers = {"Authorization": f"Bearer {self.token}"} if self.token else {}
        doc = _http_json(url, headers, timeout=10.0, insecure=self.insecure)
        if doc.get("status") != "success":
            raise RuntimeError(f"prometheus query failed: {doc.get('error', doc)}")
        data = doc.get("data") or {}
        if data.get("resultType") != "vector":
            raise RuntimeError(f"The Prometheus results should not be type: {data.get('resultType')}")
        return data.get("result") or []

    @staticmethod
    def build_query(host: str, metric: str, method: str, rollup: str) -> str:
        # prometheus.go buildPromQuery
        if host == "all":
            return f"{method}({metric}[{rollup}])"
        return f'{method}({metric}{{{PROM_HOST_KEY}="{host}"}}[{rollup}])'

    def fetch_all_hosts_metrics(self, win: dict) -> dict[str, list[dict]]:
        out: dict[str, list[dict]] = {}
        err: Exception | None = None
        rollup = win["duration"]
        for method, op in (("avg_over_time", "AVG"), ("stddev_over_time", "STD")):
            for metric, typ in ((PROM_CPU, "CPU"), (PROM_MEM, "Memory")):
                try:
                    res = self._query(self.build_query("all", metric, method, rollup))
                except Exception as e:  # noqa: BLE001 - one failing series does not drop the others
                    log.error("error querying Prometheus for %s: %s", metric, e)
                    err = e
                    continue
                for r in res:
                    host = (r.get("metric") or {}).get(PROM_HOST_KEY, "")
                    out.setdefault(host, []).append({"name": metric, "type": typ, "operator": op, "rollup": rollup,
                                                     "value": float(r["value"][1]) * 100.0})
            if self.gpu:
                gpu_series = (
                    (PROM_GPU_BUSY, "GPU", f"avg by ({PROM_GPU_HOST_KEY}) ({method}({PROM_GPU_BUSY}[{rollup}]))"),
                    ("gpu_vram_utilization", "GPUMemory",
                     f"avg by ({PROM_GPU_HOST_KEY}) ({method}((100 * {PROM_GPU_VRAM_USED} / {PROM_GPU_VRAM_TOTAL})"
                     f"[{rollup}:1m]))"),
                )
                for name, typ, q in gpu_series:
                    try:
                        res = self._query(q)
                    except Exception as e:  # noqa: BLE001 - no GPU exporter is not an error for CPU metrics
                        log.debug("no GPU series %s: %s", name, e)
                        continue
                    for r in res:
                        host = (r.get("metric") or {}).get(PROM_GPU_HOST_KEY, "")
                        out.setdefault(host, []).append({"name": name, "type": typ, "operator": op, "rollup": rollup,
                                                         "value": float(r["value"][1])})
        if not out and err is not None:
            raise err
        return out

    def health(self) -> bool:
        return _head_ok(self.address)


# -------------------------------------------------------------- SignalFx ----
class SignalFxProvider:
    name = SIGNALFX_CLIENT_NAME

    def __init__(self, address: str = "", token: str = "", host_suffix: str = "", cluster: str = "",
                 insecure_skip_verify: bool = False):
        if not token:
            raise ValueError("No auth token found to connect with SignalFx server")
        self.address = (address or DEFAULT_SIGNALFX_ADDRESS).rstrip("/")
        self.token, self.suffix, self.cluster = token, host_suffix, cluster
        self.insecure = insecure_skip_verify

    def _get(self, path: str, q: dict):
        return _http_json(f"{self.address}{path}?" + urllib.parse.urlencode(q),
                          {"X-SF-Token": self.token, "Content-Type": "application/json"}, timeout=55.0,
                          insecure=self.insecure)

    @staticmethod
    def _host_name(fqdn: str) -> str:
        return fqdn.split(".", 1)[0]

    def fetch_all_hosts_metrics(self, win: dict) -> dict[str, list[dict]]:
        host_filter = f"host:*{self.suffix}"
        cluster_filter = f"cluster:{self.cluster}"
        out: dict[str, list[dict]] = {}
        for metric, typ in ((SFX_CPU, "CPU"), (SFX_MEM, "Memory")):
            query = f"{host_filter} AND {cluster_filter} AND {metric}"
            data = self._get("/v1/timeserieswindow", {"query": query, "startMs": win["start"] * 1000,
                                                      "endMs": win["end"] * 1000, "resolution": 60000})
            meta = self._get("/v2/metrictimeseries", {"query": query, "limit": 10000})
            tsid_host = {}
            for r in meta.get("results") or []:
                host = ((r or {}).get("dimensions") or {}).get("host")
                if r.get("id") and isinstance(host, str):
                    tsid_host[r["id"]] = self._host_name(host)
            for tsid, points in (data.get("data") or {}).items():
                if tsid not in tsid_host or not points:
                    continue
                vals = [p[1] for p in points if isinstance(p, list) and len(p) >= 2 and isinstance(p[1], (int, float))]
                if not vals:
                    continue
                out.setdefault(tsid_host[tsid], []).append({"name": metric, "type": typ, "operator": "AVG",
                                                            "rollup": "", "value": sum(vals) / len(vals)})
        return out

    def health(self) -> bool:
        return _head_ok(self.address)


def new_provider(metric_provider: dict, client=None) -> MetricsProvider:
    """metricProvider args (apis/config/types.go MetricProviderSpec) -> provider."""
    typ = metric_provider.get("type") or K8S_CLIENT_NAME
    if typ == PROM_CLIENT_NAME:
        return PrometheusProvider(metric_provider.get("address", ""), metric_provider.get("token", ""),
                                  bool(metric_provider.get("insecureSkipVerify", True)))
    if typ == SIGNALFX_CLIENT_NAME:
        return SignalFxProvider(metric_provider.get("address", ""), metric_provider.get("token", ""),
                                insecure_skip_verify=bool(metric_provider.get("insecureSkipVerify", False)))
    if typ == K8S_CLIENT_NAME:
        if client is None:
            raise ValueError("KubernetesMetricsServer provider needs an API client")
        return KubernetesMetricsServerProvider(client)
    raise ValueError(f"unknown metric provider type {typ!r}")


# --------------------------------------------------------------- Watcher ----
class Watcher:
    """In-process load-watcher over one provider (watcher.go:104-203)."""

    CACHE_SIZE = 5

    def __init__(self, provider: MetricsProvider, period: float = 60.0, clock: Callable[[], float] = time.time):
        self.provider, self.period, self.clock = provider, period, clock
        self._cache: dict[str, deque] = {d: deque(maxlen=self.CACHE_SIZE) for d in (FIFTEEN, TEN, FIVE)}
        self._mu = threading.RLock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._sinks: list[Callable[[dict], None]] = []
        self.errors = 0

    def fetch_once(self, duration: str) -> bool:
        win = window(duration, self.clock())
        try:
            host_metrics = self.provider.fetch_all_hosts_metrics(win)
        except Exception as e:  # noqa: BLE001
            self.errors += 1
            log.error("received error while fetching metrics: %s", e)
            return False
        doc = {"timestamp": int(self.clock()), "window": win, "source": self.provider.name,
               "data": {"NodeMetricsMap": {h: {"metrics": ms} for h, ms in sorted(host_metrics.items())}}}
        with self._mu:
            self._cache[duration].append(doc)
        return True

    def fetch_all(self) -> None:
        for d in (FIFTEEN, TEN, FIVE):
            self.fetch_once(d)
        latest = self.latest(FIFTEEN)
        if latest is not None:
            for sink in self._sinks:
                try:
                    sink(latest)
                except Exception as e:  # noqa: BLE001
                    log.warning("watcher sink failed: %s", e)

    def latest(self, duration: str = FIFTEEN) -> dict | None:
        """GetLatestWatcherMetrics: 15m, else 10m, else 5m (deep copy)."""
        with self._mu:
            if duration == FIFTEEN and self._cache[FIFTEEN]:
                d = self._cache[FIFTEEN][-1]
            elif duration in (FIFTEEN, TEN) and self._cache[TEN]:
                d = self._cache[TEN][-1]
            elif duration in (TEN, FIVE) and self._cache[FIVE]:
                d = self._cache[FIVE][-1]
            else:
                return None
            return json.loads(json.dumps(d))

    def publish_to(self, client, name: str) -> "Watcher":
        from .telemetry import publish

        self._sinks.append(lambda doc: publish(client, dict(doc, metadata={"name": name})))
        return self

    def serve(self, http) -> "Watcher":
        """GET /watcher[?host=] and /watcher/health on a ServiceHTTP."""

        def handler(q, body):
            doc = self.latest(FIFTEEN)
            if doc is None:
                return 404, "application/json", ""
            host = q.get("host")
            if host:
                nm = doc["data"]["NodeMetricsMap"].get(host)
                if nm is None:
                    return 404, "application/json", ""
                doc["data"] = {"NodeMetricsMap": {host: nm}}
            return 200, "application/json", doc

        http.add_route("GET", "/watcher", handler)
        http.add_route("GET", "/watcher/health",
                       lambda q, b: (200, "text/plain", "") if self.provider.health() else (503, "text/plain", ""))
        return self

    def start(self) -> "Watcher":
        self.fetch_all()  # populate the cache before returning (watcher.go:149-153)

        def run():
            while not self._stop.wait(self.period):
                self.fetch_all()

        self._thread = threading.Thread(target=run, name="load-watcher", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
