"""Load telemetry in the load-watcher wire format, MI355X-aware.

The reference's Trimaran plugins consume `WatcherMetrics` from the vendored
paypal/load-watcher (vendor/github.com/paypal/load-watcher/pkg/watcher/
watcher.go:38-101): per node, metrics {name, type CPU|Memory, operator
AVG|STD|Latest, rollup, value %} over 15/10/5-minute windows, refreshed every
minute from metrics-server/Prometheus/SignalFx, served at GET /watcher.

Here each node agent samples its own host — CPU from /proc/stat, memory from
/proc/meminfo, and per-GPU counters from amd-smi (the native libamd_smi
sampler, gpu/amdsmi.py: GFX and HBM-controller activity, VRAM, xGMI link
traffic) or, without it, amdgpu sysfs (gpu_busy_percent,
mem_info_vram_used/total) — keeps rolling windows, and publishes one
WatcherMetrics document per node into the API store
(`loadwatchermetrics/<node>`), which the C++ Trimaran plugins merge
(csrc/plugins/trimaran.cc). GPU metric types extend the set: "GPU" (busy %),
"GPUMemory" (HBM used %), and with amd-smi "GPUMemoryBandwidth" (HBM
controller activity %) and "XGMI" (xGMI traffic as % of the up links'
capacity). `LoadWatcherService` re-serves the cluster
union at GET /watcher (+ ?host=, /watcher/health) for any consumer that
speaks the original service mode, and `WatcherFetcher` does the reverse for a
scheduler pointed at an external load-watcher (`watcherAddress`).
"""
from __future__ import annotations

import json
import logging
import math
import os
import threading
import time
import urllib.request
from collections import deque
from dataclasses import dataclass

from .discovery import _read, _read_int

log = logging.getLogger(__name__)

WINDOWS = {"15m": 900, "10m": 600, "5m": 300}


@dataclass
class Sample:
    t: float
    cpu: float | None = None
    memory: float | None = None
    gpu: float | None = None
    gpu_memory: float | None = None
    hbm_bandwidth: float | None = None
    xgmi: float | None = None


def _mean(xs) -> float | None:
    xs = [x for x in xs if x is not None]
    return sum(xs) / len(xs) if xs else None


@dataclass
class GpuReading:
    """One GPU's utilisation percentages at one sample."""
    index: int
    gfx: float | None = None          # GFX engine busy
    vram_used_pct: float | None = None
    umc: float | None = None          # HBM controller activity
    xgmi_pct: float | None = None


def aggregate(readings: list[GpuReading], t: float, cpu: float | None = None,
              memory: float | None = None) -> Sample:
    """A node's Sample from its GPUs' readings: the mean of each counter over
    the GPUs that report it (what the node agent publishes for the node)."""
    return Sample(t, cpu, memory, _mean(r.gfx for r in readings), _mean(r.vram_used_pct for r in readings),
                  _mean(r.umc for r in readings), _mean(r.xgmi_pct for r in readings))


class HostSampler:
    """Reads utilisation percentages of the local host (or a sysfs root).

    GPU counters come from amd-smi when it is usable on the live host
    (`gpu_source="auto"` with root "/", or "amdsmi"; `smi` injects a sampler
    for tests), else from amdgpu sysfs. `gpu_source` reports which."""

    def __init__(self, root: str = "/", cards: list[str] | None = None, gpu_source: str = "auto", smi=None):
        self.root = root
        self._prev_cpu: tuple[int, int] | None = None
        if cards is None:
            from .discovery import discover_gpus
            cards = [g.card for g in discover_gpus(root)]
        self.cards = cards
        self.smi = smi
        if self.smi is None and (gpu_source == "amdsmi" or (gpu_source == "auto" and root == "/")):
            from .amdsmi import AmdSmiSampler, native_status
            ok, err = native_status()
            if ok:
                self.smi = AmdSmiSampler()
            elif gpu_source == "amdsmi":
                raise RuntimeError(f"amd-smi unavailable: {err}")
        self.gpu_source = "amdsmi" if self.smi is not None else "sysfs"

    def _cpu(self) -> float | None:
        line = _read(os.path.join(self.root, "proc/stat")).splitlines()[:1]
        if not line or not line[0].startswith("cpu "):
            return None
        vals = [int(x) for x in line[0].split()[1:]]
        idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
        total = sum(vals[:8])
        prev, self._prev_cpu = self._prev_cpu, (idle, total)
        if prev is None or total <= prev[1]:
            return None
        return 100.0 * (1.0 - (idle - prev[0]) / (total - prev[1]))

    def _memory(self) -> float | None:
        info = {}
        for line in _read(os.path.join(self.root, "proc/meminfo")).splitlines():
            k, _, v = line.partition(":")
            if v.strip():
                info[k] = int(v.split()[0])
        tot, avail = info.get("MemTotal"), info.get("MemAvailable")
        if not tot or avail is None:
            return None
        return 100.0 * (tot - avail) / tot

    def gpu_samples(self) -> list[tuple[int | None, float | None]]:
        out = []
        for c in self.cards:
            dev = os.path.join(self.root, "sys/class/drm", c, "device")
            busy = _read_int(os.path.join(dev, "gpu_busy_percent"))
            tot = _read_int(os.path.join(dev, "mem_info_vram_total"), 0) or 0
            used = _read_int(os.path.join(dev, "mem_info_vram_used"), 0) or 0
            out.append((busy, 100.0 * used / tot if tot else None))
        return out

    def per_gpu(self) -> list[GpuReading]:
        """Every visible GPU's reading, in amd-smi / sysfs card order."""
        if self.smi is not None:
            return [GpuReading(i, c.gfx, c.vram_used_pct, c.umc, c.xgmi_pct) for i, c in enumerate(self.smi.sample())]
        return [GpuReading(i, None if b is None else float(b), m) for i, (b, m) in enumerate(self.gpu_samples())]

    def sample(self) -> Sample:
        return aggregate(self.per_gpu(), time.time(), self._cpu(), self._memory())


class RollingWindow:
    def __init__(self, seconds: float):
        self.seconds = seconds
        self.points: deque[tuple[float, float]] = deque()

    def add(self, t: float, v: float | None) -> None:
        if v is None:
            return
        self.points.append((t, v))
        self.trim(t)

    def trim(self, now: float) -> None:
        while self.points and self.points[0][0] < now - self.seconds:
            self.points.popleft()

    def stats(self) -> tuple[float, float, float] | None:
        if not self.points:
            return None
        vals = [v for _, v in self.points]
        mu = sum(vals) / len(vals)
        sd = math.sqrt(sum((v - mu) ** 2 for v in vals) / len(vals))
        return mu, sd, vals[-1]


_TYPES = (("cpu", "CPU"), ("memory", "Memory"), ("gpu", "GPU"), ("gpu_memory", "GPUMemory"),
          ("hbm_bandwidth", "GPUMemoryBandwidth"), ("xgmi", "XGMI"))


class NodeTelemetry:
    """Rolling 15/10/5-minute windows for one node."""

    def __init__(self, node: str, sampler=None, source: str = "xsched-node-agent"):
        self.node, self.sampler, self.source = node, sampler, source
        self.windows = {d: {f: RollingWindow(s) for f, _ in _TYPES} for d, s in WINDOWS.items()}

    def add(self, s: Sample) -> None:
        for wins in self.windows.values():
            for f, _ in _TYPES:
                wins[f].add(s.t, getattr(s, f))

    def sample(self) -> Sample:
        s = self.sampler.sample()
        self.add(s)
        return s

    def metrics(self, duration: str = "15m") -> list[dict]:
        out = []
        for f, typ in _TYPES:
            st = self.windows[duration][f].stats()
            if st is None:
                continue
            mu, sd, last = st
            # Latest before AVG: TargetLoadPacking takes the last AVG-or-Latest
            # metric of a type (targetloadpacking.go:216-221), so it sees the
            # window mean; LVRB reads AVG and STD by operator.
            out.append({"name": f"{f}_utilization", "type": typ, "operator": "Latest", "rollup": "LATEST",
                        "value": round(last, 4)})
            out.append({"name": f"{f}_utilization", "type": typ, "operator": "AVG", "rollup": "AVERAGE",
                        "value": round(mu, 4)})
            out.append({"name": f"{f}_utilization", "type": typ, "operator": "STD", "rollup": "AVERAGE",
                        "value": round(sd, 4)})
        return out

    def watcher_metrics(self, duration: str = "15m", now: float | None = None) -> dict:
        end = int(now if now is not None else time.time())
        return {"metadata": {"name": self.node}, "timestamp": end,
                "window": {"duration": duration, "start": end - WINDOWS[duration], "end": end},
                "source": self.source, "data": {"NodeMetricsMap": {self.node: {"metrics": self.metrics(duration)}}}}


def publish(client, doc: dict) -> None:
    """Create-or-replace the node's document in the API store."""
    name = doc["metadata"]["name"]
    cur = client.get("loadwatchermetrics", "", name)
    if cur is None:
        try:
            client.create("loadwatchermetrics", doc)
            return
        except Exception as e:  # noqa: BLE001
            if getattr(e, "code", 0) != 409:
                raise
            cur = client.get("loadwatchermetrics", "", name)
    body = dict(doc)
    body["metadata"] = dict(doc["metadata"], resourceVersion=cur["metadata"].get("resourceVersion"))
    client.update("loadwatchermetrics", body)


def merge_documents(docs: list[dict]) -> dict | None:
    """Union of WatcherMetrics documents (freshest window per node)."""
    best: dict[str, tuple[int, dict]] = {}
    latest = None
    for d in docs:
        end = int(((d.get("window") or {}).get("end")) or 0)
        nmm = ((d.get("data") or {}).get("NodeMetricsMap")) or {}
        for node, nm in nmm.items():
            if node not in best or best[node][0] < end:
                best[node] = (end, nm)
        if latest is None or end > int(latest["window"]["end"]):
            latest = d
    if latest is None:
        return None
    return {"timestamp": latest.get("timestamp", 0), "window": latest["window"], "source": latest.get("source", ""),
            "data": {"NodeMetricsMap": {n: v for n, (_, v) in sorted(best.items())}}}


class LoadWatcherService:
    """GET /watcher[?host=] and /watcher/health over the published documents."""

    def __init__(self, client, http):
        self.client = client
        http.add_route("GET", "/watcher", self._watcher)
        http.add_route("GET", "/watcher/health", lambda q, b: (200, "text/plain", ""))

    def _watcher(self, q, body):
        docs, _ = self.client.list("loadwatchermetrics")
        merged = merge_documents(docs)
        if merged is None:
            return 404, "application/json", ""
        host = q.get("host")
        if host:
            nm = merged["data"]["NodeMetricsMap"].get(host)
            if nm is None:
                return 404, "application/json", ""
            merged = dict(merged, data={"NodeMetricsMap": {host: nm}})
        return 200, "application/json", merged


class WatcherFetcher:
    """Poll an external load-watcher (`watcherAddress`) every `period`
    seconds (targetloadpacking.go:125-154 refreshes every 30 s) and store the
    document as `loadwatchermetrics/<name>` for the native plugins."""

    def __init__(self, address: str, store_client, name: str = "load-watcher", period: float = 30.0):
        self.url = address.rstrip("/") + "/watcher"
        self.client, self.name, self.period = store_client, name, period
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.fetches = 0
        self.errors = 0

    def fetch_once(self) -> bool:
        try:
            with urllib.request.urlopen(self.url, timeout=10) as r:
                doc = json.loads(r.read())
        except Exception as e:  # noqa: BLE001
            self.errors += 1
            log.warning("load-watcher fetch %s failed: %s", self.url, e)
            return False
        doc = dict(doc, metadata={"name": self.name})
        publish(self.client, doc)
        self.fetches += 1
        return True

    def _run(self) -> None:
        while not self._stop.is_set():
            self.fetch_once()
            self._stop.wait(self.period)

    def start(self) -> "WatcherFetcher":
        self._thread = threading.Thread(target=self._run, name="watcher-fetch", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
