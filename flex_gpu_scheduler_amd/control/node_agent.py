"""MI355X node agent: advertises a GPU node to the scheduler.

Plays the roles the reference delegates to the NVIDIA device plugin + the NRT
exporter + metrics-server:
  * discovers the box from sysfs (gpu/discovery.py) — GPUs, compute/memory
    partition modes, HBM, NUMA locality, xGMI hive;
  * registers/updates the Node: allocatable `amd.com/gpu` (whole SPX GPUs),
    `amd.com/gpu-xcd` (XCD slices), `amd.com/gpu-memory` (HBM GiB), the
    compute-partition label and the `amd.com/gpu-topology` annotation FlexGPU
    reads (csrc/plugins/flexgpu.cc), plus a Ready heartbeat condition;
  * publishes the NodeResourceTopology CR (one zone per CPU socket holding its
    GPUs) for NodeResourceTopologyMatch;
  * optionally runs the HIP health probe (ops/hip_probe.py: pattern write +
    checksum per GPU) and withholds unhealthy GPUs from allocatable, tainting
    the node when none are healthy;
  * samples load (gpu/telemetry.py) and publishes its WatcherMetrics document
    for the Trimaran plugins.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from datetime import datetime, timezone
from typing import Callable

from ..gpu.discovery import HostInfo, discover_host
from ..gpu.telemetry import HostSampler, NodeTelemetry, publish
from ..models.mi355x import (GPU, GPU_MEMORY, GPU_XCD, TOPOLOGY_ANNOTATION, XCDS_PER_GPU, mi355x_node,
                             mi355x_nrt)
from .client import Client, is_conflict

log = logging.getLogger(__name__)

# Per-GPU HBM bandwidth by compute-partition size (NodeAgent.measure_bandwidth).
BANDWIDTH_ANNOTATION = "amd.com/gpu-hbm-bandwidth"
UNHEALTHY_TAINT = {"key": "amd.com/gpu-unhealthy", "value": "true", "effect": "NoSchedule"}
MEMORY_PARTITION_LABEL = "amd.com/gpu.memory-partition"
HIVE_LABEL = "amd.com/xgmi.hive"


def _now() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


class NodeAgent:
    def __init__(self, client: Client, node_name: str, *, host_fn: Callable[[], HostInfo] | None = None,
                 root: str = "/", labels: dict | None = None, reserved_cpu: int = 0, reserved_memory_gib: int = 0,
                 heartbeat: float = 10.0, telemetry_period: float = 60.0, publish_metrics: bool = True,
                 health_fn: Callable[[int], bool] | None = None, sampler=None, kubelet_managed: bool = False,
                 bandwidth_fn: Callable[[int], dict] | None = None):
        self.client, self.name = client, node_name
        self.host_fn = host_fn or (lambda: discover_host(root))
        self.labels = dict(labels or {})
        self.reserved_cpu, self.reserved_memory_gib = reserved_cpu, reserved_memory_gib
        self.heartbeat, self.telemetry_period = heartbeat, telemetry_period
        self.health_fn = health_fn
        # HBM bandwidth per compute-partition size, per GPU (ops/hip_probe.py
        # partition_table): measured once per GPU and published with the node.
        self.bandwidth_fn = bandwidth_fn
        self.bandwidth: dict[int, dict] = {}
        # A GPU whose probe failed is not probed again on every heartbeat
        # (each attempt streams GiBs through a GPU that may be serving
        # tenants): GPU index -> time.monotonic() of the next attempt.
        self.bandwidth_retry_s = 600.0
        self._bandwidth_retry_at: dict[int, float] = {}
        self.publish_metrics = publish_metrics
        self._sampler = sampler
        self._root = root
        self.telemetry: NodeTelemetry | None = None
        self.unhealthy: set[int] = set()
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.host: HostInfo | None = None
        # With a kubelet on the node, the device plugins advertise amd.com/*
        # capacity; the agent must not write those fields (kubelet owns them).
        self.kubelet_managed = kubelet_managed
        self.device_plugins: list = []

    # --------------------------------------------------------------- objects
    def check_health(self, host: HostInfo) -> set[int]:
        if self.health_fn is None:
            return set()
        bad = set()
        # HIP ordinals follow the KFD node order of the GPUs this process can
        # open; GPUs whose KFD node is hidden (other containers' devices) are
        # not probed. With no KFD info at all (fake hosts) use the index.
        visible = sorted((g for g in host.gpus if g.kfd_node is not None), key=lambda g: g.kfd_node)
        targets = [(i, g) for i, g in enumerate(visible)] if visible else [(g.index, g) for g in host.gpus]
        for ordinal, g in targets:
            try:
                if not self.health_fn(ordinal):
                    bad.add(g.index)
            except Exception as e:  # noqa: BLE001
                log.warning("health probe GPU %d failed: %s", g.index, e)
                bad.add(g.index)
        return bad

    def measure_bandwidth(self, host: HostInfo) -> None:
        """Partition bandwidth table per healthy GPU (HIP ordinal order, as
        check_health), measured the first time a GPU is seen."""
        if self.bandwidth_fn is None:
            return
        visible = sorted((g for g in host.gpus if g.kfd_node is not None), key=lambda g: g.kfd_node)
        targets = [(i, g) for i, g in enumerate(visible)] if visible else [(g.index, g) for g in host.gpus]
        now = time.monotonic()
        for ordinal, g in targets:
            if g.index in self.bandwidth or g.index in self.unhealthy:
                continue
            if now < self._bandwidth_retry_at.get(g.index, 0.0):
                continue
            try:
                self.bandwidth[g.index] = self.bandwidth_fn(ordinal)
                self._bandwidth_retry_at.pop(g.index, None)
            except Exception as e:  # noqa: BLE001
                log.warning("bandwidth probe GPU %d failed (next try in %.0f s): %s", g.index,
                            self.bandwidth_retry_s, e)
                self._bandwidth_retry_at[g.index] = now + self.bandwidth_retry_s

    def build_node(self, host: HostInfo, unhealthy: set[int] = frozenset()) -> dict:
        healthy = [g for g in host.gpus if g.index not in unhealthy]
        infos = [g.to_gpu_info() for g in healthy]
        mem_kib = max(0, host.memory_bytes // 1024 - self.reserved_memory_gib * (1 << 20))
        labels = dict(self.labels)
        parts = {g.memory_partition for g in host.gpus}
        if len(parts) == 1:
            labels[MEMORY_PARTITION_LABEL] = parts.pop()
        if host.xgmi_hive:
            labels[HIVE_LABEL] = f"{host.xgmi_hive:x}"
        node = mi355x_node(self.name, gpus=infos, cpu=str(max(1, host.cpus - self.reserved_cpu)),
                           memory=f"{mem_kib}Ki", pods=max(110, host.cpus), labels=labels,
                           taints=[UNHEALTHY_TAINT] if host.gpus and not healthy else None)
        if not host.gpus:  # a CPU-only node carries no GPU identity labels
            for k in ("amd.com/gpu.compute-partition", "amd.com/gpu.product", "amd.com/gpu.family"):
                node["metadata"]["labels"].pop(k, None)
        topo = json.loads(node["metadata"]["annotations"][TOPOLOGY_ANNOTATION])
        by_index = {g.index: g for g in healthy}
        for i, entry in enumerate(topo["gpus"]):
            g = by_index[infos[i].index]
            entry.update(bdf=g.bdf, uniqueId=g.unique_id, memoryPartition=g.memory_partition,
                         computePartition=g.compute_partition, xgmiLinks=len(g.xgmi_links),
                         xgmiLinkMBps=max((lk.bandwidth_mbps for lk in g.xgmi_links), default=0))
        topo["unhealthy"] = sorted(unhealthy)
        node["metadata"]["annotations"][TOPOLOGY_ANNOTATION] = json.dumps(topo, sort_keys=True)
        if self.bandwidth:
            node["metadata"]["annotations"][BANDWIDTH_ANNOTATION] = json.dumps(
                {str(i): t for i, t in sorted(self.bandwidth.items()) if i not in unhealthy}, sort_keys=True)
        # Capacity reports the hardware; allocatable withholds unhealthy GPUs.
        cap = dict(node["status"]["allocatable"])
        cap[GPU] = str(len(host.gpus))
        cap[GPU_XCD] = str(XCDS_PER_GPU * len(host.gpus))
        cap[GPU_MEMORY] = str(sum(g.hbm_gib for g in host.gpus))
        node["status"]["capacity"] = cap
        if self.kubelet_managed:
            for k in (GPU, GPU_XCD, GPU_MEMORY):
                node["status"]["allocatable"].pop(k, None)
                node["status"]["capacity"].pop(k, None)
        node["status"]["conditions"] = [self._ready_condition()]
        node["status"]["nodeInfo"] = {"architecture": "amd64", "operatingSystem": "linux",
                                      "kubeletVersion": "v1.23.3-xsched-agent"}
        return node

    @staticmethod
    def _ready_condition() -> dict:
        now = _now()
        return {"type": "Ready", "status": "True", "reason": "AgentReady", "message": "MI355X node agent is posting",
                "lastHeartbeatTime": now, "lastTransitionTime": now}

    def build_nrt(self, host: HostInfo, unhealthy: set[int] = frozenset()) -> dict:
        sockets = max(1, len(host.numa_nodes))
        cpus = [len(host.numa_cpus.get(s, [])) or host.cpus // sockets for s in range(sockets)]
        mem_gib = host.memory_bytes // (1 << 30) // sockets
        gpus = [g.to_gpu_info() for g in host.gpus if g.index not in unhealthy]
        nrt = mi355x_nrt(self.name, gpus=gpus, cpu_per_socket=min(cpus), memory_per_socket_gib=mem_gib,
                         sockets=sockets)
        for z, c in zip(nrt["zones"], cpus):
            for r in z["resources"]:
                if r["name"] == "cpu":
                    r["capacity"] = r["allocatable"] = r["available"] = str(c)
        return nrt

    # --------------------------------------------------------------- publish
    def _upsert(self, kind: str, obj: dict, keep_spec: bool) -> None:
        name = obj["metadata"]["name"]
        for _ in range(5):
            cur = self.client.get(kind, "", name)
            if cur is None:
                try:
                    self.client.create(kind, obj)
                    return
                except Exception as e:  # noqa: BLE001
                    if not is_conflict(e):
                        raise
                    continue
            body = json.loads(json.dumps(obj))
            if keep_spec:
                # Node spec (cordon, admin taints) belongs to the cluster, not
                # the agent; keep it, only manage our own taint.
                spec = dict(cur.get("spec") or {})
                taints = [t for t in spec.get("taints") or [] if t.get("key") != UNHEALTHY_TAINT["key"]]
                taints += [t for t in (obj.get("spec") or {}).get("taints") or []]
                if taints:
                    spec["taints"] = taints
                else:
                    spec.pop("taints", None)
                body["spec"] = spec
                md = body["metadata"]
                md["labels"] = {**(cur["metadata"].get("labels") or {}), **(md.get("labels") or {})}
                md["annotations"] = {**(cur["metadata"].get("annotations") or {}), **(md.get("annotations") or {})}
            body["metadata"]["resourceVersion"] = cur["metadata"].get("resourceVersion")
            try:
                self.client.update(kind, body)
                return
            except Exception as e:  # noqa: BLE001
                if not is_conflict(e):
                    raise
        raise RuntimeError(f"could not update {kind}/{name}: persistent conflicts")

    def sync(self) -> HostInfo:
        host = self.host_fn()
        self.unhealthy = self.check_health(host)
        self.measure_bandwidth(host)
        for dp in self.device_plugins:
            dp.host = host
            dp.set_unhealthy(self.unhealthy)
        self._upsert("nodes", self.build_node(host, self.unhealthy), keep_spec=True)
        self._upsert("noderesourcetopologies", self.build_nrt(host, self.unhealthy), keep_spec=False)
        self.host = host
        return host

    def post_heartbeat(self) -> None:
        self.client.patch("nodes", "", self.name, {"status": {"conditions": [self._ready_condition()]}})

    def sample_and_publish(self) -> dict | None:
        if self.telemetry is None:
            self.telemetry = NodeTelemetry(self.name, self._sampler or HostSampler(self._root))
        self.telemetry.sample()
        doc = self.telemetry.watcher_metrics("15m")
        if self.publish_metrics:
            publish(self.client, doc)
        return doc

    # ------------------------------------------------------------------ run
    def _loop(self, period: float, fn: Callable[[], object]) -> None:
        while not self._stop.wait(period):
            try:
                fn()
            except Exception:  # noqa: BLE001
                log.exception("node agent %s: periodic task failed", self.name)

    def start(self) -> "NodeAgent":
        self.sync()
        if self.publish_metrics:
            self.sample_and_publish()
        loops = [(self.heartbeat, self._heartbeat_and_resync)]
        if self.publish_metrics:
            loops.append((self.telemetry_period, self.sample_and_publish))
        for period, fn in loops:
            t = threading.Thread(target=self._loop, args=(period, fn), daemon=True, name="node-agent")
            t.start()
            self._threads.append(t)
        return self

    def _heartbeat_and_resync(self) -> None:
        host = self.host_fn()
        unhealthy = self.check_health(host)
        changed = (self.host is None or [g.to_gpu_info() for g in host.gpus] != [g.to_gpu_info() for g in self.host.gpus]
                   or unhealthy != self.unhealthy)
        if changed:
            self.sync()
        else:
            self.post_heartbeat()

    def stop(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)


def hip_health_fn() -> Callable[[int], bool]:
    """Health callback backed by the HIP probes (HBM pattern + checksum and an
    MFMA tile check per GPU)."""
    from ..ops.hip_probe import probe

    p = probe()
    # HBM pattern/checksum and an exact-integer MFMA tile: a GPU whose matrix
    # cores mis-compute is withheld even if its memory checks out.
    return lambda dev: bool(p.health(dev)["healthy"]) and bool(p.mfma_check(dev)["healthy"])


def hip_bandwidth_fn(nbytes: int = 1 << 30, iters: int = 10) -> Callable[[int], dict]:
    """Partition bandwidth table backed by the HIP XCD-pinned streaming probe
    (read and copy over a 1 GiB working set per CPX/QPX/DPX/SPX XCD set)."""
    from ..ops.hip_probe import probe

    p = probe()
    return lambda dev: p.partition_table(dev, nbytes, iters)


def run_forever(agent: NodeAgent) -> None:  # pragma: no cover - CLI
    agent.start()
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        agent.stop()
