"""Kubelet device plugin for MI355X resources (the device-plugin role of the
node agent).

The scheduler picks concrete GPUs / partitions / HBM slices and records them
on the pod (`amd.com/gpu-index`, `amd.com/gpu-partitions`, carried by the
Binding). Kubelet, however, asks a device plugin to `Allocate` N fungible
device IDs per container without saying which pod they are for. As in the
reference's NVIDIA flex stack (and gpushare-style plugins), `Allocate`
therefore resolves the pod: the oldest bound, not-yet-started pod on this node
whose request of the resource equals N and that carries the scheduler's
placement annotations but no `amd.com/gpu-assigned` mark. It returns:

  * device specs: /dev/kfd plus the DRM render node of each chosen GPU
    (renderD(128+N) for cardN) or partition p (renderD(128+N+p): the amdgpu
    `xcp` partition nodes follow their GPU's primary node);
  * envs: HIP_VISIBLE_DEVICES (container-local ordinals), XSCHED_GPU_INDEX,
    XSCHED_GPU_PARTITIONS and, for HBM slices, XSCHED_HBM_LIMIT_GIB;

and marks the pod so a second Allocate cannot reuse it. Devices are
advertised per resource: `amd.com/gpu` (untouched SPX GPUs), `amd.com/gpu-xcd`
(8 per GPU) and `amd.com/gpu-memory` (1 per GiB of HBM), each with its NUMA
node so kubelet's topology manager can align them.
"""
from __future__ import annotations

import logging
import os
import threading
from concurrent import futures

import grpc

from ..gpu.discovery import HostInfo
from ..models.mi355x import GPU, GPU_MEMORY, GPU_XCD, INDEX_ANNOTATION, PARTITION_ANNOTATION, XCDS_PER_GPU
from .client import Client
from .deviceplugin_api import DEVICE_PLUGIN_PATH, HEALTHY, KUBELET_SOCKET, UNHEALTHY, VERSION, method_path, pb

log = logging.getLogger(__name__)

ASSIGNED_ANNOTATION = "amd.com/gpu-assigned"


def _card_minor(card: str) -> int:
    return int(card[4:]) if card.startswith("card") and card[4:].isdigit() else 0


def render_node(host: HostInfo, gpu: int, partition: int = 0, dev_root: str = "/dev") -> str:
    g = host.gpus[gpu]
    return f"{dev_root}/dri/renderD{128 + _card_minor(g.card) + partition}"


class GpuDevicePlugin:
    def __init__(self, resource: str, host: HostInfo, client: Client, node_name: str, *,
                 socket_dir: str = DEVICE_PLUGIN_PATH, dev_root: str = "/dev", unhealthy: set[int] | None = None):
        if resource not in (GPU, GPU_XCD, GPU_MEMORY):
            raise ValueError(f"unsupported resource {resource}")
        self.resource, self.host, self.client, self.node = resource, host, client, node_name
        self.socket_dir, self.dev_root = socket_dir, dev_root
        short = resource.split("/")[-1]
        self.endpoint = f"xsched-{short}.sock"
        self.unhealthy = set(unhealthy or ())
        self._server: grpc.Server | None = None
        self._cv = threading.Condition()
        self._gen = 0
        self._stop = threading.Event()
        self._alloc_lock = threading.Lock()
        self.allocations = 0

    # ---------------------------------------------------------------- devices
    def devices(self) -> list:
        out = []
        for g in self.host.gpus:
            health = UNHEALTHY if g.index in self.unhealthy else HEALTHY
            topo = pb.TopologyInfo(nodes=[pb.NUMANode(ID=max(0, g.numa))])
            if self.resource == GPU:
                if g.partitions == 1:
                    out.append(pb.Device(ID=f"gpu-{g.index}", health=health, topology=topo))
            elif self.resource == GPU_XCD:
                out += [pb.Device(ID=f"xcd-{g.index}-{k}", health=health, topology=topo) for k in range(XCDS_PER_GPU)]
            else:
                out += [pb.Device(ID=f"mem-{g.index}-{i}", health=health, topology=topo) for i in range(g.hbm_gib)]
        return out

    def set_unhealthy(self, gpus: set[int]) -> None:
        with self._cv:
            if gpus != self.unhealthy:
                self.unhealthy = set(gpus)
                self._gen += 1
                self._cv.notify_all()

    # ------------------------------------------------------------ allocation
    def _demand(self, pod: dict) -> int:
        total = 0
        for c in (pod.get("spec") or {}).get("containers") or []:
            lim = ((c.get("resources") or {}).get("limits") or {}).get(self.resource)
            req = ((c.get("resources") or {}).get("requests") or {}).get(self.resource)
            v = lim if lim is not None else req
            if v is not None:
                total += int(str(v))
        return total

    @staticmethod
    def _scheduled_at(pod: dict) -> str:
        for c in (pod.get("status") or {}).get("conditions") or []:
            if c.get("type") == "PodScheduled" and c.get("status") == "True":
                return c.get("lastTransitionTime") or ""
        return (pod.get("metadata") or {}).get("creationTimestamp") or ""

    def find_pod(self, n: int) -> dict | None:
        pods, _ = self.client.list("pods", "", field_selector=f"spec.nodeName={self.node}")
        cands = []
        for p in pods:
            md = p.get("metadata") or {}
            ann = md.get("annotations") or {}
            if (p.get("status") or {}).get("phase", "Pending") != "Pending" or md.get("deletionTimestamp"):
                continue
            if INDEX_ANNOTATION not in ann or ann.get(ASSIGNED_ANNOTATION) == "true":
                continue
            if self._demand(p) != n:
                continue
            cands.append(p)
        cands.sort(key=self._scheduled_at)
        return cands[0] if cands else None

    def container_response(self, pod: dict):
        ann = pod["metadata"].get("annotations") or {}
        gpus = [int(x) for x in ann.get(INDEX_ANNOTATION, "").split(",") if x.strip()]
        parts = [tuple(int(v) for v in x.split(":")) for x in ann.get(PARTITION_ANNOTATION, "").split(",") if ":" in x]
        targets = parts if parts else [(g, 0) for g in gpus]
        devs = [pb.DeviceSpec(container_path=f"{self.dev_root}/kfd", host_path=f"{self.dev_root}/kfd",
                              permissions="rw")]
        for g, p in targets:
            if 0 <= g < len(self.host.gpus):
                path = render_node(self.host, g, p, self.dev_root)
                devs.append(pb.DeviceSpec(container_path=path, host_path=path, permissions="rw"))
        envs = {"HIP_VISIBLE_DEVICES": ",".join(str(i) for i in range(len(targets))),
                "XSCHED_GPU_INDEX": ann.get(INDEX_ANNOTATION, ""),
                "XSCHED_GPU_PARTITIONS": ann.get(PARTITION_ANNOTATION, "")}
        if self.resource == GPU_MEMORY:
            envs["XSCHED_HBM_LIMIT_GIB"] = str(self._demand(pod))
        return pb.ContainerAllocateResponse(envs=envs, devices=devs,
                                            annotations={"xsched.amd.com/pod": f"{pod['metadata'].get('namespace')}/"
                                                                               f"{pod['metadata'].get('name')}"})

    # ------------------------------------------------------------------ gRPC
    def _get_options(self, req, ctx):
        return pb.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def _list_and_watch(self, req, ctx):
        last = -1
        while not self._stop.is_set() and ctx.is_active():
            with self._cv:
                if self._gen == last:
                    self._cv.wait(timeout=1.0)
                    if self._gen == last:
                        continue
                last = self._gen
            yield pb.ListAndWatchResponse(devices=self.devices())

    def _preferred(self, req, ctx):
        resp = pb.PreferredAllocationResponse()
        for cr in req.container_requests:
            must = list(cr.must_include_deviceIDs)
            rest = [d for d in cr.available_deviceIDs if d not in must]
            resp.container_responses.add(deviceIDs=(must + rest)[: cr.allocation_size])
        return resp

    def _allocate(self, req, ctx):
        resp = pb.AllocateResponse()
        with self._alloc_lock:
            for cr in req.container_requests:
                n = len(cr.devicesIDs)
                pod = self.find_pod(n)
                if pod is None:
                    ctx.abort(grpc.StatusCode.FAILED_PRECONDITION,
                              f"no pod on {self.node} with a scheduler placement requesting {n} {self.resource}")
                resp.container_responses.append(self.container_response(pod))
                md = pod["metadata"]
                self.client.patch("pods", md.get("namespace", "default"), md["name"],
                                  {"metadata": {"annotations": {ASSIGNED_ANNOTATION: "true"}}})
                self.allocations += 1
        return resp

    def _prestart(self, req, ctx):
        return pb.PreStartContainerResponse()

    def _handler(self):
        def uu(fn, req, resp):
            return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req.FromString,
                                                       response_serializer=resp.SerializeToString)
        return grpc.method_handlers_generic_handler(f"{VERSION}.DevicePlugin", {
            "GetDevicePluginOptions": uu(self._get_options, pb.Empty, pb.DevicePluginOptions),
            "ListAndWatch": grpc.unary_stream_rpc_method_handler(
                self._list_and_watch, request_deserializer=pb.Empty.FromString,
                response_serializer=pb.ListAndWatchResponse.SerializeToString),
            "GetPreferredAllocation": uu(self._preferred, pb.PreferredAllocationRequest, pb.PreferredAllocationResponse),
            "Allocate": uu(self._allocate, pb.AllocateRequest, pb.AllocateResponse),
            "PreStartContainer": uu(self._prestart, pb.PreStartContainerRequest, pb.PreStartContainerResponse),
        })

    @property
    def socket_path(self) -> str:
        return os.path.join(self.socket_dir, self.endpoint)

    def serve(self) -> "GpuDevicePlugin":
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        self._server.add_generic_rpc_handlers((self._handler(),))
        self._server.add_insecure_port(f"unix://{self.socket_path}")
        self._server.start()
        return self

    def register(self, timeout: float = 10.0) -> None:
        kubelet = os.path.join(self.socket_dir, KUBELET_SOCKET)
        with grpc.insecure_channel(f"unix://{kubelet}") as ch:
            call = ch.unary_unary(method_path("Registration", "Register"),
                                  request_serializer=pb.RegisterRequest.SerializeToString,
                                  response_deserializer=pb.Empty.FromString)
            call(pb.RegisterRequest(version=VERSION, endpoint=self.endpoint, resource_name=self.resource,
                                    options=pb.DevicePluginOptions(get_preferred_allocation_available=True)),
                 timeout=timeout)

    def run(self, poll: float = 5.0) -> None:
        """Serve + register, re-registering whenever kubelet restarts (kubelet
        wipes the plugin directory, removing our socket)."""
        while not self._stop.is_set():
            try:
                self.serve()
                self.register()
                log.info("device plugin %s registered at %s", self.resource, self.socket_path)
            except Exception as e:  # noqa: BLE001 - kubelet not up yet
                log.warning("device plugin %s: registration failed: %s", self.resource, e)
                self.stop_server()
                self._stop.wait(poll)
                continue
            while not self._stop.wait(poll):
                if not os.path.exists(self.socket_path):
                    log.info("device plugin %s: socket removed (kubelet restart); re-registering", self.resource)
                    break
            self.stop_server()

    def stop_server(self) -> None:
        if self._server is not None:
            self._server.stop(grace=0.5)
            self._server = None

    def stop(self) -> None:
        self._stop.set()
        with self._cv:
            self._gen += 1
            self._cv.notify_all()
        self.stop_server()


def start_plugins(host: HostInfo, client: Client, node_name: str, **kw) -> list[GpuDevicePlugin]:
    plugins = [GpuDevicePlugin(r, host, client, node_name, **kw) for r in (GPU, GPU_XCD, GPU_MEMORY)]
    for p in plugins:
        threading.Thread(target=p.run, daemon=True, name=f"devplugin-{p.endpoint}").start()
    return plugins
