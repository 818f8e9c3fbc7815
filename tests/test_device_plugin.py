"""Kubelet device-plugin API: registration, ListAndWatch, Allocate resolving
the scheduler's placement into render nodes and env (the node agent's
device-plugin role), against a fake kubelet over unix sockets."""
import os
import threading
import time
from concurrent import futures

import grpc
import pytest

from flex_gpu_scheduler_amd.control import LocalClient
from flex_gpu_scheduler_amd.control.device_plugin import ASSIGNED_ANNOTATION, GpuDevicePlugin, render_node
from flex_gpu_scheduler_amd.control.deviceplugin_api import VERSION, method_path, pb
from flex_gpu_scheduler_amd.gpu import discover_host
from flex_gpu_scheduler_amd.gpu.discovery import fake_host
from flex_gpu_scheduler_amd.models import GPU, GPU_MEMORY, GPU_XCD, make_pod

BOX = os.path.join(os.path.dirname(__file__), "fixtures", "mi355x_box", "root")


class FakeKubelet:
    def __init__(self, d):
        self.registrations = []
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))

        def register(req, ctx):
            self.registrations.append(req)
            return pb.Empty()
        h = grpc.method_handlers_generic_handler(f"{VERSION}.Registration", {
            "Register": grpc.unary_unary_rpc_method_handler(register, request_deserializer=pb.RegisterRequest.FromString,
                                                            response_serializer=pb.Empty.SerializeToString)})
        self.server.add_generic_rpc_handlers((h,))
        self.server.add_insecure_port(f"unix://{d}/kubelet.sock")
        self.server.start()

    def stub(self, sock, method, req_cls, resp_cls, stream=False):
        ch = grpc.insecure_channel(f"unix://{sock}")
        f = (ch.unary_stream if stream else ch.unary_unary)(
            method_path("DevicePlugin", method), request_serializer=req_cls.SerializeToString,
            response_deserializer=resp_cls.FromString)
        return ch, f


@pytest.fixture
def sockdir():
    # unix socket paths must stay short
    import tempfile
    d = tempfile.mkdtemp(prefix="dp", dir="/tmp")
    yield d


def bound_pod(store, name, node, res, amount, gpu_index, partitions=None):
    p = make_pod(name, limits={res: str(amount)}, requests={res: str(amount)})
    store.create("pods", p)
    ann = {"amd.com/gpu-index": gpu_index}
    if partitions:
        ann["amd.com/gpu-partitions"] = partitions
    store.bind("default", name, "", node, ann)


def test_render_nodes_follow_drm_minors():
    h = discover_host(BOX)
    # card8 -> renderD136 (its partitions: renderD137..), card40 -> renderD168
    g0 = h.gpus[0]
    assert g0.card == "card8" and render_node(h, 0) == "/dev/dri/renderD136"
    assert render_node(h, 0, 3) == "/dev/dri/renderD139"
    vis = next(g for g in h.gpus if g.kfd_node is not None)
    assert render_node(h, vis.index).endswith(f"renderD{vis.render_minor}")  # KFD agrees


def test_register_list_and_allocate(store, sockdir):
    kubelet = FakeKubelet(sockdir)
    host = fake_host(8, "SPX")
    client = LocalClient(store)
    plugin = GpuDevicePlugin(GPU, host, client, "node-a", socket_dir=sockdir)
    t = threading.Thread(target=plugin.run, kwargs={"poll": 0.1}, daemon=True)
    t.start()
    try:
        deadline = time.time() + 10
        while time.time() < deadline and not kubelet.registrations:
            time.sleep(0.02)
        (reg,) = kubelet.registrations
        assert reg.resource_name == GPU and reg.version == VERSION and reg.endpoint == "xsched-gpu.sock"
        sock = os.path.join(sockdir, reg.endpoint)
        ch, law = kubelet.stub(sock, "ListAndWatch", pb.Empty, pb.ListAndWatchResponse, stream=True)
        it = law(pb.Empty())
        first = next(it)
        assert [d.ID for d in first.devices] == [f"gpu-{i}" for i in range(8)]
        assert first.devices[5].topology.nodes[0].ID == 1
        plugin.set_unhealthy({2})
        second = next(it)
        assert [d.health for d in second.devices].count("Unhealthy") == 1
        ch.close()

        bound_pod(store, "train-0", "node-a", GPU, 2, "4,5")
        bound_pod(store, "elsewhere", "node-b", GPU, 2, "0,1")
        ch, alloc = kubelet.stub(sock, "Allocate", pb.AllocateRequest, pb.AllocateResponse)
        resp = alloc(pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devicesIDs=["gpu-0", "gpu-1"])]))
        (cr,) = resp.container_responses
        paths = sorted(d.host_path for d in cr.devices)
        assert paths == ["/dev/dri/renderD160", "/dev/dri/renderD168", "/dev/kfd"]  # cards 32 and 40
        assert cr.envs["HIP_VISIBLE_DEVICES"] == "0,1" and cr.envs["XSCHED_GPU_INDEX"] == "4,5"
        assert store.get("pods", "default", "train-0")["metadata"]["annotations"][ASSIGNED_ANNOTATION] == "true"
        # A second Allocate finds no unassigned pod on this node.
        with pytest.raises(grpc.RpcError) as e:
            alloc(pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devicesIDs=["gpu-2", "gpu-3"])]))
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION
        ch.close()
    finally:
        plugin.stop()
        kubelet.server.stop(0)
        t.join(timeout=5)


def test_partition_and_memory_allocation(store, sockdir):
    host = fake_host(8, "CPX")
    client = LocalClient(store)
    xcd = GpuDevicePlugin(GPU_XCD, host, client, "n", socket_dir=sockdir)
    assert len(xcd.devices()) == 64
    bound_pod(store, "quarter", "n", GPU_XCD, 2, "3", "3:4,3:5")
    r = xcd.container_response(xcd.find_pod(2))
    assert sorted(d.host_path for d in r.devices)[:2] == ["/dev/dri/renderD156", "/dev/dri/renderD157"]
    assert r.envs["XSCHED_GPU_PARTITIONS"] == "3:4,3:5"
    mem = GpuDevicePlugin(GPU_MEMORY, host, client, "n", socket_dir=sockdir)
    assert len(mem.devices()) == 8 * 288
    bound_pod(store, "slice", "n", GPU_MEMORY, 36, "6", "6:0")
    r = mem.container_response(mem.find_pod(36))
    assert r.envs["XSCHED_HBM_LIMIT_GIB"] == "36"
    # An SPX-only resource: no CPX GPU is a whole-GPU device.
    assert GpuDevicePlugin(GPU, host, client, "n", socket_dir=sockdir).devices() == []


def test_agent_kubelet_managed_leaves_capacity_to_plugins(store):
    from flex_gpu_scheduler_amd.control.node_agent import NodeAgent
    agent = NodeAgent(LocalClient(store), "n", host_fn=lambda: fake_host(8), publish_metrics=False, kubelet_managed=True)
    agent.sync()
    st = store.get("nodes", "", "n")["status"]
    assert GPU not in st["allocatable"] and GPU_XCD not in st["capacity"]
    assert st["allocatable"]["cpu"] == "256"
