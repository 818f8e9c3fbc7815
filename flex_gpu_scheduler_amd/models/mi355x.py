"""MI355X node model: what one 8x MI355X server looks like to the scheduler.

The reference models a GPU node as two extended-resource integers
(`nvidia.flex.com/gpu` and `.../memory`, pkg/flexgpu/gpu_node.go:30-65). An
MI355X node additionally has compute partitions (SPX/DPX/QPX/CPX split the
8 XCDs of each GPU into 1/2/4/8 devices), 288 GB of HBM3E per GPU, two CPU
sockets with four GPUs each, and a full xGMI mesh (7 links x ~153 GB/s per
GPU). The node agent (control/node_agent.py) publishes exactly these objects
from sysfs; this module builds them synthetically for tests and benches.
"""
from __future__ import annotations

import json
from dataclasses import dataclass

from .objects import make_node, make_nrt, nrt_zone

XCDS_PER_GPU = 8
CUS_PER_XCD = 32
HBM_GIB_PER_GPU = 288
XGMI_LINKS_PER_GPU = 7
XGMI_LINK_GBPS = 153.0
GPUS_PER_NODE = 8
PARTITIONS = {"spx": 1, "dpx": 2, "qpx": 4, "cpx": 8}

GPU = "amd.com/gpu"
GPU_MEMORY = "amd.com/gpu-memory"
GPU_XCD = "amd.com/gpu-xcd"
INDEX_ANNOTATION = "amd.com/gpu-index"
PARTITION_ANNOTATION = "amd.com/gpu-partitions"
PARTITION_LABEL = "amd.com/gpu.compute-partition"
TOPOLOGY_ANNOTATION = "amd.com/gpu-topology"


@dataclass
class GpuInfo:
    index: int
    partition_mode: str = "spx"
    hbm_gib: int = HBM_GIB_PER_GPU
    numa: int = 0
    cus: int = XCDS_PER_GPU * CUS_PER_XCD

    @property
    def partitions(self) -> int:
        return PARTITIONS[self.partition_mode]


def default_gpus(n: int = GPUS_PER_NODE, mode: str = "spx", sockets: int = 2) -> list[GpuInfo]:
    per = max(1, n // sockets)
    return [GpuInfo(i, mode, numa=min(sockets - 1, i // per)) for i in range(n)]


def mi355x_node(name: str, *, gpus: list[GpuInfo] | None = None, n_gpus: int = GPUS_PER_NODE, mode: str = "spx",
                cpu: str = "256", memory: str = "3Ti", pods: int = 256, labels: dict | None = None,
                taints: list[dict] | None = None) -> dict:
    """A Node object as the MI355X node agent advertises it.

    amd.com/gpu = physical GPUs; amd.com/gpu-xcd = 8 x GPUs; amd.com/gpu-memory
    = total HBM in GiB (the FlexGPU memory path splits it evenly per GPU).
    """
    gpus = gpus if gpus is not None else default_gpus(n_gpus, mode)
    modes = {g.partition_mode for g in gpus}
    lab = {PARTITION_LABEL: modes.pop() if len(modes) == 1 else "mixed", "amd.com/gpu.product": "MI355X",
           "amd.com/gpu.family": "CDNA4", **(labels or {})}
    topo = {"gpus": [{"index": g.index, "partitions": g.partitions, "numa": g.numa, "hbmGiB": g.hbm_gib, "cus": g.cus}
                     for g in gpus],
            "xgmi": {"links": XGMI_LINKS_PER_GPU, "linkGBps": XGMI_LINK_GBPS, "topology": "fullmesh"}}
    alloc = {"cpu": cpu, "memory": memory, "pods": str(pods), GPU: str(len(gpus)),
             GPU_MEMORY: str(sum(g.hbm_gib for g in gpus)), GPU_XCD: str(XCDS_PER_GPU * len(gpus))}
    return make_node(name, alloc, labels=lab, annotations={TOPOLOGY_ANNOTATION: json.dumps(topo)}, taints=taints)


def mi355x_nrt(name: str, *, gpus: list[GpuInfo] | None = None, cpu_per_socket: int = 128,
               memory_per_socket_gib: int = 1536, sockets: int = 2,
               policies=("SingleNUMANodeContainerLevel",)) -> dict:
    """NodeResourceTopology CR with one zone per CPU socket holding its GPUs.

    xGMI is a full mesh inside the node, so GPU-to-GPU distance is uniform;
    what differs is socket locality (CPU/host memory/NIC) and same-node vs
    cross-node. Zone costs encode that: local socket 10, remote socket 32.
    """
    gpus = gpus if gpus is not None else default_gpus()
    zones = []
    for s in range(sockets):
        mine = [g for g in gpus if g.numa == s]
        res = {"cpu": cpu_per_socket, "memory": f"{memory_per_socket_gib}Gi", GPU: len(mine),
               GPU_XCD: XCDS_PER_GPU * len(mine), GPU_MEMORY: sum(g.hbm_gib for g in mine)}
        costs = {f"node-{o}": (10 if o == s else 32) for o in range(sockets)}
        zones.append(nrt_zone(s, res, costs=costs))
    return make_nrt(name, zones, policies)
