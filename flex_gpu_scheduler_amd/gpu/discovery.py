"""MI355X hardware discovery from sysfs (amdgpu DRM + KFD topology).

This is the node agent's view of the box — the device-plugin role the
reference leaves to NVIDIA's stack (it only reads the advertised integers,
pkg/flexgpu/gpu_node.go:30-65). Sources, all plain files (no SMI process on
the hot path, no root needed):

  /sys/class/drm/cardN/device/        physical GPU = PCI function (uevent
      PCI_SLOT_NAME), current_compute_partition (SPX/DPX/QPX/CPX),
      current_memory_partition (NPS1/NPS2), numa_node, local_cpulist,
      mem_info_vram_total/used, gpu_busy_percent, unique_id, product_name.
      `amdgpu_xcp_*` platform cards are partition render nodes, not GPUs.
  /sys/class/kfd/kfd/topology/nodes/N/properties   compute topology of every
      agent the process may see: simd_count (4 SIMD per CU), num_xcc,
      location_id/domain (PCI address), hive_id (xGMI hive), and io_links of
      type 11 (XGMI) with their bandwidth.

A capture of a real 8x MI355X box (tests/fixtures/mi355x_box) backs the CPU
tests: 8 SPX GPUs with 288 GiB each, two NUMA nodes (4 GPUs each), NPS1, a
7-link xGMI full mesh at 76 GB/s per link and direction.
"""
from __future__ import annotations

import glob
import os
import re
from dataclasses import dataclass, field

from ..models.mi355x import CUS_PER_XCD, XCDS_PER_GPU, GpuInfo

KFD_LINK_XGMI = 11
KFD_LINK_PCIE = 2
_BDF = re.compile(r"^[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-7]$")


def _read(path: str, default: str = "") -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def _read_int(path: str, default: int | None = None) -> int | None:
    s = _read(path)
    try:
        return int(s, 0) if s else default
    except ValueError:
        return default


def _kv(path: str) -> dict[str, str]:
    out = {}
    for line in _read(path).splitlines():
        parts = line.split(None, 1)
        if len(parts) == 2:
            out[parts[0]] = parts[1].strip()
    return out


def parse_cpulist(s: str) -> list[int]:
    cpus: list[int] = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


@dataclass
class XgmiLink:
    peer_node: int
    bandwidth_mbps: int
    weight: int


@dataclass
class GpuDevice:
    index: int
    bdf: str
    card: str
    product: str = ""
    unique_id: str = ""
    numa: int = 0
    local_cpus: list[int] = field(default_factory=list)
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    available_compute_partitions: list[str] = field(default_factory=list)
    available_memory_partitions: list[str] = field(default_factory=list)
    vram_bytes: int = 0
    vram_used_bytes: int = 0
    busy_percent: int | None = None
    kfd_node: int | None = None
    gpu_id: int | None = None
    render_minor: int | None = None
    num_xcc: int | None = None
    simd_count: int | None = None
    gfx_target_version: int | None = None
    hive_id: int | None = None
    xgmi_links: list[XgmiLink] = field(default_factory=list)

    @property
    def cus(self) -> int:
        return (self.simd_count // 4) if self.simd_count else XCDS_PER_GPU * CUS_PER_XCD

    @property
    def hbm_gib(self) -> int:
        # The driver reserves a few MiB: 288 GiB parts report 287.98 GiB.
        return round(self.vram_bytes / (1 << 30))

    @property
    def partitions(self) -> int:
        return {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}.get(self.compute_partition.upper(), 1)

    def to_gpu_info(self) -> GpuInfo:
        mode = self.compute_partition.lower() if self.compute_partition.lower() in ("spx", "dpx", "qpx", "cpx") \
            else "spx"
        return GpuInfo(self.index, mode, hbm_gib=self.hbm_gib or 288, numa=max(self.numa, 0), cus=self.cus)


@dataclass
class HostInfo:
    cpus: int
    memory_bytes: int
    numa_nodes: list[int]
    numa_cpus: dict[int, list[int]]
    gpus: list[GpuDevice]

    @property
    def xgmi_hive(self) -> int | None:
        hives = {g.hive_id for g in self.gpus if g.hive_id}
        return hives.pop() if len(hives) == 1 else None


def _pci_from_location(domain: int, location_id: int) -> str:
    bus, devfn = (location_id >> 8) & 0xFF, location_id & 0xFF
    return f"{domain:04x}:{bus:02x}:{devfn >> 3:02x}.{devfn & 7}"


def _kfd_nodes(root: str) -> dict[str, dict]:
    """PCI address -> KFD GPU node info (readable nodes only)."""
    out = {}
    for nd in glob.glob(os.path.join(root, "sys/class/kfd/kfd/topology/nodes/*")):
        props = _kv(os.path.join(nd, "properties"))
        if not props or int(props.get("simd_count", "0")) == 0:
            continue
        node_id = int(os.path.basename(nd))
        links = []
        for lp in sorted(glob.glob(os.path.join(nd, "io_links/*/properties"))):
            lk = _kv(lp)
            if int(lk.get("type", "0")) == KFD_LINK_XGMI:
                links.append(XgmiLink(int(lk.get("node_to", "0")), int(lk.get("max_bandwidth", "0")),
                                      int(lk.get("weight", "0"))))
        bdf = _pci_from_location(int(props.get("domain", "0")), int(props.get("location_id", "0")))
        out[bdf.lower()] = {
            "kfd_node": node_id, "gpu_id": _read_int(os.path.join(nd, "gpu_id")),
            "render_minor": int(props.get("drm_render_minor", "0")) or None,
            "num_xcc": int(props.get("num_xcc", "0")) or None, "simd_count": int(props.get("simd_count", "0")),
            "gfx_target_version": int(props.get("gfx_target_version", "0")) or None,
            "hive_id": int(props.get("hive_id", "0")) or None, "xgmi_links": links,
        }
    return out


def discover_gpus(root: str = "/") -> list[GpuDevice]:
    """Physical AMD GPUs, indexed in PCI-address order (the order amd-smi and
    HIP_VISIBLE_DEVICES use on a default system)."""
    kfd = _kfd_nodes(root)
    found = []
    for card in glob.glob(os.path.join(root, "sys/class/drm/card*")):
        name = os.path.basename(card)
        if not re.fullmatch(r"card\d+", name):
            continue
        dev = os.path.join(card, "device")
        ue = dict(line.split("=", 1) for line in _read(os.path.join(dev, "uevent")).splitlines() if "=" in line)
        bdf = ue.get("PCI_SLOT_NAME", "")
        if not _BDF.match(bdf) or ue.get("DRIVER", "amdgpu") != "amdgpu":
            continue
        vendor = _read(os.path.join(dev, "vendor"), "0x1002")
        if vendor.lower() not in ("0x1002", ""):
            continue
        found.append((bdf.lower(), name, dev))
    gpus = []
    for idx, (bdf, name, dev) in enumerate(sorted(found)):
        k = kfd.get(bdf, {})
        g = GpuDevice(
            index=idx, bdf=bdf, card=name, product=_read(os.path.join(dev, "product_name")),
            unique_id=_read(os.path.join(dev, "unique_id")),
            numa=_read_int(os.path.join(dev, "numa_node"), 0) or 0,
            local_cpus=parse_cpulist(_read(os.path.join(dev, "local_cpulist"))),
            compute_partition=_read(os.path.join(dev, "current_compute_partition"), "SPX") or "SPX",
            memory_partition=_read(os.path.join(dev, "current_memory_partition"), "NPS1") or "NPS1",
            available_compute_partitions=[p.strip() for p in _read(
                os.path.join(dev, "available_compute_partitions")).split(",") if p.strip()],
            available_memory_partitions=[p.strip() for p in _read(
                os.path.join(dev, "available_memory_partition")).split(",") if p.strip()],
            vram_bytes=_read_int(os.path.join(dev, "mem_info_vram_total"), 0) or 0,
            vram_used_bytes=_read_int(os.path.join(dev, "mem_info_vram_used"), 0) or 0,
            busy_percent=_read_int(os.path.join(dev, "gpu_busy_percent")),
            **k)
        gpus.append(g)
    return gpus


def visible_gpu_count(root: str = "/", env: dict | None = None) -> int:
    """GPUs this process may use, counted from amdgpu sysfs / KFD without
    touching HIP: the physical GPUs, narrowed by the first visibility list
    that is set (ROCR_VISIBLE_DEVICES, HIP_VISIBLE_DEVICES,
    CUDA_VISIBLE_DEVICES). 0 when sysfs shows no GPU."""
    env = os.environ if env is None else env
    n = len(discover_gpus(root))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            return min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def discover_host(root: str = "/") -> HostInfo:
    gpus = discover_gpus(root)
    nodes = parse_cpulist(_read(os.path.join(root, "sys/devices/system/node/online"), "0"))
    numa_cpus = {n: parse_cpulist(_read(os.path.join(root, f"sys/devices/system/node/node{n}/cpulist")))
                 for n in nodes}
    if not any(numa_cpus.values()):
        # Not captured / unreadable: derive from the GPUs' local_cpulist.
        for g in gpus:
            numa_cpus.setdefault(g.numa, [])
            numa_cpus[g.numa] = sorted(set(numa_cpus[g.numa]) | set(g.local_cpus))
    all_cpus = sorted({c for v in numa_cpus.values() for c in v})
    ncpu = len(all_cpus) or _count_processors(root) or (os.cpu_count() or 1)
    mem_kb = 0
    for line in _read(os.path.join(root, "proc/meminfo")).splitlines():
        if line.startswith("MemTotal:"):
            mem_kb = int(line.split()[1])
    return HostInfo(cpus=ncpu, memory_bytes=mem_kb * 1024, numa_nodes=nodes or [0], numa_cpus=numa_cpus, gpus=gpus)


def _count_processors(root: str) -> int:
    return sum(1 for line in _read(os.path.join(root, "proc/cpuinfo")).splitlines() if line.startswith("processor"))


def fake_host(n_gpus: int = 8, mode: str = "SPX", sockets: int = 2, cpus: int = 256,
              memory_gib: int = 3072) -> HostInfo:
    """A synthetic MI355X host for tests and dry runs (no sysfs)."""
    per = max(1, n_gpus // sockets)
    gpus = []
    for i in range(n_gpus):
        numa = min(sockets - 1, i // per)
        gpus.append(GpuDevice(index=i, bdf=f"0000:{0x10 + i * 0x10:02x}:00.0", card=f"card{i * 8}",
                              product="AMD Instinct MI355 OAM", numa=numa, compute_partition=mode,
                              vram_bytes=288 << 30, num_xcc=8, simd_count=1024, hive_id=1,
                              xgmi_links=[XgmiLink(j, 76000, 15) for j in range(n_gpus) if j != i]))
    cpn = cpus // sockets
    return HostInfo(cpus=cpus, memory_bytes=memory_gib << 30, numa_nodes=list(range(sockets)),
                    numa_cpus={s: list(range(s * cpn, (s + 1) * cpn)) for s in range(sockets)}, gpus=gpus)
