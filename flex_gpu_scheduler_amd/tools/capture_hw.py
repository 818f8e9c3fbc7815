"""Capture the GPU-relevant sysfs tree and SMI tool output of an MI355X box.

The node agent (gpu/discovery.py) reads KFD topology and DRM device
attributes; CPU-side tests replay a capture taken on a real box through
gpurun, so discovery is tested against real MI355X sysfs rather than guesses.

    python -m flex_gpu_scheduler_amd.tools.capture_hw gpurun_out/hwcapture
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import subprocess
import sys

KFD_FILES = ("properties", "gpu_id", "name")
DRM_ATTRS = ("current_compute_partition", "available_compute_partitions", "current_memory_partition",
             "available_memory_partition", "numa_node", "gpu_busy_percent", "mem_info_vram_total",
             "mem_info_vram_used", "mem_info_vis_vram_total", "unique_id", "product_name", "product_number",
             "vendor", "device", "revision", "uevent", "mem_busy_percent", "local_cpulist", "power_dpm_force_performance_level",
             "pp_dpm_sclk", "pp_dpm_mclk", "serial_number")


def _copy(src: str, dst_root: str) -> bool:
    try:
        with open(src, "rb") as f:
            data = f.read(1 << 20)
    except OSError:
        return False
    dst = os.path.join(dst_root, src.lstrip("/"))
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "wb") as f:
        f.write(data)
    return True


def capture_sysfs(out: str, root: str = "/") -> dict:
    n = 0
    topo = os.path.join(root, "sys/class/kfd/kfd/topology")
    for node in sorted(glob.glob(os.path.join(topo, "nodes", "*"))):
        for f in KFD_FILES:
            n += _copy(os.path.join(node, f), out)
        for sub in ("mem_banks", "io_links", "p2p_links"):
            for p in glob.glob(os.path.join(node, sub, "*", "properties")):
                n += _copy(p, out)
    n += _copy(os.path.join(topo, "system_properties"), out)
    n += _copy(os.path.join(topo, "generation_id"), out)
    links = {}
    for card in sorted(glob.glob(os.path.join(root, "sys/class/drm/card*"))):
        dev = os.path.join(card, "device")
        if not os.path.isdir(dev):
            continue
        try:
            links[os.path.basename(card)] = os.path.basename(os.path.realpath(dev))
        except OSError:
            pass
        for a in DRM_ATTRS:
            n += _copy(os.path.join(dev, a), out)
    for rd in sorted(glob.glob(os.path.join(root, "sys/class/drm/renderD*"))):
        try:
            links[os.path.basename(rd)] = os.path.basename(os.path.realpath(os.path.join(rd, "device")))
        except OSError:
            pass
    with open(os.path.join(out, "drm_links.json"), "w") as f:
        json.dump(links, f, indent=1, sort_keys=True)
    for p in ("proc/cpuinfo", "proc/meminfo", "sys/devices/system/node/online"):
        n += _copy(os.path.join(root, p), out)
    for p in glob.glob(os.path.join(root, "sys/devices/system/node/node*/cpulist")):
        n += _copy(p, out)
    return {"files": n, "drm_links": links}


SMI_COMMANDS = {
    "amd-smi_static.json": ["amd-smi", "static", "--json"],
    "amd-smi_partition.json": ["amd-smi", "partition", "--json"],
    "amd-smi_metric.json": ["amd-smi", "metric", "--json"],
    "amd-smi_topology.json": ["amd-smi", "topology", "--json"],
    "amd-smi_list.json": ["amd-smi", "list", "--json"],
    "rocm-smi_showall.json": ["rocm-smi", "--showuse", "--showmemuse", "--showmeminfo", "vram", "--json"],
    "rocm-smi_topo.json": ["rocm-smi", "--showtopo", "--json"],
    "rocminfo.txt": ["rocminfo"],
}


def capture_smi(out: str, timeout: float = 60.0) -> dict:
    res = {}
    os.makedirs(os.path.join(out, "smi"), exist_ok=True)
    for fname, cmd in SMI_COMMANDS.items():
        if shutil.which(cmd[0]) is None and not os.path.exists(f"/opt/rocm/bin/{cmd[0]}"):
            res[fname] = "missing"
            continue
        exe = shutil.which(cmd[0]) or f"/opt/rocm/bin/{cmd[0]}"
        try:
            p = subprocess.run([exe] + cmd[1:], capture_output=True, text=True, timeout=timeout)
            with open(os.path.join(out, "smi", fname), "w") as f:
                f.write(p.stdout)
            if p.stderr:
                with open(os.path.join(out, "smi", fname + ".stderr"), "w") as f:
                    f.write(p.stderr[-20000:])
            res[fname] = p.returncode
        except subprocess.TimeoutExpired:
            res[fname] = "timeout"
    return res


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    out = argv[0] if argv else "gpurun_out/hwcapture"
    os.makedirs(out, exist_ok=True)
    summary = {"sysfs": capture_sysfs(os.path.join(out, "root")), "smi": capture_smi(out)}
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
