"""One-shot node-agent run on a real box: discover the MI355X host from sysfs,
run the HIP health probe on the visible GPU(s), publish Node + NRT +
WatcherMetrics into an in-process store and print what a scheduler would see.

    python -m flex_gpu_scheduler_amd.tools.agent_check > gpurun_out/agent_check.json
"""
from __future__ import annotations

import json
import socket
import sys
import time


def main() -> int:
    from .. import Store
    from ..control.client import LocalClient
    from ..control.node_agent import NodeAgent, hip_health_fn

    store = Store()
    health = None
    try:
        health = hip_health_fn()
    except Exception as e:  # noqa: BLE001 - no HIP probe on this host
        print(f"# health probe unavailable: {e}", file=sys.stderr)
    agent = NodeAgent(LocalClient(store), socket.gethostname(), health_fn=health)
    t0 = time.perf_counter()
    host = agent.sync()
    sync_s = time.perf_counter() - t0
    agent.sample_and_publish()
    time.sleep(1.0)
    doc = agent.sample_and_publish()
    node = store.get("nodes", "", agent.name)
    out = {
        "gpus": [{"index": g.index, "bdf": g.bdf, "numa": g.numa, "partition": g.compute_partition,
                  "memory_partition": g.memory_partition, "hbm_gib": g.hbm_gib, "busy": g.busy_percent,
                  "kfd_node": g.kfd_node, "cus": g.cus, "xgmi_links": len(g.xgmi_links)} for g in host.gpus],
        "cpus": host.cpus, "numa_nodes": host.numa_nodes, "unhealthy": sorted(agent.unhealthy),
        "allocatable": node["status"]["allocatable"], "labels": node["metadata"]["labels"],
        "nrt_zones": [z["name"] for z in store.get("noderesourcetopologies", "", agent.name)["zones"]],
        "metrics": doc["data"]["NodeMetricsMap"][agent.name]["metrics"], "sync_seconds": round(sync_s, 4),
    }
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
