"""TargetLoadPacking on live MI355X load (the GPU tier's Trimaran check).

Two node agents' telemetry come from this host's real GPU through amd-smi
(csrc/telemetry/amdsmi_sampler.cc): "mi355x-idle" is sampled while the GPU is
idle, "mi355x-busy" while a device copy loop keeps it busy. Both publish
load-watcher documents (gpu/telemetry.py, the reference's WatcherMetrics,
vendor/github.com/paypal/load-watcher/pkg/watcher/watcher.go:63-101) into a
store; a scheduler scoring with TargetLoadPacking in GPU mode
(pkg/trimaran/targetloadpacking/targetloadpacking.go) explains a one-GPU pod,
then schedules it. Prints one JSON line: both nodes' GPU busy means, their
TLP scores, the node explain() predicts and the node the pod was bound to.

    python -m flex_gpu_scheduler_amd.tools.tlp_live [--seconds 2]
"""
from __future__ import annotations

import argparse
import json
import threading
import time

IDLE, BUSY = "mi355x-idle", "mi355x-busy"


def tlp_config() -> dict:
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta3", "kind": "KubeSchedulerConfiguration",
            "profiles": [{"schedulerName": "default-scheduler",
                          "plugins": {"filter": {"enabled": [{"name": "FlexGPU"}]},
                                      "score": {"enabled": [{"name": "TargetLoadPacking"}], "disabled": [{"name": "*"}]},
                                      "reserve": {"enabled": [{"name": "FlexGPU"}]}},
                          "pluginConfig": [{"name": "TargetLoadPacking",
                                            "args": {"resourceType": "GPU", "targetUtilization": 40}}]}]}


def sample_for(tel, seconds: float, period: float) -> int:
    n, t_end = 0, time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        tel.sample()
        n += 1
        time.sleep(period)
    return n


def copy_loop_load(device: int = 0):
    """Keeps cuda:`device` busy with 1 GiB device copies until the returned
    stop()."""
    import torch

    x = torch.empty(1 << 30, dtype=torch.uint8, device=f"cuda:{device}")
    y = torch.empty_like(x)
    stop = threading.Event()

    def loop():
        while not stop.is_set():
            for _ in range(8):
                y.copy_(x)
            torch.cuda.synchronize(device)

    th = threading.Thread(target=loop, daemon=True)
    th.start()

    def end():
        stop.set()
        th.join(timeout=30)
    return end


def run(seconds: float = 2.0, period: float = 0.05, *, sampler=None, start_load=copy_loop_load) -> dict:
    """`sampler` / `start_load` default to amd-smi and a torch copy loop on
    cuda:0; the CPU tests inject stand-ins."""
    from .. import load_config, new_scheduler
    from ..gpu.telemetry import HostSampler, NodeTelemetry
    from ..models import GPU, make_pod, mi355x_node
    from ..scheduler import Store

    hs = sampler if sampler is not None else HostSampler(gpu_source="amdsmi")
    idle, busy = NodeTelemetry(IDLE, hs), NodeTelemetry(BUSY, hs)
    n_idle = sample_for(idle, min(1.0, seconds / 2), period)
    end_load = start_load()
    try:
        time.sleep(0.3)  # let the activity counters ramp
        n_busy = sample_for(busy, seconds, period)
    finally:
        end_load()

    def gpu_avg(tel):
        m = [d for d in tel.metrics() if d["type"] == "GPU" and d["operator"] == "AVG"]
        return m[0]["value"] if m else None

    store = Store()
    for n in (IDLE, BUSY):
        store.create("nodes", json.dumps(mi355x_node(n)))
    s = new_scheduler(store, load_config(tlp_config()))
    s.start()
    try:
        for tel in (idle, busy):
            store.create("loadwatchermetrics", json.dumps(tel.watcher_metrics()))
        pod = make_pod("first-gpu-pod", limits={GPU: "1"})
        s.sync_informers(50)
        ex = s.explain(pod)
        scores = {n: v.get("TargetLoadPacking*1") for n, v in (ex.get("scores") or {}).items()}
        store.create("pods", json.dumps(pod))
        deadline = time.time() + 10
        landed = ""
        while time.time() < deadline and not landed:
            landed = (store.get("pods", "default", "first-gpu-pod") or {}).get("spec", {}).get("nodeName", "")
            time.sleep(0.01)
    finally:
        s.stop()
    return {"gpu_source": getattr(hs, "gpu_source", "injected"), "samples": {"idle": n_idle, "busy": n_busy},
            "gpu_busy_avg": {IDLE: gpu_avg(idle), BUSY: gpu_avg(busy)}, "tlp_scores": scores,
            "predicted": ex.get("selected") or ex.get("node"), "landed": landed}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    print(json.dumps(run(a.seconds)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
