"""Checks that the amd-smi telemetry provider sees load on this host's
MI355X: samples idle, then while a device-to-device copy loop keeps HBM busy
(torch on cuda:0), and prints per-phase maxima of GFX / HBM-controller
activity, power and xGMI traffic as one JSON line.

    python -m flex_gpu_scheduler_amd.tools.amdsmi_probe [--seconds 2]
"""
from __future__ import annotations

import argparse
import json
import threading
import time


def sample_while(sampler, stop: threading.Event, period: float, out: list) -> None:
    while not stop.is_set():
        out.append(sampler.sample())
        time.sleep(period)


def summarize(frames: list) -> dict:
    if not frames:
        return {}
    n = len(frames[0])
    res = {}
    for key in ("gfx", "umc", "power_w", "xgmi_gbps", "vram_used_pct"):
        vals = [getattr(f[i], key) for f in frames for i in range(min(n, len(f)))]
        vals = [v for v in vals if v is not None]
        res[f"max_{key}"] = round(max(vals), 2) if vals else None
    return res


def run(seconds: float = 2.0, period: float = 0.05) -> dict:
    from ..gpu.amdsmi import AmdSmiSampler, native_status

    ok, err = native_status()
    if not ok:
        return {"available": False, "error": err}
    smi = AmdSmiSampler()
    first = smi.sample()
    out = {"available": True, "gpus": len(first),
           "gpu0": {"bdf": first[0].bdf, "links_up": first[0].links_up, "xcc": len(first[0].xcc_busy)} if first else None}
    idle: list = []
    stop = threading.Event()
    th = threading.Thread(target=sample_while, args=(smi, stop, period, idle))
    th.start()
    time.sleep(min(1.0, seconds / 2))
    stop.set()
    th.join()
    out["idle"] = summarize(idle)
    try:
        import torch
    except ImportError:
        return out
    if not torch.cuda.is_available():
        return out
    x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")  # 1 GiB
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    busy: list = []
    stop = threading.Event()
    th = threading.Thread(target=sample_while, args=(smi, stop, period, busy))
    th.start()
    t0 = time.perf_counter()
    copies = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            y.copy_(x)
        torch.cuda.synchronize()
        copies += 8
    dt = time.perf_counter() - t0
    stop.set()
    th.join()
    out["load"] = summarize(busy)
    out["load"]["copy_GBps"] = round(2 * copies * x.numel() / dt / 1e9, 1)  # read + write
    out["samples"] = {"idle": len(idle), "load": len(busy)}
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    print(json.dumps(run(a.seconds)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
