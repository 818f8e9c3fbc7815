"""Live MI355X counters through the native amd-smi sampler
(csrc/telemetry/amdsmi_sampler.cc, libamd_smi loaded with dlopen).

`AmdSmiSampler.sample()` returns one `GpuCounters` per GPU with the rates the
load-watcher provider publishes (gpu/telemetry.py):

* `gfx` — GFX engine activity % (what `gpu_busy_percent` reports in sysfs);
* `umc` — memory-controller (HBM3E) activity %, the bandwidth-pressure signal
  sysfs does not expose;
* `vram_used_pct` — VRAM used / total;
* `xgmi_gbps` — xGMI traffic (read + write, all links) from the firmware's
  per-link data accumulators differenced between two samples, and
  `xgmi_pct` — that traffic over the capacity of the links that are up
  (`XGMI_LINK_GBPS` per direction per link);
* `power_w`, `hotspot_c`, per-XCC busy %.

The reference's Trimaran consumes load-watcher's CPU/Memory metrics from
metrics-server / Prometheus / SignalFx
(vendor/github.com/paypal/load-watcher/pkg/watcher/watcher.go:116-160);
these GPU counters are the MI355X-side replacement for DCGM.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

# One xGMI link of an MI355X carries ~76.8 GB/s per direction (the KFD
# io_links of the captured 8x MI355X host report 76 GB/s per direction;
# 7 links x 2 directions x 76.8 = 1075 GB/s aggregate).
XGMI_LINK_GBPS = 76.8


@dataclass
class GpuCounters:
    index: int
    bdf: str
    gfx: float | None
    umc: float | None
    vram_used_pct: float | None
    xgmi_gbps: float | None
    xgmi_pct: float | None
    power_w: float | None
    hotspot_c: float | None
    xcc_busy: list[float] = field(default_factory=list)
    links_up: int = 0


def _pct(x: float) -> float | None:
    return None if x is None or x < 0 else float(x)


def native_status() -> tuple[bool, str]:
    try:
        from .._native import native
    except Exception as e:  # noqa: BLE001 - extension not built
        return False, f"native core unavailable: {e}"
    ok, err = native().amdsmi_status()
    return bool(ok), str(err)


class AmdSmiSampler:
    """Stateful: keeps the previous accumulators to turn them into rates."""

    def __init__(self, reader=None, clock=time.monotonic):
        if reader is None:
            from .._native import native
            reader = native().amdsmi_sample
        self._read = reader
        self._clock = clock
        self._prev: dict[int, tuple[float, int]] = {}

    def sample(self) -> list[GpuCounters]:
        now = self._clock()
        out = []
        for d in self._read():
            idx = int(d["index"])
            up = [u for u in d.get("xgmi_link_up", []) if u == 1]
            acc_kb = sum(int(x) for x in d.get("xgmi_read_kb", [])) + sum(int(x) for x in d.get("xgmi_write_kb", []))
            gbps = pct = None
            prev = self._prev.get(idx)
            if prev is not None and now > prev[0] and acc_kb >= prev[1]:
                gbps = (acc_kb - prev[1]) * 1024.0 / (now - prev[0]) / 1e9
                if up:
                    pct = min(100.0, 100.0 * gbps / (len(up) * 2 * XGMI_LINK_GBPS))
            self._prev[idx] = (now, acc_kb)
            tot, used = int(d.get("vram_total_mb", -1)), int(d.get("vram_used_mb", -1))
            out.append(GpuCounters(
                index=idx, bdf=str(d.get("bdf", "")), gfx=_pct(d.get("gfx_activity")), umc=_pct(d.get("umc_activity")),
                vram_used_pct=100.0 * used / tot if tot > 0 and used >= 0 else None, xgmi_gbps=gbps, xgmi_pct=pct,
                power_w=_pct(d.get("socket_power_w")), hotspot_c=_pct(d.get("temp_hotspot_c")),
                xcc_busy=[float(x) for x in d.get("xcc_busy", [])], links_up=len(up)))
        return out
