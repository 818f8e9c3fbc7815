"""HBM / partition bandwidth sweep with the HIP probe (for rocprofv3 runs).

Prints one JSON line: device props, XCD census, health, the streaming-kernel
tuning sweep (unroll x cache policy x workgroups/CU) per mode, and the
bandwidth a CPX/QPX/DPX-sized partition (1/2/4 XCDs) can pull.
"""
from __future__ import annotations

import json
import sys

from ..ops.hip_probe import probe


def main() -> int:
    dev = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    pr = probe()
    out = {"props": pr.props(dev), "census": pr.xcd_census(dev, 4096), "health": pr.health(dev, 256 << 20)}
    out["tuning"] = {m: pr.tune(dev, m, 2 << 30, 10) for m in ("read", "write", "copy", "triad")}
    parts = []
    for label, mask in (("cpx-1xcd", 0x01), ("qpx-2xcd", 0x03), ("dpx-4xcd", 0x0F), ("spx-8xcd", 0xFF)):
        for mode in ("read", "write", "copy"):
            bw = pr.hbm_bandwidth_xcd(dev, mask, 2 << 30, 10, mode)
            parts.append({"partition": label, "mode": mode, "GBps": round(bw.gbps, 1), "ms": round(bw.ms_per_iter, 4)})
    out["partitions"] = parts
    out["mfma_check"] = pr.mfma_check(dev, 256)
    out["mfma_bf16"] = []
    for label, mask in (("cpx-1xcd", 0x01), ("qpx-2xcd", 0x03), ("dpx-4xcd", 0x0F), ("spx-8xcd", 0xFF)):
        r = pr.mfma_peak(dev, mask, iters=8192)
        out["mfma_bf16"].append({"partition": label, "TFLOPs": round(r["tflops"], 1), "ms": round(r["ms"], 3),
                                 "active_blocks": r["active_blocks"]})
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
