"""HBM / partition bandwidth sweep with the HIP probe (for rocprofv3 runs).

Prints one JSON line: device props, XCD census, and GB/s for read / write /
copy / triad at full-device and partition-sized (32-CU, one XCD) budgets.
"""
from __future__ import annotations

import json
import sys

from ..ops.hip_probe import probe


def main() -> int:
    dev = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    pr = probe()
    out = {"props": pr.props(dev), "census": pr.xcd_census(dev, 4096), "health": pr.health(dev, 256 << 20)}
    sweep = []
    for cu in (0, 128, 64, 32):
        for mode in ("read", "write", "copy", "triad"):
            bw = pr.hbm_bandwidth(dev, 2 << 30, iters=20, cu_limit=cu, mode=mode)
            sweep.append({"cu_limit": cu or out["props"]["computeUnits"], "mode": mode, "GBps": round(bw.gbps, 1),
                          "ms": round(bw.ms_per_iter, 4)})
    out["bandwidth"] = sweep
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
