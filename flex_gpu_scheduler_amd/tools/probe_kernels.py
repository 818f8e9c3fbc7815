"""Run one HIP probe kernel family in isolation (for rocprofv3 --pmc passes).

    python -m flex_gpu_scheduler_amd.tools.probe_kernels mfma|hbm-read|hbm-copy [device]

Prints the probe's own measurement as one JSON line, so a counter pass can be
cross-checked against the timing the probe reports.
"""
from __future__ import annotations

import json
import sys

from ..ops.hip_probe import probe


def main() -> int:
    what = sys.argv[1] if len(sys.argv) > 1 else "mfma"
    dev = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    pr = probe()
    if what == "mfma":
        r = pr.mfma_peak(dev, 0xFF, iters=8192)
        out = {"kernel": "k_mfma_peak", "TFLOPs": round(r["tflops"], 1), "ms": round(r["ms"], 3)}
    elif what in ("hbm-read", "hbm-copy"):
        bw = pr.hbm_bandwidth(dev, 2 << 30, iters=5, mode=what.split("-")[1])
        out = {"kernel": what, "bytes": 2 << 30, "GBps": round(bw.gbps, 1), "ms": round(bw.ms_per_iter, 4)}
    else:
        raise SystemExit(f"unknown probe {what!r}")
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
