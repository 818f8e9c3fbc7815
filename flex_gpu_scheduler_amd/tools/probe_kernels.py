"""Run one HIP probe kernel family in isolation (for rocprofv3 --pmc passes).

    python -m flex_gpu_scheduler_amd.tools.probe_kernels PROBE [device] [iters]

    PROBE: mfma | hbm-read | hbm-copy | hbm-triad | hbm-write
           | xcd-read-K | xcd-copy-K   (k_pinned on the first K XCDs: K=1 is
             one CPX partition's CUs, 2 QPX, 4 DPX, 8 the whole GPU)
           | partitions                (the node agent's per-partition table)
           | seg-{read,write}[-nt]-SEG  (k_segments: 2^18 segments of SEG bytes,
             one per 4 KiB, for counter calibration)

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
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    pr = probe()
    if what == "mfma":
        r = pr.mfma_peak(dev, 0xFF, iters=8192)
        flops = r["tflops"] * 1e12 * r["ms"] * 1e-3  # per dispatch: every dispatch runs the same tile loop
        out = {"kernel": "k_mfma_peak", "TFLOPs": round(r["tflops"], 1), "ms": round(r["ms"], 3),
               "flops_per_dispatch": round(flops), "mfma_insts_per_dispatch": round(flops / (2 * 32 * 32 * 16))}
    elif what in ("hbm-read", "hbm-copy", "hbm-triad", "hbm-write"):
        mode = what.split("-")[1]
        bw = pr.hbm_bandwidth(dev, 2 << 30, iters=iters, mode=mode)
        arrays = {"read": 1, "write": 1, "copy": 2, "triad": 3}[mode]
        reads, writes = {"read": (1, 0), "write": (0, 1), "copy": (1, 1), "triad": (2, 1)}[mode]
        out = {"kernel": what, "iters": iters, "bytes_per_array": 2 << 30, "arrays": arrays,
               "read_bytes": reads * (2 << 30), "write_bytes": writes * (2 << 30),
               "GBps": round(bw.gbps, 1), "ms": round(bw.ms_per_iter, 4), "best_GBps": round(bw.best_gbps, 1),
               "batch_GBps": round(bw.batch_gbps, 1), "pct_of_8TBps": round(bw.gbps / 80.0, 1)}
    elif what.startswith("xcd-"):
        _, mode, k = what.split("-")
        mask = (1 << int(k)) - 1
        bw = pr.hbm_bandwidth_xcd(dev, mask, 1 << 30, iters=iters, mode=mode)
        out = {"kernel": f"k_pinned[{mode}]", "iters": iters, "xcds": int(k), "xcd_mask": mask, "bytes": 1 << 30,
               "read_bytes": 1 << 30, "write_bytes": (1 << 30) if mode == "copy" else 0,
               "GBps": round(bw.gbps, 1), "ms": round(bw.ms_per_iter, 4), "best_GBps": round(bw.best_gbps, 1),
               "batch_GBps": round(bw.batch_gbps, 1), "pct_of_8TBps": round(bw.gbps / 80.0, 1)}
    elif what.startswith("seg-"):
        parts = what.split("-")
        out = pr.segment_access(dev, parts[1], int(parts[-1]), 4096, 1 << 18, iters, nontemporal="nt" in parts)
    elif what == "partitions":
        out = pr.partition_table(dev, 1 << 30, iters)
    else:
        raise SystemExit(f"unknown probe {what!r}")
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
