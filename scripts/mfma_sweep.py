"""Sweep the dense bf16 MFMA probe over launch size and run length.

Tells a latency-bound probe (TFLOP/s grows with waves per SIMD) from a
clock/power-bound one (flat across launch sizes, falling with run length).
Prints one JSON line per point. Usage: python scripts/mfma_sweep.py [out.jsonl]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flex_gpu_scheduler_amd.ops.hip_probe import probe  # noqa: E402


def main() -> int:
    p = probe()
    props = p.props(0)
    cus = int(props.get("computeUnits", 256))
    print(json.dumps({"clockRateKHz": props.get("clockRateKHz"), "computeUnits": cus}), flush=True)
    rows = []
    for per_cu in (1, 2, 4, 8):
        for iters in (4096, 16384, 65536):
            r = p.mfma_peak(0, 0xFF, iters=iters, blocks=per_cu * cus)
            # A 32x32x16 bf16 MFMA issues every 32 cycles per SIMD at peak (1024
            # flop/clk/SIMD): the clock at which this rate would be issue-bound.
            r.update(blocks_per_cu=per_cu, iters=iters,
                     issue_bound_ghz=round(r["tflops"] * 1e3 / (cus * 4 * 1024), 3))
            rows.append(r)
            print(json.dumps(r), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
