"""Summarise `scripts/pmc_round.sh` output into a markdown table.

    python -m flex_gpu_scheduler_amd.tools.pmc_summary gpurun_out/r3a > profiles/r3a_pmc_probe_summary.md

For every counter pass (`pmc_<name>/pmc_counter_collection.csv` plus the
probe's own JSON line in `pmc_<name>.log`) it lists, per kernel, the number
of dispatches and the counters per dispatch, and derives the HBM traffic:
FETCH_SIZE and WRITE_SIZE are in KiB, so bytes per dispatch against the
bytes the kernel must move tells whether it over-fetches, and the probe's
timing turns the bytes into GB/s and % of the 8 TB/s HBM3E peak.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

HBM_PEAK_GBPS = 8000.0


def _short(kernel: str) -> str:
    m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", kernel)
    return m.group(1) if m else kernel.split("(")[0][-60:]


def _probe_line(log: str) -> dict:
    try:
        with open(log) as f:
            for line in f:
                if line.startswith("{"):
                    return json.loads(line)
    except OSError:
        pass
    return {}


def summarize(root: str) -> str:
    rows = []
    for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        name = os.path.basename(d)[4:]
        csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not csvs:
            continue
        per: dict[str, dict] = defaultdict(lambda: {"dispatches": {}, "counters": defaultdict(float)})
        with open(csvs[0]) as f:
            for r in csv.DictReader(f):
                k = _short(r["Kernel_Name"])
                per[k]["dispatches"][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                per[k]["counters"][r["Counter_Name"]] += float(r["Counter_Value"])
        probe = _probe_line(os.path.join(root, f"pmc_{name}.log"))
        for k, v in per.items():
            nd = len(v["dispatches"])
            cnt = {c: val / nd for c, val in v["counters"].items()}
            ns = sum(v["dispatches"].values()) / nd
            rows.append((name, k, nd, cnt, ns, probe))
    out = ["| pass | kernel | dispatches | counters per dispatch | HBM bytes per dispatch | counter GB/s "
           "(bytes / dispatch time) | probe-reported |",
           "|---|---|---|---|---|---|---|"]
    for name, k, nd, cnt, ns, probe in rows:
        if k.startswith("__amd_rocclr"):
            continue  # runtime fills/copies around the probe
        cs = ", ".join(f"{c}={v:,.0f}" for c, v in sorted(cnt.items()))
        moved, nbytes = [], 0.0
        if "FETCH_SIZE" in cnt:
            # gfx950 counts 64 B per 128-B read request in FETCH_SIZE: every
            # streaming read reports exactly half its bytes (r1f and r3
            # passes), so the read traffic is 2 x FETCH_SIZE.
            nbytes += 2 * cnt["FETCH_SIZE"] * 1024
            moved.append(f"read {2 * cnt['FETCH_SIZE'] * 1024 / 2**30:.3f} GiB (2 x FETCH_SIZE)")
        if "WRITE_SIZE" in cnt:
            nbytes += cnt["WRITE_SIZE"] * 1024
            moved.append(f"written {cnt['WRITE_SIZE'] * 1024 / 2**30:.3f} GiB")
        cgb = f"{nbytes / ns:,.0f}" if nbytes and ns > 0 and nbytes > (1 << 20) else ""
        pr = ""
        # The probe's line belongs to the measured kernel, not the buffer fill.
        if probe and "k_write<4, true>" not in k:
            gbps = probe.get("GBps") or 0
            pr = f"{gbps:,.0f} GB/s = {100 * gbps / HBM_PEAK_GBPS:.1f}% of 8 TB/s" if gbps else \
                json.dumps(probe)
        out.append(f"| {name} | `{k}` | {nd} | {cs} | {'; '.join(moved)} | {cgb} | {pr} |")
    return "\n".join(out) + "\n"


def main() -> int:
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    sys.stdout.write(summarize(root))
    return 0


if __name__ == "__main__":
    sys.exit(main())
