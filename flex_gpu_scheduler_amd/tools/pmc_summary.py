"""Summarise `scripts/pmc_round.sh` output into markdown tables.

    python -m flex_gpu_scheduler_amd.tools.pmc_summary gpurun_out/r4d > profiles/r4d_pmc_probe_summary.md

Every streaming probe ran in two counter passes, FETCH_SIZE and WRITE_SIZE
(`pmc_<probe>_fetch`, `pmc_<probe>_write`; one pass for read-only probes),
each with --kernel-trace and the probe's own JSON line in `pmc_<name>.log`.
Per probe the table gives:

* the bytes the counters saw per dispatch against the bytes the kernel must
  move (the probe's read_bytes / write_bytes): FETCH_SIZE and WRITE_SIZE are
  in KiB, and gfx950 counts 64 B per 128-B read request in FETCH_SIZE, so the
  read traffic is 2 x FETCH_SIZE;
* the median dispatch time of the measured kernel, from a --kernel-trace
  only run when scripts/probe_timing.sh left one (`trace_<probe>`), else from
  the counter passes, and the GB/s it implies for the counted bytes
  ("counter GB/s");
* the probe's own figure: the median of its per-launch event pairs, from a
  plain run when there is one (`plain_<probe>.log`), else from the passes;
* the difference between the two (the probe must agree within 5 %).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import statistics
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


def _pass(d: str) -> dict[str, dict]:
    """kernel -> {"ns": [dispatch ns...], "counters": {name: per-dispatch mean}}."""
    csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not csvs:
        return {}
    per: dict[str, dict] = defaultdict(lambda: {"disp": {}, "sum": defaultdict(float)})
    with open(csvs[0]) as f:
        for r in csv.DictReader(f):
            k = _short(r["Kernel_Name"])
            per[k]["disp"][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per[k]["sum"][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, v in per.items():
        nd = len(v["disp"])
        out[k] = {"ns": sorted(v["disp"].values()), "counters": {c: s / nd for c, s in v["sum"].items()}}
    return out


def _trace(d: str) -> dict[str, dict]:
    """kernel -> {"ns": [dispatch ns...]} from a --kernel-trace-only run."""
    csvs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not csvs:
        return {}
    out: dict[str, dict] = defaultdict(lambda: {"ns": [], "counters": {}})
    with open(csvs[0]) as f:
        for r in csv.DictReader(f):
            out[_short(r["Kernel_Name"])]["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return dict(out)


def _measured_kernel(kernels: dict[str, dict], probe: dict) -> str | None:
    """The probe's kernel in a pass: not the runtime's fills, not the warm-up
    write of the buffers (k_write<4, true>) unless the probe is a write."""
    want = "k_pinned" if str(probe.get("kernel", "")).startswith("k_pinned") else None
    best = None
    for k, v in kernels.items():
        if k.startswith("__amd_rocclr"):
            continue
        if want and not k.startswith(want):
            continue
        if not want and k == "k_write<4, true>" and probe.get("kernel") != "hbm-write":
            continue
        if best is None or len(v["ns"]) > len(kernels[best]["ns"]):
            best = k
    return best


def summarize(root: str) -> str:
    passes: dict[str, dict[str, str]] = defaultdict(dict)  # probe -> {"fetch"|"write"|"": dir}
    for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        name = os.path.basename(d)[4:]
        m = re.match(r"(.+)_(fetch|write)$", name)
        probe, kind = (m.group(1), m.group(2)) if m else (name, "")
        passes[probe][kind] = d
    lines = ["| probe | kernel | bytes to move per dispatch | counted per dispatch | median dispatch | "
             "counter GB/s | probe GB/s (median launch) | probe vs counter | timing from |",
             "|---|---|---|---|---|---|---|---|---|"]
    other = []
    for probe, kinds in sorted(passes.items()):
        ns_all: list[int] = []
        read_b = write_b = None
        kernel = None
        pj: dict = {}
        for kind, d in sorted(kinds.items()):
            kern = _pass(d)
            pj = _probe_line(d + ".log") or pj
            k = _measured_kernel(kern, pj)
            if k is None:
                continue
            kernel = k
            ns_all += kern[k]["ns"][1:] if len(kern[k]["ns"]) > 2 else kern[k]["ns"]  # first: cold
            c = kern[k]["counters"]
            if "FETCH_SIZE" in c:
                read_b = 2 * c["FETCH_SIZE"] * 1024
            if "WRITE_SIZE" in c:
                write_b = c["WRITE_SIZE"] * 1024
            if not ("FETCH_SIZE" in c or "WRITE_SIZE" in c):
                other.append(f"| {probe} | `{k}` | " + ", ".join(f"{n}={v:,.0f}" for n, v in sorted(c.items())) +
                             f" | {json.dumps(pj)} |")
        if kernel is None or "read_bytes" not in pj:
            continue
        want_r, want_w = pj["read_bytes"], pj["write_bytes"]
        counted = (read_b or 0) + (write_b or 0)
        # Timing from the counter-free runs when present (scripts/probe_timing.sh):
        # counter collection serializes dispatches and stretches the probe's
        # own event timing, so the comparison is made without it.
        timing = "pmc pass"
        tdir = os.path.join(root, f"trace_{probe}")
        plain = _probe_line(os.path.join(root, f"plain_{probe}.log"))
        if os.path.isdir(tdir):
            tr = _trace(tdir)
            k = _measured_kernel(tr, pj)
            if k is not None and tr[k]["ns"]:
                ns_all = tr[k]["ns"][1:] if len(tr[k]["ns"]) > 2 else tr[k]["ns"]
                timing = "kernel trace"
        if plain.get("GBps"):
            pj = plain
            timing += ", plain probe"
        med = statistics.median(ns_all) if ns_all else 0
        cgb = counted / med if med else 0.0
        pgb = float(pj.get("GBps") or 0)
        diff = f"{100 * (pgb - cgb) / cgb:+.1f}%" if cgb else ""
        lines.append(
            f"| {probe} | `{kernel}` | read {want_r / 2**30:.2f} GiB, write {want_w / 2**30:.2f} GiB | "
            f"read {0 if read_b is None else read_b / 2**30:.3f} GiB, "
            f"write {0 if write_b is None else write_b / 2**30:.3f} GiB | {med / 1e3:,.1f} us | {cgb:,.0f} | "
            f"{pgb:,.0f} ({100 * pgb / HBM_PEAK_GBPS:.1f}% of 8 TB/s) | {diff} | {timing} |")
    out = "\n".join(lines) + "\n"
    if other:
        out += "\n| pass | kernel | counters per dispatch | probe |\n|---|---|---|---|\n" + "\n".join(other) + "\n"
    return out


def _calib_pass(root: str, name: str, prefix: str | None = None, with_ns: bool = False):
    """(per-dispatch counters of the measured kernel, probe JSON line) of one
    calibration pass `pmc_<name>`; `prefix` selects the kernel by name. With
    `with_ns`, also the kernel's dispatch durations (ns)."""
    d = os.path.join(root, f"pmc_{name}")
    kern = _pass(d)
    pj = _probe_line(d + ".log")
    if prefix:
        ks = [k for k in kern if k.startswith(prefix)]
        k = max(ks, key=lambda x: len(kern[x]["ns"])) if ks else None
    else:
        k = _measured_kernel(kern, pj)
    if with_ns:
        return (kern[k]["counters"] if k else {}), pj, (kern[k]["ns"] if k else [])
    return (kern[k]["counters"] if k else {}), pj


def calibration(root: str) -> str:
    """scripts/pmc_calibrate.sh output (`<root>/pmc_*`) as markdown: the L2
    memory-side request counters per dispatch of k_segments (known bytes and
    128-B lines), the raw request counters of the streaming probes, and the
    MFMA instruction counters of k_mfma_peak against the probe's own count."""
    out = ["### Reads: k_segments, 2^18 segments per dispatch, one per 4 KiB",
           "", "| segment | policy | bytes | 128-B lines | TCC_EA0_RDREQ | of which 32B | TCC_BUBBLE (128B) | "
           "RDREQ_DRAM | RDREQ per line | FETCH_SIZE x1024 / bytes |", "|---|---|---|---|---|---|---|---|---|---|"]
    for seg in (16, 32, 64, 128, 256, 1024):
        for pol, tag in (("default", ""), ("nt", "nt-")):
            c, pj = _calib_pass(root, f"seg-read-{tag}{seg}_req", "k_segments")
            if not c:
                continue
            f, _ = _calib_pass(root, f"seg-read-{tag}{seg}_fetch", "k_segments")
            lines_, bytes_ = pj.get("lines128_per_dispatch", 0), pj.get("bytes_per_dispatch", 0)
            rd = c.get("TCC_EA0_RDREQ_sum", 0)
            fs = f"{f['FETCH_SIZE'] * 1024 / bytes_:.3f}" if f.get("FETCH_SIZE") and bytes_ else "-"
            out.append(f"| {seg} B | {pol} | {bytes_:,} | {lines_:,} | {rd:,.0f} | {c.get('TCC_EA0_RDREQ_32B_sum', 0):,.0f} | "
                       f"{c.get('TCC_BUBBLE_sum', 0):,.0f} | {c.get('TCC_EA0_RDREQ_DRAM_sum', 0):,.0f} | "
                       f"{rd / lines_ if lines_ else 0:.3f} | {fs} |")
    out += ["", "### Writes: k_segments", "", "| segment | policy | bytes | 128-B lines | TCC_EA0_WRREQ | of which 64B | "
            "WRREQ_DRAM | WRREQ per line | WRITE_SIZE x1024 / bytes |", "|---|---|---|---|---|---|---|---|---|"]
    for seg in (16, 32, 64, 128, 256, 1024):
        for pol, tag in (("default", ""), ("nt", "nt-")):
            c, pj = _calib_pass(root, f"seg-write-{tag}{seg}_req", "k_segments")
            if not c:
                continue
            w, _ = _calib_pass(root, f"seg-write-{tag}{seg}_wsize", "k_segments")
            lines_, bytes_ = pj.get("lines128_per_dispatch", 0), pj.get("bytes_per_dispatch", 0)
            wr = c.get("TCC_EA0_WRREQ_sum", 0)
            ws = f"{w['WRITE_SIZE'] * 1024 / bytes_:.3f}" if w.get("WRITE_SIZE") and bytes_ else "-"
            out.append(f"| {seg} B | {pol} | {bytes_:,} | {lines_:,} | {wr:,.0f} | {c.get('TCC_EA0_WRREQ_64B_sum', 0):,.0f} | "
                       f"{c.get('TCC_EA0_WRREQ_DRAM_sum', 0):,.0f} | {wr / lines_ if lines_ else 0:.3f} | {ws} |")
    out += ["", "### Streaming probes: raw request counters per dispatch", "",
            "| probe | kernel bytes read / written | TCC_EA0_RDREQ | 32B | BUBBLE | read requests x 128 B / bytes read | "
            "TCC_EA0_WRREQ | 64B | write requests x 64 B / bytes written |", "|---|---|---|---|---|---|---|---|---|"]
    for probe in ("hbm-read", "hbm-copy", "hbm-write"):
        r, pj = _calib_pass(root, f"{probe}_req")
        w, _ = _calib_pass(root, f"{probe}_wreq")
        if not (r or w):
            continue
        rb, wb = pj.get("read_bytes", 0), pj.get("write_bytes", 0)
        rd, wr = r.get("TCC_EA0_RDREQ_sum", 0), w.get("TCC_EA0_WRREQ_sum", 0)
        out.append(f"| {probe} | {rb / 2**30:.2f} GiB / {wb / 2**30:.2f} GiB | {rd:,.0f} | "
                   f"{r.get('TCC_EA0_RDREQ_32B_sum', 0):,.0f} | {r.get('TCC_BUBBLE_sum', 0):,.0f} | "
                   f"{rd * 128 / rb if rb else 0:.3f} | {wr:,.0f} | "
                   f"{w.get('TCC_EA0_WRREQ_64B_sum', 0):,.0f} | {wr * 64 / wb if wb else 0:.3f} |")
    c, pj, ns = _calib_pass(root, "mfma_insts", "k_mfma_peak", with_ns=True)
    if c:
        insts, mops = c.get("SQ_INSTS_VALU_MFMA_BF16", 0), c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0)
        want_i, want_f = pj.get("mfma_insts_per_dispatch", 0), pj.get("flops_per_dispatch", 0)
        # Counted FLOPs over the profiler's own dispatch times (the fastest
        # dispatch: the first ones run while the clock ramps).
        t = min(ns) if ns else 0
        out += ["", "### MFMA: k_mfma_peak counters per dispatch vs the probe's own count", "",
                "| SQ_INSTS_VALU_MFMA_BF16 | probe MFMA instructions | ratio | SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 | "
                "probe FLOPs | ratio | SQ_WAVES | fastest dispatch (trace) | counted FLOPs / dispatch time | "
                "probe TFLOP/s (event timing) |", "|---|---|---|---|---|---|---|---|---|---|",
                f"| {insts:,.0f} | {want_i:,} | {insts / want_i if want_i else 0:.4f} | {mops * 512:,.0f} | {want_f:,} | "
                f"{mops * 512 / want_f if want_f else 0:.4f} | {c.get('SQ_WAVES', 0):,.0f} | {t / 1e6:.3f} ms | "
                f"{mops * 512 / t / 1e3 if t else 0:,.1f} TFLOP/s | {pj.get('TFLOPs')} |"]
    return "\n".join(out) + "\n"


def main() -> int:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    root = args[0] if args else "gpurun_out"
    sys.stdout.write(calibration(root) if "--calibration" in sys.argv else summarize(root))
    return 0


if __name__ == "__main__":
    sys.exit(main())
