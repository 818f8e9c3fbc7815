"""Per-millisecond activity of a scheduler Chrome trace (Scheduler set_trace):
events and busy time per phase in 1 ms bins, plus the longest events of each
phase. Used to find what stalls the binding cycles in an open-loop run
(scripts/openloop_probe.py --trace-run K).

Usage: python scripts/trace_bins.py trace.json [--bin-us 1000] [--top 12]
"""
import argparse
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bin-us", type=float, default=1000.0)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    with open(a.trace) as f:
        evs = json.load(f)
    if isinstance(evs, dict):
        evs = evs.get("traceEvents", [])
    t0 = min(float(e["ts"]) for e in evs)
    bins = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    by_name = defaultdict(list)
    for e in evs:
        s, d = float(e["ts"]) - t0, float(e.get("dur", 0))
        b = int(s // a.bin_us)
        c = bins[b][e["name"]]
        c[0] += 1
        c[1] += d
        by_name[e["name"]].append((d, s, e.get("args", {}).get("pod", e.get("args", {})), e.get("args", {})))
    names = sorted(by_name)
    print("bin_ms " + " ".join(f"{n}(n,ms)" for n in names))
    for b in range(max(bins) + 1):
        row = bins.get(b, {})
        print(f"{b * a.bin_us / 1000:7.1f} " + " ".join(
            f"{row[n][0]},{row[n][1] / 1000:.1f}" if n in row else "0,0" for n in names))
    for n in names:
        top = sorted(by_name[n], key=lambda x: -x[0])[:a.top]
        print(f"\nlongest {n}:")
        for d, s, pod, args in top:
            print(f"  {d / 1000:8.3f} ms at {s / 1000:8.3f} ms  {json.dumps(args)[:160]}")


if __name__ == "__main__":
    main()
