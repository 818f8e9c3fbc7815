"""Per-wave timeline of a scheduler Chrome trace (`bench.py --trace FILE`).

Waves are told apart by the gap in scheduling cycles while a wave is deleted
and drained (no cycle for >= --gap-us). For each wave it prints the
scheduling thread's busy time inside the wave's span, the informer's busy
time, the binder's, and the idle stretches of the scheduling thread: before
its first cycle (waiting for the first pods), inside the wave, and after its
last cycle (binding tail, deletion, drain).

Usage: python scripts/trace_timeline.py trace.json [--gap-us 400]
"""
import argparse
import json


def merge(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def busy_in(iv, lo, hi):
    return sum(max(0, min(e, hi) - max(s, lo)) for s, e in iv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=400.0)
    a = ap.parse_args()
    with open(a.trace) as f:
        evs = json.load(f)
    if isinstance(evs, dict):
        evs = evs.get("traceEvents", [])
    sched, inf, bind = [], [], []
    for e in evs:
        s, d = float(e["ts"]), float(e.get("dur", 0))
        if e["name"] in ("schedule", "assume_reserve_permit", "cycle_setup", "snapshot"):
            sched.append((s, s + d))
        elif e["name"] == "informer_batch":
            inf.append((s, s + d))
        elif e["name"] == "bind":
            bind.append((s, s + d))
    sched, inf, bind = merge(sched), merge(inf), merge(bind)
    waves, cur = [], [sched[0]]
    for iv in sched[1:]:
        if iv[0] - cur[-1][1] >= a.gap_us:
            waves.append(cur)
            cur = []
        cur.append(iv)
    waves.append(cur)
    print(f"{len(waves)} waves, {len(sched)} sched intervals, {len(inf)} informer batches, {len(bind)} binds")
    for i, w in enumerate(waves):
        lo, hi = w[0][0], w[-1][1]
        nxt = waves[i + 1][0][0] if i + 1 < len(waves) else None
        s_busy = sum(e - s for s, e in w)
        print(f"wave {i}: sched span {hi - lo:7.0f} us, sched busy {s_busy:7.0f} us ({s_busy / max(1, hi - lo):.0%}), "
              f"informer busy in span {busy_in(inf, lo, hi):6.0f} us, bind busy {busy_in(bind, lo, hi):6.0f} us"
              + (f", gap to next wave {nxt - hi:6.0f} us (informer busy {busy_in(inf, hi, nxt):5.0f}, "
                 f"bind {busy_in(bind, hi, nxt):5.0f})" if nxt else ""))


if __name__ == "__main__":
    main()
