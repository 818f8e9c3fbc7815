"""Symbolize and summarize a CPU-sample dump of the native stress driver
(csrc/tools/sampler.h; `XSCHED_SAMPLE=<file> build/xsched_stress <dir> N`).

Samples are wall-clock (every thread, fixed rate). A sample whose stack is
parked in a condition-variable wait or a sleep is idle; the rest are busy
(lock contention counts as busy). Per thread role (xs-sched, xs-bind,
xs-informer, xs-filter, xs-timer, main): busy fraction, and over busy samples
the top functions by self time (leaf frame), by self time with library frames
charged to their caller in our code, and by inclusive time.

    python -m flex_gpu_scheduler_amd.tools.sample_report <dump> [--exe build/xsched_stress] [--top 25] [--json out]
    python -m flex_gpu_scheduler_amd.tools.sample_report <dump> --exe flex_gpu_scheduler_amd/_xsched*.so \
        --timeline 1 [--roles xs-sched,xs-bind,xs-informer]

Dumps from the Python extension (`native().sampler_start/_dump`, used by
scripts/openloop_probe.py --sample-run) carry a timestamp per sample:
`--timeline BIN_MS` prints, per time bin and thread role, the busy share and
the most common first own-code frame of the busy samples (a stall shows as
bins where every role sits in the same lock), and `--window A B` restricts the
summary to [A, B) ms from the first sample.
"""
from __future__ import annotations

import argparse
import bisect
import collections
import json
import re
import subprocess
import sys


class SymbolTable:
    def __init__(self, path: str, dynamic: bool = False):
        args = ["nm", "-C", "-n", "--defined-only"] + (["-D"] if dynamic else []) + [path]
        try:
            out = subprocess.run(args, capture_output=True, text=True, check=False).stdout
        except OSError:
            out = ""
        self.addrs: list[int] = []
        self.names: list[str] = []
        for line in out.splitlines():
            parts = line.split(" ", 2)
            if len(parts) < 3 or parts[1] not in "tTwW":
                continue
            self.addrs.append(int(parts[0], 16))
            self.names.append(parts[2])

    def lookup(self, off: int) -> str | None:
        i = bisect.bisect_right(self.addrs, off) - 1
        return self.names[i] if i >= 0 else None


def short(name: str, width: int = 110) -> str:
    name = re.sub(r"std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> >", "std::string", name)
    name = re.sub(r"\(__gnu_cxx::_Lock_policy\)2", "2", name)
    return name if len(name) <= width else name[: width - 3] + "..."


def load(dump: str, exe: str):
    base = 0
    maps: list[tuple[int, int, int, str]] = []
    samples: list[tuple[str, list[int], int]] = []
    with open(dump) as f:
        for line in f:
            if line.startswith("exe_base "):
                base = int(line.split()[1], 16)
            elif line.startswith("map "):
                m = line.split()
                lo, hi = (int(x, 16) for x in m[1].split("-"))
                maps.append((lo, hi, int(m[3], 16), m[6] if len(m) > 6 else "?"))
            else:
                parts = line.split()
                if len(parts) < 3:
                    continue
                t = 0
                if parts[2].startswith("@"):
                    t = int(parts[2][1:])
                    parts = parts[:2] + parts[3:]
                samples.append((parts[1], [int(x, 16) for x in parts[2:]], t))
    exe_syms = SymbolTable(exe)
    lib_syms: dict[str, SymbolTable] = {}
    cache: dict[int, str] = {}

    def resolve(pc: int) -> str:
        if pc in cache:
            return cache[pc]
        name = None
        for lo, hi, off, path in maps:
            if lo <= pc < hi:
                if path.endswith(exe.split("/")[-1]):
                    # the executable at its load base, or a shared object
                    # (the Python extension) at its mapping
                    name = exe_syms.lookup(pc - lo + off if ".so" in path else pc - base)
                else:
                    tab = lib_syms.get(path)
                    if tab is None:
                        tab = lib_syms[path] = SymbolTable(path, dynamic=True)
                    sym = tab.lookup(pc - lo + off)
                    name = f"{sym or '?'} [{path.split('/')[-1]}]"
                break
        cache[pc] = name or f"?{pc:x}"
        return cache[pc]

    return samples, resolve


IDLE_MARKERS = ("pthread_cond_wait", "pthread_cond_timedwait", "pthread_cond_clockwait",
                "std::condition_variable::wait", "nanosleep", "clock_nanosleep", "std::this_thread::sleep")


def is_idle(frames: list[str]) -> bool:
    return any(f.startswith(IDLE_MARKERS) for f in frames[:6])


def frames_of(pcs: list[int], resolve) -> list[str]:
    # frames[0] is the handler, [1] the signal trampoline; [2] is the interrupted pc.
    return [resolve(pc if i == 2 else pc - 1) for i, pc in enumerate(pcs) if i >= 2]


def timeline(dump: str, exe: str, bin_ms: float, roles: list[str]) -> list[str]:
    samples, resolve = load(dump, exe)
    if not samples:
        return []
    t0 = min(t for _, _, t in samples)
    bins: dict = collections.defaultdict(lambda: collections.defaultdict(list))
    for tname, pcs, t in samples:
        role = re.sub(r"\d+$", "", tname)
        if role in roles:
            bins[int((t - t0) / 1e6 // bin_ms)][role].append(frames_of(pcs, resolve))
    out = []
    for b in sorted(bins):
        cells = []
        for role in roles:
            stacks = bins[b].get(role, [])
            busy = [s for s in stacks if not is_idle(s)]
            own = collections.Counter(next((f for f in s if "[lib" not in f), "?") for s in busy if s)
            leaf = collections.Counter(s[0] for s in busy if s)
            top = own.most_common(1)[0][0] if own else "-"
            lf = leaf.most_common(1)[0][0] if leaf else "-"
            cells.append(f"{role} {len(busy)}/{len(stacks)} {short(top, 60)} <{short(lf, 40)}>")
        out.append(f"{b * bin_ms:8.1f} | " + " | ".join(cells))
    return out


def summarize(dump: str, exe: str, top: int = 25, window: tuple[float, float] | None = None) -> dict:
    samples, resolve = load(dump, exe)
    if window and samples:
        t0 = min(t for _, _, t in samples)
        samples = [s for s in samples if window[0] <= (s[2] - t0) / 1e6 < window[1]]
    by_thread: dict[str, list[list[str]]] = collections.defaultdict(list)
    for tname, pcs, _t in samples:
        # frames[0] is the handler, [1] the signal trampoline; [2] is the interrupted pc.
        frames = [resolve(pc if i == 2 else pc - 1) for i, pc in enumerate(pcs) if i >= 2]
        role = re.sub(r"\d+$", "", tname)
        by_thread[role].append(frames)
    total = sum(len(v) for v in by_thread.values())
    out: dict = {"samples": total, "threads": {}}
    for role, all_stacks in sorted(by_thread.items(), key=lambda kv: -len(kv[1])):
        stacks = [s for s in all_stacks if not is_idle(s)]
        self_c = collections.Counter(s[0] for s in stacks if s)
        # First frame in our own code: charges libc/libstdc++ time (malloc,
        # locks, atomics) to the function that called into it.
        own_c = collections.Counter(next((f for f in s if "[lib" not in f), "?") for s in stacks if s)
        incl_c: collections.Counter = collections.Counter()
        for s in stacks:
            incl_c.update(set(s))
        n = max(1, len(stacks))
        out["threads"][role] = {
            "samples": len(all_stacks),
            "busy": round(len(stacks) / max(1, len(all_stacks)), 4),
            "self": [[round(c / n, 4), short(f)] for f, c in self_c.most_common(top)],
            "self_own_code": [[round(c / n, 4), short(f)] for f, c in own_c.most_common(top)],
            "inclusive": [[round(c / n, 4), short(f)] for f, c in incl_c.most_common(top)],
        }
    return out


def lines(dump: str, exe: str, func: str, top: int = 25) -> list[tuple[float, str]]:
    """Source lines (addr2line on a -g build) of the busy samples whose leaf
    frame is in our code and whose function name contains `func`, as
    fractions of those samples. Works for the stress executable and for the
    Python extension (a shared object: offsets from its mapping)."""
    samples, resolve = load(dump, exe)
    base = 0
    maps: list[tuple[int, int, int, str]] = []
    with open(dump) as f:
        for line in f:
            if line.startswith("exe_base "):
                base = int(line.split()[1], 16)
            elif line.startswith("map "):
                m = line.split()
                lo, hi = (int(x, 16) for x in m[1].split("-"))
                maps.append((lo, hi, int(m[3], 16), m[6] if len(m) > 6 else "?"))
    exe_name = exe.split("/")[-1]

    def file_offset(pc: int) -> int | None:
        for lo, hi, off, path in maps:
            if lo <= pc < hi and path.endswith(exe_name):
                return pc - lo + off if ".so" in path else pc - base
        return None

    offs: collections.Counter = collections.Counter()
    for _tname, pcs, _t in samples:
        if len(pcs) < 3:
            continue
        frames = frames_of(pcs, resolve)
        if not frames or is_idle(frames):
            continue
        if func in frames[0] and "[lib" not in frames[0]:
            o = file_offset(pcs[2])
            if o is not None:
                offs[o] += 1
    addrs = list(offs)
    if not addrs:
        return []
    out = subprocess.run(["addr2line", "-C", "-e", exe, *[hex(a) for a in addrs]], capture_output=True,
                         text=True, check=False).stdout.splitlines()
    by_line: collections.Counter = collections.Counter()
    for a, loc in zip(addrs, out):
        by_line[loc.split(" (")[0]] += offs[a]
    matched = sum(offs.values())  # fractions of the matched function(s)' own samples
    return [(c / max(1, matched), loc) for loc, c in by_line.most_common(top)]


def callers(dump: str, exe: str, func: str, top: int = 25) -> list[tuple[float, str]]:
    """For busy samples whose first frame in our code matches `func`: the
    next frame in our code (who called it), as fractions of those samples."""
    samples, resolve = load(dump, exe)
    by: collections.Counter = collections.Counter()
    for _tname, pcs, _t in samples:
        frames = [resolve(pc if i == 2 else pc - 1) for i, pc in enumerate(pcs) if i >= 2]
        if not frames or is_idle(frames):
            continue
        own = [f for f in frames if "[lib" not in f]
        if len(own) >= 1 and func in own[0]:
            by[short(own[1]) if len(own) > 1 else "?"] += 1
    total = sum(by.values())
    return [(c / max(1, total), f) for f, c in by.most_common(top)]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("dump")
    ap.add_argument("--exe", default="build/xsched_stress")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json", default="")
    ap.add_argument("--lines", default="", help="per source line of the leaf frames in functions matching this")
    ap.add_argument("--callers", default="", help="callers of the functions matching this (first own-code frame)")
    ap.add_argument("--timeline", type=float, default=0.0, help="per-bin view (bin width in ms)")
    ap.add_argument("--roles", default="xs-sched,xs-bind,xs-informer,python")
    ap.add_argument("--window", type=float, nargs=2, default=None, help="summary over [A, B) ms only")
    a = ap.parse_args()
    if a.timeline:
        for line in timeline(a.dump, a.exe, a.timeline, a.roles.split(",")):
            print(line)
        return 0
    if a.callers:
        for frac, f in callers(a.dump, a.exe, a.callers, a.top):
            print(f"{100 * frac:5.1f}%  {f}")
        return 0
    if a.lines:
        for frac, loc in lines(a.dump, a.exe, a.lines, a.top):
            print(f"{100 * frac:5.1f}%  {loc}")
        return 0
    rep = summarize(a.dump, a.exe, a.top, tuple(a.window) if a.window else None)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)
    print(f"samples: {rep['samples']}")
    for role, t in rep["threads"].items():
        print(f"\n== {role}: {t['samples']} samples, {100 * t['busy']:.1f}% busy (profiles below: busy samples)")
        print("  self:")
        for frac, f in t["self"]:
            print(f"    {100 * frac:5.1f}%  {f}")
        print("  self, library time charged to its caller in our code:")
        for frac, f in t["self_own_code"]:
            print(f"    {100 * frac:5.1f}%  {f}")
        print("  inclusive:")
        for frac, f in t["inclusive"]:
            print(f"    {100 * frac:5.1f}%  {f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
