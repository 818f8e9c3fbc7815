"""CPU placement for a scheduler shard.

A shard is a handful of latency-bound threads (informer, scheduling loop,
Filter/Score helpers, binders) that hand work to each other many thousand
times a second. Left to float over a 256-CPU host they wake on whatever core
is idle, often in another L3 domain or socket, and every hand-off then pays a
cross-CCD cache miss. Pinning the shard to whole L3 domains keeps the
snapshot, queue and listers in one L3.

`pick(mode, rank)`:
  * "none": leave the affinity alone;
  * "l3" / "l3xK": the K (default 1) least-busy L3 domains of the CPUs we may
    use, measured over a short /proc/stat window; ranks on one host take
    disjoint domains in rank order (rank r gets domains [r*K, (r+1)*K) of the
    idle-sorted list), so 8 shards on one 8-GPU node do not collide.
"""
from __future__ import annotations

import glob
import os
import re
import time


def _parse_list(s: str) -> set[int]:
    out: set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def l3_domains(allowed: set[int] | None = None) -> list[list[int]]:
    """CPU lists sharing an L3 cache, restricted to `allowed` (default: the
    process affinity). Falls back to one domain of all allowed CPUs."""
    allowed = set(os.sched_getaffinity(0)) if allowed is None else allowed
    seen: dict[frozenset, None] = {}
    for path in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/cache/index3/shared_cpu_list"):
        try:
            with open(path) as f:
                dom = frozenset(_parse_list(f.read()) & allowed)
        except OSError:
            continue
        if dom:
            seen[dom] = None
    doms = sorted((sorted(d) for d in seen), key=lambda d: d[0])
    return doms or [sorted(allowed)]


def _cpu_busy(window_s: float) -> dict[int, float]:
    def snap() -> dict[int, tuple[int, int]]:
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                m = re.match(r"cpu(\d+)\s+(.*)", line)
                if m:
                    v = [int(x) for x in m.group(2).split()]
                    idle = v[3] + (v[4] if len(v) > 4 else 0)
                    out[int(m.group(1))] = (sum(v), idle)
        return out

    a = snap()
    time.sleep(window_s)
    b = snap()
    busy = {}
    for c, (tot, idle) in b.items():
        t0, i0 = a.get(c, (tot, idle))
        dt = tot - t0
        busy[c] = 1.0 - (idle - i0) / dt if dt > 0 else 0.0
    return busy


def ranked_domains(window_s: float = 0.1) -> list[list[int]]:
    """L3 domains, least busy first (ties by first CPU)."""
    doms = l3_domains()
    try:
        busy = _cpu_busy(window_s)
    except OSError:
        busy = {}
    doms.sort(key=lambda d: (sum(busy.get(c, 0.0) for c in d) / len(d), d[0]))
    return doms


def pick(mode: str, rank: int = 0, window_s: float = 0.1, order: list[list[int]] | None = None) -> list[int] | None:
    """CPUs for this shard under `mode` (see module doc), or None to keep the
    current affinity. `order` is a shared `ranked_domains()` result, so ranks
    of one host that measured at slightly different times still agree."""
    if not mode or mode == "none":
        return None
    m = re.fullmatch(r"l3(?:x(\d+))?", mode)
    if not m:
        return sorted(_parse_list(mode))
    k = int(m.group(1) or 1)
    doms = order if order is not None else ranked_domains(window_s)
    if len(doms) <= 1:
        return None
    start = (rank * k) % len(doms)
    chosen = [c for d in (doms + doms)[start:start + k] for c in d]
    return sorted(chosen)


_original: set[int] | None = None  # the affinity before apply() pinned the shard
_pinned: list[int] | None = None

# Child processes that must not share the shard's CPUs (the service-mode API
# server, load generators) read their CPU list from this variable at start.
CHILD_ENV = "XSCHED_CHILD_CPUS"


def apply(mode: str, rank: int = 0, order: list[list[int]] | None = None) -> list[int] | None:
    """Pin the calling thread (and every thread it creates afterwards, i.e.
    the scheduler's) to `pick(mode, rank)`. Returns the CPU list or None."""
    global _original, _pinned
    cpus = pick(mode, rank, order=order)
    if cpus:
        if _original is None:
            _original = set(os.sched_getaffinity(0))
        os.sched_setaffinity(0, cpus)
        _pinned = cpus
    return cpus


def child_env(env: dict | None = None) -> dict:
    """`env` (default os.environ) plus CHILD_ENV naming the CPUs this process
    could use before its shard was pinned, minus the shard's own CPUs (all of
    them if nothing was pinned or nothing else is left)."""
    out = dict(os.environ if env is None else env)
    if _original and _pinned:
        rest = sorted(_original - set(_pinned)) or sorted(_original)
        out[CHILD_ENV] = ",".join(map(str, rest))
    return out


def adopt_child_cpus() -> None:
    """In a child process: take the CPU list CHILD_ENV names, if any."""
    v = os.environ.get(CHILD_ENV)
    if v:
        try:
            os.sched_setaffinity(0, _parse_list(v))
        except OSError:
            pass
