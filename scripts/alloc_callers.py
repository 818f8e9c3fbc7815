"""Who allocates on one thread of a sampler dump: for busy samples with
malloc / operator new / free in the top frames, the first own-code frame.

    python scripts/alloc_callers.py DUMP EXE THREAD
"""
import collections, sys
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), ".."))
from flex_gpu_scheduler_amd.tools.sample_report import load, is_idle, short
samples, resolve = load(sys.argv[1], sys.argv[2])
by = collections.Counter(); tot = 0; busy = 0
for tname, pcs, _t in samples:
    if tname != sys.argv[3]:
        continue
    frames = [resolve(pc if i == 2 else pc - 1) for i, pc in enumerate(pcs) if i >= 2]
    if not frames or is_idle(frames):
        continue
    busy += 1
    if not any(("malloc" in f or "operator new" in f or "morecore" in f or "free@" in f) for f in frames[:4]):
        continue
    tot += 1
    own = [f for f in frames if "[lib" not in f and "operator new" not in f]
    by[short(own[0]) if own else "?"] += 1
print(f"alloc samples {tot} of {busy} busy ({tot/max(1,busy):.1%})")
for f, c in by.most_common(30):
    print(f"{c/max(1,tot):6.1%}  {f[:150]}")
