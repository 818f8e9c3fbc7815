"""Headline bench waves under the timestamped sampler, as bench.py runs them
(Python Shard.run: chunked creates, wait for binds, delete, cache drain).

    python scripts/sample_bench_waves.py OUTDIR [--nodes 64] [--waves 40]

Writes OUTDIR/bench_waves.samples (symbolize against the extension .so) and
OUTDIR/bench_waves_split.json (per-wave create / to_bound / delete_drain ms).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from flex_gpu_scheduler_amd._native import native  # noqa: E402
from flex_gpu_scheduler_amd.utils.benchrun import Shard  # noqa: E402
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply  # noqa: E402
from flex_gpu_scheduler_amd.utils.workload import ClusterSpec  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--waves", type=int, default=40)
    ap.add_argument("--hz", type=int, default=4000)
    ap.add_argument("--colocation", default="Preferred", help="NRT gangColocation of the flagship profile")
    ap.add_argument("--tag", default="bench_waves")
    ap.add_argument("--pin", default="l3", help="shard CPU placement (utils/cpuaffinity.py): l3 | l3x2 | none")
    ap.add_argument("--options", default="{}", help="scheduler options JSON, e.g. '{\"bindWorkers\": 8}'")
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    apply(a.pin)
    from flex_gpu_scheduler_amd.utils.workload import flagship_config

    shard = Shard(ClusterSpec(nodes=a.nodes), namespace="sample", seed=a.seed, options=json.loads(a.options),
                  config=flagship_config(gang_colocation=a.colocation))
    try:
        ws = [shard.wave(i) for i in range(a.waves + 4)]
        prepared = [w.chunks_json() for w in ws]
        for i in range(4):
            shard.run(ws[i], prepared=prepared[i], collect_gangs=False)
        native().sampler_start(a.hz, 4_000_000)
        split = []
        for i in range(4, a.waves + 4):
            r = shard.run(ws[i], prepared=prepared[i], collect_gangs=False)
            split.append({k: round(v, 3) for k, v in r.split_ms.items()})
        native().sampler_dump(os.path.join(a.out, f"{a.tag}.samples"))
    finally:
        shard.close()
    tot = {k: round(sum(s[k] for s in split) / len(split), 3) for k in split[0]}
    with open(os.path.join(a.out, f"{a.tag}_split.json"), "w") as f:
        json.dump({"nodes": a.nodes, "waves": a.waves, "mean_ms": tot, "per_wave": split}, f)
    print(json.dumps({"nodes": a.nodes, "waves": a.waves, "mean_ms": tot}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
