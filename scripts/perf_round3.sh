#!/usr/bin/env bash
# Default 1-GPU bench (L3-pinned shard) x2, pinned phase profile and score bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 240 python bench.py > "$OUT/bench_pinned_$i.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_pinned_$i.log" | cut -c1-420
done
timeout -k 10 120 python -c "
import json, os
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply
cpus = apply('l3')
from flex_gpu_scheduler_amd.tools.phase_profile import profile
r = profile(64, 8); r['cpus'] = cpus
print(json.dumps(r))" > "$OUT/phase_pinned.json" || exit $?
cat "$OUT/phase_pinned.json"
