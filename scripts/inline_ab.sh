#!/usr/bin/env bash
# Filter/Score on the scheduling thread vs the parallelizer at 256/1024 nodes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
for n in 256 1024; do
  for inl in 128 1000000; do  # 128 = default (cost model decides above it)
    timeout -k 10 200 python -c "
import json
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply
apply('l3')
from flex_gpu_scheduler_amd.tools.phase_profile import profile
r = profile($n, 2, warmup=1, options={'parallelInlineBelow': $inl})
print(json.dumps({'nodes': $n, 'inline_below': $inl, 'pods_per_s': r['pods_per_s'], 'filter_us': r['phases_us_per_pod']['filter'], 'schedule_us': r['phases_us_per_pod']['schedule']}))" >> "$OUT/inline_ab2.txt" || exit $?
  done
done
cat "$OUT/inline_ab2.txt"
