#!/usr/bin/env bash
# Scheduler perf evidence on the GPU box's CPUs: phase profile (cache on/off),
# eq-cache A/B bench runs, then the standard 1-GPU bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 120 python -m flex_gpu_scheduler_amd.tools.phase_profile --waves 8 > "$OUT/phase_on.json" || exit $?
timeout -k 10 120 python -m flex_gpu_scheduler_amd.tools.phase_profile --waves 8 --options '{"equivalenceCache": false}' > "$OUT/phase_off.json" || exit $?
for i in 1 2 3; do
  for eq in true false; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-scenarios \
      --sched-options "{\"equivalenceCache\": $eq}" > "$OUT/ab_${eq}_$i.json" 2> "$OUT/ab_${eq}_$i.err" || exit $?
    python -c "import json; d=json.loads(open('$OUT/ab_${eq}_$i.json').read().splitlines()[-1]); print('eq=$eq', d['value'], d['config']['p99_gang_admit_ms'], d['config']['eq_cache_filter_hit_rate'])" | tee -a "$OUT/ab_summary.txt"
  done
done
timeout -k 10 240 python bench.py > "$OUT/bench1.log" 2>&1 || exit $?
tail -1 "$OUT/bench1.log"
