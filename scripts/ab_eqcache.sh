#!/usr/bin/env bash
# A/B of the scheduler equivalence cache on the GPU box's CPUs (bench.py, 1 rank).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for eq in true false; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-scenarios \
      --sched-options "{\"equivalenceCache\": $eq}" > gpurun_out/ab_${eq}_$i.json 2> gpurun_out/ab_${eq}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${eq}_$i.json').read().splitlines()[-1]); print('eq=$eq', d['value'], d['config']['p99_gang_admit_ms'], d['config']['eq_cache_filter_hit_rate'])" | tee -a gpurun_out/ab_summary.txt
  done
done
nproc >> gpurun_out/ab_summary.txt
