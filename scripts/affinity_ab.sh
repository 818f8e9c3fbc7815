#!/usr/bin/env bash
# A/B of shard CPU placement (utils/cpuaffinity.py) on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
S="$OUT/affinity_ab.txt"
python -c "
from flex_gpu_scheduler_amd.utils import cpuaffinity as c
d = c.l3_domains(); print('l3 domains', len(d), 'sizes', sorted({len(x) for x in d}), 'first', d[0])
print('pick l3', c.pick('l3')); print('pick l3x2', c.pick('l3x2'))" > "$S" 2>&1 || exit $?
for i in 1 2 3; do
  for mode in none l3 l3x2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-scenarios --cpus $mode > "$OUT/aff_${mode}_$i.json" 2>/dev/null || exit $?
    python -c "import json; d=json.loads(open('$OUT/aff_${mode}_$i.json').read().splitlines()[-1]); print('$mode', d['value'], d['config']['p99_gang_admit_ms'], d['config'].get('cpus'))" >> "$S"
  done
done
cat "$S"
