#!/usr/bin/env bash
# What CPU budget does a GPU-box command get? cgroup quota, throttling during
# bench runs, and bench variance.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
{
  echo "nproc=$(nproc) affinity=$(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
  cat /proc/self/cgroup
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpuset.cpus.effective; do echo "== $f"; cat "$f" 2>/dev/null; done
  uptime
} > "$OUT/cpu_env.txt" 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-scenarios > "$OUT/var_$i.json" 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('$OUT/var_$i.json').read().splitlines()[-1]); print('run $i', d['value'], d['config']['p99_gang_admit_ms'])" >> "$OUT/cpu_env.txt"
  echo "== cpu.stat after run $i" >> "$OUT/cpu_env.txt"; cat /sys/fs/cgroup/cpu.stat >> "$OUT/cpu_env.txt" 2>/dev/null
done
cat "$OUT/cpu_env.txt"
