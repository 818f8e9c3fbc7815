#!/usr/bin/env bash
# Scheduler-core throughput sweep on the GPU box's CPUs (native stress driver,
# no Python in the loop): Filter/Score inline threshold, parallelism and bind
# workers. Usage: bash scripts/perf_sweep.sh  (writes gpurun_out/perf_sweep.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
timeout -k 10 300 python -m flex_gpu_scheduler_amd.build_ext --stress > "$OUT/perf_build.log" 2>&1 || exit $?
python -m flex_gpu_scheduler_amd.tools.stress /tmp/xs_stress_in --parallelism 16 || exit $?
nproc > "$OUT/perf_sweep.txt"
for opt in "parallelInlineBelow=128" "parallelInlineBelow=32" "parallelInlineBelow=16" "parallelism=8" "bindWorkers=4" "bindWorkers=32"; do
  k=${opt%%=*}; v=${opt##*=}
  python - "$k" "$v" <<'PY'
import json, sys
p = "/tmp/xs_stress_in/config.json"
c = json.load(open(p))
o = c.setdefault("options", {})
for key in ("parallelInlineBelow", "parallelism", "bindWorkers"):
    o.pop(key, None)
o["parallelism"] = 16
o[sys.argv[1]] = int(sys.argv[2])
json.dump(c, open(p, "w"))
PY
  for i in 1 2 3; do
    echo "$opt $(timeout -k 5 120 build/xsched_stress /tmp/xs_stress_in 12 2>&1 | tail -1)" >> "$OUT/perf_sweep.txt" || exit $?
  done
done
