#!/usr/bin/env bash
# Scheduling-thread timeline (pinned), GPU test tier, smoke, default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 120 python -m flex_gpu_scheduler_amd.tools.timeline > "$OUT/timeline_$i.json" || exit $?
done
cat "$OUT/timeline_1.json"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || exit $?
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit $?
tail -1 "$OUT/smoke.txt"
timeout -k 10 240 python bench.py > "$OUT/bench1.log" 2>&1 || exit $?
tail -1 "$OUT/bench1.log" | cut -c1-300
