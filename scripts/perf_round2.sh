#!/usr/bin/env bash
# Scheduler perf evidence on the GPU box: phase profiles (with the
# assume/reserve/permit span), the Score micro-benchmark, the 1-GPU bench
# and the GPU test tier.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 120 python -m flex_gpu_scheduler_amd.tools.phase_profile --waves 8 > "$OUT/phase_$i.json" || exit $?
done
timeout -k 10 300 python -m flex_gpu_scheduler_amd.tools.score_bench --iterations 200 --mi355x > "$OUT/score_bench.json" || exit $?
timeout -k 10 240 python bench.py > "$OUT/bench1.log" 2>&1 || exit $?
tail -1 "$OUT/bench1.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || exit $?
tail -3 "$OUT/pytest_gpu.txt"
