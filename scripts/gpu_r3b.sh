#!/usr/bin/env bash
# Probe timing investigation: event-timed bandwidth vs. iteration count, and
# kernel-trace durations of the same launches; the new per-XCD k_pinned.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3b
mkdir -p "$OUT"
for it in 5 20 100; do
  for p in hbm-read hbm-copy hbm-triad xcd-read-1 xcd-read-8 xcd-copy-1; do
    timeout -k 5 60 python -m flex_gpu_scheduler_amd.tools.probe_kernels $p 0 $it >> "$OUT/iters.jsonl" 2>> "$OUT/iters.err" || { echo "fail $p $it"; exit 1; }
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace_read" -o tr -- python3 -m flex_gpu_scheduler_amd.tools.probe_kernels hbm-read 0 20 > "$OUT/trace_read.log" 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace_xcd8" -o tr -- python3 -m flex_gpu_scheduler_amd.tools.probe_kernels xcd-read-8 0 20 > "$OUT/trace_xcd8.log" 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k pinned > "$OUT/pytest_pinned.txt" 2>&1
echo "exit=$?"
