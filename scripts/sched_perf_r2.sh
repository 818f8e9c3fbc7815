#!/usr/bin/env bash
# scheduler_perf-style matrix on the GPU box's host CPUs (one L3 domain), at
# 500 nodes / 1,000 pods and 5,000 nodes / 5,000 pods.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
tag=${1:-r2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 500 --pods 1000 --cpus l3 > "$OUT/${tag}_sched_perf_500.jsonl" 2>&1 || exit $?
timeout -k 10 700 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 5000 --cpus l3 > "$OUT/${tag}_sched_perf_5000.jsonl" 2>&1 || exit $?
cat "$OUT/${tag}_sched_perf_500.jsonl" "$OUT/${tag}_sched_perf_5000.jsonl" | cut -c1-200
