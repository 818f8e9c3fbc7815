#!/usr/bin/env bash
# Service-mode throughput on the GPU box's host CPUs (scheduler and API
# server in separate processes over HTTP): native REST IO vs the Python
# mirror/writer, plain pods and 8-rank gangs. Usage: bash scripts/remote_bench_r2.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
tag=${1:-r2}
mkdir -p "$OUT"
f="$OUT/${tag}_remote_bench.jsonl"
: > "$f"
for io in "" "--python-io"; do
  timeout -k 10 200 python -m flex_gpu_scheduler_amd.tools.remote_bench --pods 4000 $io >> "$f" 2>/dev/null || exit $?
  timeout -k 10 200 python -m flex_gpu_scheduler_amd.tools.remote_bench --pods 512 --gangs $io >> "$f" 2>/dev/null || exit $?
done
cut -c1-240 "$f"
