#!/usr/bin/env bash
# CPU-sample profile of the scheduling core on the GPU box's host CPUs: the
# native stress driver (no Python in the loop) pinned to one idle L3 domain,
# sampled with csrc/tools/sampler.h, summarized per thread role by
# tools/sample_report.py. Usage: bash scripts/perf_r2.sh <tag> [nodes...]
# Writes gpurun_out/<tag>_stress_<n>.txt and <tag>_samples_<n>.{txt,json}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
tag=${1:-r2}
shift || true
nodes=${*:-64 1024}
timeout -k 10 300 python -m flex_gpu_scheduler_amd.build_ext --stress > "$OUT/${tag}_build.log" 2>&1 || exit $?
cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import apply; print(','.join(map(str, apply('l3') or [])))")
echo "cpus: $cpus" > "$OUT/${tag}_env.txt"
for n in $nodes; do
  python -m flex_gpu_scheduler_amd.tools.stress /tmp/xs_$n --nodes "$n" --parallelism 16 || exit $?
  waves=40
  [ "$n" -ge 512 ] && waves=8
  timeout -k 5 200 taskset -c "$cpus" build/xsched_stress /tmp/xs_$n "$waves" > "$OUT/${tag}_stress_$n.txt" 2>&1 || exit $?
  XSCHED_SAMPLE=/tmp/samples_$n.txt XSCHED_SAMPLE_HZ=5000 timeout -k 5 200 taskset -c "$cpus" build/xsched_stress /tmp/xs_$n "$waves" \
    >> "$OUT/${tag}_stress_$n.txt" 2>&1 || exit $?
  python -m flex_gpu_scheduler_amd.tools.sample_report /tmp/samples_$n.txt --top 40 \
    --json "$OUT/${tag}_samples_$n.json" > "$OUT/${tag}_samples_$n.txt" || exit $?
  grep total "$OUT/${tag}_stress_$n.txt"
done
