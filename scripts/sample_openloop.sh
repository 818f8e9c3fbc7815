#!/usr/bin/env bash
# Open-loop arrivals (tools/stress.py --openloop RATE) on the native stress
# driver under the wall-clock thread sampler, pinned to one idle L3 domain.
# Usage: bash scripts/sample_openloop.sh TAG RATE [SECONDS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; rate=$2; secs=${3:-1}
OUT=gpurun_out/$tag
mkdir -p "$OUT"
python -m flex_gpu_scheduler_amd.tools.stress /tmp/s_ol --nodes 64 --openloop "$rate" --seconds "$secs" || exit 1
cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))")
XSCHED_SAMPLE_HZ=2000 XSCHED_SAMPLE="$OUT/openloop_$rate.samples" timeout -k 5 120 taskset -c "$cpus" \
  abbin/xsched_stress_prof /tmp/s_ol > "$OUT/openloop_$rate.run.txt" 2>&1
echo "rc=$?" >> "$OUT/openloop_$rate.run.txt"
