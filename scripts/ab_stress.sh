#!/usr/bin/env bash
# A/B of two native stress binaries (abbin/xsched_stress_{base,new}) on one
# scheduler_perf workload, alternating runs pinned to one idle L3 domain.
# Usage: bash scripts/ab_stress.sh TAG WORKLOAD NODES PODS [RUNS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; wl=$2; nodes=$3; pods=$4; runs=${5:-3}
OUT=gpurun_out/$tag
mkdir -p "$OUT"
dir=/tmp/ab_$wl
if [ "$wl" = bench ]; then  # the headline bench waves; PODS = number of waves
  python -m flex_gpu_scheduler_amd.tools.stress "$dir" --nodes "$nodes" || exit 1
  waves=$pods
else
  python -m flex_gpu_scheduler_amd.tools.stress "$dir" --workload "$wl" --nodes "$nodes" --pods "$pods" || exit 1
  waves=1
fi
cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import ranked_domains; print(','.join(map(str, ranked_domains()[0])))")
echo "cpus=$cpus" | tee "$OUT/ab_${wl}.txt"
for i in $(seq "$runs"); do
  for v in base new; do
    r=$(timeout -k 5 300 taskset -c "$cpus" "abbin/xsched_stress_$v" "$dir" "$waves" 2>&1 | tail -1) || exit 1
    echo "$v $r" | tee -a "$OUT/ab_${wl}.txt"
  done
done
