#!/usr/bin/env bash
# A/B of glibc malloc tunables on the native stress driver, pinned to one L3
# domain: per-thread cache for larger blocks (Pods, NodeInfos are 1-4 KiB)
# against the defaults. Usage: bash scripts/ab_malloc.sh <tag> [nodes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
tag=${1:-r2}
n=${2:-64}
timeout -k 10 300 python -m flex_gpu_scheduler_amd.build_ext --stress > "$OUT/${tag}_build.log" 2>&1 || exit $?
cpus=$(python -c "from flex_gpu_scheduler_amd.utils.cpuaffinity import apply; print(','.join(map(str, apply('l3') or [])))")
python -m flex_gpu_scheduler_amd.tools.stress /tmp/xs_$n --nodes "$n" --parallelism 16 || exit $?
waves=40
[ "$n" -ge 512 ] && waves=8
T="glibc.malloc.tcache_max=8192:glibc.malloc.tcache_count=512"
for i in 1 2 3 4; do
  echo "default $(timeout -k 5 200 taskset -c "$cpus" build/xsched_stress /tmp/xs_$n "$waves" 2>&1 | tail -1)" >> "$OUT/${tag}_ab_malloc_$n.txt" || exit $?
  echo "tcache  $(GLIBC_TUNABLES=$T timeout -k 5 200 taskset -c "$cpus" build/xsched_stress /tmp/xs_$n "$waves" 2>&1 | tail -1)" >> "$OUT/${tag}_ab_malloc_$n.txt" || exit $?
done
cat "$OUT/${tag}_ab_malloc_$n.txt"
