#!/usr/bin/env bash
# Host-only sanitizer runs of the native stress driver (no GPU code):
# ThreadSanitizer and AddressSanitizer+UBSan builds over the bench waves and
# the scheduler_perf shapes that exercise preemption, topology spreading and
# inter-pod affinity. Usage: bash scripts/sanitizers.sh OUTFILE
set -u
cd "$(dirname "$0")/.."
out=${1:-profiles/r3_sanitizers.txt}
python -m flex_gpu_scheduler_amd.build_ext --tsan > /dev/null || exit 1
python -m flex_gpu_scheduler_amd.build_ext --asan > /dev/null || exit 1
export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0"
export ASAN_OPTIONS="detect_leaks=1 halt_on_error=0" UBSAN_OPTIONS="print_stacktrace=1 halt_on_error=0"
python -m flex_gpu_scheduler_amd.tools.stress /tmp/san_bench --nodes 64 > /dev/null || exit 1
: > "$out"
run() {  # name dir waves
  for s in tsan asan; do
    log=/tmp/san_${s}_$1.log
    timeout -k 10 1200 "build/xsched_stress_$s" "$2" "$3" > "$log" 2>&1
    rc=$?
    if [ "$s" = tsan ]; then n=$(grep -c "WARNING: ThreadSanitizer" "$log"); else
      n=$(grep -c "ERROR: AddressSanitizer\|runtime error:\|ERROR: LeakSanitizer" "$log"); fi
    echo "$s  $1  rc=$rc  reports=$n  $(tail -1 "$log")" | tee -a "$out"
  done
}
run bench64 /tmp/san_bench 3
# The 1,024-node headline waves: gang window, Filter scan memo, column
# equivalence table, snapshot arrays (one wave of 12k pods).
python -m flex_gpu_scheduler_amd.tools.stress /tmp/san_1024 --nodes 1024 > /dev/null || exit 1
run n1024 /tmp/san_1024 1
run apiserver apiserver 4   # native HTTP API server: 4 REST clients, 2 watch streams, mirror, stop
# Open-loop arrivals: gangs created and deleted one by one while they are
# scheduled (run_open_loop, batched gang deletion, gang-record cleanup).
python -m flex_gpu_scheduler_amd.tools.stress /tmp/san_ol --nodes 16 --openloop 2000 --seconds 0.5 > /dev/null || exit 1
run openloop /tmp/san_ol 1
for spec in "PreemptionBasic 200 400" "SchedulingBasic 500 1000" "TopologySpreading 300 600" \
            "SchedulingPodAntiAffinity 300 300" "Unschedulable 300 600" "MI355X-Gang8 200 800" "MI355X-FlexGPUMix 200 800" \
            "CapacityScheduling-Reclaim 300 300"; do
  set -- $spec
  python -m flex_gpu_scheduler_amd.tools.stress "/tmp/san_$1" --workload "$1" --nodes "$2" --pods "$3" > /dev/null \
    || { echo "skip $1 (no such workload)" | tee -a "$out"; continue; }
  run "$1_$2" "/tmp/san_$1" 1
done
