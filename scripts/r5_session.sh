#!/usr/bin/env bash
# One GPU-box session: the GPU test tier, the 5,000-node preemption rows, the
# counter calibration and the probe counter passes. Each step runs under its
# own time limit; a test failure does not stop the later steps, but a crash,
# abort or time limit (124/134/137/139) ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUTDIR:-gpurun_out/r5}
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac; }
step() {  # name limit command...
  local name=$1 limit=$2; shift 2
  echo "[session] $name start $(date +%T)" | tee -a "$OUT/session.log"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc $(date +%T)" | tee -a "$OUT/session.log"
  if fatal $rc; then echo "[session] stopping after $name" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}
for s in ${STEPS:-pytest sched5000 calib pmc}; do
  case $s in
    pytest) step pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    sched5000) step sched_perf_5000 500 python -u -m flex_gpu_scheduler_amd.tools.sched_perf --nodes 5000 --pods 5000 \
                 --only PreemptionBasic CapacityScheduling-Reclaim --cpus l3 ;;
    calib) OUTDIR="$OUT" step calib 500 bash scripts/pmc_calibrate.sh ;;
    pmc) OUTDIR="$OUT" step pmc 450 bash scripts/pmc_round.sh ;;
    bench) step bench 600 python -u bench.py --steps 20 --warmup 3 ;;
  esac
done
echo "[session] done" | tee -a "$OUT/session.log"
