#!/usr/bin/env bash
# Hardware-counter passes over the HIP probe kernels (one rocprofv3 --pmc run
# per counter group, each under its own SIGKILL timeout; no tracing domains).
# Every streaming probe gets a FETCH_SIZE pass and, when it writes, a
# WRITE_SIZE pass (the two do not fit one pass: 3 + 2 TCC counters), so
# tools/pmc_summary.py can check the bytes each dispatch moves and compare
# the probe's own median launch time with the dispatch times of the trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUTDIR:-gpurun_out}
mkdir -p "$OUT"
run() {  # name probe counters...
  local name=$1 probe=$2; shift 2
  echo "[pmc] $name: $*" | tee -a "$OUT/pmc_steps.log"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/pmc_$name" -o pmc \
    -- python3 -m flex_gpu_scheduler_amd.tools.probe_kernels "$probe" > "$OUT/pmc_$name.log" 2>&1
  local rc=$?
  echo "[pmc] $name rc=$rc" | tee -a "$OUT/pmc_steps.log"
  return $rc
}
run mfma mfma SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
for p in hbm-read xcd-read-1 xcd-read-2 xcd-read-4 xcd-read-8; do
  run "${p}_fetch" "$p" FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
done
for p in hbm-copy hbm-triad hbm-write xcd-copy-1 xcd-copy-2 xcd-copy-4 xcd-copy-8; do
  run "${p}_fetch" "$p" FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
  run "${p}_write" "$p" WRITE_SIZE GRBM_GUI_ACTIVE || exit $?
done
OUTDIR="$OUT" bash scripts/probe_timing.sh || exit $?
echo "[pmc] done" | tee -a "$OUT/pmc_steps.log"
