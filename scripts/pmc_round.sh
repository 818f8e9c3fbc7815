#!/usr/bin/env bash
# Hardware-counter passes over the HIP probe kernels (one rocprofv3 --pmc run
# per counter group, each under its own SIGKILL timeout; no tracing domains).
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
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/pmc_list_avail.txt" 2>&1 || true
run mfma mfma SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run hbm_read hbm-read FETCH_SIZE GRBM_GUI_ACTIVE &&
run hbm_copy hbm-copy WRITE_SIZE GRBM_GUI_ACTIVE &&
run triad_fetch hbm-triad FETCH_SIZE GRBM_GUI_ACTIVE &&
run triad_write hbm-triad WRITE_SIZE GRBM_GUI_ACTIVE &&
run xcd1_read xcd-read-1 FETCH_SIZE GRBM_GUI_ACTIVE &&
run xcd2_read xcd-read-2 FETCH_SIZE GRBM_GUI_ACTIVE &&
run xcd4_read xcd-read-4 FETCH_SIZE GRBM_GUI_ACTIVE &&
run xcd8_read xcd-read-8 FETCH_SIZE GRBM_GUI_ACTIVE &&
run xcd1_copy xcd-copy-1 WRITE_SIZE GRBM_GUI_ACTIVE
echo "[pmc] done" | tee -a "$OUT/pmc_steps.log"
