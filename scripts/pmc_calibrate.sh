#!/usr/bin/env bash
# Calibrate the L2 memory-side request counters that FETCH_SIZE / WRITE_SIZE
# are built from, on kernels of known request count (k_segments: 2^18
# segments of SEG bytes, one per 4 KiB slot, so every dispatch moves
# 2^18 x SEG bytes in 2^18 x ceil(SEG/128) lines), then read the raw
# request counters of the streaming probes and the MFMA instruction counters
# of the MFMA probe. One rocprofv3 --pmc run per counter group, each under
# its own SIGKILL timeout, no tracing domains; at most 4 TCC counters a pass.
# tools/pmc_summary.py --calibration renders the result.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUTDIR:-gpurun_out}/calib
mkdir -p "$OUT"
run() {  # name probe counters...
  local name=$1 probe=$2; shift 2
  echo "[calib] $name: $*" | tee -a "$OUT/steps.log"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/pmc_$name" -o pmc \
    -- python3 -m flex_gpu_scheduler_amd.tools.probe_kernels "$probe" 0 5 > "$OUT/pmc_$name.log" 2>&1
  local rc=$?
  echo "[calib] $name rc=$rc" | tee -a "$OUT/steps.log"
  return $rc
}
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum"
WR="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum"
for seg in 16 32 64 128 256 1024; do
  run "seg-read-${seg}_req" "seg-read-$seg" $RD || exit $?
  run "seg-read-${seg}_fetch" "seg-read-$seg" FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
  run "seg-write-${seg}_req" "seg-write-$seg" $WR || exit $?
  run "seg-write-${seg}_wsize" "seg-write-$seg" WRITE_SIZE GRBM_GUI_ACTIVE || exit $?
done
for seg in 128 1024; do
  run "seg-read-nt-${seg}_req" "seg-read-nt-$seg" $RD || exit $?
  run "seg-write-nt-${seg}_req" "seg-write-nt-$seg" $WR || exit $?
done
for p in hbm-read hbm-copy hbm-write; do
  run "${p}_req" "$p" $RD || exit $?
  run "${p}_wreq" "$p" $WR || exit $?
done
run mfma_insts mfma SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVES GRBM_GUI_ACTIVE || exit $?
echo "[calib] done" | tee -a "$OUT/steps.log"
