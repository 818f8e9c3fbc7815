#!/usr/bin/env bash
# Probe timing without counters (companion of scripts/pmc_round.sh): each
# streaming probe once plain (its own per-launch event timing, as the node
# agent runs it) and once under --kernel-trace only (the dispatch times the
# counted bytes are divided by in tools/pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUTDIR:-gpurun_out}
mkdir -p "$OUT"
for p in hbm-read hbm-copy hbm-triad hbm-write xcd-read-1 xcd-read-2 xcd-read-4 xcd-read-8 \
         xcd-copy-1 xcd-copy-2 xcd-copy-4 xcd-copy-8; do
  echo "[pmc] plain+trace $p" | tee -a "$OUT/pmc_steps.log"
  timeout -s KILL 60 python3 -m flex_gpu_scheduler_amd.tools.probe_kernels "$p" > "$OUT/plain_$p.log" 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$p" -o trace \
    -- python3 -m flex_gpu_scheduler_amd.tools.probe_kernels "$p" > "$OUT/trace_$p.log" 2>&1 || exit $?
done
