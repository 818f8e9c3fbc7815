#!/usr/bin/env bash
# A/B of the probes' clock warm-up (XS_PROBE_WARM_MS=0 vs the default), each
# probe in a fresh process, variants alternating. Usage: probe_warm_ab.sh OUT
set -euo pipefail
out=${1:-gpurun_out/probe_warm_ab.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
export PYTHONPATH=.
for rep in 1 2; do
  for p in hbm-read hbm-copy hbm-triad hbm-write xcd-read-1 xcd-read-8 mfma; do
    for warm in 0 20; do
      line=$(XS_PROBE_WARM_MS=$warm timeout -k 10 60 python -m flex_gpu_scheduler_amd.tools.probe_kernels "$p" 0 20 | tail -n 1)
      echo "{\"rep\": $rep, \"warm_ms\": $warm, \"probe\": \"$p\", \"r\": $line}" | tee -a "$out"
    done
  done
done
