#!/usr/bin/env bash
# One GPU-box session: gpu tests, 1-GPU bench, rocprofv3 kernel stats of the
# HIP probes and of the bench. Every GPU step has its own time limit; after a
# fault / abort / timeout nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[gpu_round] $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[gpu_round] $name rc=$rc" | tee -a "$OUT/steps.log"
  case $rc in
    0|1) return 0 ;;               # pass / test failures: keep going
    *) echo "[gpu_round] stopping after rc=$rc" | tee -a "$OUT/steps.log"; exit $rc ;;
  esac
}
step pytest_gpu 420 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step agent_check 120 python -m flex_gpu_scheduler_amd.tools.agent_check
step bench1 240 python bench.py
step probe_sweep 120 python -m flex_gpu_scheduler_amd.tools.probe_bench
step rocprof_probe 180 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_probe" -o probe -- python3 -m flex_gpu_scheduler_amd.tools.probe_bench
step rocprof_bench 200 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_bench" -o bench -- python3 bench.py --steps 5 --warmup 1
echo "[gpu_round] done" | tee -a "$OUT/steps.log"
