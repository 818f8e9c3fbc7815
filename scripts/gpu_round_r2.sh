#!/usr/bin/env bash
# Round-2 GPU-box session: GPU test tier, smoke(), 1-GPU bench with the
# BASELINE scenarios, amd-smi probe, rocprofv3 kernel stats of the HIP probes
# and of the bench. Each GPU step has its own time limit; after a fault,
# abort or timeout nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
tag=${1:-r2}
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[gpu_round] $name: $*" | tee -a "$OUT/${tag}_steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/${tag}_$name.log" 2>&1
  local rc=$?
  echo "[gpu_round] $name rc=$rc" | tee -a "$OUT/${tag}_steps.log"
  case $rc in
    0|1) return 0 ;;
    *) echo "[gpu_round] stopping after rc=$rc" | tee -a "$OUT/${tag}_steps.log"; exit $rc ;;
  esac
}
step pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 240 python bench.py
step amdsmi_probe 120 python -m flex_gpu_scheduler_amd.tools.amdsmi_probe --seconds 2
step rocprof_probe 180 rocprofv3 --kernel-trace --stats -d "$OUT/${tag}_rocprof_probe" -o probe -- python3 -m flex_gpu_scheduler_amd.tools.probe_bench
step rocprof_bench 200 rocprofv3 --kernel-trace --stats -d "$OUT/${tag}_rocprof_bench" -o bench -- python3 bench.py --steps 5 --warmup 1
echo "[gpu_round] done" | tee -a "$OUT/${tag}_steps.log"
