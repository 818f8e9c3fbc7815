#!/usr/bin/env bash
# Round-3 GPU pass: GPU tier (incl. kernel numerics and live placement), the
# default 1-GPU bench, and the hardware-counter passes. Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3a
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 &&
timeout -k 10 300 python -u bench.py > "$OUT/bench1.json" 2> "$OUT/bench1.err" &&
OUTDIR="$OUT" bash scripts/pmc_round.sh
echo "exit=$?"
