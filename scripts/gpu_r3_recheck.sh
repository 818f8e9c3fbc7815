#!/usr/bin/env bash
# Re-check of a freshly rebuilt tree on the box: GPU tier, smoke, two default
# bench runs and a rocprofv3 kernel table of the bench. Each GPU step has its
# own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/recheck
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1 || exit $?
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit $?
tail -1 "$OUT/smoke.txt"
for i in 1 2; do
  timeout -k 10 240 python bench.py > "$OUT/bench_$i.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$i.log" | cut -c1-400
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_bench" -o bench -- python3 bench.py --steps 5 --warmup 1 > "$OUT/rocprof_bench.log" 2>&1 || exit $?
echo "recheck done"
