#!/usr/bin/env bash
# Three default bench runs on one box: spread of the open-loop capacity and
# of the burst headline. Each run has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/capacity
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > "$OUT/bench_$i.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$i.log" | cut -c1-200
done
echo "capacity done"
