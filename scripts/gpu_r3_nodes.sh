#!/usr/bin/env bash
# Headline workload on larger clusters (one shard): 256 and 1,024 nodes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/nodes
mkdir -p "$OUT"
for n in 256 1024; do
  timeout -k 10 300 python bench.py --nodes $n --steps 10 --warmup 2 --no-scenarios > "$OUT/bench_$n.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$n.log" | cut -c1-200
done
echo "nodes done"
