#!/usr/bin/env bash
# Larger clusters (parallel Filter/Score above 128 nodes), default bench, GPU tier.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
for n in 256 1024; do
  timeout -k 10 200 python -c "
import json
from flex_gpu_scheduler_amd.utils.cpuaffinity import apply
cpus = apply('l3')
from flex_gpu_scheduler_amd.tools.phase_profile import profile
r = profile($n, 2, warmup=1); r['cpus'] = len(cpus or []); r['nodes'] = $n
print(json.dumps(r))" > "$OUT/phase_nodes_$n.json" || exit $?
  head -c 400 "$OUT/phase_nodes_$n.json"; echo
done
timeout -k 10 240 python bench.py > "$OUT/bench1.log" 2>&1 || exit $?
tail -1 "$OUT/bench1.log" | cut -c1-300
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || exit $?
tail -1 "$OUT/pytest_gpu.txt"
